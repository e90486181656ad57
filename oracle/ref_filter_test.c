/*
 * ref_filter_test.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The reference's own filter tests, run unmodified on either implementation: this unit
 * #includes vmware/splinterdb tests/functional/filter_test.c exactly as it lies under
 * /root/reference (nothing is copied) and exports its two static test bodies,
 *
 *   test_filter_basic  (filter_test.c:22-148): num_values incremental routing_filter_add
 *                      calls, estimate_unique_keys per step, estimate_unique_fp across the
 *                      chain, every inserted key looked up, false positives of unused keys
 *   test_filter_perf   (filter_test.c:150-273): num_trees chains of num_values adds, then
 *                      positive and negative lookups of every key
 *
 * on the page stack of ref_harness.c (its clockcache, rc_allocator and in-memory device).
 * oracle/Makefile links this unit twice: with the reference's src/routing_filter.c
 * (_ref/libfilter_test_ref.so) and with shim/routing_filter_amd.c in its place
 * (_ref/libfilter_test_shim.so). filter_test() itself -- argument parsing, laio device,
 * task system -- needs sources this image cannot build (libaio) and is never called: it is
 * renamed below and dropped by the linker (--gc-sections, only rfr_* exported).
 */
#define filter_test unused_filter_test_driver
#include "filter_test.c"
#undef filter_test

/* the stack's pieces and its log redirection (ref_harness.c; this unit may not use stdio:
   filter_test.c includes poison.h) */
typedef struct rfr_stack rfr_stack;
cache            *rfr_cache(rfr_stack *s);
routing_config   *rfr_routing_config(rfr_stack *s);
platform_heap_id  rfr_heap(rfr_stack *s);
int               rfr_log_begin(const char *log_path);
void              rfr_log_end(void);

int
rfr_filter_test_basic(rfr_stack  *s,
                      uint64      key_size,
                      uint64      num_fingerprints,
                      uint64      num_values,
                      const char *log_path)
{
   if (rfr_log_begin(log_path)) {
      return -1;
   }
   platform_status rc = test_filter_basic(
      rfr_cache(s), rfr_routing_config(s), rfr_heap(s), key_size, num_fingerprints, num_values);
   rfr_log_end();
   return rc.r;
}

int
rfr_filter_test_perf(rfr_stack  *s,
                     uint64      key_size,
                     uint64      num_fingerprints,
                     uint64      num_values,
                     uint64      num_trees,
                     const char *log_path)
{
   if (rfr_log_begin(log_path)) {
      return -1;
   }
   platform_status rc = test_filter_perf(rfr_cache(s),
                                         rfr_routing_config(s),
                                         rfr_heap(s),
                                         key_size,
                                         num_fingerprints,
                                         num_values,
                                         num_trees);
   rfr_log_end();
   return rc.r;
}
