/*
 * ref_kvs.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The reference's whole key-value store as the caller of the routing filter: splinterdb.c,
 * core.c, trunk.c, btree.c, memtable.c and the rest of vmware/splinterdb src/, compiled
 * unmodified from /root/reference by oracle/Makefile, once with the reference's
 * routing_filter.c (_ref/libkvs_ref.so) and once with the drop-in shim/routing_filter_amd.c
 * in its place (_ref/libkvs_shim.so). The storage device is ref_harness.c's in-memory device
 * (io_handle_create below replaces platform_io.c, which needs libaio).
 *
 * Inserts through splinterdb_insert flush memtables into the trunk, whose compactions build
 * maplets through maplet_compaction_task -> routing_filter_add (src/trunk.c:3780-3927);
 * splinterdb_lookup reaches routing_filter_lookup through trunk_ondisk_bundle_merge_lookup
 * (src/trunk.c:6008-6110), core_lookup_async reaches routing_filter_lookup_async (:6136).
 * The link wraps routing_filter_add / _lookup / _lookup_async (-Wl,--wrap) to record every
 * filter the trunk builds -- descriptor, and an XXH64 of its index slots and data pages read
 * back through the cache -- and to count the filter lookups, so the two stacks can be
 * compared call for call. Background threads are off (tasks run on the inserting thread), so
 * both stacks issue the same calls in the same order.
 */
#define _GNU_SOURCE
#include "platform.h"
#include "splinterdb/splinterdb.h"
#include "splinterdb/default_data_config.h"
#include "splinterdb_tests_private.h"
#include "routing_filter.h"
#include "core.h"
#include "lookup_result.h"
#include "clockcache.h"

#include <stdatomic.h>
#include <time.h>
#include <xxhash.h>

/* ---- recording wrappers ------------------------------------------------------------- */
typedef struct rfk_add_rec {
   uint64 old_addr, num_new, value, rc;
   uint64 addr, meta_head, num_fingerprints, num_unique, value_size;
   uint64 digest; /* XXH64 over the index slots and every data page */
} rfk_add_rec;

static rfk_add_rec   *g_adds;
static uint64         g_nadds, g_cap_adds;
static _Atomic uint64 g_nlookups, g_nlookups_async;
static pthread_mutex_t g_rec_mu = PTHREAD_MUTEX_INITIALIZER;
static int             g_record_digest = 1;

platform_status
__real_routing_filter_add(cache                *cc,
                          const routing_config *cfg,
                          routing_filter       *old_filter,
                          routing_filter       *filter,
                          uint32               *new_fp_arr,
                          uint64                num_new_fp,
                          uint16                value);
platform_status
__real_routing_filter_lookup(cache                *cc,
                             const routing_config *cfg,
                             routing_filter       *filter,
                             key                   target,
                             uint64               *found_values);
async_status
__real_routing_filter_lookup_async(routing_filter_lookup_async_state *state);

/* the filter's bytes as the cache holds them: its index slots (absolute page addresses, the
 * allocation order included) and each distinct data page once, in slot order */
static uint64
filter_digest(cache *cc, const routing_config *cfg, const routing_filter *f)
{
   if (f->addr == 0) {
      return 0;
   }
   const uint64 ps  = cache_config_page_size(cfg->cache_cfg);
   const uint64 app = ps / sizeof(uint64);
   const uint32 lnb = 31 - __builtin_clz(f->num_fingerprints);
   const uint32 lb  = lnb > cfg->log_index_size ? lnb : cfg->log_index_size;
   const uint64 ni  = 1ull << (lb - cfg->log_index_size);
   XXH64_state_t *st = XXH64_createState();
   XXH64_reset(st, 0);
   uint64 last_page = UINT64_MAX;
   for (uint64 i = 0; i < ni; i++) {
      page_handle *ip   = cache_get(cc, f->addr + ps * (i / app), TRUE, PAGE_TYPE_FILTER);
      const uint64 slot = ((const uint64 *)ip->data)[i % app];
      cache_unget(cc, ip);
      XXH64_update(st, &slot, sizeof(slot));
      const uint64 page = slot - slot % ps;
      if (page != last_page) {
         page_handle *pg = cache_get(cc, page, TRUE, PAGE_TYPE_FILTER);
         XXH64_update(st, pg->data, ps);
         cache_unget(cc, pg);
         last_page = page;
      }
   }
   const uint64 d = XXH64_digest(st);
   XXH64_freeState(st);
   return d;
}

platform_status
__wrap_routing_filter_add(cache                *cc,
                          const routing_config *cfg,
                          routing_filter       *old_filter,
                          routing_filter       *filter,
                          uint32               *new_fp_arr,
                          uint64                num_new_fp,
                          uint16                value)
{
   const uint64    old_addr = old_filter->addr;
   platform_status rc =
      __real_routing_filter_add(cc, cfg, old_filter, filter, new_fp_arr, num_new_fp, value);
   rfk_add_rec r = {.old_addr         = old_addr,
                    .num_new          = num_new_fp,
                    .value            = value,
                    .rc               = (uint64)rc.r,
                    .addr             = filter->addr,
                    .meta_head        = filter->meta_head,
                    .num_fingerprints = filter->num_fingerprints,
                    .num_unique       = filter->num_unique,
                    .value_size       = filter->value_size};
   if (SUCCESS(rc) && g_record_digest) {
      r.digest = filter_digest(cc, cfg, filter);
   }
   pthread_mutex_lock(&g_rec_mu);
   if (g_nadds == g_cap_adds) {
      g_cap_adds = g_cap_adds ? 2 * g_cap_adds : 1024;
      g_adds     = realloc(g_adds, sizeof(*g_adds) * g_cap_adds);
      platform_assert(g_adds != NULL);
   }
   g_adds[g_nadds++] = r;
   pthread_mutex_unlock(&g_rec_mu);
   return rc;
}

platform_status
__wrap_routing_filter_lookup(cache                *cc,
                             const routing_config *cfg,
                             routing_filter       *filter,
                             key                   target,
                             uint64               *found_values)
{
   atomic_fetch_add(&g_nlookups, 1);
   return __real_routing_filter_lookup(cc, cfg, filter, target, found_values);
}

async_status
__wrap_routing_filter_lookup_async(routing_filter_lookup_async_state *state)
{
   if (state->__async_state_stack[0] == ASYNC_STATE_INIT) {
      atomic_fetch_add(&g_nlookups_async, 1);
   }
   return __real_routing_filter_lookup_async(state);
}

/* ---- the in-memory device as the kvstore's io handle (platform_io.c's constructor) ---- */
extern uint64 g_rfr_kvs_disk_bytes; /* ref_harness.c */
io_handle *
rfr_mem_io_create(io_config *cfg, uint64 bytes);
void
rfr_mem_io_destroy(io_handle *ioh);

io_handle *
io_handle_create(io_config *cfg, platform_heap_id hid)
{
   (void)hid;
   return rfr_mem_io_create(cfg, g_rfr_kvs_disk_bytes);
}

void
io_handle_destroy(io_handle *ioh)
{
   rfr_mem_io_destroy(ioh);
}

/* ---- the kvstore ------------------------------------------------------------------------ */
typedef struct rfk_kvs {
   splinterdb       *kvs;
   data_config       data_cfg;
   splinterdb_config cfg;
} rfk_kvs;

rfk_kvs *
rfk_open(uint64 cache_mib,
         uint64 disk_mib,
         uint64 memtable_mib,
         uint32 filter_hash_size,
         uint32 filter_log_index_size,
         int    record_digest)
{
   rfk_kvs *k = calloc(1, sizeof(*k));
   if (!k) {
      return NULL;
   }
   default_data_config_init(&k->data_cfg);
   k->cfg.filename                = "rfk-memory-device";
   k->cfg.cache_size              = cache_mib << 20;
   k->cfg.disk_size               = disk_mib << 20;
   k->cfg.data_cfg                = &k->data_cfg;
   k->cfg.memtable_capacity       = memtable_mib << 20;
   k->cfg.filter_hash_size        = filter_hash_size;
   k->cfg.filter_log_index_size   = filter_log_index_size;
   k->cfg.num_memtable_bg_threads = 0; /* every task on the inserting thread: both stacks */
   k->cfg.num_normal_bg_threads   = 0; /* issue the same filter calls in the same order */
   k->cfg.use_log                 = FALSE;
   g_record_digest                = record_digest;
   g_rfr_kvs_disk_bytes           = k->cfg.disk_size;
   if (splinterdb_create(&k->cfg, &k->kvs) != 0) {
      free(k);
      return NULL;
   }
   return k;
}

/* the shim's release of a cache whose page buffer took images directly, and its registration
 * counters (weak: absent from the reference's own library) */
__attribute__((weak)) void
routing_filter_amd_cache_release(cache *cc);
__attribute__((weak)) void
routing_filter_amd_direct_stats(uint64 *out);
__attribute__((weak)) void
routing_filter_amd_add_breakdown(uint64 *out);
__attribute__((weak)) int
routing_filter_amd_cache_attach(cache *cc);

/* the shim's routing_filter_add breakdown (out[0..10], zeros with the reference) */
void
rfk_add_breakdown(uint64 *out)
{
   for (int i = 0; i < 11; i++) {
      out[i] = 0;
   }
   if (routing_filter_amd_add_breakdown) {
      routing_filter_amd_add_breakdown(out);
   }
}

/* the shim's engine made now and this store's cache attached: its page buffer registered for
 * direct placement (-1 with the reference, or when the shim keeps the bounce path) */
int
rfk_attach(rfk_kvs *k)
{
   return routing_filter_amd_cache_attach
             ? routing_filter_amd_cache_attach((cache *)splinterdb_get_cache_handle(k->kvs))
             : -1;
}

/* release = 0 closes the store as the unmodified reference does: without telling the shim */
void
rfk_close_ex(rfk_kvs *k, int release)
{
   if (k) {
      if (release && routing_filter_amd_cache_release) {
         routing_filter_amd_cache_release((cache *)splinterdb_get_cache_handle(k->kvs));
      }
      splinterdb_close(&k->kvs);
      free(k);
   }
}

void
rfk_close(rfk_kvs *k)
{
   rfk_close_ex(k, 1);
}

/* out[0] caches registered now, out[1] registrations found stale, out[2] adds placing now
 * (zeros without the shim); out[3] the address of the store's cache page buffer */
void
rfk_direct_stats(rfk_kvs *k, uint64 *out)
{
   out[0] = out[1] = out[2] = 0;
   if (routing_filter_amd_direct_stats) {
      routing_filter_amd_direct_stats(out);
   }
   out[3] = k ? (uint64)(uintptr_t)((clockcache *)splinterdb_get_cache_handle(k->kvs))->data : 0;
}

/* n inserts of key i = keys[i * key_len ...], value i = values[i * val_len ...] */
int
rfk_insert(rfk_kvs *k, const uint8 *keys, uint32 key_len, const uint8 *values, uint32 val_len, uint64 n)
{
   for (uint64 i = 0; i < n; i++) {
      int rc = splinterdb_insert(k->kvs,
                                 slice_create(key_len, keys + i * key_len),
                                 slice_create(val_len, values + i * val_len),
                                 NULL);
      if (rc) {
         return rc;
      }
   }
   return 0;
}

static double
now_s(void)
{
   struct timespec ts;
   clock_gettime(CLOCK_MONOTONIC, &ts);
   return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* synchronous lookups (splinterdb_lookup): found[i] = 1 and the first 8 value bytes into
 * value8[i] when key i is found; returns the seconds spent in the lookup calls, < 0 on error */
double
rfk_lookup(rfk_kvs *k, const uint8 *keys, uint32 key_len, uint64 n, uint8 *found, uint64 *value8)
{
   splinterdb_lookup_result res;
   splinterdb_lookup_result_init(k->kvs, &res, SPLINTERDB_LOOKUP_VALUE, 0, NULL);
   double t = 0;
   for (uint64 i = 0; i < n; i++) {
      const double t0 = now_s();
      int          rc = splinterdb_lookup(k->kvs, slice_create(key_len, keys + i * key_len), &res);
      t += now_s() - t0;
      if (rc) {
         splinterdb_lookup_result_deinit(&res);
         return -1;
      }
      found[i]  = splinterdb_lookup_found(&res);
      value8[i] = 0;
      if (found[i]) {
         slice v;
         splinterdb_lookup_result_value(&res, &v);
         memcpy(&value8[i], slice_data(v), slice_length(v) < 8 ? slice_length(v) : 8);
      }
   }
   splinterdb_lookup_result_deinit(&res);
   return t;
}

/* asynchronous lookups through core_lookup_async (src/core.c:1669), at most max_inflight in
 * flight, each re-called only after its callback fired -- the tests/functional/test_async.c
 * pattern; same outputs as rfk_lookup, returns the wall seconds */
typedef struct rfk_actx {
   core_lookup_async_state  st;
   splinterdb_lookup_result res;
   uint64                  i;
   _Atomic int             ready;
   struct rfk_actx        *next;
} rfk_actx;

static void
rfk_actx_cb(void *arg)
{
   atomic_store(&((rfk_actx *)arg)->ready, 1);
}

double
rfk_lookup_async(rfk_kvs     *k,
                 const uint8 *keys,
                 uint32       key_len,
                 uint64       n,
                 uint8       *found,
                 uint64      *value8,
                 uint32       max_inflight)
{
   core_handle *spl  = (core_handle *)splinterdb_get_trunk_handle(k->kvs);
   rfk_actx    *ctx  = calloc(max_inflight, sizeof(*ctx));
   rfk_actx   **live = calloc(max_inflight, sizeof(*live));
   if (!ctx || !live) {
      free(ctx);
      free(live);
      return -1;
   }
   for (uint32 c = 0; c < max_inflight; c++) {
      splinterdb_lookup_result_init(k->kvs, &ctx[c].res, SPLINTERDB_LOOKUP_VALUE, 0, NULL);
   }
   uint64       next = 0, done = 0;
   uint32       nlive = 0, nfree = max_inflight;
   rfk_actx   **freel = calloc(max_inflight, sizeof(*freel));
   for (uint32 c = 0; c < max_inflight; c++) {
      freel[c] = &ctx[c];
   }
   const double t0  = now_s();
   int          err = 0;
#define RFK_FINISH(c)                                                                         \
   do {                                                                                      \
      if (!SUCCESS((c)->st.__async_result)) {                                                \
         err = 1;                                                                            \
      }                                                                                      \
      found[(c)->i]  = splinterdb_lookup_found(&(c)->res);                                   \
      value8[(c)->i] = 0;                                                                    \
      if (found[(c)->i]) {                                                                   \
         slice v;                                                                            \
         splinterdb_lookup_result_value(&(c)->res, &v);                                      \
         memcpy(&value8[(c)->i], slice_data(v), slice_length(v) < 8 ? slice_length(v) : 8);  \
      }                                                                                      \
      freel[nfree++] = (c);                                                                  \
      done++;                                                                                \
   } while (0)
   while (done < n && !err) {
      while (nfree && next < n) {
         rfk_actx *c = freel[--nfree];
         c->i        = next++;
         atomic_store(&c->ready, 0);
         lookup_result *lr = lookup_result_from_splinterdb(&c->res);
         lookup_result_reset(lr);
         key target = key_create(FALSE, key_len, keys + c->i * key_len);
         core_lookup_async_state_init(&c->st, spl, target, lr, rfk_actx_cb, c);
         if (core_lookup_async(&c->st) == ASYNC_STATUS_DONE) {
            RFK_FINISH(c);
         } else {
            live[nlive++] = c;
         }
      }
      for (uint32 j = 0; j < nlive;) {
         rfk_actx *c = live[j];
         if (atomic_load(&c->ready)) {
            atomic_store(&c->ready, 0);
            if (core_lookup_async(&c->st) == ASYNC_STATUS_DONE) {
               live[j] = live[--nlive];
               RFK_FINISH(c);
               continue;
            }
         }
         j++;
      }
      cache_cleanup((cache *)splinterdb_get_cache_handle(k->kvs));
   }
#undef RFK_FINISH
   const double t = now_s() - t0;
   for (uint32 c = 0; c < max_inflight; c++) {
      splinterdb_lookup_result_deinit(&ctx[c].res);
   }
   free(ctx);
   free(live);
   free(freel);
   return err ? -1 : t;
}

/* recorded filter adds (up to cap records into out; returns how many there are) and the
 * filter lookups counted so far; reset clears both */
uint64
rfk_adds(rfk_add_rec *out, uint64 cap, uint64 *lookups, uint64 *lookups_async, int reset)
{
   pthread_mutex_lock(&g_rec_mu);
   const uint64 n = g_nadds;
   if (out) {
      memcpy(out, g_adds, sizeof(*out) * (n < cap ? n : cap));
   }
   *lookups       = atomic_load(&g_nlookups);
   *lookups_async = atomic_load(&g_nlookups_async);
   if (reset) {
      g_nadds = 0;
      atomic_store(&g_nlookups, 0);
      atomic_store(&g_nlookups_async, 0);
   }
   pthread_mutex_unlock(&g_rec_mu);
   return n;
}
