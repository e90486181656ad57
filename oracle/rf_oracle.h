/*
 * rf_oracle.h -- CPU restatement of SplinterDB's routing filter (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X routing-filter engine. It is NOT part of the
 * product: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker / the CPU baseline. The product path (splinterdb_amd/) never
 * links or calls it.
 *
 * What it restates (reference = vmware/splinterdb, files relative to its root):
 *   - XXH32 (xxHash 0.8.x, the unvendored libxxhash the reference links, Makefile:94),
 *     reached via data_key_hash (src/data_internal.h:673-683) -> key_hash
 *     (src/default_data_config.c:30-35) -> platform_hash32 (platform_linux/platform_hash.h:23)
 *   - PackedArray pack/unpack/get        src/PackedArray.c:205-299, 386-538
 *   - RadixSort                          src/routing_filter.c:54-131
 *   - routing_filter_add                 src/routing_filter.c:337-656
 *   - routing_get_bucket_bounds / counts src/routing_filter.c:230-306
 *   - routing_filter_lookup              src/routing_filter.c:985-1073
 *   - routing_filter_estimate_unique_fp  src/routing_filter.c:702-848
 *   - routing_filter_estimate_unique_keys_from_count src/routing_filter.c:1119-1139
 *
 * Parity pinning (see DESIGN.md "Oracle"): the reference's own tests hold no golden bytes
 * and its routing_filter.c cannot be built here without header stand-ins (xxhash.h is
 * absent from the image), so this restatement is pinned by (a) the reference's
 * PackedArray.c compiled from its own sources into oracle/_ref/, (b) XXH32 vectors from
 * the image's libxxhash.so.0 and python-xxhash, and (c) the known-answer facts the survey
 * recorded from running the reference.
 *
 * Filter images are relocatable: an index slot holds  data_page_no * page_size + offset
 * instead of the absolute disk address the reference stores (src/routing_filter.c:620).
 */
#ifndef RF_ORACLE_H
#define RF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rfo_config {
   uint32_t fingerprint_size; /* routing_config.fingerprint_size (26)   */
   uint32_t log_index_size;   /* routing_config.log_index_size (8 / 9)  */
   uint32_t seed;             /* routing_config.seed (42)               */
   uint32_t page_size;        /* cache page size (4096)                 */
   uint32_t pages_per_extent; /* extent_size / page_size (32)           */
} rfo_config;

/* In-memory, relocatable filter image. */
typedef struct rfo_filter {
   uint32_t num_fingerprints; /* routing_filter.num_fingerprints */
   uint32_t num_unique;       /* routing_filter.num_unique       */
   uint32_t value_size;       /* routing_filter.value_size       */
   uint32_t num_indices;
   uint32_t num_pages;        /* data pages                      */
   uint32_t pages_cap;
   uint64_t *slots;           /* pages_per_extent*page_size/8 u64 (the index extent) */
   uint8_t  *pages;           /* num_pages * page_size bytes     */
} rfo_filter;

/* hashing */
uint32_t rfo_xxh32(const void *input, size_t len, uint32_t seed);
void     rfo_hash_fixed(const uint8_t *keys, uint64_t n, uint32_t key_len, uint32_t seed,
                        uint32_t *out);
void     rfo_hash_var(const uint8_t *bytes, const uint64_t *offs, uint64_t n, uint32_t seed,
                      uint32_t *out);

/* PackedArray codec */
void     rfo_pack(uint32_t *a, uint32_t offset, const uint32_t *in, uint32_t count,
                  uint32_t bits);
void     rfo_unpack(const uint32_t *a, uint32_t offset, uint32_t *out, uint32_t count,
                    uint32_t bits);
uint32_t rfo_get(const uint32_t *a, uint32_t offset, uint32_t bits);

/* filter build / query. Returns 0 on success, 12 (ENOMEM), 22 (EINVAL). */
int      rfo_filter_add(const rfo_config *cfg, const rfo_filter *old_filter, rfo_filter *out,
                        uint32_t *new_fp_arr, uint64_t num_new_fp, uint16_t value);
void     rfo_filter_release(rfo_filter *f);
uint64_t rfo_filter_lookup_hash(const rfo_config *cfg, const rfo_filter *f, uint32_t hash);
void     rfo_filter_lookup_hashes(const rfo_config *cfg, const rfo_filter *f,
                                  const uint32_t *hashes, uint64_t n, uint64_t *found);
int      rfo_estimate_unique_fp(const rfo_config *cfg, const rfo_filter *filters,
                                uint64_t num_filters, uint32_t *num_unique_fp);
uint32_t rfo_estimate_unique_keys_from_count(const rfo_config *cfg, uint64_t num_unique);
uint64_t rfo_space_use_bytes(const rfo_config *cfg, const rfo_filter *f);
void     rfo_bucket_counts(const rfo_config *cfg, const uint8_t *hdr, uint32_t *count);
/* RadixSort (returns pData or pTemp: the buffer holding the result) and
 * routing_get_bucket_bounds, exposed for the pinning tests */
uint32_t *rfo_radix_sort(uint32_t *pData, uint32_t *pTemp, uint32_t count, uint32_t fp_size);
void     rfo_bucket_bounds(const uint8_t *encoding, uint64_t len, uint64_t bucket_offset, uint64_t *start,
                           uint64_t *end);

/* handle-style helpers for ctypes */
rfo_filter *rfo_filter_new(void);
void        rfo_filter_delete(rfo_filter *f);

/*
 * Multi-threaded CPU baseline: builds `num_filters` independent filters, filter f from
 * keys [key_start[f], key_start[f]+key_count[f]) of a fixed-length key array, one
 * routing_filter_add per task on `threads` worker threads (the reference's
 * TASK_TYPE_NORMAL model, src/trunk.c:3932). If hash_keys==0, `keys` is read as u32
 * hashes. Returns elapsed seconds. Filters are released unless `keep` is non-NULL.
 */
double rfo_bench_build(const rfo_config *cfg, const uint8_t *keys, uint32_t key_len,
                       int hash_keys, const uint64_t *key_start, const uint32_t *key_count,
                       uint32_t num_filters, uint16_t value, int threads, rfo_filter *keep);
double rfo_bench_probe(const rfo_config *cfg, const rfo_filter *filters,
                       const uint8_t *keys, uint32_t key_len, const uint32_t *filter_id,
                       uint64_t n, int threads, uint64_t *found);
/* variable-length keys (bytes + n+1 offsets, default_data_config hashing) */
double rfo_bench_build_var(const rfo_config *cfg, const uint8_t *bytes, const uint64_t *offs,
                           const uint64_t *key_start, const uint32_t *key_count,
                           uint32_t num_filters, uint16_t value, int threads, rfo_filter *keep);
double rfo_bench_probe_var(const rfo_config *cfg, const rfo_filter *filters, const uint8_t *bytes,
                           const uint64_t *offs, const uint32_t *filter_id, uint64_t n,
                           int threads, uint64_t *found);

#ifdef __cplusplus
}
#endif
#endif
