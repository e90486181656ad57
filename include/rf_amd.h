/*
 * rf_amd.h -- C ABI of the MI355X routing-filter engine.
 *
 * Drop-in boundary for SplinterDB's routing filter (reference: vmware/splinterdb,
 * src/routing_filter.h). Plain C types only: device pointers are `void *` / typed
 * pointers into HIP device memory, streams are `hipStream_t` passed as `void *`.
 * Errors follow platform_status (src/platform_linux/platform_status.h): 0 = STATUS_OK,
 * ENOMEM = STATUS_NO_MEMORY, EINVAL = STATUS_BAD_PARAM, ENODEV = no HIP device.
 *
 * Filter images are bit-exact with the reference's page bytes (src/routing_filter.c
 * :599-633 layout, src/PackedArray.c packing). Index slots are RELOCATABLE:
 * slot = data_page_no * page_size + byte_offset; the integration shim
 * adds the mini_alloc'd page address, restoring the reference's absolute slot
 * (src/routing_filter.c:620).
 */
#ifndef RF_AMD_H
#define RF_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RF_AMD_OK        0
#define RF_AMD_ENOMEM    12
#define RF_AMD_ENODEV    19
#define RF_AMD_EINVAL    22

/* per-filter error bits reported in rf_amd_filter_info.error */
#define RF_AMD_ERR_INDEX_OVERFLOW 1u /* > 4096 entries in one index (ref: fp_buffer overflow, :596) */
#define RF_AMD_ERR_BLOCK_TOO_BIG  2u /* one index block > page (ref: writes past page, :603-610) */
#define RF_AMD_ERR_PAGE_CAP       4u /* internal page bound exceeded (never expected)           */
#define RF_AMD_ERR_GEOMETRY       8u /* invalid geometry                                         */

/* mirrors routing_config (src/routing_filter.h:32-40); key_hash is always XXH32 */
typedef struct rf_amd_config {
   uint32_t fingerprint_size; /* 26 (splinterdb.c:147-152, tests/config.c:29) */
   uint32_t log_index_size;   /* 9 library default, 8 tests                   */
   uint32_t seed;             /* 42                                           */
   uint32_t page_size;        /* 4096                                         */
   uint32_t pages_per_extent; /* 32                                           */
} rf_amd_config;

/* mirrors the routing_filter descriptor (src/routing_filter.h:66-72) + image geometry */
typedef struct rf_amd_filter_info {
   uint32_t num_fingerprints;
   uint32_t num_unique;
   uint32_t value_size;
   uint32_t num_indices;
   uint32_t num_pages; /* data pages in the image */
   uint32_t error;     /* RF_AMD_ERR_* bits, 0 on success */
} rf_amd_filter_info;

typedef struct rf_amd_engine rf_amd_engine;
typedef struct rf_amd_batch  rf_amd_batch;

/* ---- engine ------------------------------------------------------------------------ */
int         rf_amd_engine_create(int device, rf_amd_engine **out);
void        rf_amd_engine_destroy(rf_amd_engine *e);
const char *rf_amd_last_error(void);

/* ---- batched device-resident build (the throughput path) ----------------------------
 * A batch = F independent filters, filter f built from the f-th run of `num_new[f]`
 * inputs (runs concatenated in filter order), tagged with value[f]. This coalesces the
 * concurrent routing_filter_add calls SplinterDB issues from its TASK_TYPE_NORMAL
 * workers (src/trunk.c:3821-3835) into one launch sequence. `old` (may be NULL) gives,
 * per filter, a previously built filter (batch, index) whose entries are merged in
 * (routing_filter_add's old_filter, src/routing_filter.c:355-368, 496-544); pass
 * old_batch[f] = NULL for a fresh filter.
 */
int rf_amd_batch_create(rf_amd_engine *e, const rf_amd_config *cfg, uint32_t num_filters,
                        const uint32_t *num_new, const uint16_t *value,
                        rf_amd_batch *const *old_batch, const uint32_t *old_index,
                        rf_amd_batch **out);
/* synchronises the device, then releases the batch's memory (routing_filter_dec_ref's
 * release of a superseded filter, src/routing_filter.c:1101-1109) */
void rf_amd_batch_destroy(rf_amd_batch *b);
/* stream-ordered destroy: the caller has ordered every use of b before the current end of
 * `stream` (NULL = engine's); the memory becomes reusable once the stream passes that point.
 * Does not wait. */
int rf_amd_batch_destroy_on(rf_amd_batch *b, void *stream);

/* inputs are DEVICE pointers; all calls are asynchronous on `stream` (NULL = engine's) */
int rf_amd_batch_build_keys(rf_amd_batch *b, const void *d_keys, uint32_t key_len,
                            void *stream);
int rf_amd_batch_build_var_keys(rf_amd_batch *b, const uint8_t *d_bytes,
                                const uint64_t *d_offsets, void *stream);
int rf_amd_batch_build_hashes(rf_amd_batch *b, const uint32_t *d_hashes, void *stream);

/* probes: probe i looks up key i in filter d_filter_id[i]; result = routing_filter_lookup's
 * found_values bit-vector (src/routing_filter.c:985-1073) */
int rf_amd_batch_probe_keys(rf_amd_batch *b, const void *d_keys, uint32_t key_len,
                            const uint32_t *d_filter_id, uint64_t n, uint64_t *d_found,
                            void *stream);
int rf_amd_batch_probe_var_keys(rf_amd_batch *b, const uint8_t *d_bytes,
                                const uint64_t *d_offsets, const uint32_t *d_filter_id,
                                uint64_t n, uint64_t *d_found, void *stream);
int rf_amd_batch_probe_hashes(rf_amd_batch *b, const uint32_t *d_hashes,
                              const uint32_t *d_filter_id, uint64_t n, uint64_t *d_found,
                              void *stream);
/* probes grouped by filter, in filter order: filter f's h_counts[f] probes follow those of
 * filters < f (one batch of routing_filter_lookup calls per filter). The filter of each
 * probe follows from its position: no per-probe filter id is read. */
int rf_amd_batch_probe_keys_runs(rf_amd_batch *b, const void *d_keys, uint32_t key_len,
                                 const uint64_t *h_counts, uint64_t *d_found, void *stream);
int rf_amd_batch_probe_hashes_runs(rf_amd_batch *b, const uint32_t *d_hashes, const uint64_t *h_counts,
                                   uint64_t *d_found, void *stream);

/* Host-buffer forms (synchronous), for callers that hold no device memory, e.g. the
 * routing_filter.h shim (shim/routing_filter_amd.c): build batch b from its keys_total host
 * hashes (staged through the engine's pinned buffer, on the engine stream), and probe n host
 * hashes (filter h_filter_id[i], or filter 0 when NULL; ids >= the batch's filters find
 * nothing) into h_found.
 * Lookups (this and the two calls below) are ONE kernel launch per call on one of the
 * engine's lookup slots (own stream, pinned device-mapped buffers, a completion word the
 * host polls): small calls are read by the kernel straight from pinned host memory, large
 * ones copied in once; results are written by the kernel into pinned host memory. They are
 * thread-safe and concurrent callers run concurrently. Batches must be built (a build issued
 * on the engine stream is waited for). */
int rf_amd_batch_build_hashes_host(rf_amd_batch *b, const uint32_t *h_hashes);
/* the same in two steps, for callers that fill the pinned staging buffer themselves (e.g.
 * each thread of a coalesced add copying its own fingerprints, in parallel): stage_begin
 * takes the engine's staging buffer (filter f's hashes at its run offset, runs in filter
 * order) and returns its host address; stage_build uploads it, builds, waits and releases
 * it; stage_abort releases it without building. */
int  rf_amd_batch_stage_begin(rf_amd_batch *b, uint32_t **h_stage);
int  rf_amd_batch_stage_build(rf_amd_batch *b);
void rf_amd_batch_stage_abort(rf_amd_batch *b);
int rf_amd_batch_probe_hashes_host(rf_amd_batch *b, const uint32_t *h_hashes, const uint32_t *h_filter_id,
                                   uint64_t n, uint64_t *h_found);
/* lookups against many resident filters -- of any batches of the engine -- in ONE launch:
 * probe i looks up h_hashes[i] in filter filter_index[g] (NULL: 0) of batches[g], where
 * g = h_group[i] (NULL: 0); g >= num_groups finds nothing. The form of a flush of queued
 * routing_filter_lookup_async states (src/routing_filter.h:130-155) and of trunk_merge_lookup's
 * per-bundle routing_filter_lookup calls (src/trunk.c:6008-6075; routing_filter.h:87-92)
 * gathered together. Each group is probed with its own batch's routing config, so filters of
 * differently configured kvstores may share a call. */
int rf_amd_probe_filters_host(rf_amd_engine *e, rf_amd_batch *const *batches, const uint32_t *filter_index,
                              uint32_t num_groups, const uint32_t *h_hashes, const uint32_t *h_group,
                              uint64_t n, uint64_t *h_found);
/* the same with the probes grouped: group g probes counts[g] consecutive hashes */
int rf_amd_probe_many_hashes_host(rf_amd_engine *e, rf_amd_batch *const *batches,
                                  const uint32_t *filter_index, const uint64_t *counts,
                                  uint32_t num_groups, const uint32_t *h_hashes, uint64_t *h_found);
/* The engine's lookup server: single lookups -- routing_filter_lookup (src/routing_filter.h:
 * 87-92) and routing_filter_lookup_async states (:130-155) -- without a kernel launch per
 * call. A persistent wave (started on demand on a queue of its own, exiting after 400 us
 * without requests and after an 800 us lifetime -- so a device-wide synchronisation waits at
 * most that long for it; relaunched while lookups continue) polls a ring of requests in
 * device memory that the host writes through its BAR mapping (RF_AMD_SRV_RING=host: pinned
 * host memory) and
 * answers each with filter filter_index of batch b, in submission order. submit queues the
 * lookup of `hash` and returns its ticket; the batch must stay alive until the result is
 * taken. A NULL tag: the caller takes the result with rf_amd_lookup_wait (blocking). A
 * non-NULL tag: the result is delivered by rf_amd_lookup_reap, which returns up to max
 * answered tagged lookups in ticket order (tags[i], found_values[i]) without blocking (0 if
 * none is ready or another thread is reaping). Thread-safe. */
#define RF_AMD_SERVER_RING 4096 /* requests in flight at most (a submit beyond waits for a slot) */
int rf_amd_lookup_submit(rf_amd_engine *e, rf_amd_batch *b, uint32_t filter_index, uint32_t hash,
                         void *tag, uint64_t *ticket);
int rf_amd_lookup_wait(rf_amd_engine *e, uint64_t ticket, uint64_t *found_values);
uint64_t rf_amd_lookup_reap(rf_amd_engine *e, void **tags, uint64_t *found_values, uint64_t max);
/* the server's first error (0: none; sticky: a launch that failed, a faulted stream). Once it
 * is set, submit and wait return it, and rf_amd_lookup_server_failed hands back (consumes) the
 * tags of tagged lookups that will not be answered, so their owners can complete them with an
 * error instead of waiting */
int rf_amd_lookup_server_error(rf_amd_engine *e);
uint64_t rf_amd_lookup_server_failed(rf_amd_engine *e, void **tags, uint64_t max);
/* idle exit and lifetime (microseconds) of the server waves launched from now on (defaults
 * 400 / 800; RF_AMD_SERVER_IDLE_US / _LIFE_US): a host-controlled keep-alive */
int rf_amd_lookup_server_set_times(rf_amd_engine *e, uint64_t idle_us, uint64_t life_us);
/* device-allocation pool of the engine (batch work buffers are recycled across batches; up
 * to RF_AMD_POOL_MIB MiB stay pooled, by default a quarter of the device memory free at
 * engine creation and at most 16 GiB); trim hands pooled blocks back to the device until at
 * most keep_bytes stay pooled */
int rf_amd_engine_pool_stats(rf_amd_engine *e, uint64_t *pooled_bytes, uint64_t *hits, uint64_t *misses);
int rf_amd_engine_pool_trim(rf_amd_engine *e, uint64_t keep_bytes);
/* the most device memory the pool keeps parked for reuse (default: RF_AMD_POOL_MIB, else a
 * quarter of the free memory at creation, at most 16 GiB); trims to it now */
int rf_amd_engine_set_pool_limit(rf_amd_engine *e, uint64_t bytes);
/* the engine's stream (NULL-stream arguments, host-buffer builds and imports run there) and
 * its synchronisation (only that stream, not the device) */
void *rf_amd_engine_stream(rf_amd_engine *e);
int   rf_amd_engine_sync(rf_amd_engine *e);
/* pinned host memory: a read-back target that the DMA engines write at full PCIe rate (a
 * copy into pageable memory goes through the driver's staging buffers) */
int  rf_amd_host_alloc(rf_amd_engine *e, uint64_t bytes, void **out);
void rf_amd_host_free(rf_amd_engine *e, void *p);
/* a completion point after the work queued on the engine stream so far (e.g. one filter's
 * image read-back); fence_wait blocks until it has passed and releases it (once) */
int rf_amd_engine_fence(rf_amd_engine *e, uint64_t *fence);
/* host memory the kernels may write directly (e.g. a page cache's buffer, registered once):
 * rf_amd_batch_place_image stores images there without a staging copy */
int rf_amd_host_register(rf_amd_engine *e, void *p, uint64_t bytes);
int rf_amd_host_unregister(rf_amd_engine *e, void *p);
/* filter f's image straight into host pages (replaces the reference's page fill,
 * src/routing_filter.c:603-633): `table` (rf_amd_host_alloc'd) holds the destination of each
 * of the num_pages image pages (inside registered memory), then each page's disk address,
 * then the destinations of the ceil(num_indices / addrs_per_page) index pages. One call writes
 * pages [first_page, first_page + count) and, with_index, the absolute index slots; the
 * destinations it uses are translated in place. Stream-ordered (NULL: the engine stream):
 * wait with rf_amd_engine_fence before using the pages */
int rf_amd_batch_place_image(rf_amd_batch *b, uint32_t f, uint64_t *table, uint32_t num_pages,
                             uint32_t first_page, uint32_t count, int with_index, uint32_t addrs_per_page,
                             void *stream);
int rf_amd_engine_fence_wait(rf_amd_engine *e, uint64_t fence);
/* Residency control for callers that keep many built batches (the shim's registry):
 * device_bytes = the device memory the batch holds; trim drops its build work buffers,
 * keeping pages, slots, probe lines and plans (lookups, image reads, estimates and use as an
 * old filter through an image decode keep working; incremental adds lose the in-place read
 * of its sorted entries). Stream-ordered on `stream` (NULL = engine's), like destroy_on. */
uint64_t rf_amd_batch_device_bytes(const rf_amd_batch *b);
int      rf_amd_batch_trim(rf_amd_batch *b, void *stream);

/* synchronising accessors */
int rf_amd_batch_info(rf_amd_batch *b, uint32_t f, rf_amd_filter_info *out);
/* all rf_amd_batch_num_filters(b) infos at once: one synchronisation, with `stream` (the
 * build's stream) or, if NULL, the whole device */
int rf_amd_batch_infos(rf_amd_batch *b, rf_amd_filter_info *out, void *stream);
/* copy filter f's image to host: num_pages*page_size bytes and num_indices slots */
int rf_amd_batch_read_image(rf_amd_batch *b, uint32_t f, uint8_t *h_pages,
                            uint64_t pages_bytes, uint64_t *h_slots, uint32_t num_slots);
/* asynchronous D2H of filter f's first pages_bytes of pages and num_slots slots on
 * `stream` (e.g. into hipHostRegister'ed clockcache page buffers); the caller knows the
 * sizes from a previous rf_amd_batch_info or sizes by the reservation */
int rf_amd_batch_read_image_async(rf_amd_batch *b, uint32_t f, void *h_pages, uint64_t pages_bytes,
                                  void *h_slots, uint32_t num_slots, void *stream);
/* device pointers of filter f's image (pages, slots) for zero-copy consumers */
int rf_amd_batch_image_ptrs(rf_amd_batch *b, uint32_t f, void **d_pages, void **d_slots);
uint32_t rf_amd_batch_num_filters(const rf_amd_batch *b);

/* per-stage timing with HIP events recorded on the launch stream. Stages of the last
 * build: 0 partition (fresh builds: fused hash + coarse-bucket partition; incremental: hash
 * + histogram), 1 count/scan (fresh: spill fallback only), 2 scatter (fresh: spill fallback
 * only), 3 bucket sort, 4 big-bucket sort, 5 layout, 6 page assembly + probe lines, 7 whole
 * build; 8 = last probe kernel.
 * Milliseconds, -1 if a stage did not run. */
#define RF_AMD_NUM_TIMINGS 9
/* enable = number of event sets kept (0 = off): each build starts the next set of a ring,
 * so the stages of the last `enable` build+probe rounds can be read without synchronising
 * between them (rf_amd_batch_timings_back: back = 0 is the latest round). A negative
 * enable keeps -enable sets but records only the probe's start and end (every build stage
 * reads back as -1): 2 event records per round instead of 10. */
int rf_amd_batch_set_timing(rf_amd_batch *b, int enable);
int rf_amd_batch_timings_back(rf_amd_batch *b, uint32_t back, float *ms, uint32_t n);
int rf_amd_batch_timings(rf_amd_batch *b, float *ms, uint32_t n);

/* XXH32(key, cfg->seed) of n device-resident keys into d_hashes (data_key_hash as
 * btree_pack computes a compaction's fingerprints, src/btree.c:4020-4024); asynchronous */
int rf_amd_hash_keys(rf_amd_engine *e, const rf_amd_config *cfg, const void *d_keys, uint32_t key_len,
                     uint64_t n, uint32_t *d_hashes, void *stream);
int rf_amd_hash_var_keys(rf_amd_engine *e, const rf_amd_config *cfg, const uint8_t *d_bytes,
                         const uint64_t *d_offsets, uint64_t n, uint32_t *d_hashes, void *stream);

/* Import filter images as a built, probe-only batch (e.g. images all-gathered from the
 * other ranks when probes are replicated rather than routed). Filter f's
 * pages are the infos[f].num_pages * page_size bytes after those of filters < f in
 * `pages`; its relocatable index slots the infos[f].num_indices u64 after those of
 * filters < f in `slots`. device_resident: the buffers are HIP device memory (else host).
 * The batch copies them; probe lines are cut on the device. */
int rf_amd_batch_export(rf_amd_batch *b, void *d_pages, uint64_t pages_bytes, uint64_t *d_slots,
                        uint64_t num_slots, void *stream); /* all filters, packed as import reads them */
int rf_amd_batch_import(rf_amd_engine *e, const rf_amd_config *cfg, uint32_t num_filters,
                        const rf_amd_filter_info *infos, const void *pages, const uint64_t *slots,
                        int device_resident, rf_amd_batch **out);

/* ---- routed probes across ranks (multi-GPU serving) --------------------
 * Each rank owns the filters of a contiguous key range (one filter per trunk pivot,
 * src/trunk.c:4133-4170); a probe may arrive on any rank. rf_amd_route_probes partitions
 * n probes (hash, global filter id) stably by owning rank, d_route[g] = local_id << 8 |
 * rank, into d_pairs = (local_id << 32 | hash) grouped by rank (h_counts[r] pairs for
 * rank r) plus d_perm (pair j came from probe d_perm[j]); it synchronises on the stream
 * to return h_counts. One all-to-all of d_pairs (RCCL, by the caller) hands every rank
 * its probes; rf_amd_batch_probe_pairs probes them against the owner's batch; the
 * reverse all-to-all returns found_values in pair order, and rf_amd_unroute_found
 * scatters them back (d_found[d_perm[j]] = d_back[j]). d_scratch holds
 * rf_amd_route_scratch_bytes(n, world) bytes. Bad filter ids / ranks: EINVAL. */
#define RF_AMD_ROUTE_MAX_WORLD 16
uint64_t rf_amd_route_scratch_bytes(uint64_t n, uint32_t world);
int rf_amd_route_probes(rf_amd_engine *e, const uint32_t *d_hashes, const uint32_t *d_filter_id, uint64_t n,
                        const uint32_t *d_route, uint32_t num_filters, uint32_t world, uint64_t *d_pairs,
                        uint32_t *d_perm, void *d_scratch, uint64_t *h_counts, void *stream);
int rf_amd_batch_probe_pairs(rf_amd_batch *b, const uint64_t *d_pairs, uint64_t n, uint64_t *d_found,
                             void *stream);
int rf_amd_unroute_found(rf_amd_engine *e, const uint64_t *d_back, const uint32_t *d_perm, uint64_t n,
                         uint64_t *d_found, void *stream);

/* ---- drop-in single-filter calls on HOST buffers ------------------------------------
 * rf_amd_filter_add replaces routing_filter_add (src/routing_filter.h:78-85): hashes
 * (32-bit XXH32 of the keys, as btree_pack produces them, src/btree.c:4020-4024) in,
 * relocatable image out. `old_pages/old_slots/old_info` describe old_filter (NULL for
 * NULL_ROUTING_FILTER). Unlike the reference, new_fp_arr is not modified.
 * The image buffers are allocated with malloc and freed with rf_amd_image_free.
 */
typedef struct rf_amd_image {
   rf_amd_filter_info info;
   uint8_t           *pages; /* info.num_pages * page_size bytes */
   uint64_t          *slots; /* info.num_indices slots           */
} rf_amd_image;

int  rf_amd_filter_add(rf_amd_engine *e, const rf_amd_config *cfg, const rf_amd_image *old_filter,
                       rf_amd_image *filter, const uint32_t *new_fp_arr, uint64_t num_new_fp,
                       uint16_t value);
/* replaces routing_filter_lookup (src/routing_filter.h:87-92) for a batch of hashed keys */
int  rf_amd_filter_lookup_hashes(rf_amd_engine *e, const rf_amd_config *cfg,
                                 const rf_amd_image *filter, const uint32_t *hashes, uint64_t n,
                                 uint64_t *found_values);
/* keys-in form: hashes each fixed-length key (XXH32, cfg->seed) on the GPU, as
 * routing_filter_lookup does with data_key_hash (src/routing_filter.c:1011) */
int  rf_amd_filter_lookup_keys(rf_amd_engine *e, const rf_amd_config *cfg,
                               const rf_amd_image *filter, const void *keys, uint32_t key_len,
                               uint64_t n, uint64_t *found_values);
void rf_amd_image_free(rf_amd_image *img);

/* ---- routing_filter_estimate_unique_fp (src/routing_filter.h:169-175, .c:702-848) ------
 * Distinct fingerprints among the first 1/16 of the indices of up to 32 filters, times 16
 * (leaf-split sizing, src/trunk.c:4506). Filters with pages == NULL (filter.addr == 0) or
 * fewer than 16 indices contribute nothing, as in the reference. EINVAL: NULL out-param
 * (STATUS_BAD_PARAM, :710-714), more than MAX_FILTERS = 32 filters, or more decoded entries
 * than num_fingerprints / 12 (the reference asserts, :776-780). */
int rf_amd_estimate_unique_fp(rf_amd_engine *e, const rf_amd_config *cfg, const rf_amd_image *filters,
                              uint64_t num_filters, uint32_t *num_unique_fp);
/* same over device-resident filters: filter i = (batches[i], filter_index[i]); a NULL
 * batches[i] is NULL_ROUTING_FILTER. All batches share one engine and routing config. */
int rf_amd_batch_estimate_unique_fp(rf_amd_batch *const *batches, const uint32_t *filter_index,
                                    uint64_t num_filters, uint32_t *num_unique_fp);
/* routing_filter_estimate_unique_keys (src/routing_filter.h:165-167, .c:1141-1146) */
uint32_t rf_amd_estimate_unique_keys(const rf_amd_filter_info *filter, const rf_amd_config *cfg);

/* ---- asynchronous lookups (routing_filter_lookup_async, src/routing_filter.h:130-155,
 * .c:895-972) ---------------------------------------------------------------------------
 * The reference's lookup coroutine returns ASYNC_STATUS_RUNNING while it waits for a page
 * and calls callback(callback_arg) when it can be resumed. Here one call starts a whole
 * batch of lookups against a built (device-resident) batch: host keys are staged through
 * pinned memory to HBM, probed, and the found_values bit-vectors copied back into h_found,
 * all on `stream` (NULL = the engine's). When h_found is complete, callback(callback_arg)
 * runs on a HIP runtime thread (it must not call HIP). h_filter_id == NULL probes filter 0.
 * poll returns RF_AMD_ASYNC_RUNNING / RF_AMD_ASYNC_DONE (async_status order); free waits for
 * completion first. The keys buffer may be reused as soon as rf_amd_lookup_async returns. */
#define RF_AMD_ASYNC_RUNNING 0
#define RF_AMD_ASYNC_DONE    1
typedef void (*rf_amd_callback_fn)(void *arg);
typedef struct rf_amd_lookup_async_state rf_amd_lookup_async_state;
int  rf_amd_lookup_async(rf_amd_batch *b, const void *h_keys, uint32_t key_len,
                         const uint32_t *h_filter_id, uint64_t n, uint64_t *h_found,
                         rf_amd_callback_fn callback, void *callback_arg, void *stream,
                         rf_amd_lookup_async_state **state);
int  rf_amd_lookup_async_poll(rf_amd_lookup_async_state *state);
int  rf_amd_lookup_async_wait(rf_amd_lookup_async_state *state);
void rf_amd_lookup_async_free(rf_amd_lookup_async_state *state);

/* ---- debug functions (src/routing_filter.h:185-192) ------------------------------------
 * rf_amd_filter_verify replaces routing_filter_verify (.c:1163-1183): every key must find
 * `value`; returns EINVAL (the reference asserts) with *num_missing keys that did not.
 * rf_amd_filter_print replaces routing_filter_print (.c:1260-1286), same text (slots are
 * relocatable), to out_file (a FILE *, NULL = stdout). */
int rf_amd_filter_verify(rf_amd_engine *e, const rf_amd_config *cfg, const rf_amd_image *filter,
                         const void *keys, uint32_t key_len, uint64_t n, uint16_t value,
                         uint64_t *num_missing);
int rf_amd_filter_print(const rf_amd_config *cfg, const rf_amd_image *filter, void *out_file);
/* the same text with the reference's absolute addresses: the filter's index extent address
 * and each index slot as stored on the index pages (src/routing_filter.c:1201-1226) */
int rf_amd_filter_print_abs(const rf_amd_config *cfg, const rf_amd_image *filter, uint64_t filter_addr,
                            const uint64_t *abs_slots, void *out_file);

/* host-side helpers mirroring routing_filter.h (no GPU work) */
uint64_t rf_amd_max_fingerprints(const rf_amd_config *cfg);              /* .h:120-127  */
uint32_t rf_amd_estimate_unique_keys_from_count(const rf_amd_config *cfg,
                                                uint64_t num_unique);     /* .c:1119-1139 */
uint64_t rf_amd_space_use_bytes(const rf_amd_config *cfg, uint32_t num_pages); /* .c:1149 */

#ifdef __cplusplus
}
#endif
#endif
