/*
 * routing_filter_amd.c -- drop-in replacement for vmware/splinterdb's src/routing_filter.c.
 *
 * Compiled in SplinterDB's tree against its own headers (src/routing_filter.h,
 * src/mini_allocator.h, src/cache.h, ...) in place of routing_filter.c, it defines every
 * function routing_filter.h declares, with the reference's signatures, and runs the filter
 * work on the MI355X engine through its C ABI (include/rf_amd.h, librf_amd.so):
 *
 *   routing_filter_add                  routing_filter.h:78-85   build on the GPU (concurrent
 *                                        calls coalesced into one batch), then the reference's
 *                                        page allocation sequence, page by page
 *   routing_filter_lookup               :87-92     hash via data_config (the application's
 *                                        callback, as the reference), one GPU round trip
 *   routing_filter_lookup_async         :130-155   states queued and probed together, many
 *                                        filters per launch (see "async" below)
 *   routing_filter_inc_ref / _dec_ref   :157-162   the reference's mini_allocator refcounts
 *   routing_filter_estimate_unique_*    :163-175   GPU decode + distinct count
 *   routing_filter_space_use_bytes      :177-178   mini_space_use_bytes
 *   routing_filter_verify / _print      :182-192   GPU lookups / the reference's text
 *
 * Page bytes and addresses. The GPU returns a relocatable image (data pages in placement
 * order, slot = page_no * page_size + offset). routing_filter_add then allocates exactly
 * as the reference does (src/routing_filter.c:429-456, :603-610): the meta extent with
 * allocator_alloc, an unkeyed mini_allocator, the 32-page index extent, then one data page
 * per image page through mini_alloc + cache_alloc; it copies each image page into its cache
 * page and writes the absolute index slots (page address + offset, :620). From the same
 * cache/allocator state the filter descriptor (addr, meta_head, num_fingerprints,
 * num_unique, value_size) and every written page byte equal the reference's; bytes the
 * reference leaves untouched on a data page are zero here (they are zero on a fresh cache
 * page there, SURVEY finding 4). Each thread's allocation runs in its own call, in the
 * reference's order, after the shared GPU build.
 *
 * Differences a caller can see: new_fp_arr is not shifted/sorted in place (no caller reads
 * it afterwards; the trunk frees it, src/trunk.c:2825-2826); inputs the reference treats as
 * undefined behaviour (zero fingerprints, a block larger than a page) return
 * STATUS_BAD_PARAM instead of corrupting memory; without a HIP device every call that needs
 * one returns ENODEV (there is no CPU fallback).
 *
 * Concurrent adds. SplinterDB calls routing_filter_add from many TASK_TYPE_NORMAL workers at
 * once (src/trunk.c:3932, :4168). The first caller to find the engine idle becomes the
 * combiner: it takes every add queued so far -- its own and those that arrived while the
 * previous batch was building -- builds them as ONE multi-filter batch (rf_amd_batch_create
 * with F filters), reads each image back and hands it to its caller, which then allocates
 * its pages in the reference's order. No artificial wait: under load, batches form by
 * themselves; a lone caller builds alone.
 *
 * Device residency. Each filter this process builds stays on the GPU -- its whole batch, so a
 * later incremental add onto it reads the old entries in place instead of decoding the image
 * -- in a registry keyed by (cache, index-extent address); lookups never re-read it. A
 * filter not in the registry (built before a restart, or evicted) is read back through
 * cache_get once and imported. The registry is bounded (RF_AMD_REGISTRY_MIB, default 8 GiB
 * of device memory): past the bound the least recently used batches are first trimmed to
 * their probe-only state, then evicted; batches in use by a running call are pinned and
 * never released under it. dec_ref drops the device copy when the reference's refcount
 * reaches zero.
 *
 * Lookups. routing_filter_lookup and routing_filter_lookup_async go to the engine's lookup
 * server (rf_amd_lookup_submit): a ring of requests in device memory, written by the host
 * through the BAR, that a persistent GPU wave polls, so a single lookup costs no kernel
 * launch and needs no batching.
 * routing_filter_lookup waits for its answer. routing_filter_lookup_async's first call on a
 * state hashes the key, submits it and returns ASYNC_STATUS_RUNNING without touching the
 * state again (async.h:115-125: it may be completed on another thread at once). A completion
 * thread reaps the answers in submission order, stores found_values and the result, marks
 * the state done, then calls its callback(callback_arg) -- from that thread, registered with
 * the platform like any SplinterDB thread -- and the state's next call returns
 * ASYNC_STATUS_DONE. A state called again while still running (a polling owner) reaps in its
 * own thread and returns ASYNC_STATUS_RUNNING: a call never both fires its state's callback
 * and returns DONE. routing_filter_amd_lookup_batch (many keys at once) stays one launch over
 * every filter they name.
 */
#include "routing_filter.h"
#include "clockcache.h"
#include "mini_allocator.h"
#include "iterator.h"
#include "platform_assert.h"
#include "platform_threads.h"
#include "platform_typed_alloc.h"

#include <pthread.h>
#include <sched.h>
#include <x86intrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rf_amd.h"
#include "routing_filter_amd.h"

/* ---- engine ------------------------------------------------------------------------- */
static rf_amd_engine  *g_eng;
static int             g_eng_rc;
static pthread_once_t  g_eng_once = PTHREAD_ONCE_INIT;

static uint64 g_engine_ns, g_register_ns; /* one-time costs: engine creation, cache registrations */

static uint64
mono_ns(void)
{
   struct timespec ts;
   clock_gettime(CLOCK_MONOTONIC, &ts);
   return (uint64)ts.tv_sec * 1000000000ull + (uint64)ts.tv_nsec;
}

static void shim_at_exit(void);

static void
engine_init(void)
{
   const uint64 t0 = mono_ns();
   const char  *d  = getenv("RF_AMD_DEVICE");
   g_eng_rc        = rf_amd_engine_create(d ? atoi(d) : 0, &g_eng);
   if (g_eng_rc == 0) {
      /* registered after the engine library's own exit handler (rf_amd_engine_create), so it
         runs first: the shim's threads stop before the engine is torn down */
      (void)atexit(shim_at_exit);
   }
   /* a storage engine links this: its pool keeps at most 2 GiB parked unless
      RF_AMD_POOL_MIB says otherwise (one add's batch is at most a few hundred MB) */
   if (g_eng_rc == 0 && !getenv("RF_AMD_POOL_MIB")) {
      (void)rf_amd_engine_set_pool_limit(g_eng, 2048ull << 20);
   }
   g_engine_ns = mono_ns() - t0;
}

static rf_amd_engine *
engine(void)
{
   pthread_once(&g_eng_once, engine_init);
   return g_eng_rc == 0 ? g_eng : NULL;
}

static platform_status
status_of(int rc)
{
   platform_status s = {.r = rc};
   return s;
}

static rf_amd_config
amd_config(const routing_config *cfg)
{
   rf_amd_config c;
   c.fingerprint_size = cfg->fingerprint_size;
   c.log_index_size   = cfg->log_index_size;
   c.seed             = cfg->seed;
   c.page_size        = cache_config_page_size(cfg->cache_cfg);
   c.pages_per_extent = cache_config_pages_per_extent(cfg->cache_cfg);
   return c;
}

static uint32
num_indices_of(const routing_config *cfg, uint32 num_fingerprints)
{
   uint32 lnb = 31 - __builtin_clz(num_fingerprints);
   if (lnb < cfg->log_index_size) {
      lnb = cfg->log_index_size;
   }
   return 1u << (lnb - cfg->log_index_size);
}

static uint64
now_ns(void)
{
   struct timespec ts;
   clock_gettime(CLOCK_MONOTONIC, &ts);
   return (uint64)ts.tv_sec * 1000000000ull + (uint64)ts.tv_nsec;
}

static uint64
env_u64(const char *name, uint64 dflt)
{
   const char *s = getenv(name);
   return s ? (uint64)atoll(s) : dflt;
}

/* ---- registry of device-resident filters, keyed by (cache, index-extent address) -------- */
/* An engine batch shared by the filters built (or imported) together. `entries` counts the
 * registry entries naming it, `pins` the running calls using it; it is destroyed when both
 * are zero. Its device bytes count against the registry bound while entries > 0. */
typedef struct shim_batch {
   rf_amd_batch *b;
   uint32        entries;
   uint32        pins;
   uint64        bytes;
   int           full; /* build work buffers kept (entries in place for incremental adds) */
} shim_batch;

typedef struct resident_filter {
   const cache            *cc;
   uint64                  addr;
   shim_batch             *sb;
   uint32                  f;
   struct resident_filter *next;                /* hash chain */
   struct resident_filter *lru_prev, *lru_next; /* most recently used first */
} resident_filter;

#define REGISTRY_BUCKETS 4096
static resident_filter *g_registry[REGISTRY_BUCKETS];
static resident_filter  g_lru = {.lru_prev = &g_lru, .lru_next = &g_lru};
static pthread_mutex_t  g_registry_mu = PTHREAD_MUTEX_INITIALIZER;
static uint64           g_registry_bytes;
static uint64           g_registry_evictions, g_registry_trims;

static uint64 g_registry_limit; /* bytes; 0 = not yet read from RF_AMD_REGISTRY_MIB */

static uint64
registry_limit(void)
{
   if (!g_registry_limit) {
      g_registry_limit = env_u64("RF_AMD_REGISTRY_MIB", 8192) << 20;
   }
   return g_registry_limit;
}

static uint64
registry_bucket(const cache *cc, uint64 addr)
{
   return ((addr >> 12) ^ (uint64)(uintptr_t)cc) * 0x9E3779B97F4A7C15ull >> 52;
}

static void
lru_unlink(resident_filter *r)
{
   r->lru_prev->lru_next = r->lru_next;
   r->lru_next->lru_prev = r->lru_prev;
}

static void
lru_push_front(resident_filter *r)
{
   r->lru_next             = g_lru.lru_next;
   r->lru_prev             = &g_lru;
   g_lru.lru_next->lru_prev = r;
   g_lru.lru_next          = r;
}

static shim_batch *
shim_batch_new(rf_amd_batch *b, uint32 pins, int full)
{
   shim_batch *sb = malloc(sizeof(*sb));
   platform_assert(sb != NULL);
   sb->b       = b;
   sb->entries = 0;
   sb->pins    = pins;
   sb->bytes   = rf_amd_batch_device_bytes(b);
   sb->full    = full;
   return sb;
}

/* releases of batches decided under the registry lock, done after it is dropped */
typedef struct release_list {
   shim_batch **sb;
   uint32       n, cap;
} release_list;

static void
release_run(release_list *rl)
{
   for (uint32 i = 0; i < rl->n; i++) {
      rf_amd_batch_destroy_on(rl->sb[i]->b, NULL); /* stream-ordered, no device-wide wait */
      free(rl->sb[i]);
   }
   free(rl->sb);
   rl->sb = NULL;
   rl->n = rl->cap = 0;
}

/* the caller holds g_registry_mu; sb loses one entry or pin */
static void
shim_batch_drop_locked(shim_batch *sb, int entry, release_list *rl)
{
   if (entry) {
      platform_assert(sb->entries > 0);
      if (--sb->entries == 0) {
         g_registry_bytes -= sb->bytes;
      }
   } else {
      platform_assert(sb->pins > 0);
      sb->pins--;
   }
   if (sb->entries == 0 && sb->pins == 0) {
      if (rl->n == rl->cap) {
         rl->cap = rl->cap ? 2 * rl->cap : 8;
         rl->sb  = realloc(rl->sb, sizeof(*rl->sb) * rl->cap);
         platform_assert(rl->sb != NULL);
      }
      rl->sb[rl->n++] = sb;
   }
}

static void
registry_remove_locked(resident_filter *r, release_list *rl)
{
   for (resident_filter **pp = &g_registry[registry_bucket(r->cc, r->addr)]; *pp; pp = &(*pp)->next) {
      if (*pp == r) {
         *pp = r->next;
         break;
      }
   }
   lru_unlink(r);
   shim_batch *sb = r->sb;
   free(r);
   shim_batch_drop_locked(sb, 1, rl);
}

/* Keeps the registry under its bound: least recently used first, a batch that still holds
 * its build buffers is trimmed to its probe-only state, then filters are evicted. Pinned
 * batches are left alone. `keep` (may be NULL) is never evicted. */
static void
registry_evict_locked(const resident_filter *keep, uint64 limit, release_list *rl)
{
   /* pass 1 trims (least recently used first), pass 2 evicts */
   for (int pass = 0; pass < 2; pass++) {
      resident_filter *r = g_lru.lru_prev;
      while (g_registry_bytes > limit && r != &g_lru) {
         resident_filter *prev = r->lru_prev;
         shim_batch      *sb   = r->sb;
         if (r != keep && sb->pins == 0) {
            if (pass == 0 && sb->full) {
               rf_amd_batch_trim(sb->b, NULL);
               const uint64 nb = rf_amd_batch_device_bytes(sb->b);
               if (sb->entries) {
                  g_registry_bytes -= sb->bytes - nb;
               }
               sb->bytes = nb;
               sb->full  = 0;
               g_registry_trims++;
            } else if (pass == 1) {
               registry_remove_locked(r, rl);
               g_registry_evictions++;
            }
         }
         r = prev;
      }
   }
}

/* the filter's batch and index, pinned (registry_unpin when done), or NULL */
static shim_batch *
registry_find_pin(const cache *cc, uint64 addr, uint32 *f)
{
   shim_batch *sb = NULL;
   pthread_mutex_lock(&g_registry_mu);
   for (resident_filter *r = g_registry[registry_bucket(cc, addr)]; r; r = r->next) {
      if (r->cc == cc && r->addr == addr) {
         sb = r->sb;
         *f = r->f;
         sb->pins++;
         lru_unlink(r);
         lru_push_front(r);
         break;
      }
   }
   pthread_mutex_unlock(&g_registry_mu);
   return sb;
}

/* n pins dropped under one lock (the async completion path: one acquisition per reap, not
 * per state) */
static void
registry_unpin_many(shim_batch *const *sb, uint64 n)
{
   release_list rl = {NULL, 0, 0};
   pthread_mutex_lock(&g_registry_mu);
   for (uint64 i = 0; i < n; i++) {
      if (sb[i]) {
         shim_batch_drop_locked(sb[i], 0, &rl);
      }
   }
   pthread_mutex_unlock(&g_registry_mu);
   release_run(&rl);
}

static void
registry_unpin(shim_batch *sb)
{
   if (!sb) {
      return;
   }
   release_list rl = {NULL, 0, 0};
   pthread_mutex_lock(&g_registry_mu);
   shim_batch_drop_locked(sb, 0, &rl);
   pthread_mutex_unlock(&g_registry_mu);
   release_run(&rl);
}

/*
 * Registers filter f of sb for (cc, addr), turning one of the caller's pins into the entry.
 * replace = 0 (a filter imported from the cache): an entry present already wins; the
 * caller's pin moves to that entry's batch, which is returned (*f updated). replace = 1 (a
 * filter just built at addr): any entry there is stale -- its pages were freed and
 * reallocated without our dec_ref seeing it reach zero -- and is dropped.
 */
static shim_batch *
registry_insert(const cache *cc, uint64 addr, shim_batch *sb, uint32 *f, int replace, int keep_pin)
{
   release_list rl = {NULL, 0, 0};
   pthread_mutex_lock(&g_registry_mu);
   resident_filter **head = &g_registry[registry_bucket(cc, addr)];
   for (resident_filter *r = *head; r; r = r->next) {
      if (r->cc == cc && r->addr == addr) {
         if (!replace) {
            shim_batch *have = r->sb;
            *f               = r->f;
            have->pins++;
            shim_batch_drop_locked(sb, 0, &rl); /* ours is not needed */
            if (!keep_pin) {
               shim_batch_drop_locked(have, 0, &rl);
            }
            lru_unlink(r);
            lru_push_front(r);
            pthread_mutex_unlock(&g_registry_mu);
            release_run(&rl);
            return have;
         }
         registry_remove_locked(r, &rl);
         break;
      }
   }
   resident_filter *r = malloc(sizeof(*r));
   platform_assert(r != NULL);
   r->cc   = cc;
   r->addr = addr;
   r->sb   = sb;
   r->f    = *f;
   r->next = *head;
   *head   = r;
   lru_push_front(r);
   if (sb->entries++ == 0) {
      g_registry_bytes += sb->bytes;
   }
   if (!keep_pin) {
      shim_batch_drop_locked(sb, 0, &rl);
   }
   registry_evict_locked(r, registry_limit(), &rl);
   pthread_mutex_unlock(&g_registry_mu);
   release_run(&rl);
   return sb;
}

static void
registry_drop(const cache *cc, uint64 addr)
{
   release_list rl = {NULL, 0, 0};
   pthread_mutex_lock(&g_registry_mu);
   for (resident_filter *r = g_registry[registry_bucket(cc, addr)]; r; r = r->next) {
      if (r->cc == cc && r->addr == addr) {
         registry_remove_locked(r, &rl);
         break;
      }
   }
   pthread_mutex_unlock(&g_registry_mu);
   release_run(&rl);
}

/* every unpinned filter out (device memory ran out) */
static void
registry_evict_all(void)
{
   release_list rl = {NULL, 0, 0};
   pthread_mutex_lock(&g_registry_mu);
   registry_evict_locked(NULL, 0, &rl);
   pthread_mutex_unlock(&g_registry_mu);
   release_run(&rl);
   rf_amd_engine_sync(engine());
   rf_amd_engine_pool_trim(engine(), 0);
}

void
routing_filter_amd_registry_set_limit(uint64 mib)
{
   release_list rl = {NULL, 0, 0};
   pthread_mutex_lock(&g_registry_mu);
   g_registry_limit = mib << 20;
   registry_evict_locked(NULL, g_registry_limit, &rl);
   pthread_mutex_unlock(&g_registry_mu);
   release_run(&rl);
}

void
routing_filter_amd_registry_stats(uint64 *bytes, uint64 *evictions, uint64 *trims)
{
   pthread_mutex_lock(&g_registry_mu);
   *bytes     = g_registry_bytes;
   *evictions = g_registry_evictions;
   *trims     = g_registry_trims;
   pthread_mutex_unlock(&g_registry_mu);
}

/* ---- a filter read back through the cache (the image of a filter built elsewhere) ------ */
/*
 * Walks the index slots of the index extent (src/routing_filter.c:178-198) and copies each
 * data page once, in placement order. img->pages / img->slots are malloc'd; abs_slots (may
 * be NULL) receives the absolute slots as stored.
 */
static platform_status
rf_read_image(cache                *cc,
              const routing_config *cfg,
              const routing_filter *f,
              rf_amd_image         *img,
              uint64              **abs_slots_out)
{
   memset(img, 0, sizeof(*img));
   const uint64 ps             = cache_config_page_size(cfg->cache_cfg);
   const uint64 addrs_per_page = ps / sizeof(uint64);
   const uint32 ni             = num_indices_of(cfg, f->num_fingerprints);
   uint64      *abs_slots      = malloc(sizeof(uint64) * ni);
   uint64      *page_addr      = malloc(sizeof(uint64) * ni);
   uint64      *slots          = malloc(sizeof(uint64) * ni);
   if (!abs_slots || !page_addr || !slots) {
      free(abs_slots);
      free(page_addr);
      free(slots);
      return STATUS_NO_MEMORY;
   }
   uint32 np = 0;
   for (uint32 i = 0; i < ni; i++) {
      if (i % addrs_per_page == 0) {
         page_handle *ip = cache_get(cc, f->addr + ps * (i / addrs_per_page), TRUE, PAGE_TYPE_FILTER);
         uint32       m  = ni - i < addrs_per_page ? ni - i : (uint32)addrs_per_page;
         memcpy(abs_slots + i, ip->data, m * sizeof(uint64));
         cache_unget(cc, ip);
      }
      const uint64 page = abs_slots[i] - abs_slots[i] % ps;
      if (np == 0 || page_addr[np - 1] != page) {
         page_addr[np++] = page;
      }
      slots[i] = (uint64)(np - 1) * ps + abs_slots[i] % ps;
   }
   uint8 *pages = malloc(ps * np + 16);
   if (!pages) {
      free(abs_slots);
      free(page_addr);
      free(slots);
      return STATUS_NO_MEMORY;
   }
   for (uint32 k = 0; k < np; k++) {
      page_handle *pg = cache_get(cc, page_addr[k], TRUE, PAGE_TYPE_FILTER);
      memcpy(pages + k * ps, pg->data, ps);
      cache_unget(cc, pg);
   }
   free(page_addr);
   img->info.num_fingerprints = f->num_fingerprints;
   img->info.num_unique       = f->num_unique;
   img->info.value_size       = f->value_size;
   img->info.num_indices      = ni;
   img->info.num_pages        = np;
   img->pages                 = pages;
   img->slots                 = slots;
   if (abs_slots_out) {
      *abs_slots_out = abs_slots;
   } else {
      free(abs_slots);
   }
   return STATUS_OK;
}

/* The filter's device-resident batch and index, pinned: from the registry, or imported from
 * the cache (probe-only). An import that finds the device full evicts the registry and
 * retries once, so a lookup does not fail while evictable filters hold the memory. */
static platform_status
resident_pin(cache *cc, const routing_config *cfg, const routing_filter *f, shim_batch **out, uint32 *fi)
{
   *out = registry_find_pin(cc, f->addr, fi);
   if (*out) {
      return STATUS_OK;
   }
   rf_amd_engine *e = engine();
   if (!e) {
      return status_of(RF_AMD_ENODEV);
   }
   rf_amd_image    img;
   platform_status rc = rf_read_image(cc, cfg, f, &img, NULL);
   if (!SUCCESS(rc)) {
      return rc;
   }
   rf_amd_config c = amd_config(cfg);
   rf_amd_batch *b = NULL;
   int           r = rf_amd_batch_import(e, &c, 1, &img.info, img.pages, img.slots, 0, &b);
   if (r == RF_AMD_ENOMEM) {
      registry_evict_all();
      r = rf_amd_batch_import(e, &c, 1, &img.info, img.pages, img.slots, 0, &b);
   }
   rf_amd_image_free(&img);
   if (r) {
      return status_of(r);
   }
   *fi  = 0;
   *out = registry_insert(cc, f->addr, shim_batch_new(b, 1, 0), fi, 0, 1);
   return STATUS_OK;
}

static inline void
unlock_and_unget_page(cache *cc, page_handle *page)
{
   cache_unlock(cc, page);
   cache_unclaim(cc, page);
   cache_unget(cc, page);
}

/* ---- routing_filter_add: concurrent calls coalesced into one GPU batch ----------------- */
typedef struct add_req {
   rf_amd_config      c;
   shim_batch        *old_sb; /* pinned by the caller, or NULL */
   uint32             old_f;
   const uint32      *hashes;
   uint32             n;
   uint16             value;
   /* results */
   int                rc;
   rf_amd_filter_info info;
   uint8             *pages; /* pinned read-back buffer: pages, then slots */
   uint64            *slots;
   uint64             pin_cap; /* bytes of the pinned buffer (returned to the pool) */
   uint64             fence;   /* the read-back's completion point on the engine stream */
   uint32             direct;  /* 1 + registration slot: no read-back, the adding thread places the image itself */
   shim_batch        *sb; /* the built batch, pinned once for this request */
   uint32             f;
   int                done;
   struct add_req    *next;
   /* staging: where this request's fingerprints go in the engine's pinned buffer; whichever
      thread claims the copy first (the request's own thread, or the combiner) makes it */
   uint32            *stage_dst;
   int                claim, copied; /* atomic */
} add_req;

static pthread_mutex_t g_add_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t  g_add_cv = PTHREAD_COND_INITIALIZER;
static add_req        *g_add_head, *g_add_tail;
static int             g_add_busy;
static uint64          g_add_batches, g_add_filters;
/* where routing_filter_add spends its time (routing_filter_amd_add_breakdown): per combiner
 * batch -- batch creation, the staging copies, the build, the info read-back, the image
 * read-back; per add -- the wait for its batch, the page allocation and fill */
enum { AB_CALLS, AB_BATCHES, AB_CREATE, AB_STAGE, AB_BUILD, AB_INFOS, AB_READBACK, AB_WAIT, AB_PLACE, AB_N };
static uint64 g_add_ns[AB_N];
#define AB_ADD(k, v) __atomic_fetch_add(&g_add_ns[k], (v), __ATOMIC_RELAXED)

/* out[0..8] as AB_*, out[9] ns creating the engine, out[10] ns registering cache buffers */
void
routing_filter_amd_add_breakdown(uint64 *out)
{
   for (int k = 0; k < AB_N; k++) {
      out[k] = __atomic_load_n(&g_add_ns[k], __ATOMIC_RELAXED);
   }
   out[AB_N]     = g_engine_ns;
   out[AB_N + 1] = g_register_ns;
}

/* copies a request's fingerprints into its staging slot, unless another thread has claimed it */
static void
add_copy(add_req *q)
{
   if (q->stage_dst && __atomic_exchange_n(&q->claim, 1, __ATOMIC_ACQ_REL) == 0) {
      memcpy(q->stage_dst, q->hashes, sizeof(uint32) * q->n);
      __atomic_store_n(&q->copied, 1, __ATOMIC_RELEASE);
   }
}

/* pinned read-back buffers, recycled: an image is read straight into one by the DMA engine
 * (a read-back into malloc'd memory goes through the driver's staging copies), then copied
 * into the cache pages by its adding thread */
#define PIN_POOL 16
static struct {
   void  *p;
   uint64 cap;
} g_pin_pool[PIN_POOL];
static uint32          g_pin_n;
static uint64          g_pin_bytes; /* bytes held by the pool */
static pthread_mutex_t g_pin_mu = PTHREAD_MUTEX_INITIALIZER;

/* RF_SHIM_PIN_POOL_MIB (default 256): the pinned bytes the pool may keep between adds; a
 * buffer that would take it over the cap is freed instead of pooled */
static uint64
pin_pool_cap(void)
{
   static uint64 v = 0;
   if (!v) {
      const char *s = getenv("RF_SHIM_PIN_POOL_MIB");
      uint64      m = s ? strtoull(s, NULL, 10) : 256;
      v             = (m << 20) + 1;
   }
   return v - 1;
}

/* RF_SHIM_PINNED=0: read-backs into malloc'd memory after one engine-wide sync (A/B) */
static int
pin_enabled(void)
{
   static int v = -1;
   if (v < 0) {
      const char *s = getenv("RF_SHIM_PINNED");
      v             = (s && s[0] == '0') ? 0 : 1;
   }
   return v;
}

static void *
pin_take_any(rf_amd_engine *e, uint64 bytes, uint64 *cap, int force)
{
   if (!force && !pin_enabled()) {
      *cap = bytes;
      return malloc(bytes);
   }
   pthread_mutex_lock(&g_pin_mu);
   for (uint32 i = 0; i < g_pin_n; i++) { /* the smallest that fits */
      if (g_pin_pool[i].cap >= bytes) {
         uint32 best = i;
         for (uint32 j = i + 1; j < g_pin_n; j++) {
            if (g_pin_pool[j].cap >= bytes && g_pin_pool[j].cap < g_pin_pool[best].cap) {
               best = j;
            }
         }
         void *p = g_pin_pool[best].p;
         *cap    = g_pin_pool[best].cap;
         g_pin_bytes -= *cap;
         g_pin_pool[best] = g_pin_pool[--g_pin_n];
         pthread_mutex_unlock(&g_pin_mu);
         return p;
      }
   }
   pthread_mutex_unlock(&g_pin_mu);
   const uint64 c = bytes < (1ull << 20) ? (1ull << 20) : bytes + bytes / 4;
   void        *p = NULL;
   if (rf_amd_host_alloc(e, c, &p)) {
      return NULL;
   }
   *cap = c;
   return p;
}

static void
pin_give_any(rf_amd_engine *e, void *p, uint64 cap, int force)
{
   if (!p) {
      return;
   }
   if (!force && !pin_enabled()) {
      free(p);
      return;
   }
   pthread_mutex_lock(&g_pin_mu);
   if (g_pin_n < PIN_POOL && g_pin_bytes + cap <= pin_pool_cap()) {
      g_pin_pool[g_pin_n].p   = p;
      g_pin_pool[g_pin_n].cap = cap;
      g_pin_n++;
      g_pin_bytes += cap;
      p = NULL;
   }
   pthread_mutex_unlock(&g_pin_mu);
   if (p) {
      rf_amd_host_free(e, p);
   }
}

static void *
pin_take(rf_amd_engine *e, uint64 bytes, uint64 *cap)
{
   return pin_take_any(e, bytes, cap, 0);
}

static void
pin_give(rf_amd_engine *e, void *p, uint64 cap)
{
   pin_give_any(e, p, cap, 0);
}

/* ---- images placed straight into the cache's pages -----------------------------------------
 * A cache attached by routing_filter_amd_cache_attach has its page buffer (clockcache.c:3426,
 * one platform_buffer of cfg->capacity bytes) registered with the engine; an add then writes
 * its image into the pages it allocated with one kernel (its stores cross PCIe), instead of a
 * read-back into a bounce buffer and a memcpy per page (src/routing_filter.c:603-633 fills the
 * pages in place too). The cache is a clockcache (SplinterDB's only cache); every destination
 * is checked against the registered range by the engine before the launch.
 * Registration is opt-in because only the caller knows the buffer's lifetime: the unmodified
 * reference unmaps it in splinterdb_close (clockcache.c:3546 -> platform_buffer.c:86) without
 * telling the shim, and a GPU store through a registration whose pages were unmapped is a GPU
 * memory fault, not a detectable miss. So caches are never registered implicitly: an
 * unmodified caller gets the bounce-buffer path; a caller that attaches a cache after opening
 * the store releases it (routing_filter_amd_cache_release) before closing it.
 * RF_SHIM_DIRECT=0 keeps the bounce-buffer path even for attached caches. */
#define DIRECT_CACHES 16
static struct {
   const cache *cc;
   char        *base;
   uint64       bytes;
   int          ok;       /* attached and registered: placements go straight into its pages */
   int          stale;    /* a placement's canary showed its stores did not reach the host's pages */
   uint32       inflight; /* adds placing through this registration now */
} g_direct[DIRECT_CACHES];
static uint32          g_direct_n;
static uint64          g_direct_stale_seen; /* registrations found stale (routing_filter_amd_direct_stats) */
static pthread_mutex_t g_direct_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t  g_direct_cv = PTHREAD_COND_INITIALIZER;

static int
direct_enabled(void)
{
   static int v = -1;
   if (v < 0) {
      const char *s = getenv("RF_SHIM_DIRECT");
      v             = (s && s[0] == '0') ? 0 : 1;
   }
   return v;
}

/* registers cc's page buffer (caller holds g_direct_mu) */
static int
direct_register(rf_amd_engine *e, uint32 i, char *base, uint64 bytes)
{
   /* registering pins the whole buffer (once, ~proportional to its size): caches over
      RF_SHIM_DIRECT_MAX_MIB (default 65,536) keep the bounce-buffer path */
   const uint64 max_b = env_u64("RF_SHIM_DIRECT_MAX_MIB", 65536) << 20;
   const uint64 t0    = mono_ns();
   g_direct[i].base  = base;
   g_direct[i].bytes = bytes;
   g_direct[i].stale = 0;
   g_direct[i].ok    = base && bytes && bytes <= max_b && rf_amd_host_register(e, base, bytes) == 0;
   g_register_ns += mono_ns() - t0;
   return g_direct[i].ok;
}

/* The registration an add places through: 1 + its slot when cc is attached and its page
 * buffer is the one registered, 0 for the bounce-buffer path. The caller owns one in-flight
 * count on the slot until direct_done. */
static uint32
cache_direct(cache *cc)
{
   if (!direct_enabled()) {
      return 0;
   }
   uint32      slot = 0;
   clockcache *ccc  = (clockcache *)cc;
   pthread_mutex_lock(&g_direct_mu);
   for (uint32 i = 0; i < g_direct_n; i++) {
      if (g_direct[i].cc == cc) {
         /* a placement found stale, or another buffer behind the same cache struct (attached
            and not released): the bounce path until the cache is attached again */
         if (g_direct[i].ok && !g_direct[i].stale && g_direct[i].base == ccc->data
             && ccc->cfg && g_direct[i].bytes == ccc->cfg->capacity)
         {
            slot = i + 1;
            g_direct[i].inflight++;
         }
         break;
      }
   }
   pthread_mutex_unlock(&g_direct_mu);
   return slot;
}

/* an add is done placing through its registration (stale: its canary showed the stores did
 * not reach the host's pages) */
static void
direct_done(uint32 slot, int stale)
{
   if (!slot) {
      return;
   }
   pthread_mutex_lock(&g_direct_mu);
   g_direct[slot - 1].inflight--;
   if (stale && !g_direct[slot - 1].stale) {
      g_direct[slot - 1].stale = 1;
      g_direct_stale_seen++;
   }
   pthread_cond_broadcast(&g_direct_cv);
   pthread_mutex_unlock(&g_direct_mu);
}

/* waits until no add places through slot i, then drops its registration (caller holds
 * g_direct_mu) */
static void
direct_drop(uint32 i)
{
   const int was_ok = g_direct[i].ok;
   g_direct[i].ok   = 0; /* no new add takes this registration */
   while (g_direct[i].inflight) {
      pthread_cond_wait(&g_direct_cv, &g_direct_mu);
   }
   if (was_ok) {
      rf_amd_engine *e = engine();
      if (e) {
         (void)rf_amd_host_unregister(e, g_direct[i].base);
      }
   }
}

/* Attach: the engine now (not inside the store's first routing_filter_add) and cc's page
 * buffer registered, so adds place their images straight into its pages. Call after the
 * store opened; release before it closes. 0 = attached, -1 = the bounce path stays (no GPU,
 * the buffer over RF_SHIM_DIRECT_MAX_MIB, the registration failed, or too many caches). */
int
routing_filter_amd_cache_attach(cache *cc)
{
   rf_amd_engine *e = engine();
   if (!e || !cc || !direct_enabled()) {
      /* RF_SHIM_DIRECT=0: nothing is registered (a caller that sees -1 need not release;
         ADVICE r5: a registration here outlived the buffer's munmap) */
      return -1;
   }
   clockcache *ccc   = (clockcache *)cc;
   char       *base  = ccc->data;
   uint64      bytes = ccc->cfg ? ccc->cfg->capacity : 0;
   int         ok    = 0;
   pthread_mutex_lock(&g_direct_mu);
   uint32 i = 0;
   while (i < g_direct_n && g_direct[i].cc != cc) {
      i++;
   }
   if (i < g_direct_n) { /* attached before: registered anew (same or another buffer) */
      direct_drop(i);
   } else if (g_direct_n < DIRECT_CACHES) {
      g_direct_n++;
      g_direct[i].cc       = cc;
      g_direct[i].inflight = 0;
   } else {
      pthread_mutex_unlock(&g_direct_mu);
      return -1;
   }
   ok = direct_register(e, i, base, bytes);
   pthread_mutex_unlock(&g_direct_mu);
   return ok ? 0 : -1;
}

/* out[0] = caches registered now, out[1] = registrations found stale by a placement */
void
routing_filter_amd_direct_stats(uint64 *out)
{
   pthread_mutex_lock(&g_direct_mu);
   uint64 n = 0, fl = 0;
   for (uint32 i = 0; i < g_direct_n; i++) {
      n += g_direct[i].ok != 0;
      fl += g_direct[i].inflight;
   }
   out[0] = n;
   out[1] = g_direct_stale_seen;
   out[2] = fl;
   pthread_mutex_unlock(&g_direct_mu);
}

/* a cache is going away (its buffer will be unmapped): unregister it once no add still
 * places through it; later adds through cc take the bounce-buffer path until it is attached
 * again */
void
routing_filter_amd_cache_release(cache *cc)
{
   pthread_mutex_lock(&g_direct_mu);
   for (uint32 i = 0; i < g_direct_n; i++) {
      if (g_direct[i].cc == cc) {
         direct_drop(i);
         break;
      }
   }
   pthread_mutex_unlock(&g_direct_mu);
}

/* builds k requests of one config as one batch; a batch that cannot be created (one
 * request's geometry, or memory) is retried request by request so each gets its own error */
static void
run_adds(rf_amd_engine *e, add_req **rq, uint32 k)
{
   uint32        *num_new = malloc(sizeof(uint32) * k);
   uint16        *value   = malloc(sizeof(uint16) * k);
   rf_amd_batch **old     = malloc(sizeof(*old) * k);
   uint32        *old_idx = malloc(sizeof(uint32) * k);
   platform_assert(num_new && value && old && old_idx);
   uint64 total = 0;
   int    any_old = 0;
   for (uint32 i = 0; i < k; i++) {
      num_new[i] = rq[i]->n;
      value[i]   = rq[i]->value;
      old[i]     = rq[i]->old_sb ? rq[i]->old_sb->b : NULL;
      old_idx[i] = rq[i]->old_f;
      any_old |= old[i] != NULL;
      total += rq[i]->n;
   }
   rf_amd_batch *b  = NULL;
   uint64        tp = now_ns();
   int           r = rf_amd_batch_create(e, &rq[0]->c, k, num_new, value, any_old ? old : NULL,
                               any_old ? old_idx : NULL, &b);
   if (r == RF_AMD_ENOMEM) {
      registry_evict_all();
      r = rf_amd_batch_create(e, &rq[0]->c, k, num_new, value, any_old ? old : NULL, any_old ? old_idx : NULL, &b);
   }
   free(num_new);
   free(value);
   free(old);
   free(old_idx);
   if (r && k > 1) {
      for (uint32 i = 0; i < k; i++) {
         run_adds(e, rq + i, 1);
      }
      return;
   }
   if (r) {
      rq[0]->rc = r;
      return;
   }
   /* the fingerprints go straight into the engine's pinned staging buffer, each request's
      copy made by its own waiting thread or by this one, whichever claims it first */
   uint32 *stage = NULL;
   r             = rf_amd_batch_stage_begin(b, &stage);
   uint64 tn     = now_ns();
   AB_ADD(AB_CREATE, tn - tp);
   tp = tn;
   if (!r) {
      pthread_mutex_lock(&g_add_mu);
      uint64 at = 0;
      for (uint32 i = 0; i < k; i++) {
         rq[i]->stage_dst = stage + at;
         at += rq[i]->n;
      }
      pthread_cond_broadcast(&g_add_cv);
      pthread_mutex_unlock(&g_add_mu);
      for (uint32 i = 0; i < k; i++) {
         add_copy(rq[i]);
      }
      for (uint32 i = 0; i < k; i++) {
         while (!__atomic_load_n(&rq[i]->copied, __ATOMIC_ACQUIRE)) {
            __builtin_ia32_pause();
         }
      }
      tn = now_ns();
      AB_ADD(AB_STAGE, tn - tp);
      tp = tn;
      r = rf_amd_batch_stage_build(b);
      tn = now_ns();
      AB_ADD(AB_BUILD, tn - tp);
      tp = tn;
   }
   (void)total;
   rf_amd_filter_info *infos = malloc(sizeof(*infos) * k);
   platform_assert(infos != NULL);
   if (!r) {
      r = rf_amd_batch_infos(b, infos, rf_amd_engine_stream(e));
      tn = now_ns();
      AB_ADD(AB_INFOS, tn - tp);
      tp = tn;
   }
   const uint64 ps = rq[0]->c.page_size;
   for (uint32 i = 0; i < k && !r; i++) {
      add_req *q = rq[i];
      q->info    = infos[i];
      if (q->info.error) {
         q->rc = RF_AMD_EINVAL; /* a block over a page: undefined behaviour in the reference */
         continue;
      }
      if (q->direct) {
         continue; /* its thread writes the image into its cache pages */
      }
      /* the image and its slots into a pinned buffer; each request gets its own completion
         point, so its thread places its pages while the next images are still in flight */
      const uint64 pb = (ps * q->info.num_pages + 15) & ~15ull;
      q->pages        = pin_take(e, pb + sizeof(uint64) * q->info.num_indices, &q->pin_cap);
      if (!q->pages) {
         r = RF_AMD_ENOMEM;
         break;
      }
      q->slots = (uint64 *)(q->pages + pb);
      r        = rf_amd_batch_read_image_async(b, i, q->pages, ps * q->info.num_pages, q->slots,
                                        q->info.num_indices, NULL);
      if (!r && pin_enabled()) {
         r = rf_amd_engine_fence(e, &q->fence);
      }
   }
   if (!r && !pin_enabled()) {
      r = rf_amd_engine_sync(e);
   }
   AB_ADD(AB_READBACK, now_ns() - tp);
   AB_ADD(AB_BATCHES, 1);
   free(infos);
   if (r) {
      (void)rf_amd_engine_sync(e); /* read-backs already queued land before their buffers go */
      for (uint32 i = 0; i < k; i++) {
         rq[i]->rc = r;
         if (rq[i]->fence) {
            (void)rf_amd_engine_fence_wait(e, rq[i]->fence);
            rq[i]->fence = 0;
         }
         pin_give(e, rq[i]->pages, rq[i]->pin_cap);
         rq[i]->pages = NULL;
         rq[i]->slots = NULL;
      }
      rf_amd_batch_destroy_on(b, NULL);
      return;
   }
   uint32 ok = 0;
   for (uint32 i = 0; i < k; i++) {
      ok += rq[i]->rc == 0;
   }
   if (ok == 0) {
      rf_amd_batch_destroy_on(b, NULL);
      return;
   }
   shim_batch *sb = shim_batch_new(b, ok, 1);
   for (uint32 i = 0; i < k; i++) {
      if (rq[i]->rc == 0) {
         rq[i]->sb = sb;
         rq[i]->f  = i;
      }
   }
   __atomic_fetch_add(&g_add_batches, 1, __ATOMIC_RELAXED);
   __atomic_fetch_add(&g_add_filters, k, __ATOMIC_RELAXED);
}

/* the combiner's pass over the requests it took: one batch per distinct config */
static void
run_add_list(rf_amd_engine *e, add_req *list)
{
   uint32 n = 0;
   for (add_req *q = list; q; q = q->next) {
      n++;
   }
   add_req **rq = malloc(sizeof(*rq) * n);
   platform_assert(rq != NULL);
   uint32 m = 0;
   for (add_req *q = list; q; q = q->next) {
      rq[m++] = q;
   }
   for (uint32 s = 0; s < n;) {
      uint32 t = s + 1; /* gather the requests sharing rq[s]'s config to the front */
      for (uint32 i = s + 1; i < n; i++) {
         if (memcmp(&rq[i]->c, &rq[s]->c, sizeof(rf_amd_config)) == 0) {
            add_req *x = rq[t];
            rq[t++]    = rq[i];
            rq[i]      = x;
         }
      }
      run_adds(e, rq + s, t - s);
      s = t;
   }
   free(rq);
}

/* queue the request; build it (and whatever else is queued) if the engine is idle, else wait
 * for the combiner that takes it */
static void
add_submit(rf_amd_engine *e, add_req *q)
{
   pthread_mutex_lock(&g_add_mu);
   q->next = NULL;
   if (g_add_tail) {
      g_add_tail->next = q;
   } else {
      g_add_head = q;
   }
   g_add_tail = q;
   while (!q->done) {
      if (!g_add_busy) {
         g_add_busy    = 1;
         add_req *list = g_add_head;
         g_add_head = g_add_tail = NULL;
         pthread_mutex_unlock(&g_add_mu);
         run_add_list(e, list);
         pthread_mutex_lock(&g_add_mu);
         for (add_req *x = list; x; x = x->next) {
            x->done = 1;
         }
         g_add_busy = 0;
         pthread_cond_broadcast(&g_add_cv);
      } else {
         pthread_cond_wait(&g_add_cv, &g_add_mu);
         if (q->stage_dst && !__atomic_load_n(&q->claim, __ATOMIC_ACQUIRE)) {
            pthread_mutex_unlock(&g_add_mu); /* our share of the staging copy */
            add_copy(q);
            pthread_mutex_lock(&g_add_mu);
         }
      }
   }
   pthread_mutex_unlock(&g_add_mu);
}

void
routing_filter_amd_add_stats(uint64 *batches, uint64 *filters)
{
   *batches = __atomic_load_n(&g_add_batches, __ATOMIC_RELAXED);
   *filters = __atomic_load_n(&g_add_filters, __ATOMIC_RELAXED);
}

/* pages held write-locked at once while their images land (the reference holds one) */
#define PLACE_CHUNK 512

/* Allocates q's data pages in the reference's order (mini_alloc + cache_alloc per page,
 * :603-610) and has the engine write the image into them and the absolute index slots into
 * the index pages (:612-633), PLACE_CHUNK pages per launch, each chunk unlocked once its
 * images have landed. A launch the engine refuses (a page outside the registered buffer)
 * falls back to a read-back of the image and a copy per page. */
static int
place_direct(rf_amd_engine  *e,
             cache          *cc,
             add_req        *q,
             mini_allocator *mini,
             page_handle   **index_page,
             uint64          addrs_per_page,
             uint64         *page_addr)
{
   const uint64 np  = q->info.num_pages, ni = q->info.num_indices;
   const uint64 nip = (ni + addrs_per_page - 1) / addrs_per_page;
   const uint64 ps  = q->c.page_size;
   rf_amd_batch *b  = q->sb->b;
   uint64        tcap = 0, bcap = 0;
   uint64       *table = pin_take_any(e, sizeof(uint64) * (2 * np + nip + 1), &tcap, 1);
   uint8        *bounce = NULL; /* the fallback's read-back: pages, then slots */
   page_handle **ph     = malloc(sizeof(*ph) * (np ? np : 1));
   platform_assert(table && ph);
   for (uint64 i = 0; i < nip; i++) {
      table[2 * np + i] = (uint64)(uintptr_t)index_page[i]->data;
   }
   /* canary: a word the host writes into the first data page of each chunk (and into index
      slot 0 before the last chunk) before the launch; once the chunk's images have landed it
      must be gone. If it is not, the registration no longer maps these pages (the buffer was
      unmapped and mapped again at the same address): the chunk and the rest of the
      image take the bounce path and the registration is replaced on the next add. */
   const uint64 canary = 0x5bd1e9955bd1e995ull ^ now_ns() ^ (uint64)(uintptr_t)q;
   int          stale  = 0;
   for (uint64 k0 = 0; k0 < np || k0 == 0; k0 += PLACE_CHUNK) {
      const uint64 cnt  = np - k0 < PLACE_CHUNK ? np - k0 : PLACE_CHUNK;
      const int    last = k0 + cnt == np;
      for (uint64 k = k0; k < k0 + cnt; k++) {
         page_addr[k]     = mini_alloc(mini, 0, NULL);
         ph[k]            = cache_alloc(cc, page_addr[k], PAGE_TYPE_FILTER);
         table[k]         = (uint64)(uintptr_t)ph[k]->data;
         table[np + k]    = page_addr[k];
      }
      volatile uint64 *cw0 = cnt ? (volatile uint64 *)ph[k0]->data : NULL;
      volatile uint64 *cw1 = last && ni ? (volatile uint64 *)index_page[0]->data : NULL;
      if (!bounce) {
         if (cw0) {
            *cw0 = canary;
         }
         if (cw1) {
            *cw1 = canary;
         }
      }
      int r = bounce ? 1
                     : rf_amd_batch_place_image(b, q->f, table, (uint32)np, (uint32)k0, (uint32)cnt, last,
                                                (uint32)addrs_per_page, NULL);
      uint64 fence = 0;
      if (!r) {
         r = rf_amd_engine_fence(e, &fence);
      }
      if (!r) {
         r = rf_amd_engine_fence_wait(e, fence);
      }
      if (!r && ((cw0 && *cw0 == canary) || (cw1 && *cw1 == canary))) {
         stale = 1;
         r     = 1;
      }
      if (r) {
         if (!bounce) { /* one read-back of the whole image and its slots */
            const uint64 pb = (ps * np + 15) & ~15ull;
            bounce          = pin_take_any(e, pb + sizeof(uint64) * ni + 8, &bcap, 1);
            platform_assert(bounce != NULL);
            platform_assert(rf_amd_batch_read_image_async(b, q->f, bounce, ps * np, bounce + pb, (uint32)ni,
                                                          NULL)
                            == 0);
            platform_assert(rf_amd_engine_sync(e) == 0);
         }
         for (uint64 k = k0; k < k0 + cnt; k++) {
            memcpy(ph[k]->data, bounce + k * ps, ps);
         }
         if (last) {
            const uint64 *slots = (const uint64 *)(bounce + ((ps * np + 15) & ~15ull));
            for (uint64 i = 0; i < ni; i++) {
               uint64 *cursor = (uint64 *)index_page[i / addrs_per_page]->data + i % addrs_per_page;
               *cursor        = page_addr[slots[i] / ps] + slots[i] % ps;
            }
         }
      }
      for (uint64 k = k0; k < k0 + cnt; k++) {
         unlock_and_unget_page(cc, ph[k]);
      }
      if (last) {
         break;
      }
   }
   free(ph);
   pin_give_any(e, table, tcap, 1);
   pin_give_any(e, bounce, bcap, 1);
   return stale;
}

platform_status
routing_filter_add(cache                *cc,
                   const routing_config *cfg,
                   routing_filter       *old_filter,
                   routing_filter       *filter,
                   uint32               *new_fp_arr,
                   uint64                num_new_fp,
                   uint16                value)
{
   ZERO_CONTENTS(filter);
   rf_amd_engine *e = engine();
   if (!e) {
      return status_of(RF_AMD_ENODEV);
   }
   const uint64 nfp = num_new_fp + old_filter->num_fingerprints;
   if (nfp == 0 || nfp > routing_filter_max_fingerprints(cfg->cache_cfg, cfg)) {
      return STATUS_BAD_PARAM; /* the reference: __builtin_clz(0) / index-extent overflow */
   }
   add_req q;
   memset(&q, 0, sizeof(q));
   q.c      = amd_config(cfg);
   q.hashes = new_fp_arr;
   q.n      = (uint32)num_new_fp;
   q.value  = value;
   if (old_filter->addr != 0) {
      mini_prefetch(cc, PAGE_TYPE_FILTER, old_filter->meta_head); /* as :356 */
      platform_status rc = resident_pin(cc, cfg, old_filter, &q.old_sb, &q.old_f);
      if (!SUCCESS(rc)) {
         return rc;
      }
   }

   /* the image, on the GPU (coalesced with concurrent adds) */
   q.direct        = cache_direct(cc);
   const uint64 tw = now_ns();
   add_submit(e, &q);
   if (q.fence) { /* this request's image has landed in its pinned buffer */
      int fr = rf_amd_engine_fence_wait(e, q.fence);
      if (fr && !q.rc) {
         q.rc = fr;
      }
   }
   const uint64 tpl = now_ns();
   AB_ADD(AB_WAIT, tpl - tw);
   AB_ADD(AB_CALLS, 1);
   registry_unpin(q.old_sb);
   if (q.rc) {
      direct_done(q.direct, 0);
      pin_give(e, q.pages, q.pin_cap);
      registry_unpin(q.sb);
      return status_of(q.rc);
   }
   const rf_amd_filter_info info  = q.info;
   const uint8             *pages = q.pages;
   const uint64            *slots = q.slots;
   const uint64             ps    = cache_config_page_size(cfg->cache_cfg);

   /* the reference's page allocation sequence, :429-456 */
   allocator *al = cache_get_allocator(cc);
   uint64     meta_head;
   platform_status rc = allocator_alloc(al, &meta_head, PAGE_TYPE_FILTER);
   platform_assert_status_ok(rc);
   filter->meta_head = meta_head;
   mini_allocator mini;
   mini_init(&mini, cc, filter->meta_head, 0, 1, PAGE_TYPE_FILTER);

   const uint64 extent_size      = cache_config_extent_size(cfg->cache_cfg);
   const uint64 pages_per_extent = cache_config_pages_per_extent(cfg->cache_cfg);
   const uint64 addrs_per_page   = ps / sizeof(uint64);
   page_handle *index_page[MAX_PAGES_PER_EXTENT];
   uint64       index_addr = mini_alloc(&mini, 0, NULL);
   platform_assert(index_addr % extent_size == 0);
   index_page[0] = cache_alloc(cc, index_addr, PAGE_TYPE_FILTER);
   for (uint64 i = 1; i < pages_per_extent; i++) {
      uint64 next_index_addr = mini_alloc(&mini, 0, NULL);
      platform_assert(next_index_addr == index_addr + i * ps);
      index_page[i] = cache_alloc(cc, next_index_addr, PAGE_TYPE_FILTER);
   }
   filter->addr = index_addr;

   /* data pages in placement order (:453-455, :603-610), each filled from the image */
   uint64 *page_addr = malloc(sizeof(uint64) * info.num_pages);
   platform_assert(page_addr != NULL);
   if (q.direct) {
      direct_done(q.direct, place_direct(e, cc, &q, &mini, index_page, addrs_per_page, page_addr));
   } else {
      for (uint32 k = 0; k < info.num_pages; k++) {
         page_addr[k]      = mini_alloc(&mini, 0, NULL);
         page_handle *page = cache_alloc(cc, page_addr[k], PAGE_TYPE_FILTER);
         memcpy(page->data, pages + k * ps, ps);
         unlock_and_unget_page(cc, page);
      }
      /* absolute index slots (:612-620) */
      for (uint32 i = 0; i < info.num_indices; i++) {
         uint64 *cursor = (uint64 *)index_page[i / addrs_per_page]->data + i % addrs_per_page;
         *cursor        = page_addr[slots[i] / ps] + slots[i] % ps;
      }
   }
   for (uint64 i = 0; i < pages_per_extent; i++) {
      unlock_and_unget_page(cc, index_page[i]);
   }
   mini_release(&mini);
   free(page_addr);
   pin_give(e, q.pages, q.pin_cap);

   filter->num_fingerprints = (uint32)nfp;
   filter->num_unique       = info.num_unique;
   filter->value_size       = info.value_size;

   AB_ADD(AB_PLACE, now_ns() - tpl);
   /* keep the filter on the device, its whole batch (the pin becomes the registry entry) */
   registry_insert(cc, filter->addr, q.sb, &q.f, 1, 0);
   return STATUS_OK;
}

/* ---- lookups ----------------------------------------------------------------------------- */
platform_status
routing_filter_lookup(cache                *cc,
                      const routing_config *cfg,
                      routing_filter       *filter,
                      key                   target,
                      uint64               *found_values)
{
   if (filter->addr == 0) {
      *found_values = 0;
      return STATUS_OK;
   }
   uint32          h = data_key_hash(cfg->data_cfg, target, cfg->seed);
   shim_batch     *sb;
   uint32          f;
   platform_status rc = resident_pin(cc, cfg, filter, &sb, &f);
   if (!SUCCESS(rc)) {
      return rc;
   }
   /* one request to the engine's lookup server: no kernel launch (a launch round trip is
      ~6.5 us, the server's ~3.8 us, profiles/r04_pingpong.txt) */
   uint64 ticket;
   rc = status_of(rf_amd_lookup_submit(engine(), sb->b, f, h, NULL, &ticket));
   if (SUCCESS(rc)) {
      rc = status_of(rf_amd_lookup_wait(engine(), ticket, found_values));
   }
   registry_unpin(sb);
   return rc;
}

/* ---- grouping of lookups by filter: an open-addressing map (cache, addr) -> group ---------- */
typedef struct group_map {
   uint64       *key_addr;
   const cache **key_cc;
   uint32       *gid;
   uint64        mask;
} group_map;

static void
group_map_init(group_map *m, uint64 n)
{
   uint64 cap = 16;
   while (cap < 2 * n) {
      cap <<= 1;
   }
   m->key_addr = malloc(sizeof(uint64) * cap);
   m->key_cc   = malloc(sizeof(*m->key_cc) * cap);
   m->gid      = malloc(sizeof(uint32) * cap);
   platform_assert(m->key_addr && m->key_cc && m->gid);
   memset(m->gid, 0xff, sizeof(uint32) * cap);
   m->mask = cap - 1;
}

static void
group_map_deinit(group_map *m)
{
   free(m->key_addr);
   free(m->key_cc);
   free(m->gid);
}

/* the group of (cc, addr); *is_new when this call created it as group `next`. The start slot
 * takes all 64 bits of the mix (registry_bucket keeps only 12: tables over 4,096 slots would
 * cluster in their first 4,096) */
static uint32
group_map_get(group_map *m, const cache *cc, uint64 addr, uint32 next, int *is_new)
{
   uint64 x = ((addr >> 12) ^ (uint64)(uintptr_t)cc) * 0x9E3779B97F4A7C15ull;
   uint64 s = (x ^ (x >> 29)) & m->mask;
   for (;; s = (s + 1) & m->mask) {
      if (m->gid[s] == UINT32_MAX) {
         m->key_addr[s] = addr;
         m->key_cc[s]   = cc;
         m->gid[s]      = next;
         *is_new        = 1;
         return next;
      }
      if (m->key_addr[s] == addr && m->key_cc[s] == cc) {
         *is_new = 0;
         return m->gid[s];
      }
   }
}

/*
 * n lookups: hashes h[i] against filters[i] (each given by a representative descriptor and
 * cache), in ONE GPU launch over every filter they name. Per lookup: found[i] and rc[i].
 */
static void
lookup_many(cache *const          *ccs,
            const routing_config *const *cfgs,
            const routing_filter *const *filters,
            const uint32         *h,
            uint64                n,
            uint64               *found,
            platform_status      *rc)
{
   group_map m;
   group_map_init(&m, n);
   uint32          *gid    = malloc(sizeof(uint32) * (n ? n : 1));
   uint32          *pgid   = malloc(sizeof(uint32) * (n ? n : 1));
   shim_batch     **gsb    = malloc(sizeof(*gsb) * (n ? n : 1));
   rf_amd_batch   **gb     = malloc(sizeof(*gb) * (n ? n : 1));
   uint32          *gf     = malloc(sizeof(uint32) * (n ? n : 1));
   uint32          *gprobe = malloc(sizeof(uint32) * (n ? n : 1));
   platform_status *grc    = malloc(sizeof(*grc) * (n ? n : 1));
   platform_assert(gid && pgid && gsb && gb && gf && gprobe && grc);
   uint32 ng = 0, np = 0; /* groups, groups that probe */
   for (uint64 i = 0; i < n; i++) {
      int is_new;
      gid[i] = group_map_get(&m, ccs[i], filters[i]->addr, ng, &is_new);
      if (is_new) {
         uint32 fi = 0;
         grc[ng]   = resident_pin(ccs[i], cfgs[i], filters[i], &gsb[ng], &fi);
         if (SUCCESS(grc[ng])) {
            gb[np]     = gsb[ng]->b;
            gf[np]     = fi;
            gprobe[ng] = np++;
         } else {
            gsb[ng]    = NULL;
            gprobe[ng] = UINT32_MAX; /* finds nothing; the state gets grc */
         }
         ng++;
      }
      pgid[i] = gprobe[gid[i]];
   }
   platform_status prc = status_of(rf_amd_probe_filters_host(engine(), gb, gf, np, h, pgid, n, found));
   for (uint64 i = 0; i < n; i++) {
      rc[i] = SUCCESS(grc[gid[i]]) ? prc : grc[gid[i]];
      if (!SUCCESS(rc[i])) {
         found[i] = 0;
      }
   }
   for (uint32 g = 0; g < ng; g++) {
      registry_unpin(gsb[g]);
   }
   group_map_deinit(&m);
   free(gid);
   free(pgid);
   free(gsb);
   free(gb);
   free(gf);
   free(gprobe);
   free(grc);
}

/* ---- async: states answered by the engine's lookup server, or in batches ------------------- */
/*
 * routing_filter_lookup_async hashes the key and, while fewer than AQ_SERVER_MAX states wait
 * on the engine's lookup server, pins the filter's device batch and submits ONE request to it
 * (rf_amd_lookup_submit: a ring in device memory that a persistent GPU wave polls -- no
 * kernel launch, no batching delay: the latency path of callers that keep a few lookups in
 * flight). Beyond that the state goes onto a lock-free stack instead (one compare-and-swap):
 * the batch thread takes the whole stack whenever it is free and answers it with ONE launch
 * over every filter the states name (lookup_many) -- a burst of thousands of states costs one
 * push each instead of one ring request each. Either way the call returns
 * ASYNC_STATUS_RUNNING without touching the state again (async.h:115-125); a completion
 * thread registered with the platform stores each result, marks the state done and fires its
 * callback; the next call returns DONE. A polling owner's re-call completes what it can in
 * its own thread. The server state's pin (its batch stays resident until answered) is kept
 * in its filter_page local, a queued state's next pointer in index_page: locals the shim's
 * coroutine never uses otherwise.
 */
static char g_queued_marker;
#define ASYNC_STATE_QUEUED ((async_state)&g_queued_marker)
typedef routing_filter_lookup_async_state rf_state;

/* The submitting threads and the completion thread run on different cores: what each side
 * writes sits on 128-byte blocks of its own (a written line moving between the host's CCDs
 * costs ~300 ns; profiles/r06_async_submit.txt) */
#define SHIM_LINE __attribute__((aligned(128)))
/* submitted, not yet completed (atomic; the completion thread subtracts once per reap) */
static uint64 g_aq_outstanding SHIM_LINE;
static uint64 g_async_submit_ns; /* ns spent submitting: hash, pin, ring (submitters) */
static int    g_aq_sleeping SHIM_LINE; /* the completion thread waits on g_aq_cv (atomic) */
static pthread_mutex_t g_aq_mu SHIM_LINE = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t  g_aq_cv = PTHREAD_COND_INITIALIZER;
static pthread_once_t  g_aq_once = PTHREAD_ONCE_INIT;
/* reaps that returned states, states completed, ns spent reaping and firing callbacks
 * (routing_filter_amd_async_breakdown; the completion thread's) */
static uint64 g_async_batches SHIM_LINE, g_async_probes, g_async_reap_ns, g_async_cb_ns;
/* RF_SHIM_SUBMIT_PROFILE=1 (diagnostics; set at the first async call): submit steps, and the
 * server states outstanding whenever a reap finds answers (completion thread only) */
static int    g_subprof = -1;
static uint64 g_reap_outstanding_sum, g_reap_outstanding_n;

#define AQ_PIN(st) (*(shim_batch **)&(st)->filter_page)

#define AQ_SERVER_MAX 64 /* server requests outstanding beyond which states are batched */
/* first calls of this thread since one of its calls last returned DONE */
static __thread uint32 g_tl_first_calls;
static rf_state *g_bq_head;     /* the stack of batched states (atomic) */
static uint64    g_bq_count;    /* states on it (atomic) */
static uint64    g_bq_pending;  /* batched states not yet completed (atomic) */
static int       g_bq_sleeping; /* batch threads waiting on g_bq_cv (atomic) */
static pthread_mutex_t g_bq_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t  g_bq_cv = PTHREAD_COND_INITIALIZER;
/* launches and states of the batch path, ns in lookup_many (host work + GPU round trip) */
static uint64 g_bq_batches, g_bq_probes, g_bq_ns;
#define AQ_NEXT(st) (*(rf_state **)&(st)->index_page)

/* probe and complete the n states of a taken stack (their filters in one launch); each
 * state's callback fires after it is marked done */
static void
complete_states(rf_state *list, uint64 n)
{
   if (n == 0) {
      return;
   }
   rf_state             **q    = malloc(sizeof(*q) * n);
   cache               **ccs   = malloc(sizeof(*ccs) * n);
   const routing_config **cfgs = malloc(sizeof(*cfgs) * n);
   const routing_filter **fl   = malloc(sizeof(*fl) * n);
   uint32               *h     = malloc(sizeof(uint32) * n);
   uint64               *found = malloc(sizeof(uint64) * n);
   platform_status      *rc    = malloc(sizeof(*rc) * n);
   platform_assert(q && ccs && cfgs && fl && h && found && rc);
   uint64 m = 0;
   for (rf_state *st = list; st && m < n; st = AQ_NEXT(st)) {
      q[m]    = st;
      ccs[m]  = st->cc;
      cfgs[m] = st->cfg;
      fl[m]   = &st->filter;
      h[m]    = st->fp; /* the full 32-bit hash, stored when queued */
      m++;
   }
   const uint64 t0 = now_ns();
   lookup_many(ccs, cfgs, fl, h, m, found, rc);
   __atomic_fetch_add(&g_bq_ns, now_ns() - t0, __ATOMIC_RELAXED);
   for (uint64 i = 0; i < m; i++) {
      rf_state         *st  = q[i];
      async_callback_fn cb  = st->callback;
      void             *arg = st->callback_arg;
      *st->found_values     = found[i];
      st->__async_result    = rc[i];
      /* from here the owner may resume (and reuse) the state: it is not touched again */
      __atomic_store_n(&st->__async_state_stack[0], ASYNC_STATE_DONE, __ATOMIC_RELEASE);
      __atomic_sub_fetch(&g_bq_pending, 1, __ATOMIC_RELEASE);
      if (cb) {
         cb(arg);
      }
   }
   __atomic_fetch_add(&g_bq_batches, 1, __ATOMIC_RELAXED);
   __atomic_fetch_add(&g_bq_probes, m, __ATOMIC_RELAXED);
   free(q);
   free(ccs);
   free(cfgs);
   free(fl);
   free(h);
   free(found);
   free(rc);
}

/* takes every batched state: the stack's head and how many states it holds */
static rf_state *
bq_take(uint64 *n)
{
   rf_state *list = __atomic_exchange_n(&g_bq_head, NULL, __ATOMIC_ACQUIRE);
   uint64    c    = 0;
   for (rf_state *st = list; st; st = AQ_NEXT(st)) {
      c++;
   }
   __atomic_fetch_sub(&g_bq_count, c, __ATOMIC_RELAXED);
   *n = c;
   return list;
}

static uint64
bq_complete(void)
{
   uint64    n;
   rf_state *list = bq_take(&n);
   complete_states(list, n);
   return n;
}

/* the batch thread: takes the whole stack whenever it is free -- what arrived during one GPU
 * round trip goes out in the next; a burst of submissions settles first (no arrival for a
 * microsecond, at most 4) */
/* the shim's threads (completion, batch): joinable, stopped by shim_at_exit */
#define SHIM_THREADS_MAX 9
static pthread_t g_threads[SHIM_THREADS_MAX];
static uint32    g_nthreads;
static int       g_stopping SHIM_LINE; /* atomic: the threads leave their loops */

static void *
batch_main(void *arg)
{
   (void)arg;
   platform_ensure_thread_registered(); /* callbacks and cache_get (imports) run here */
   for (;;) {
      if (!__atomic_load_n(&g_bq_head, __ATOMIC_ACQUIRE)) {
         const uint64 t0 = now_ns();
         while (!__atomic_load_n(&g_bq_head, __ATOMIC_ACQUIRE) && now_ns() - t0 < 30000) {
            __builtin_ia32_pause();
         }
         pthread_mutex_lock(&g_bq_mu);
         __atomic_add_fetch(&g_bq_sleeping, 1, __ATOMIC_SEQ_CST);
         while (!__atomic_load_n(&g_bq_head, __ATOMIC_SEQ_CST) && !__atomic_load_n(&g_stopping, __ATOMIC_SEQ_CST)) {
            pthread_cond_wait(&g_bq_cv, &g_bq_mu);
         }
         __atomic_sub_fetch(&g_bq_sleeping, 1, __ATOMIC_SEQ_CST);
         pthread_mutex_unlock(&g_bq_mu);
      }
      if (__atomic_load_n(&g_stopping, __ATOMIC_SEQ_CST)) {
         break;
      }
      uint64       c0 = __atomic_load_n(&g_bq_count, __ATOMIC_RELAXED);
      const uint64 t0 = now_ns();
      uint64       tc = t0, t = t0;
      while (t - t0 < 4000 && t - tc < 1000) {
         __builtin_ia32_pause();
         t               = now_ns();
         const uint64 c1 = __atomic_load_n(&g_bq_count, __ATOMIC_RELAXED);
         if (c1 != c0) {
            c0 = c1;
            tc = t;
         }
      }
      bq_complete();
   }
   return NULL;
}

/* take what the server has answered and complete those states; returns how many */
static uint64
async_reap_complete(void)
{
   enum { REAP = 256 };
   void  *tags[REAP];
   uint64 found[REAP];
   const uint64 t0 = now_ns();
   uint64       n  = rf_amd_lookup_reap(engine(), tags, found, REAP);
   if (n == 0) {
      /* a dead lookup server (a launch failed, its stream faulted) never answers: complete
         its states with the error instead of leaving their owners waiting. The
         server's sticky error word is read first: it is read-mostly, the outstanding count is
         written by every submit */
      const int err = rf_amd_lookup_server_error(engine());
      uint64    k   = err && __atomic_load_n(&g_aq_outstanding, __ATOMIC_ACQUIRE)
                         ? rf_amd_lookup_server_failed(engine(), tags, REAP)
                         : 0;
      for (uint64 i = 0; i < k; i++) {
         rf_state         *st  = tags[i];
         async_callback_fn cb  = st->callback;
         void             *arg = st->callback_arg;
         shim_batch       *sb  = AQ_PIN(st);
         *st->found_values     = 0;
         st->__async_result    = status_of(err);
         __atomic_store_n(&st->__async_state_stack[0], ASYNC_STATE_DONE, __ATOMIC_RELEASE);
         __atomic_sub_fetch(&g_aq_outstanding, 1, __ATOMIC_RELAXED);
         registry_unpin(sb);
         if (cb) {
            cb(arg);
         }
      }
      return k;
   }
   const uint64 t1 = now_ns();
   shim_batch       *pins[REAP];
   async_callback_fn cbs[REAP];
   void             *args[REAP];
   for (uint64 i = 0; i < n && i < 4; i++) {
      __builtin_prefetch(tags[i], 1, 3);
   }
   for (uint64 i = 0; i < n; i++) {
      if (i + 4 < n) {
         __builtin_prefetch(tags[i + 4], 1, 3); /* the owners' states: misses overlapped */
      }
      rf_state *st       = tags[i];
      cbs[i]             = st->callback;
      args[i]            = st->callback_arg;
      pins[i]            = AQ_PIN(st);
      *st->found_values  = found[i];
      st->__async_result = STATUS_OK;
      /* from here the owner may resume (and reuse) the state: it is not touched again */
      __atomic_store_n(&st->__async_state_stack[0], ASYNC_STATE_DONE, __ATOMIC_RELEASE);
   }
   /* one update of the shared count per reap, before the callbacks (a callback that submits
      and finds the ring nearly full reaps in place: the count must not hold these) */
   const uint64 outstanding = __atomic_fetch_sub(&g_aq_outstanding, n, __ATOMIC_RELEASE);
   if (g_subprof > 0) { /* diagnostics: server states outstanding when a reap finds answers */
      g_reap_outstanding_sum += outstanding;
      g_reap_outstanding_n++;
   }
   for (uint64 i = 0; i < n; i++) {
      if (cbs[i]) {
         cbs[i](args[i]);
      }
   }
   registry_unpin_many(pins, n); /* the batches stay pinned until their answers are stored */
   __atomic_fetch_add(&g_async_reap_ns, t1 - t0, __ATOMIC_RELAXED);
   __atomic_fetch_add(&g_async_cb_ns, now_ns() - t1, __ATOMIC_RELAXED);
   __atomic_fetch_add(&g_async_batches, 1, __ATOMIC_RELAXED);
   __atomic_fetch_add(&g_async_probes, n, __ATOMIC_RELAXED);
   return n;
}

static void *
completion_main(void *arg)
{
   (void)arg;
   platform_ensure_thread_registered(); /* callbacks and cache_get (imports) run here */
   uint32 idle = 0;
   while (!__atomic_load_n(&g_stopping, __ATOMIC_SEQ_CST)) {
      if (async_reap_complete()) {
         idle = 0;
         continue;
      }
      /* answers arrive within microseconds: spin on the reap (it reads only the GPU-written
         answer line while idle) and look at the submitters' count only every 64 spins */
      if ((++idle & 63) != 0 || __atomic_load_n(&g_aq_outstanding, __ATOMIC_ACQUIRE)) {
         __builtin_ia32_pause();
         continue;
      }
      pthread_mutex_lock(&g_aq_mu);
      __atomic_store_n(&g_aq_sleeping, 1, __ATOMIC_SEQ_CST);
      while (!__atomic_load_n(&g_aq_outstanding, __ATOMIC_SEQ_CST) && !__atomic_load_n(&g_stopping, __ATOMIC_SEQ_CST)) {
         pthread_cond_wait(&g_aq_cv, &g_aq_mu);
      }
      __atomic_store_n(&g_aq_sleeping, 0, __ATOMIC_SEQ_CST);
      pthread_mutex_unlock(&g_aq_mu);
   }
   return NULL;
}

/* RF_SHIM_PIN_THREADS (default 1): the completion and batch threads run on the cores that
 * share the last-level cache with the thread that made the first async call. Every answered
 * state moves cache lines between that thread and the completion thread (the state, its
 * callback's context, the ring bookkeeping); between the host's CCDs such a move costs ~300 ns,
 * within one a fraction of it. Nothing is pinned when the process's allowed cores do not
 * include two of that cache's cores. */
static void
pin_near_caller(const pthread_t *th, uint32 n)
{
   if (!env_u64("RF_SHIM_PIN_THREADS", 1)) {
      return;
   }
   const int cpu = sched_getcpu();
   if (cpu < 0) {
      return;
   }
   char path[160], buf[1024];
   int  lvl = 0;
   snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/level", cpu);
   FILE *f = fopen(path, "r");
   if (!f) {
      return;
   }
   if (fscanf(f, "%d", &lvl) != 1) {
      lvl = 0;
   }
   fclose(f);
   if (lvl != 3) {
      return;
   }
   snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
   f = fopen(path, "r");
   if (!f) {
      return;
   }
   const char *ok = fgets(buf, sizeof(buf), f);
   fclose(f);
   if (!ok) {
      return;
   }
   cpu_set_t llc, allowed;
   CPU_ZERO(&llc);
   for (char *p = buf; *p && *p != '\n';) { /* "a-b,c,..." */
      char *e;
      long  a = strtol(p, &e, 10), b = a;
      if (e == p) {
         break;
      }
      if (*e == '-') {
         p = e + 1;
         b = strtol(p, &e, 10);
      }
      for (long c = a; c <= b && c < CPU_SETSIZE; c++) {
         CPU_SET(c, &llc);
      }
      p = (*e == ',') ? e + 1 : e;
   }
   if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) {
      return;
   }
   CPU_AND(&llc, &llc, &allowed);
   if (CPU_COUNT(&llc) < 2) {
      return;
   }
   for (uint32 i = 0; i < n; i++) {
      (void)pthread_setaffinity_np(th[i], sizeof(llc), &llc);
   }
}

static void
aq_init(void)
{
   const uint32 first = g_nthreads;
   platform_assert(pthread_create(&g_threads[g_nthreads++], NULL, completion_main, NULL) == 0);
   /* RF_SHIM_BATCH_THREADS batch threads (default 1; 2: a batch goes out while the previous
      one is on the GPU) */
   uint64 nb = env_u64("RF_SHIM_BATCH_THREADS", 1);
   for (uint64 k = 0; k < (nb >= 1 && nb <= SHIM_THREADS_MAX - 1 ? nb : 1); k++) {
      platform_assert(pthread_create(&g_threads[g_nthreads++], NULL, batch_main, NULL) == 0);
   }
   pin_near_caller(&g_threads[first], g_nthreads - first);
}

/* Process exit (atexit, registered when the engine was created): the completion and batch
 * threads leave their loops and are joined, then the engine is destroyed -- its server wave
 * stopped, streams drained, pinned rings freed, cache registrations dropped -- before HIP
 * unregisters the engine library's kernels (the heap abort in
 * __hipUnregisterFatBinary at the exit of a process running the shim). A thread that does not
 * return within 2 s (stuck in a callback or a GPU wait) leaves the engine alone. States still
 * queued at exit are not completed: their owners are gone. */
static void
shim_at_exit(void)
{
   __atomic_store_n(&g_stopping, 1, __ATOMIC_SEQ_CST);
   pthread_mutex_lock(&g_aq_mu);
   pthread_cond_broadcast(&g_aq_cv);
   pthread_mutex_unlock(&g_aq_mu);
   pthread_mutex_lock(&g_bq_mu);
   pthread_cond_broadcast(&g_bq_cv);
   pthread_mutex_unlock(&g_bq_mu);
   int joined = 1;
   for (uint32 i = 0; i < g_nthreads; i++) {
      struct timespec dl;
      clock_gettime(CLOCK_REALTIME, &dl);
      dl.tv_sec += 2;
      if (pthread_timedjoin_np(g_threads[i], NULL, &dl) != 0) {
         joined = 0;
      }
   }
   if (joined && g_eng) {
      rf_amd_engine_destroy(g_eng);
      g_eng    = NULL;
      g_eng_rc = RF_AMD_ENODEV;
   }
}

/* complete every state submitted so far, in the caller's thread (reaping with the
   completion thread) */
void
routing_filter_amd_flush(void)
{
   pthread_once(&g_aq_once, aq_init);
   /* until every submitted state is done, including batches a completion thread holds */
   while (__atomic_load_n(&g_aq_outstanding, __ATOMIC_ACQUIRE) || __atomic_load_n(&g_bq_pending, __ATOMIC_ACQUIRE)) {
      if (!bq_complete() && !async_reap_complete()) {
         __builtin_ia32_pause();
      }
   }
}

void
routing_filter_amd_async_stats(uint64 *batches, uint64 *probes)
{
   *batches = __atomic_load_n(&g_async_batches, __ATOMIC_RELAXED) + __atomic_load_n(&g_bq_batches, __ATOMIC_RELAXED);
   *probes  = __atomic_load_n(&g_async_probes, __ATOMIC_RELAXED) + __atomic_load_n(&g_bq_probes, __ATOMIC_RELAXED);
}

/* out[0..5]: reaps that completed server states, server states completed, then ns totals:
 * submitting (hash, pin, ring write), the batch path's lookup_many, reaping, callbacks */
void
routing_filter_amd_async_breakdown(uint64 *out)
{
   out[0] = __atomic_load_n(&g_async_batches, __ATOMIC_RELAXED);
   out[1] = __atomic_load_n(&g_async_probes, __ATOMIC_RELAXED);
   out[2] = __atomic_load_n(&g_async_submit_ns, __ATOMIC_RELAXED);
   out[3] = __atomic_load_n(&g_bq_ns, __ATOMIC_RELAXED);
   out[4] = __atomic_load_n(&g_async_reap_ns, __ATOMIC_RELAXED);
   out[5] = __atomic_load_n(&g_async_cb_ns, __ATOMIC_RELAXED);
}

uint64
routing_filter_amd_async_probe_ns(void)
{
   return __atomic_load_n(&g_async_reap_ns, __ATOMIC_RELAXED) + __atomic_load_n(&g_bq_ns, __ATOMIC_RELAXED);
}

/* RF_SHIM_SUBMIT_PROFILE=1 (diagnostics): TSC cycles of each step of a server submission --
   hash, registry pin, ring-space wait and bookkeeping, rf_amd_lookup_submit, wake-up -- summed
   and printed to stderr at exit */
static uint64 g_subprof_cyc[5], g_subprof_n;
#define SUBPROF_MARK(i)                                                                            \
   uint64 sp_##i = 0;                                                                              \
   if (g_subprof > 0) {                                                                            \
      _mm_lfence();                                                                                \
      sp_##i = __rdtsc();                                                                          \
      _mm_lfence();                                                                                \
   }
#define SUBPROF_DONE()                                                                             \
   if (g_subprof > 0) {                                                                            \
      g_subprof_cyc[0] += sp_1 - sp_0;                                                             \
      g_subprof_cyc[1] += sp_2 - sp_1;                                                             \
      g_subprof_cyc[2] += sp_3 - sp_2;                                                             \
      g_subprof_cyc[3] += sp_4 - sp_3;                                                             \
      g_subprof_cyc[4] += sp_5 - sp_4;                                                             \
      g_subprof_n++;                                                                               \
   }
static void
subprof_print(void)
{
   if (g_subprof > 0 && g_reap_outstanding_n) {
      fprintf(stderr, "rf_shim reaps: %lu with answers, %.1f server states outstanding at each\n",
              (unsigned long)g_reap_outstanding_n, (double)g_reap_outstanding_sum / g_reap_outstanding_n);
   }
   if (g_subprof > 0 && g_subprof_n) {
      fprintf(stderr,
              "rf_shim submit profile: %lu submissions, TSC cycles each: hash %.0f pin %.0f "
              "wait+book %.0f submit %.0f wake %.0f\n",
              (unsigned long)g_subprof_n, (double)g_subprof_cyc[0] / g_subprof_n,
              (double)g_subprof_cyc[1] / g_subprof_n, (double)g_subprof_cyc[2] / g_subprof_n,
              (double)g_subprof_cyc[3] / g_subprof_n, (double)g_subprof_cyc[4] / g_subprof_n);
   }
}

async_status
routing_filter_lookup_async(routing_filter_lookup_async_state *state)
{
   if (g_subprof < 0) {
      const char *v = getenv("RF_SHIM_SUBMIT_PROFILE");
      g_subprof     = v && atoi(v) > 0;
      if (g_subprof) {
         atexit(subprof_print);
      }
   }
   async_state at = __atomic_load_n(&state->__async_state_stack[0], __ATOMIC_ACQUIRE);
   if (at == ASYNC_STATE_DONE) {
      g_tl_first_calls = 0;
      return ASYNC_STATUS_DONE;
   }
   if (at == ASYNC_STATE_QUEUED) {
      /* a polling owner: complete what is answered or batched now, in this thread (this
         state among them, unless a completion thread already holds it). RUNNING either way
         -- the state's callback may have fired; the next call returns DONE */
      async_reap_complete();
      if (__atomic_load_n(&g_bq_head, __ATOMIC_RELAXED)) {
         bq_complete();
      }
      return ASYNC_STATUS_RUNNING;
   }
   /* ASYNC_STATE_INIT (:898-905) */
   if (state->filter.addr == 0) {
      *state->found_values          = 0;
      state->__async_result         = STATUS_OK;
      state->__async_state_stack[0] = ASYNC_STATE_DONE;
      return ASYNC_STATUS_DONE;
   }
   pthread_once(&g_aq_once, aq_init);
   const uint64 t0 = now_ns();
   SUBPROF_MARK(0);
   state->fp       = data_key_hash(state->cfg->data_cfg, state->target, state->cfg->seed);
   SUBPROF_MARK(1);
   /* a burst: more than AQ_SERVER_MAX first calls from this thread with no state of its
      finished in between (a caller that keeps a bounded number in flight sees DONE between
      its submissions; one that submits thousands and polls later does not). With the server
      answering in a few microseconds the outstanding count alone stays low through such a
      burst, and every state would pay a ring submission instead of a stack push */
   const int burst = ++g_tl_first_calls > AQ_SERVER_MAX;
   if (burst || __atomic_load_n(&g_aq_outstanding, __ATOMIC_RELAXED) >= AQ_SERVER_MAX
       || __atomic_load_n(&g_bq_pending, __ATOMIC_RELAXED))
   {
      /* a burst (the server's share is full, or batched states are still in flight: the
         burst stays on the batch path until it drains): onto the batch stack (the state may
         complete at once on another thread; it is not read again here) */
      state->__async_state_stack[0] = ASYNC_STATE_QUEUED;
      __atomic_add_fetch(&g_bq_pending, 1, __ATOMIC_SEQ_CST);
      rf_state *old                 = __atomic_load_n(&g_bq_head, __ATOMIC_RELAXED);
      do {
         AQ_NEXT(state) = old;
      } while (!__atomic_compare_exchange_n(&g_bq_head, &old, state, 1, __ATOMIC_SEQ_CST, __ATOMIC_RELAXED));
      __atomic_add_fetch(&g_bq_count, 1, __ATOMIC_RELAXED);
      if (old == NULL && __atomic_load_n(&g_bq_sleeping, __ATOMIC_SEQ_CST)) {
         pthread_mutex_lock(&g_bq_mu);
         pthread_cond_signal(&g_bq_cv);
         pthread_mutex_unlock(&g_bq_mu);
      }
      return ASYNC_STATUS_RUNNING;
   }
   shim_batch     *sb;
   uint32          fi;
   platform_status rc = resident_pin(state->cc, state->cfg, &state->filter, &sb, &fi);
   SUBPROF_MARK(2);
   if (!SUCCESS(rc)) {
      *state->found_values          = 0;
      state->__async_result         = rc;
      state->__async_state_stack[0] = ASYNC_STATE_DONE;
      return ASYNC_STATUS_DONE;
   }
   /* a nearly full ring: reap here first (a callback that submits from the completion thread
      must not wait for a slot only that thread would free) */
   while (__atomic_load_n(&g_aq_outstanding, __ATOMIC_ACQUIRE) >= RF_AMD_SERVER_RING - 64) {
      if (!async_reap_complete()) {
         __builtin_ia32_pause();
      }
   }
   AQ_PIN(state)                 = sb;
   state->__async_state_stack[0] = ASYNC_STATE_QUEUED;
   __atomic_add_fetch(&g_aq_outstanding, 1, __ATOMIC_SEQ_CST);
   uint64 ticket;
   SUBPROF_MARK(3);
   int    r = rf_amd_lookup_submit(engine(), sb->b, fi, state->fp, state, &ticket);
   SUBPROF_MARK(4);
   if (r) { /* not queued: nobody else saw the state */
      __atomic_sub_fetch(&g_aq_outstanding, 1, __ATOMIC_SEQ_CST);
      registry_unpin(sb);
      *state->found_values          = 0;
      state->__async_result         = status_of(r);
      state->__async_state_stack[0] = ASYNC_STATE_DONE;
      return ASYNC_STATUS_DONE;
   }
   /* the state may already be complete (another thread): it is not read again here */
   __atomic_fetch_add(&g_async_submit_ns, now_ns() - t0, __ATOMIC_RELAXED);
   if (__atomic_load_n(&g_aq_sleeping, __ATOMIC_SEQ_CST)) {
      pthread_mutex_lock(&g_aq_mu);
      pthread_cond_signal(&g_aq_cv);
      pthread_mutex_unlock(&g_aq_mu);
   }
   SUBPROF_MARK(5);
   SUBPROF_DONE();
   return ASYNC_STATUS_RUNNING;
}

/* n lookups (filters[i], keys[i]) in one GPU launch -- the batch form of the per-bundle
 * routing_filter_lookup calls of trunk_merge_lookup (src/trunk.c:6008-6075). found[i] equals
 * what routing_filter_lookup(cc, cfg, &filters[i], keys[i], &found[i]) would return. */
platform_status
routing_filter_amd_lookup_batch(cache                *cc,
                                const routing_config *cfg,
                                routing_filter       *filters,
                                const key            *keys,
                                uint64                n,
                                uint64               *found)
{
   if (n == 0) {
      return STATUS_OK;
   }
   cache               **ccs   = malloc(sizeof(*ccs) * n);
   const routing_config **cfgs = malloc(sizeof(*cfgs) * n);
   const routing_filter **fl   = malloc(sizeof(*fl) * n);
   uint32               *h     = malloc(sizeof(uint32) * n);
   uint64               *fo    = malloc(sizeof(uint64) * n);
   uint64               *idx   = malloc(sizeof(uint64) * n);
   platform_status      *rc    = malloc(sizeof(*rc) * n);
   platform_assert(ccs && cfgs && fl && h && fo && idx && rc);
   uint64 m = 0;
   for (uint64 i = 0; i < n; i++) {
      if (filters[i].addr == 0) { /* NULL filter finds nothing (:1003-1006) */
         found[i] = 0;
         continue;
      }
      ccs[m]  = cc;
      cfgs[m] = cfg;
      fl[m]   = &filters[i];
      h[m]    = data_key_hash(cfg->data_cfg, keys[i], cfg->seed);
      idx[m]  = i;
      m++;
   }
   lookup_many(ccs, cfgs, fl, h, m, fo, rc);
   platform_status ret = STATUS_OK;
   for (uint64 j = 0; j < m; j++) {
      found[idx[j]] = fo[j];
      if (!SUCCESS(rc[j]) && SUCCESS(ret)) {
         ret = rc[j];
      }
   }
   free(ccs);
   free(cfgs);
   free(fl);
   free(h);
   free(fo);
   free(idx);
   free(rc);
   return ret;
}

/* ---- reference counts, estimates, space -------------------------------------------------- */
void
routing_filter_inc_ref(cache *cc, routing_filter *filter)
{
   if (filter->num_fingerprints == 0) {
      return;
   }
   mini_inc_ref(cc, filter->meta_head);
}

void
routing_filter_dec_ref(cache *cc, routing_filter *filter)
{
   if (filter->num_fingerprints == 0) {
      return;
   }
   if (mini_dec_ref(cc, filter->meta_head, PAGE_TYPE_FILTER) == 0) {
      registry_drop(cc, filter->addr); /* the pages are gone: so is the device copy */
   }
}

uint32
routing_filter_estimate_unique_keys_from_count(const routing_config *cfg, uint64 num_unique)
{
   rf_amd_config c = amd_config(cfg);
   return rf_amd_estimate_unique_keys_from_count(&c, num_unique);
}

uint32
routing_filter_estimate_unique_keys(routing_filter *filter, routing_config *cfg)
{
   return routing_filter_estimate_unique_keys_from_count(cfg, filter->num_unique);
}

platform_status
routing_filter_estimate_unique_fp(cache                *cc,
                                  const routing_config *cfg,
                                  platform_heap_id      hid,
                                  routing_filter       *filter,
                                  uint64                num_filters,
                                  uint32               *num_unique_fp)
{
   (void)hid;
   if (num_unique_fp == NULL) {
      platform_error_log("routing_filter_estimate_unique_fp: "
                         "num_unique_fp must not be NULL\n");
      return STATUS_BAD_PARAM;
   }
   *num_unique_fp = 0;
   platform_assert(num_filters <= MAX_FILTERS);
   shim_batch     *sbs[MAX_FILTERS];
   rf_amd_batch   *batches[MAX_FILTERS];
   uint32          index[MAX_FILTERS];
   platform_status rc = STATUS_OK;
   for (uint64 i = 0; i < num_filters; i++) {
      sbs[i]     = NULL;
      batches[i] = NULL;
      index[i]   = 0;
      if (filter[i].addr != 0 && SUCCESS(rc)) {
         rc = resident_pin(cc, cfg, &filter[i], &sbs[i], &index[i]);
         if (SUCCESS(rc)) {
            batches[i] = sbs[i]->b;
         }
      }
   }
   if (SUCCESS(rc)) {
      rc = status_of(rf_amd_batch_estimate_unique_fp(batches, index, num_filters, num_unique_fp));
   }
   for (uint64 i = 0; i < num_filters; i++) {
      registry_unpin(sbs[i]);
   }
   return rc;
}

uint64
routing_filter_space_use_bytes(cache *cc, const routing_filter *filter)
{
   return mini_space_use_bytes(cc, filter->meta_head, PAGE_TYPE_FILTER);
}

/* ---- debug ------------------------------------------------------------------------------- */
void
routing_filter_verify(cache          *cc,
                      routing_config *cfg,
                      routing_filter *filter,
                      uint16          value,
                      iterator       *itor)
{
   uint64  n = 0, cap = 4096;
   uint32 *h = malloc(sizeof(uint32) * cap);
   platform_assert(h != NULL);
   while (iterator_can_next(itor)) {
      key     curr_key;
      message msg;
      iterator_curr(itor, &curr_key, &msg);
      if (n == cap) {
         cap *= 2;
         h = realloc(h, sizeof(uint32) * cap);
         platform_assert(h != NULL);
      }
      h[n++]             = data_key_hash(cfg->data_cfg, curr_key, cfg->seed);
      platform_status rc = iterator_next(itor);
      platform_assert_status_ok(rc);
   }
   uint64 *found = malloc(sizeof(uint64) * (n ? n : 1));
   platform_assert(found != NULL);
   if (n && filter->addr != 0) {
      shim_batch     *sb;
      uint32          f;
      platform_status rc = resident_pin(cc, cfg, filter, &sb, &f);
      platform_assert_status_ok(rc);
      platform_assert(rf_amd_probe_filters_host(engine(), &sb->b, &f, 1, h, NULL, n, found) == 0);
      registry_unpin(sb);
   } else {
      memset(found, 0, sizeof(uint64) * n);
   }
   for (uint64 i = 0; i < n; i++) {
      platform_assert(routing_filter_is_value_found(found[i], value));
   }
   free(found);
   free(h);
}

void
routing_filter_print(cache *cc, routing_config *cfg, routing_filter *filter)
{
   rf_amd_image img;
   uint64      *abs_slots = NULL;
   if (!SUCCESS(rf_read_image(cc, cfg, filter, &img, &abs_slots))) {
      return;
   }
   rf_amd_config c   = amd_config(cfg);
   FILE         *out = platform_get_stdout_stream(); /* platform_default_log's stream */
   fflush(out);
   rf_amd_filter_print_abs(&c, &img, filter->addr, abs_slots, out);
   free(abs_slots);
   rf_amd_image_free(&img);
}
