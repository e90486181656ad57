/*
 * routing_filter_amd.c -- drop-in replacement for vmware/splinterdb's src/routing_filter.c.
 *
 * Compiled in SplinterDB's tree against its own headers (src/routing_filter.h,
 * src/mini_allocator.h, src/cache.h, ...) in place of routing_filter.c, it defines every
 * function routing_filter.h declares, with the reference's signatures, and runs the filter
 * work on the MI355X engine through its C ABI (include/rf_amd.h, librf_amd.so):
 *
 *   routing_filter_add                  routing_filter.h:78-85   build on the GPU, then the
 *                                        reference's page allocation sequence, page by page
 *   routing_filter_lookup               :87-92     hash via data_config (the application's
 *                                        callback, as the reference), probe on the GPU
 *   routing_filter_lookup_async         :130-155   per-key coroutine states coalesced into
 *                                        one GPU probe per filter (see "async" below)
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
 * page there, SURVEY finding 4).
 *
 * Differences a caller can see: new_fp_arr is not shifted/sorted in place (no caller reads
 * it afterwards; the trunk frees it, src/trunk.c:2825-2826); inputs the reference treats as
 * undefined behaviour (zero fingerprints, a block larger than a page) return
 * STATUS_BAD_PARAM instead of corrupting memory; without a HIP device every call that needs
 * one returns ENODEV (there is no CPU fallback).
 *
 * Device residency. Each filter this process builds stays on the GPU (a probe-only batch:
 * pages, slots, probe lines) in a registry keyed by (cache, index-extent address), so lookups
 * and later incremental adds never re-read it; a filter not in the registry (built before
 * a restart) is read back through cache_get once and imported. dec_ref drops the device
 * copy when the reference's refcount reaches zero.
 *
 * async. routing_filter_lookup_async's first call on a state hashes the key, queues the
 * state and returns ASYNC_STATUS_RUNNING. The queue is flushed -- one GPU probe per filter
 * for all queued states -- when it reaches RF_SHIM_ASYNC_BATCH states (default 1024), when
 * routing_filter_amd_flush() is called, or when a queued state is called again (its owner
 * is waiting). A flush stores each state's found_values, marks it done, and calls its
 * callback(callback_arg); its next call returns ASYNC_STATUS_DONE with STATUS_OK.
 */
#include "routing_filter.h"
#include "mini_allocator.h"
#include "iterator.h"
#include "platform_assert.h"
#include "platform_threads.h"
#include "platform_typed_alloc.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rf_amd.h"
#include "routing_filter_amd.h"

/* ---- engine ------------------------------------------------------------------------- */
static rf_amd_engine  *g_eng;
static int             g_eng_rc;
static pthread_once_t  g_eng_once = PTHREAD_ONCE_INIT;

static void
engine_init(void)
{
   const char *d = getenv("RF_AMD_DEVICE");
   g_eng_rc      = rf_amd_engine_create(d ? atoi(d) : 0, &g_eng);
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

/* ---- registry of device-resident filters, keyed by (cache, index-extent address) -------- */
typedef struct resident_filter {
   const cache            *cc;
   uint64                  addr;
   rf_amd_batch           *batch;
   struct resident_filter *next;
} resident_filter;

#define REGISTRY_BUCKETS 4096
static resident_filter *g_registry[REGISTRY_BUCKETS];
static pthread_mutex_t  g_registry_mu = PTHREAD_MUTEX_INITIALIZER;

static uint64
registry_bucket(const cache *cc, uint64 addr)
{
   return ((addr >> 12) ^ (uint64)(uintptr_t)cc) * 0x9E3779B97F4A7C15ull >> 52;
}

static rf_amd_batch *
registry_find(const cache *cc, uint64 addr)
{
   rf_amd_batch *b = NULL;
   pthread_mutex_lock(&g_registry_mu);
   for (resident_filter *r = g_registry[registry_bucket(cc, addr)]; r; r = r->next) {
      if (r->cc == cc && r->addr == addr) {
         b = r->batch;
         break;
      }
   }
   pthread_mutex_unlock(&g_registry_mu);
   return b;
}

/*
 * Registers b for (cc, addr). replace = 0 (a filter imported from the cache): an entry
 * present already wins and is returned (the caller destroys b). replace = 1 (a filter just
 * built at addr): any entry there is stale -- its pages were freed and reallocated without
 * our dec_ref seeing it reach zero -- and is destroyed.
 */
static rf_amd_batch *
registry_insert(const cache *cc, uint64 addr, rf_amd_batch *b, int replace)
{
   rf_amd_batch *stale = NULL;
   pthread_mutex_lock(&g_registry_mu);
   resident_filter **head = &g_registry[registry_bucket(cc, addr)];
   for (resident_filter *r = *head; r; r = r->next) {
      if (r->cc == cc && r->addr == addr) {
         if (!replace) {
            rf_amd_batch *have = r->batch;
            pthread_mutex_unlock(&g_registry_mu);
            return have;
         }
         stale    = r->batch;
         r->batch = b;
         pthread_mutex_unlock(&g_registry_mu);
         rf_amd_batch_destroy(stale);
         return b;
      }
   }
   resident_filter *r = malloc(sizeof(*r));
   platform_assert(r != NULL);
   r->cc    = cc;
   r->addr  = addr;
   r->batch = b;
   r->next  = *head;
   *head    = r;
   pthread_mutex_unlock(&g_registry_mu);
   return b;
}

static void
registry_drop(const cache *cc, uint64 addr)
{
   rf_amd_batch *b = NULL;
   pthread_mutex_lock(&g_registry_mu);
   for (resident_filter **pp = &g_registry[registry_bucket(cc, addr)]; *pp; pp = &(*pp)->next) {
      if ((*pp)->cc == cc && (*pp)->addr == addr) {
         resident_filter *r = *pp;
         *pp                = r->next;
         b                  = r->batch;
         free(r);
         break;
      }
   }
   pthread_mutex_unlock(&g_registry_mu);
   rf_amd_batch_destroy(b);
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

/* the filter's device-resident probe-only batch (imported from the cache if needed) */
static platform_status
resident(cache *cc, const routing_config *cfg, const routing_filter *f, rf_amd_batch **out)
{
   *out = registry_find(cc, f->addr);
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
   rf_amd_image_free(&img);
   if (r) {
      return status_of(r);
   }
   *out = registry_insert(cc, f->addr, b, 0);
   if (*out != b) {
      rf_amd_batch_destroy(b);
   }
   return STATUS_OK;
}

static inline void
unlock_and_unget_page(cache *cc, page_handle *page)
{
   cache_unlock(cc, page);
   cache_unclaim(cc, page);
   cache_unget(cc, page);
}

/* ---- routing_filter_add --------------------------------------------------------------- */
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
   rf_amd_batch  *ob = NULL;
   platform_status rc;
   if (old_filter->addr != 0) {
      mini_prefetch(cc, PAGE_TYPE_FILTER, old_filter->meta_head); /* as :356 */
      rc = resident(cc, cfg, old_filter, &ob);
      if (!SUCCESS(rc)) {
         return rc;
      }
   }

   /* the image, on the GPU */
   rf_amd_config c    = amd_config(cfg);
   uint32        n32  = (uint32)num_new_fp;
   uint32        zero = 0;
   rf_amd_batch *b    = NULL;
   int           r    = rf_amd_batch_create(e, &c, 1, &n32, &value, ob ? &ob : NULL, ob ? &zero : NULL, &b);
   if (r) {
      return status_of(r);
   }
   rf_amd_filter_info info;
   r = rf_amd_batch_build_hashes_host(b, new_fp_arr);
   if (!r) {
      r = rf_amd_batch_info(b, 0, &info);
   }
   if (!r && info.error) {
      r = RF_AMD_EINVAL; /* a block over a page: undefined behaviour in the reference */
   }
   const uint64 ps    = cache_config_page_size(cfg->cache_cfg);
   uint8       *pages = NULL;
   uint64      *slots = NULL;
   if (!r) {
      pages = malloc(ps * info.num_pages);
      slots = malloc(sizeof(uint64) * info.num_indices);
      r     = (pages && slots) ? rf_amd_batch_read_image(b, 0, pages, ps * info.num_pages, slots,
                                                       info.num_indices)
                               : RF_AMD_ENOMEM;
   }
   if (r) {
      free(pages);
      free(slots);
      rf_amd_batch_destroy(b);
      return status_of(r);
   }

   /* the reference's page allocation sequence, :429-456 */
   allocator *al = cache_get_allocator(cc);
   uint64     meta_head;
   rc = allocator_alloc(al, &meta_head, PAGE_TYPE_FILTER);
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
   for (uint32 k = 0; k < info.num_pages; k++) {
      page_addr[k]        = mini_alloc(&mini, 0, NULL);
      page_handle *page   = cache_alloc(cc, page_addr[k], PAGE_TYPE_FILTER);
      memcpy(page->data, pages + k * ps, ps);
      unlock_and_unget_page(cc, page);
   }
   /* absolute index slots (:612-620) */
   for (uint32 i = 0; i < info.num_indices; i++) {
      uint64 *cursor = (uint64 *)index_page[i / addrs_per_page]->data + i % addrs_per_page;
      *cursor        = page_addr[slots[i] / ps] + slots[i] % ps;
   }
   for (uint64 i = 0; i < pages_per_extent; i++) {
      unlock_and_unget_page(cc, index_page[i]);
   }
   mini_release(&mini);
   free(page_addr);
   free(pages);
   free(slots);

   filter->num_fingerprints = (uint32)nfp;
   filter->num_unique       = info.num_unique;
   filter->value_size       = info.value_size;

   /* keep the filter on the device (probe-only copy of pages, slots and probe lines) */
   void              *d_pages = NULL, *d_slots = NULL;
   rf_amd_batch      *keep    = NULL;
   rf_amd_filter_info one     = info;
   if (rf_amd_batch_image_ptrs(b, 0, &d_pages, &d_slots) == 0
       && rf_amd_batch_import(e, &c, 1, &one, d_pages, d_slots, 1, &keep) == 0)
   {
      registry_insert(cc, filter->addr, keep, 1);
   }
   rf_amd_batch_destroy(b);
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
   uint32        h = data_key_hash(cfg->data_cfg, target, cfg->seed);
   rf_amd_batch *b;
   platform_status rc = resident(cc, cfg, filter, &b);
   if (!SUCCESS(rc)) {
      return rc;
   }
   return status_of(rf_amd_batch_probe_hashes_host(b, &h, NULL, 1, found_values));
}

/* async: a queue of waiting states; the resume marker says "queued, not yet probed" */
static char                                g_queued_marker;
#define ASYNC_STATE_QUEUED ((async_state)&g_queued_marker)
static pthread_mutex_t                     g_async_mu = PTHREAD_MUTEX_INITIALIZER;
static routing_filter_lookup_async_state **g_async_q;
static uint64                              g_async_n, g_async_cap;
static uint64                              g_async_batches, g_async_probes;

static uint64
async_batch_limit(void)
{
   const char *s = getenv("RF_SHIM_ASYNC_BATCH");
   return s ? (uint64)atoll(s) : 1024;
}

static int
cmp_state_filter(const void *a, const void *b)
{
   const routing_filter_lookup_async_state *x = *(routing_filter_lookup_async_state *const *)a;
   const routing_filter_lookup_async_state *y = *(routing_filter_lookup_async_state *const *)b;
   return x->filter.addr < y->filter.addr ? -1 : (x->filter.addr > y->filter.addr ? 1 : 0);
}

/* probe every queued state: one GPU probe per distinct filter */
void
routing_filter_amd_flush(void)
{
   pthread_mutex_lock(&g_async_mu);
   routing_filter_lookup_async_state **q = g_async_q;
   uint64                              n = g_async_n;
   g_async_q                               = NULL;
   g_async_n = g_async_cap = 0;
   pthread_mutex_unlock(&g_async_mu);
   if (n == 0) {
      return;
   }
   qsort(q, n, sizeof(*q), cmp_state_filter); /* stable grouping is enough: order unused */
   uint32          *h      = malloc(sizeof(uint32) * n);
   uint64          *found  = malloc(sizeof(uint64) * n);
   rf_amd_batch   **groups = malloc(sizeof(*groups) * n);
   uint64          *counts = malloc(sizeof(uint64) * n);
   platform_status *grc    = malloc(sizeof(*grc) * n);
   platform_assert(h && found && groups && counts && grc);
   /* every distinct filter's states form one group; all groups go to the GPU in one round
      trip (rf_amd_probe_many_hashes_host) */
   uint32 ng = 0, nok = 0;
   for (uint64 s = 0; s < n;) {
      uint64 t = s;
      while (t < n && q[t]->filter.addr == q[s]->filter.addr) {
         t++;
      }
      rf_amd_batch   *b;
      platform_status rc = resident(q[s]->cc, q[s]->cfg, &q[s]->filter, &b);
      grc[s]             = rc;
      if (SUCCESS(rc)) { /* probed groups first, in queue order */
         for (uint64 i = s; i < t; i++) {
            h[nok + (i - s)] = q[i]->fp; /* the full 32-bit hash, stored when queued */
         }
         groups[ng] = b;
         counts[ng] = t - s;
         ng++;
         nok += t - s;
      }
      s = t;
   }
   platform_status prc =
      status_of(rf_amd_probe_many_hashes_host(engine(), groups, NULL, counts, ng, h, found));
   uint64 at = 0;
   for (uint64 s = 0; s < n;) {
      uint64 t = s;
      while (t < n && q[t]->filter.addr == q[s]->filter.addr) {
         t++;
      }
      platform_status rc = SUCCESS(grc[s]) ? prc : grc[s];
      for (uint64 i = s; i < t; i++) {
         routing_filter_lookup_async_state *st = q[i];
         *st->found_values = SUCCESS(rc) ? found[at + (i - s)] : 0;
         st->__async_result = rc;
         async_callback_fn cb  = st->callback;
         void             *arg = st->callback_arg;
         __atomic_store_n(&st->__async_state_stack[0], ASYNC_STATE_DONE, __ATOMIC_RELEASE);
         if (cb) {
            cb(arg);
         }
      }
      if (SUCCESS(grc[s])) {
         at += t - s;
      }
      s = t;
   }
   __atomic_fetch_add(&g_async_batches, 1, __ATOMIC_RELAXED);
   __atomic_fetch_add(&g_async_probes, n, __ATOMIC_RELAXED);
   free(h);
   free(found);
   free(groups);
   free(counts);
   free(grc);
   free(q);
}

typedef struct lookup_ref {
   uint64 addr; /* the filter's index extent */
   uint64 i;    /* position in the caller's arrays */
} lookup_ref;

static int
cmp_lookup_ref(const void *a, const void *b)
{
   const lookup_ref *x = a, *y = b;
   if (x->addr != y->addr) {
      return x->addr < y->addr ? -1 : 1;
   }
   return x->i < y->i ? -1 : (x->i > y->i ? 1 : 0);
}

/* n lookups (filters[i], keys[i]) in one GPU round trip: the batch form of the per-bundle
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
   lookup_ref      *order  = malloc(sizeof(*order) * n);
   uint32          *h      = malloc(sizeof(uint32) * n);
   uint64          *fo     = malloc(sizeof(uint64) * n);
   rf_amd_batch   **groups = malloc(sizeof(*groups) * n);
   uint64          *counts = malloc(sizeof(uint64) * n);
   platform_assert(order && h && fo && groups && counts);
   /* group the lookups by filter */
   for (uint64 i = 0; i < n; i++) {
      order[i].addr = filters[i].addr;
      order[i].i    = i;
   }
   qsort(order, n, sizeof(*order), cmp_lookup_ref);
   platform_status rc = STATUS_OK;
   uint32          ng = 0;
   uint64          m  = 0;
   for (uint64 s = 0; s < n && SUCCESS(rc);) {
      uint64 t = s;
      while (t < n && order[t].addr == order[s].addr) {
         t++;
      }
      if (order[s].addr == 0) { /* NULL filter finds nothing (:1003-1006) */
         for (uint64 i = s; i < t; i++) {
            found[order[i].i] = 0;
         }
      } else {
         rf_amd_batch *b;
         rc = resident(cc, cfg, &filters[order[s].i], &b);
         if (SUCCESS(rc)) {
            for (uint64 i = s; i < t; i++) {
               h[m + (i - s)] = data_key_hash(cfg->data_cfg, keys[order[i].i], cfg->seed);
            }
            groups[ng] = b;
            counts[ng] = t - s;
            ng++;
            m += t - s;
         }
      }
      s = t;
   }
   if (SUCCESS(rc)) {
      rc = status_of(rf_amd_probe_many_hashes_host(engine(), groups, NULL, counts, ng, h, fo));
   }
   if (SUCCESS(rc)) {
      uint64 at = 0;
      for (uint64 i = 0; i < n; i++) {
         if (order[i].addr != 0) {
            found[order[i].i] = fo[at++];
         }
      }
   }
   free(order);
   free(h);
   free(fo);
   free(groups);
   free(counts);
   return rc;
}

void
routing_filter_amd_async_stats(uint64 *batches, uint64 *probes)
{
   *batches = __atomic_load_n(&g_async_batches, __ATOMIC_RELAXED);
   *probes  = __atomic_load_n(&g_async_probes, __ATOMIC_RELAXED);
}

async_status
routing_filter_lookup_async(routing_filter_lookup_async_state *state)
{
   async_state at = __atomic_load_n(&state->__async_state_stack[0], __ATOMIC_ACQUIRE);
   if (at == ASYNC_STATE_DONE) {
      return ASYNC_STATUS_DONE;
   }
   if (at == ASYNC_STATE_QUEUED) {
      /* the owner is waiting on it: probe everything queued so far, this state included */
      routing_filter_amd_flush();
      at = __atomic_load_n(&state->__async_state_stack[0], __ATOMIC_ACQUIRE);
      return at == ASYNC_STATE_DONE ? ASYNC_STATUS_DONE : ASYNC_STATUS_RUNNING;
   }
   /* ASYNC_STATE_INIT (:898-905) */
   if (state->filter.addr == 0) {
      *state->found_values = 0;
      state->__async_result = STATUS_OK;
      state->__async_state_stack[0] = ASYNC_STATE_DONE;
      return ASYNC_STATUS_DONE;
   }
   state->fp = data_key_hash(state->cfg->data_cfg, state->target, state->cfg->seed);
   state->__async_state_stack[0] = ASYNC_STATE_QUEUED;
   uint64 limit = async_batch_limit();
   pthread_mutex_lock(&g_async_mu);
   if (g_async_n == g_async_cap) {
      g_async_cap = g_async_cap ? 2 * g_async_cap : 256;
      g_async_q   = realloc(g_async_q, sizeof(*g_async_q) * g_async_cap);
      platform_assert(g_async_q != NULL);
   }
   g_async_q[g_async_n++] = state;
   int full               = g_async_n >= limit;
   pthread_mutex_unlock(&g_async_mu);
   if (full) {
      routing_filter_amd_flush();
   }
   return __atomic_load_n(&state->__async_state_stack[0], __ATOMIC_ACQUIRE) == ASYNC_STATE_DONE
             ? ASYNC_STATUS_DONE
             : ASYNC_STATUS_RUNNING;
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
   rf_amd_batch *batches[MAX_FILTERS];
   uint32        index[MAX_FILTERS];
   for (uint64 i = 0; i < num_filters; i++) {
      batches[i] = NULL;
      index[i]   = 0;
      if (filter[i].addr != 0) {
         platform_status rc = resident(cc, cfg, &filter[i], &batches[i]);
         if (!SUCCESS(rc)) {
            return rc;
         }
      }
   }
   return status_of(rf_amd_batch_estimate_unique_fp(batches, index, num_filters, num_unique_fp));
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
      rf_amd_batch   *b;
      platform_status rc = resident(cc, cfg, filter, &b);
      platform_assert_status_ok(rc);
      platform_assert(rf_amd_batch_probe_hashes_host(b, h, NULL, n, found) == 0);
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
