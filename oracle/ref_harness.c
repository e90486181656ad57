/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Drives the reference's OWN routing filter -- vmware/splinterdb src/routing_filter.c,
 * src/mini_allocator.c, src/clockcache.c, src/rc_allocator.c, src/PackedArray.c, compiled
 * unmodified from /root/reference by oracle/Makefile into oracle/_ref/libref_rf.so -- so
 * that the oracle restatement (rf_oracle.c) and the GPU images can be checked against
 * filters the reference itself built, byte for byte.
 *
 * The reference's storage device sits behind its abstract IO interface (io_ops,
 * src/platform_linux/platform_io.h:92-110). Its one implementation, laio.c, needs libaio,
 * which this image lacks, so laio.c and platform_io.c are NOT compiled; this file provides
 * an in-memory device behind the same interface instead (an anonymous mapping the size of
 * the configured disk), plus the two non-virtual helpers platform_io.c would provide
 * (io_config_valid, io_read_bootstrap). No libaio stand-in exists. The cache is sized to
 * hold every page, so nothing is ever written back to the device (the tests assert it) and
 * every filter page is a fresh cache page; the only device reads are incremental adds'
 * prefetch of the old filter's extents (mini_prefetch, src/routing_filter.c:356). Async
 * requests follow laio's completion protocol (mem_async_run below).
 *
 * Everything else -- routing_filter_add / _lookup / _lookup_async / _estimate_unique_fp,
 * the clockcache the pages live in, the mini_allocator that assigns their addresses -- is
 * the reference's code. rfr_filter_image() reads a built filter back through cache_get
 * (src/cache.h:268) into this repo's relocatable image form: data pages in placement order,
 * slot = data_page_no * page_size + offset (the reference stores absolute disk addresses,
 * src/routing_filter.c:620).
 */
#define _GNU_SOURCE
#include "platform.h"
#include "routing_filter.h"
#include "clockcache.h"
#include "rc_allocator.h"
#include "splinterdb/default_data_config.h"

#include <execinfo.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <pthread.h>
#include <x86intrin.h>
#include <sched.h>
#include <signal.h>
#include <stdatomic.h>
#include <sys/mman.h>
#include <sys/uio.h>
#include <time.h>

/* ---- in-memory device behind io_ops --------------------------------------------------- */
struct mem_async_state;
typedef struct mem_io {
   io_handle  super;
   io_config *cfg;
   uint8     *disk;
   uint64     size;
   _Atomic uint64 reads, writes;
   /* submitted requests whose completion callback io_cleanup has not fired yet */
   pthread_mutex_t         lock;
   struct mem_async_state *pending;
} mem_io;

static platform_status
mem_rw(mem_io *io, void *buf, uint64 bytes, uint64 addr, int wr)
{
   if (addr > io->size || bytes > io->size - addr) {
      return STATUS_IO_ERROR;
   }
   if (wr) {
      memcpy(io->disk + addr, buf, bytes);
      atomic_fetch_add(&io->writes, 1);
   } else {
      memcpy(buf, io->disk + addr, bytes);
      atomic_fetch_add(&io->reads, 1);
   }
   return STATUS_OK;
}

static platform_status
mem_read(io_handle *io, void *buf, uint64 bytes, uint64 addr)
{
   return mem_rw((mem_io *)io, buf, bytes, addr, 0);
}

static platform_status
mem_write(io_handle *io, void *buf, uint64 bytes, uint64 addr)
{
   return mem_rw((mem_io *)io, buf, bytes, addr, 1);
}

#define MEM_ASYNC_MAX_PAGES 32 /* pages_per_extent (laio.c appends at most one extent) */
typedef struct mem_async_state {
   io_async_state          super;
   mem_io                 *io;
   io_async_cmd            cmd;
   uint64                  addr;
   uint64                  iovlen;
   platform_status         rc;
   int                     submitted;
   async_callback_fn       callback;
   void                   *callback_arg;
   struct mem_async_state *next;
   struct iovec            iov[MEM_ASYNC_MAX_PAGES];
} mem_async_state;
_Static_assert(sizeof(mem_async_state) <= IO_ASYNC_STATE_BUFFER_SIZE, "async state too large");

static platform_status
mem_async_append_page(io_async_state *s, void *buf)
{
   mem_async_state *m = (mem_async_state *)s;
   if (m->iovlen == MEM_ASYNC_MAX_PAGES) {
      return STATUS_LIMIT_EXCEEDED;
   }
   m->iov[m->iovlen].iov_base = buf;
   m->iov[m->iovlen].iov_len  = m->io->cfg->page_size;
   m->iovlen++;
   return STATUS_OK;
}

/*
 * laio's protocol (src/platform_linux/laio.c:338-464): an empty request is DONE at once; a
 * submitted one returns RUNNING, its completion callback fires from a later io_cleanup
 * (laio.c:328-336), and the next run returns DONE. Callers such as clockcache's prefetch
 * (src/clockcache.c:2463-2540) ignore run's result and finish only in that callback. The
 * copy itself happens at submission; once queued the state belongs to the device.
 */
static async_status
mem_async_run(io_async_state *s)
{
   mem_async_state *m = (mem_async_state *)s;
   if (m->iovlen == 0 || m->submitted) {
      return ASYNC_STATUS_DONE;
   }
   uint64 a = m->addr;
   for (uint64 k = 0; k < m->iovlen && SUCCESS(m->rc); k++) {
      m->rc = mem_rw(m->io, m->iov[k].iov_base, m->iov[k].iov_len, a, m->cmd == io_async_pwritev);
      a += m->iov[k].iov_len;
   }
   m->submitted = 1;
   mem_io *io   = m->io;
   pthread_mutex_lock(&io->lock);
   m->next     = io->pending;
   io->pending = m;
   pthread_mutex_unlock(&io->lock);
   return ASYNC_STATUS_RUNNING;
}

static platform_status
mem_async_result(io_async_state *s)
{
   return ((mem_async_state *)s)->rc;
}

static const struct iovec *
mem_async_iovec(io_async_state *s, uint64 *iovlen)
{
   mem_async_state *m = (mem_async_state *)s;
   *iovlen            = m->iovlen;
   return m->iov;
}

static void
mem_async_deinit(io_async_state *s)
{
   (void)s;
}

static io_async_state_ops mem_async_ops = {
   .append_page = mem_async_append_page,
   .run         = mem_async_run,
   .get_result  = mem_async_result,
   .get_iovec   = mem_async_iovec,
   .deinit      = mem_async_deinit,
};

static platform_status
mem_async_init(io_async_state   *state,
               io_handle        *io,
               io_async_cmd      cmd,
               uint64            addr,
               async_callback_fn callback,
               void             *callback_arg)
{
   mem_async_state *m = (mem_async_state *)state;
   m->super.ops    = &mem_async_ops;
   m->io           = (mem_io *)io;
   m->cmd          = cmd;
   m->addr         = addr;
   m->iovlen       = 0;
   m->rc           = STATUS_OK;
   m->submitted    = 0;
   m->callback     = callback;
   m->callback_arg = callback_arg;
   m->next         = NULL;
   return STATUS_OK;
}

/* fire up to count completion callbacks (count 0: all), as laio's io_cleanup does */
static void
mem_cleanup(io_handle *ioh, uint64 count)
{
   mem_io *io = (mem_io *)ioh;
   for (uint64 done = 0; count == 0 || done < count; done++) {
      pthread_mutex_lock(&io->lock);
      mem_async_state *m = io->pending;
      if (m) {
         io->pending = m->next;
      }
      pthread_mutex_unlock(&io->lock);
      if (!m) {
         break;
      }
      if (m->callback) {
         m->callback(m->callback_arg);
      }
   }
}

static void
mem_wait_all(io_handle *io)
{
   mem_cleanup(io, 0);
}

static io_ops mem_io_ops = {
   .read             = mem_read,
   .write            = mem_write,
   .async_state_init = mem_async_init,
   .cleanup          = mem_cleanup,
   .wait_all         = mem_wait_all,
};

/* the two non-virtual io helpers of platform_io.c (not compiled: it includes laio.h) */
platform_status
io_config_valid(io_config *cfg)
{
   if (cfg->page_size != 4096 && cfg->page_size != 8192) {
      return STATUS_BAD_PARAM;
   }
   if (cfg->extent_size % cfg->page_size != 0) {
      return STATUS_BAD_PARAM;
   }
   return STATUS_OK;
}

platform_status
io_read_bootstrap(const char *filename, void *buf, uint64 bytes, uint64 addr)
{
   (void)filename;
   (void)buf;
   (void)bytes;
   (void)addr;
   return STATUS_NOTSUP; /* only used to mount an existing disk, never here */
}

/* the in-memory device as a standalone io handle: platform_io.c's io_handle_create /
 * io_handle_destroy for the kvstore harness (ref_kvs.c), sized by g_rfr_kvs_disk_bytes */
uint64 g_rfr_kvs_disk_bytes = 16ull << 30;

io_handle *
rfr_mem_io_create(io_config *cfg, uint64 bytes)
{
   mem_io *io = calloc(1, sizeof(*io));
   if (!io) {
      return NULL;
   }
   io->super.ops = &mem_io_ops;
   pthread_mutex_init(&io->lock, NULL);
   io->cfg  = cfg;
   io->size = bytes;
   io->disk = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
   if (io->disk == MAP_FAILED) {
      free(io);
      return NULL;
   }
   return &io->super;
}

void
rfr_mem_io_destroy(io_handle *ioh)
{
   mem_io *io = (mem_io *)ioh;
   if (!io) {
      return;
   }
   mem_cleanup(ioh, 0);
   munmap(io->disk, io->size);
   free(io);
}

/* ---- one reference filter stack: heap, device, allocator, clockcache, configs --------- */
typedef struct rfr_stack {
   platform_heap_id  hid;
   io_config         io_cfg;
   allocator_config  al_cfg;
   clockcache_config cc_cfg;
   mem_io            io;
   rc_allocator      al;
   clockcache        cc;
   data_config       data_cfg;
   routing_config    rcfg;
} rfr_stack;

static _Atomic int g_registered_main = 0;


/* the shim's cache attach / release (weak: absent from the reference's own library) */
__attribute__((weak)) int
routing_filter_amd_cache_attach(cache *cc);
__attribute__((weak)) void
routing_filter_amd_cache_release(cache *cc);

/* diagnostics (RFR_ABORT_BT=1): a native backtrace on SIGABRT / SIGSEGV, to stderr */
static void
rfr_crash_bt(int sig)
{
   void *f[64];
   int   n = backtrace(f, 64);
   char  msg[48];
   int   m = snprintf(msg, sizeof(msg), "rfr: signal %d, backtrace:\n", sig);
   if (m > 0) {
      (void)!write(2, msg, (size_t)m);
   }
   backtrace_symbols_fd(f, n, 2);
   signal(sig, SIG_DFL);
   raise(sig);
}

rfr_stack *
rfr_create(uint32 fingerprint_size, uint32 log_index_size, uint64 cache_mib, uint64 disk_mib)
{
   static int bt_armed;
   if (!bt_armed && getenv("RFR_ABORT_BT")) {
      bt_armed = 1;
      signal(SIGABRT, rfr_crash_bt);
      signal(SIGSEGV, rfr_crash_bt);
   }
   if (!atomic_exchange(&g_registered_main, 1)) {
      platform_register_thread();
   }
   rfr_stack *s = calloc(1, sizeof(*s));
   if (!s) {
      return NULL;
   }
   platform_status rc = platform_heap_create(platform_get_module_id(), 1024 * MiB, FALSE, &s->hid);
   if (!SUCCESS(rc)) {
      free(s);
      return NULL;
   }
   io_config_init(&s->io_cfg, 4096, 4096 * 32, O_RDWR | O_CREAT, 0600, 256, "rfr-memory-device");
   const uint64 disk = disk_mib * MiB;
   s->io.super.ops   = &mem_io_ops;
   pthread_mutex_init(&s->io.lock, NULL);
   s->io.cfg         = &s->io_cfg;
   s->io.size        = disk;
   s->io.disk        = mmap(NULL, disk, PROT_READ | PROT_WRITE,
                     MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
   if (s->io.disk == MAP_FAILED) {
      free(s);
      return NULL;
   }
   allocator_config_init(&s->al_cfg, &s->io_cfg, disk);
   rc = rc_allocator_init(&s->al, &s->al_cfg, &s->io.super, s->hid, platform_get_module_id());
   if (!SUCCESS(rc)) {
      munmap(s->io.disk, disk);
      free(s);
      return NULL;
   }
   clockcache_config_init(&s->cc_cfg, &s->io_cfg, cache_mib * MiB, "", FALSE);
   rc = clockcache_init(&s->cc, &s->cc_cfg, &s->io.super, (allocator *)&s->al, "rfr", s->hid,
                        platform_get_module_id());
   if (!SUCCESS(rc)) {
      rc_allocator_deinit(&s->al);
      munmap(s->io.disk, disk);
      free(s);
      return NULL;
   }
   default_data_config_init(&s->data_cfg);
   /* the shim: this cache attached (images placed straight into its pages; released in
      rfr_destroy before the buffer is unmapped) */
   if (routing_filter_amd_cache_attach) {
      (void)routing_filter_amd_cache_attach((cache *)&s->cc);
   }
   /* splinterdb.c:270-276 / tests/functional/test.h: hash argument ignored, seed 42 */
   routing_config_init(&s->rcfg, (cache_config *)&s->cc_cfg, &s->data_cfg, fingerprint_size,
                       log_index_size, NULL, 42);
   return s;
}


void
rfr_destroy(rfr_stack *s)
{
   if (!s) {
      return;
   }
   mem_cleanup(&s->io.super, 0); /* complete every outstanding request first */
   if (routing_filter_amd_cache_release) {
      routing_filter_amd_cache_release((cache *)&s->cc);
   }
   clockcache_deinit(&s->cc);
   rc_allocator_deinit(&s->al);
   munmap(s->io.disk, s->io.size);
   platform_heap_destroy(&s->hid);
   free(s);
}

/* device traffic: writes = pages the clockcache wrote back (evicted or flushed); reads =
 * pages read in (incremental adds prefetch the old filter's extents, mini_prefetch,
 * src/routing_filter.c:356, which includes pages never allocated -- zeros on the device) */
uint64
rfr_device_io_count(rfr_stack *s, int writes)
{
   return writes ? atomic_load(&s->io.writes) : atomic_load(&s->io.reads);
}

uint64
rfr_max_fingerprints(rfr_stack *s)
{
   return routing_filter_max_fingerprints((cache_config *)&s->cc_cfg, &s->rcfg);
}

/* routing_filter_add; fps is mutated (shifted + sorted), as the reference does */
int
rfr_filter_add(rfr_stack      *s,
               routing_filter *old_filter,
               routing_filter *filter,
               uint32         *fps,
               uint64          n,
               uint16          value)
{
   routing_filter empty = NULL_ROUTING_FILTER;
   memset(filter, 0, sizeof(*filter));
   platform_status rc = routing_filter_add(
      (cache *)&s->cc, &s->rcfg, old_filter ? old_filter : &empty, filter, fps, n, value);
   return rc.r;
}

/* one 4 KiB page of the cache into dst (cache_get / cache_unget, src/cache.h:268-311) */
static void
read_page(rfr_stack *s, uint64 addr, uint8 *dst)
{
   page_handle *pg = cache_get((cache *)&s->cc, addr, TRUE, PAGE_TYPE_FILTER);
   memcpy(dst, pg->data, s->io_cfg.page_size);
   cache_unget((cache *)&s->cc, pg);
}

/*
 * The filter as a relocatable image: the index slots of the index extent at filter->addr
 * (slot i at page i / addrs_per_page, src/routing_filter.c:178-198), their data pages in
 * order of first use (blocks are placed in index order, :599-620), each copied out whole.
 * Returns the number of indices (0 = NULL filter); *num_pages = data pages. pages must
 * hold max_pages * page_size bytes, slots num_indices entries.
 */
uint32
rfr_filter_image(rfr_stack      *s,
                 routing_filter *f,
                 uint8          *pages,
                 uint32          max_pages,
                 uint64         *slots,
                 uint32         *num_pages)
{
   *num_pages = 0;
   if (f->addr == 0) {
      return 0;
   }
   const uint64 ps  = s->io_cfg.page_size;
   const uint32 lis = s->rcfg.log_index_size;
   uint32       lnb = 31 - __builtin_clz(f->num_fingerprints);
   if (lnb < lis) {
      lnb = lis;
   }
   const uint32 num_indices    = 1u << (lnb - lis);
   const uint64 addrs_per_page = ps / sizeof(uint64);
   uint8       *ipage          = malloc(ps);
   uint64       cur_ipage      = UINT64_MAX;
   uint64       last_page      = UINT64_MAX;
   uint32       np             = 0;
   for (uint32 i = 0; i < num_indices; i++) {
      const uint64 ip = f->addr + (i / addrs_per_page) * ps;
      if (ip != cur_ipage) {
         read_page(s, ip, ipage);
         cur_ipage = ip;
      }
      const uint64 hdr  = ((uint64 *)ipage)[i % addrs_per_page];
      const uint64 page = hdr - hdr % ps;
      if (page != last_page) {
         if (np == max_pages) {
            free(ipage);
            return 0;
         }
         read_page(s, page, pages + (uint64)np * ps);
         last_page = page;
         np++;
      }
      slots[i] = (uint64)(np - 1) * ps + hdr % ps;
   }
   free(ipage);
   *num_pages = np;
   return num_indices;
}

/* routing_filter_lookup of n fixed-length keys (key i = keys[i*key_len ..]) */
void
rfr_lookup_keys(rfr_stack      *s,
                routing_filter *f,
                const uint8    *keys,
                uint32          key_len,
                uint64          n,
                uint64         *found)
{
   for (uint64 i = 0; i < n; i++) {
      key             k  = key_create(FALSE, key_len, keys + i * key_len);
      platform_status rc = routing_filter_lookup((cache *)&s->cc, &s->rcfg, f, k, &found[i]);
      if (!SUCCESS(rc)) {
         found[i] = UINT64_MAX;
      }
   }
}

/* variable-length keys: key i = bytes[offs[i] .. offs[i+1]) */
void
rfr_lookup_var_keys(rfr_stack      *s,
                    routing_filter *f,
                    const uint8    *bytes,
                    const uint64   *offs,
                    uint64          n,
                    uint64         *found)
{
   for (uint64 i = 0; i < n; i++) {
      key             k  = key_create(FALSE, offs[i + 1] - offs[i], bytes + offs[i]);
      platform_status rc = routing_filter_lookup((cache *)&s->cc, &s->rcfg, f, k, &found[i]);
      if (!SUCCESS(rc)) {
         found[i] = UINT64_MAX;
      }
   }
}

void
rfr_hash_var_keys(rfr_stack *s, const uint8 *bytes, const uint64 *offs, uint64 n, uint32 *out)
{
   for (uint64 i = 0; i < n; i++) {
      key k  = key_create(FALSE, offs[i + 1] - offs[i], bytes + offs[i]);
      out[i] = data_key_hash(&s->data_cfg, k, s->rcfg.seed);
   }
}

/* the same through the coroutine, routing_filter_lookup_async (:895-972), driven to
 * completion by polling; returns the number of ASYNC_STATUS_RUNNING yields seen */
uint64
rfr_lookup_keys_async(rfr_stack      *s,
                      routing_filter *f,
                      const uint8    *keys,
                      uint32          key_len,
                      uint64          n,
                      uint64         *found)
{
   uint64 yields = 0;
   for (uint64 i = 0; i < n; i++) {
      routing_filter_lookup_async_state st;
      key k = key_create(FALSE, key_len, keys + i * key_len);
      routing_filter_lookup_async_state_init(
         &st, (cache *)&s->cc, &s->rcfg, *f, k, &found[i], NULL, NULL);
      while (routing_filter_lookup_async(&st) != ASYNC_STATUS_DONE) {
         yields++;
         cache_cleanup((cache *)&s->cc);
      }
      if (!SUCCESS(st.__async_result)) {
         found[i] = UINT64_MAX;
      }
   }
   return yields;
}

static void
count_callback(void *arg)
{
   __atomic_fetch_add((uint64 *)arg, 1, __ATOMIC_RELAXED);
}

/*
 * n lookups issued as n concurrent coroutine states (the trunk's async lookup pattern):
 * every state is started once, then all are polled until done. Returns the number of
 * callbacks fired; *running = states whose first call returned ASYNC_STATUS_RUNNING.
 * filter_id[i] picks the filter of key i from filters[].
 */
/* phases of the last rfr_lookup_keys_async_many call (ns): starting every state, polling */
static uint64 g_many_ns[2];

void
rfr_async_many_phases(uint64 *out)
{
   out[0] = g_many_ns[0];
   out[1] = g_many_ns[1];
}

static uint64
mono_ns(void)
{
   struct timespec ts;
   clock_gettime(CLOCK_MONOTONIC, &ts);
   return (uint64)ts.tv_sec * 1000000000ull + (uint64)ts.tv_nsec;
}

uint64
rfr_lookup_keys_async_many(rfr_stack      *s,
                           routing_filter *filters,
                           const uint32   *filter_id,
                           const uint8    *keys,
                           uint32          key_len,
                           uint64          n,
                           uint64         *found,
                           uint64         *running)
{
   routing_filter_lookup_async_state *st = calloc(n ? n : 1, sizeof(*st));
   uint64                             cb = 0;
   *running                              = 0;
   const uint64                       t0 = mono_ns();
   for (uint64 i = 0; i < n; i++) {
      key k = key_create(FALSE, key_len, keys + i * key_len);
      routing_filter_lookup_async_state_init(&st[i], (cache *)&s->cc, &s->rcfg,
                                             filters[filter_id ? filter_id[i] : 0], k,
                                             &found[i], count_callback, &cb);
      if (routing_filter_lookup_async(&st[i]) != ASYNC_STATUS_DONE) {
         (*running)++;
      }
   }
   const uint64 t1 = mono_ns();
   for (uint64 i = 0; i < n; i++) {
      while (routing_filter_lookup_async(&st[i]) != ASYNC_STATUS_DONE) {
         cache_cleanup((cache *)&s->cc);
      }
      if (!SUCCESS(st[i].__async_result)) {
         found[i] = UINT64_MAX;
      }
   }
   g_many_ns[0] = t1 - t0;
   g_many_ns[1] = mono_ns() - t1;
   /* a state can be seen DONE just before its callback runs (on the completing thread):
      every state that yielded gets exactly one callback, so wait for those */
   while (__atomic_load_n(&cb, __ATOMIC_ACQUIRE) < *running) {
      cache_cleanup((cache *)&s->cc);
   }
   free(st);
   return __atomic_load_n(&cb, __ATOMIC_ACQUIRE);
}

/* the shim's flush counters (weak: absent from the reference's own library) */
__attribute__((weak)) void
routing_filter_amd_async_stats(uint64 *batches, uint64 *probes);

int
rfr_async_stats(uint64 *batches, uint64 *probes)
{
   if (!routing_filter_amd_async_stats) {
      *batches = *probes = 0;
      return 0;
   }
   routing_filter_amd_async_stats(batches, probes);
   return 1;
}

/* the shim's other counters and knobs (weak: absent from the reference's own library) */
__attribute__((weak)) void
routing_filter_amd_add_stats(uint64 *batches, uint64 *filters);
__attribute__((weak)) void
routing_filter_amd_registry_stats(uint64 *bytes, uint64 *evictions, uint64 *trims);

__attribute__((weak)) void
routing_filter_amd_flush(void);
__attribute__((weak)) void
routing_filter_amd_registry_set_limit(uint64 mib);

int
rfr_registry_set_limit(uint64 mib)
{
   if (!routing_filter_amd_registry_set_limit) {
      return 0;
   }
   routing_filter_amd_registry_set_limit(mib);
   return 1;
}

__attribute__((weak)) uint64
routing_filter_amd_async_probe_ns(void);
__attribute__((weak)) void
routing_filter_amd_async_breakdown(uint64 *out);
__attribute__((weak)) void
routing_filter_amd_add_breakdown(uint64 *out);

/* out[0..10]: the shim's routing_filter_add breakdown (calls, batches, create / stage / build /
 * infos / readback ns per batch, wait / place ns per add; ns creating the engine, registering
 * cache buffers); 0 without a shim. (Round 5 declared out[0..8] here while the shim writes 11
 * words: the Python caller's 9-word buffer was overrun by 16 bytes on every call -- the heap
 * corruption behind the two-stack latency tool's aborts) */
int
rfr_add_breakdown(uint64 *out)
{
   memset(out, 0, 11 * sizeof(uint64));
   if (!routing_filter_amd_add_breakdown) {
      return 0;
   }
   routing_filter_amd_add_breakdown(out);
   return 1;
}
int
rf_amd_diag_lookup_stats(uint64_t *out, int reset) __attribute__((weak));

/* out[0..5] = the shim's async batches, states, burst / gather / lookup / callback ns;
 * out[6..9] = the engine's lookup round trips: calls, prep / launch / wait ns. 0 without a
 * shim */
int
rfr_async_breakdown(uint64 *out)
{
   memset(out, 0, 10 * sizeof(uint64));
   if (!routing_filter_amd_async_breakdown || !rf_amd_diag_lookup_stats) {
      return 0;
   }
   routing_filter_amd_async_breakdown(out);
   rf_amd_diag_lookup_stats((uint64_t *)&out[6], 0);
   return 1;
}

/* out[0..5] = add batches, filters added, registry bytes, evictions, trims, ns spent probing
 * queued async states; 0 without a shim */
int
rfr_shim_stats(uint64 *out)
{
   memset(out, 0, 6 * sizeof(uint64));
   if (!routing_filter_amd_add_stats) {
      return 0;
   }
   routing_filter_amd_add_stats(&out[0], &out[1]);
   routing_filter_amd_registry_stats(&out[2], &out[3], &out[4]);
   out[5] = routing_filter_amd_async_probe_ns();
   return 1;
}

int
rfr_async_flush(void)
{
   if (!routing_filter_amd_flush) {
      return 0;
   }
   routing_filter_amd_flush();
   return 1;
}

/*
 * n routing_filter_lookup_async states, each started once (first call) and left queued;
 * then routing_filter_amd_flush() answers them all, and each must then be DONE on its next
 * call with its callback fired exactly once. For the "one launch per flush" check: the
 * caller sets the shim's completion thread to a batch and window it cannot reach first.
 * Returns callbacks fired, or UINT64_MAX if a state was not done after the flush.
 */
uint64
rfr_lookup_keys_async_flush(rfr_stack      *s,
                            routing_filter *filters,
                            const uint32   *filter_id,
                            const uint8    *keys,
                            uint32          key_len,
                            uint64          n,
                            uint64         *found)
{
   routing_filter_lookup_async_state *st = calloc(n ? n : 1, sizeof(*st));
   uint64                             cb = 0;
   for (uint64 i = 0; i < n; i++) {
      key k = key_create(FALSE, key_len, keys + i * key_len);
      routing_filter_lookup_async_state_init(&st[i], (cache *)&s->cc, &s->rcfg,
                                             filters[filter_id ? filter_id[i] : 0], k, &found[i],
                                             count_callback, &cb);
      routing_filter_lookup_async(&st[i]);
   }
   rfr_async_flush();
   uint64 ret = 0;
   for (uint64 i = 0; i < n; i++) {
      if (routing_filter_lookup_async(&st[i]) != ASYNC_STATUS_DONE) {
         ret = UINT64_MAX;
      }
   }
   free(st);
   return ret ? ret : __atomic_load_n(&cb, __ATOMIC_ACQUIRE);
}

/*
 * The same over filters of SEVERAL stacks (each its own cache and routing config -- e.g. two
 * kvstores with different filter_hash_size / filter_log_index_size): filter f belongs to
 * stacks[filter_stack[f]]; every state is queued first, then ONE flush answers them all.
 */
uint64
rfr_lookup_keys_async_flush_multi(rfr_stack     **stacks,
                                  routing_filter *filters,
                                  const uint32   *filter_stack,
                                  const uint32   *filter_id,
                                  const uint8    *keys,
                                  uint32          key_len,
                                  uint64          n,
                                  uint64         *found)
{
   routing_filter_lookup_async_state *st = calloc(n ? n : 1, sizeof(*st));
   uint64                             cb = 0;
   for (uint64 i = 0; i < n; i++) {
      rfr_stack *s = stacks[filter_stack[filter_id[i]]];
      key        k = key_create(FALSE, key_len, keys + i * key_len);
      routing_filter_lookup_async_state_init(&st[i], (cache *)&s->cc, &s->rcfg, filters[filter_id[i]], k,
                                             &found[i], count_callback, &cb);
      routing_filter_lookup_async(&st[i]);
   }
   rfr_async_flush();
   uint64 ret = 0;
   for (uint64 i = 0; i < n; i++) {
      if (routing_filter_lookup_async(&st[i]) != ASYNC_STATUS_DONE) {
         ret = UINT64_MAX;
      }
   }
   free(st);
   return ret ? ret : __atomic_load_n(&cb, __ATOMIC_ACQUIRE);
}

/* the shim's batched lookups (weak: absent from the reference's own library) */
__attribute__((weak)) platform_status
routing_filter_amd_lookup_batch(cache                *cc,
                                const routing_config *cfg,
                                routing_filter       *filters,
                                const key            *keys,
                                uint64                n,
                                uint64               *found);

/* n lookups (descs[filter_id[i]], key i): through routing_filter_amd_lookup_batch when the
 * linked implementation has it (returns 1), else one routing_filter_lookup per key (0) */
int
rfr_lookup_batch(rfr_stack      *s,
                 routing_filter *descs,
                 const uint32   *filter_id,
                 const uint8    *keys,
                 uint32          key_len,
                 uint64          n,
                 uint64         *found)
{
   if (!routing_filter_amd_lookup_batch) {
      for (uint64 i = 0; i < n; i++) {
         key k = key_create(FALSE, key_len, keys + i * key_len);
         routing_filter_lookup((cache *)&s->cc, &s->rcfg, &descs[filter_id[i]], k, &found[i]);
      }
      return 0;
   }
   routing_filter *fl = malloc(sizeof(*fl) * (n ? n : 1));
   key            *kl = malloc(sizeof(*kl) * (n ? n : 1));
   for (uint64 i = 0; i < n; i++) {
      fl[i] = descs[filter_id[i]];
      kl[i] = key_create(FALSE, key_len, keys + i * key_len);
   }
   platform_status rc =
      routing_filter_amd_lookup_batch((cache *)&s->cc, &s->rcfg, fl, kl, n, found);
   free(fl);
   free(kl);
   return SUCCESS(rc) ? 1 : -1;
}

/* routing_filter_print of the linked implementation, with platform_default_log pointed at
 * stdout for the call (the library's default is /dev/null, platform_log.c:15-24) */
void
rfr_print(rfr_stack *s, routing_filter *f)
{
   platform_log_handle *info = platform_get_stdout_stream();
   fflush(stdout);
   platform_set_log_streams(stdout, stderr);
   routing_filter_print((cache *)&s->cc, &s->rcfg, f);
   fflush(stdout);
   platform_set_log_streams(info, stderr);
}

/* one raw cache page (all page_size bytes) at a disk address */
void
rfr_read_page(rfr_stack *s, uint64 addr, uint8 *dst)
{
   read_page(s, addr, dst);
}

int
rfr_estimate_unique_fp(rfr_stack *s, routing_filter *filters, uint64 num, uint32 *out)
{
   return routing_filter_estimate_unique_fp((cache *)&s->cc, &s->rcfg, s->hid, filters, num, out).r;
}

uint32
rfr_estimate_unique_keys_from_count(rfr_stack *s, uint64 num_unique)
{
   return routing_filter_estimate_unique_keys_from_count(&s->rcfg, num_unique);
}

uint32
rfr_estimate_unique_keys(rfr_stack *s, routing_filter *f)
{
   return routing_filter_estimate_unique_keys(f, &s->rcfg);
}

uint64
rfr_space_use_bytes(rfr_stack *s, routing_filter *f)
{
   return routing_filter_space_use_bytes((cache *)&s->cc, f);
}

void
rfr_dec_ref(rfr_stack *s, routing_filter *f)
{
   routing_filter_dec_ref((cache *)&s->cc, f);
}

/* the header inlines, as the reference's compiler builds them (src/routing_filter.h:94-111) */
uint16
rfr_get_next_value(uint64 found_values, uint16 last_value)
{
   return routing_filter_get_next_value(found_values, last_value);
}

int
rfr_is_value_found(uint64 found_values, uint16 value)
{
   return routing_filter_is_value_found(found_values, value) ? 1 : 0;
}

/* XXH32 through the reference's data_config (data_key_hash, src/data_internal.h:673-683) */
void
rfr_hash_keys(rfr_stack *s, const uint8 *keys, uint32 key_len, uint64 n, uint32 *out)
{
   for (uint64 i = 0; i < n; i++) {
      key k  = key_create(FALSE, key_len, keys + i * key_len);
      out[i] = data_key_hash(&s->data_cfg, k, s->rcfg.seed);
   }
}

/* ---- CPU baseline: the reference's own build and lookup, P threads ------------------- */
/* One routing_filter_add per filter, filters handed to P registered threads as SplinterDB's
 * TASK_TYPE_NORMAL workers do (src/trunk.c:3932, :4168). hash_keys: 1 = hash the filter's
 * keys first (btree_pack + add, trunk semantics), 0 = keys already are 32-bit hashes
 * (filter_test semantics, tests/functional/filter_test.c:185-205). */
typedef struct rfr_bench {
   rfr_stack      *s;
   const uint8    *keys;
   const uint64   *offs; /* variable-length keys: key i = keys[offs[i] .. offs[i+1]) */
   uint32          key_len;
   int             hash_keys;
   const uint64   *start;
   const uint32   *count;
   uint32          nf;
   uint16          value;
   routing_filter *keep;
   _Atomic uint32  next;
   _Atomic int     err;
   /* compaction chain: rounds per filter, key ids (f << 32) + (v + 1) * j */
   uint32          rounds;
   uint32          chain_n;
   /* probe */
   const uint32   *filter_id;
   uint64          n;
   uint64         *found;
} rfr_bench;

static double
now_s(void)
{
   struct timespec ts;
   clock_gettime(CLOCK_MONOTONIC, &ts);
   return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *
build_worker(void *arg)
{
   rfr_bench *b = arg;
   platform_register_thread();
   for (;;) {
      uint32 f = atomic_fetch_add(&b->next, 1);
      if (f >= b->nf) {
         break;
      }
      uint32  n   = b->count[f];
      uint32 *fps = malloc((size_t)n * 4 + 4);
      if (b->hash_keys) {
         for (uint32 i = 0; i < n; i++) {
            const uint64 j = b->start[f] + i;
            key          k = b->offs ? key_create(FALSE, b->offs[j + 1] - b->offs[j], b->keys + b->offs[j])
                                     : key_create(FALSE, b->key_len, b->keys + j * b->key_len);
            fps[i] = data_key_hash(&b->s->data_cfg, k, b->s->rcfg.seed);
         }
      } else {
         memcpy(fps, (const uint32 *)b->keys + b->start[f], (size_t)n * 4);
      }
      routing_filter  empty = NULL_ROUTING_FILTER;
      platform_status rc    = routing_filter_add(
         (cache *)&b->s->cc, &b->s->rcfg, &empty, &b->keep[f], fps, n, b->value);
      if (!SUCCESS(rc)) {
         atomic_store(&b->err, rc.r);
      }
      free(fps);
   }
   platform_deregister_thread();
   return NULL;
}

static void *
probe_worker(void *arg)
{
   rfr_bench *b = arg;
   platform_register_thread();
   const uint64 chunk = 4096;
   for (;;) {
      uint64 s = (uint64)atomic_fetch_add(&b->next, 1) * chunk;
      if (s >= b->n) {
         break;
      }
      uint64 e = s + chunk < b->n ? s + chunk : b->n;
      for (uint64 i = s; i < e; i++) {
         key k = b->offs ? key_create(FALSE, b->offs[i + 1] - b->offs[i], b->keys + b->offs[i])
                         : key_create(FALSE, b->key_len, b->keys + i * b->key_len);
         routing_filter_lookup(
            (cache *)&b->s->cc, &b->s->rcfg, &b->keep[b->filter_id[i]], k, &b->found[i]);
      }
   }
   platform_deregister_thread();
   return NULL;
}

/* One filter's chain of incremental adds, as the trunk's compactions grow a branch's filter
 * (src/trunk.c:3821-3835 hashes the packed keys, routing_filter_add merges the old filter,
 * routing_filter_dec_ref drops the superseded one): round v adds chain_n 24 B keys of ids
 * (f << 32) + (v + 1) * j under value v -- for f = 0 exactly filter_test's basic chain
 * (tests/functional/filter_test.c:55-78, keys (i + 1) * j). */
static void *
chain_worker(void *arg)
{
   rfr_bench *b = arg;
   platform_register_thread();
   const uint32 n    = b->chain_n;
   uint8       *keys = calloc((size_t)n, 24);
   uint32      *fps  = malloc((size_t)n * 4 + 4);
   for (;;) {
      uint32 f = atomic_fetch_add(&b->next, 1);
      if (f >= b->nf) {
         break;
      }
      routing_filter cur = NULL_ROUTING_FILTER;
      for (uint32 v = 0; v < b->rounds; v++) {
         for (uint32 j = 0; j < n; j++) {
            uint64 id = ((uint64)f << 32) + (uint64)(v + 1) * j;
            memcpy(keys + (size_t)j * 24, &id, 8);
            fps[j] = data_key_hash(&b->s->data_cfg, key_create(FALSE, 24, keys + (size_t)j * 24),
                                   b->s->rcfg.seed);
         }
         routing_filter  next = NULL_ROUTING_FILTER;
         platform_status rc   = routing_filter_add(
            (cache *)&b->s->cc, &b->s->rcfg, &cur, &next, fps, n, (uint16)v);
         if (!SUCCESS(rc)) {
            atomic_store(&b->err, rc.r);
            break;
         }
         if (v > 0) {
            routing_filter_dec_ref((cache *)&b->s->cc, &cur);
         }
         cur = next;
      }
      b->keep[f] = cur;
   }
   free(keys);
   free(fps);
   platform_deregister_thread();
   return NULL;
}

static double
run_threads(rfr_bench *b, int threads, void *(*fn)(void *))
{
   if (threads < 1) {
      threads = 1;
   }
   pthread_t *th = malloc(sizeof(pthread_t) * threads);
   double     t0 = now_s();
   for (int t = 0; t < threads; t++) {
      pthread_create(&th[t], NULL, fn, b);
   }
   for (int t = 0; t < threads; t++) {
      pthread_join(th[t], NULL);
   }
   double t1 = now_s();
   free(th);
   return t1 - t0;
}

/* seconds, or -1 on a failed add; keep[f] = the built filters (caller releases them) */
double
rfr_bench_build(rfr_stack      *s,
                const uint8    *keys,
                const uint64   *offs,
                uint32          key_len,
                int             hash_keys,
                const uint64   *key_start,
                const uint32   *key_count,
                uint32          num_filters,
                uint16          value,
                int             threads,
                routing_filter *keep)
{
   rfr_bench b;
   memset(&b, 0, sizeof(b));
   b.s         = s;
   b.keys      = keys;
   b.offs      = offs;
   b.key_len   = key_len;
   b.hash_keys = hash_keys;
   b.start     = key_start;
   b.count     = key_count;
   b.nf        = num_filters;
   b.value     = value;
   b.keep      = keep;
   double t    = run_threads(&b, threads, build_worker);
   return atomic_load(&b.err) ? -1.0 : t;
}

double
rfr_bench_probe(rfr_stack      *s,
                routing_filter *keep,
                const uint8    *keys,
                const uint64   *offs,
                uint32          key_len,
                const uint32   *filter_id,
                uint64          n,
                int             threads,
                uint64         *found)
{
   rfr_bench b;
   memset(&b, 0, sizeof(b));
   b.s         = s;
   b.keys      = keys;
   b.offs      = offs;
   b.key_len   = key_len;
   b.keep      = keep;
   b.filter_id = filter_id;
   b.n         = n;
   b.found     = found;
   return run_threads(&b, threads, probe_worker);
}

/* seconds for num_filters chains of `rounds` incremental adds of n keys each (chain_worker),
 * or -1 on a failed add; keep[f] = each chain's last filter */
double
rfr_bench_chain(rfr_stack      *s,
                uint32          num_filters,
                uint32          rounds,
                uint32          n,
                int             threads,
                routing_filter *keep)
{
   rfr_bench b;
   memset(&b, 0, sizeof(b));
   b.s       = s;
   b.nf      = num_filters;
   b.rounds  = rounds;
   b.chain_n = n;
   b.keep    = keep;
   double t  = run_threads(&b, threads, chain_worker);
   return atomic_load(&b.err) ? -1.0 : t;
}

/* ---- the stack's pieces, for units that call the reference's own test bodies ------------- */
cache *
rfr_cache(rfr_stack *s)
{
   return (cache *)&s->cc;
}

routing_config *
rfr_routing_config(rfr_stack *s)
{
   return &s->rcfg;
}

platform_heap_id
rfr_heap(rfr_stack *s)
{
   return s->hid;
}

/* platform_default_log into a file for the duration of a test body (one at a time) */
static FILE                *g_log_file;
static platform_log_handle *g_log_saved;

int
rfr_log_begin(const char *log_path)
{
   g_log_file = fopen(log_path, "w");
   if (!g_log_file) {
      return -1;
   }
   g_log_saved = platform_get_stdout_stream();
   platform_set_log_streams(g_log_file, stderr);
   return 0;
}

void
rfr_log_end(void)
{
   fflush(g_log_file);
   platform_set_log_streams(g_log_saved, stderr);
   fclose(g_log_file);
   g_log_file = NULL;
}

/* ---- callback-driven async lookups, as tests/functional/test_async.c drives them --------- */
/*
 * A pool of max_inflight contexts (test_async.c:20-106: avail_q / ready_q). Each key is
 * submitted on a free context with a callback that moves the context to the ready queue
 * (test_async_callback, :25-30); a context is called again ONLY after its callback fired
 * (async_ctxt_process_ready, :168-196). A state whose call returns DONE is finished and its
 * context reused. Protocol violations are counted in stats[3]: a callback for a context not
 * waiting, a state both called back and returned DONE by the same call, a state called back
 * whose next call does not return DONE, or more than one callback per submission.
 * stats: [0] first calls that returned RUNNING, [1] callbacks, [2] lookups finished,
 * [3] violations. Returns 0, or -1 when no progress was made for timeout_s seconds (a state
 * whose callback never fires).
 */
typedef struct rfr_actx {
   routing_filter_lookup_async_state st;
   uint64                            i;
   _Atomic uint32                    cbs;   /* callbacks of the current submission */
   _Atomic int                       phase; /* 0 free, 1 submitted */
   struct rfr_actx                  *next;
   struct rfr_adrive                *d;
} rfr_actx;

typedef struct rfr_adrive {
   pthread_mutex_t mu;
   rfr_actx       *ready;
   _Atomic uint64  callbacks, violations;
} rfr_adrive;

static void
actx_callback(void *arg)
{
   rfr_actx   *c = arg;
   rfr_adrive *d = c->d;
   if (atomic_fetch_add(&c->cbs, 1) != 0 || atomic_load(&c->phase) != 1) {
      atomic_fetch_add(&d->violations, 1);
   } else {
      pthread_mutex_lock(&d->mu);
      c->next  = d->ready;
      d->ready = c;
      pthread_mutex_unlock(&d->mu);
   }
   /* last: the driver frees the contexts and destroys d (its stack frame) once every owed
      callback has counted itself, so nothing may touch them after this */
   atomic_fetch_add(&d->callbacks, 1);
}

int
rfr_lookup_keys_async_driven(rfr_stack      *s,
                             routing_filter *filters,
                             const uint32   *filter_id,
                             const uint8    *keys,
                             uint32          key_len,
                             uint64          n,
                             uint64         *found,
                             uint32          max_inflight,
                             uint64         *stats,
                             double          timeout_s)
{
   rfr_adrive d;
   pthread_mutex_init(&d.mu, NULL);
   d.ready = NULL;
   atomic_store(&d.callbacks, 0);
   atomic_store(&d.violations, 0);
   rfr_actx *ctx   = calloc(max_inflight, sizeof(*ctx));
   rfr_actx *avail = NULL;
   for (uint32 k = 0; k < max_inflight; k++) {
      ctx[k].d    = &d;
      ctx[k].next = avail;
      avail       = &ctx[k];
   }
   uint64 next = 0, done = 0, running = 0;
   double last = now_s();
   int    ret  = 0;
   /* RFR_DRIVE_PROF=1 (diagnostics): TSC cycles of the driving loop's parts -- first calls,
      the ready list's second calls, cleanup -- and iterations, printed to stderr */
   const int prof = getenv("RFR_DRIVE_PROF") && atoi(getenv("RFR_DRIVE_PROF")) > 0;
   uint64    pc[3] = {0, 0, 0}, iters = 0, firsts = 0, seconds = 0;
#define FINISH(c)                                                                              \
   do {                                                                                        \
      found[(c)->i] = SUCCESS((c)->st.__async_result) ? found[(c)->i] : UINT64_MAX;            \
      atomic_store(&(c)->phase, 0);                                                            \
      (c)->next = avail;                                                                       \
      avail     = (c);                                                                         \
      done++;                                                                                  \
      last = now_s();                                                                          \
   } while (0)
   while (done < n) {
      const uint64 q0 = prof ? __rdtsc() : 0;
      iters++;
      while (avail && next < n) {
         firsts++;
         rfr_actx *c = avail;
         avail       = c->next;
         c->i        = next++;
         atomic_store(&c->cbs, 0);
         atomic_store(&c->phase, 1);
         key k = key_create(FALSE, key_len, keys + c->i * key_len);
         routing_filter_lookup_async_state_init(&c->st, (cache *)&s->cc, &s->rcfg,
                                                filters[filter_id ? filter_id[c->i] : 0], k,
                                                &found[c->i], actx_callback, c);
         if (routing_filter_lookup_async(&c->st) == ASYNC_STATUS_DONE) {
            /* done without waiting: no callback may fire for it */
            if (atomic_load(&c->cbs) != 0) {
               atomic_fetch_add(&d.violations, 1);
            }
            FINISH(c);
         } else {
            running++;
         }
      }
      const uint64 q1 = prof ? __rdtsc() : 0;
      pthread_mutex_lock(&d.mu);
      rfr_actx *r = d.ready;
      d.ready     = NULL;
      pthread_mutex_unlock(&d.mu);
      while (r) {
         rfr_actx *c = r;
         r           = r->next;
         seconds++;
         if (routing_filter_lookup_async(&c->st) == ASYNC_STATUS_DONE) {
            FINISH(c);
         } else {
            atomic_fetch_add(&d.violations, 1); /* called back, yet not resumable */
         }
      }
      const uint64 q2 = prof ? __rdtsc() : 0;
      if (done < n && now_s() - last > timeout_s) {
         ret = -1;
         break;
      }
      cache_cleanup((cache *)&s->cc);
      if (prof) {
         const uint64 q3 = __rdtsc();
         pc[0] += q1 - q0;
         pc[1] += q2 - q1;
         pc[2] += q3 - q2;
      }
   }
#undef FINISH
   if (prof) {
      fprintf(stderr,
              "rfr drive profile: %lu iterations, %.2f first calls and %.2f second calls each; TSC cycles: "
              "%.0f per first call, %.0f per second call (incl. ready list), %.0f cleanup per iteration\n",
              (unsigned long)iters, (double)firsts / iters, (double)seconds / iters,
              firsts ? (double)pc[0] / firsts : 0.0, seconds ? (double)pc[1] / seconds : 0.0, (double)pc[2] / iters);
   }
   /* every callback owed has fired before the contexts go away */
   double t0 = now_s();
   while (atomic_load(&d.callbacks) < running && now_s() - t0 < timeout_s) {
      sched_yield();
   }
   stats[0] = running;
   stats[1] = atomic_load(&d.callbacks);
   stats[2] = done;
   stats[3] = atomic_load(&d.violations);
   if (ret == 0 && stats[1] < running) {
      ret = -1;
   }
   if (ret == 0) {
      free(ctx);
   } /* else leak the contexts: a late callback may still write them */
   pthread_mutex_destroy(&d.mu);
   return ret;
}

/* ---- many threads at once: adds (incremental chains) and lookups ------------------------- */
/*
 * threads x rounds chains, as SplinterDB's TASK_TYPE_NORMAL workers compact different
 * branches at the same time (src/trunk.c:3932, :4168): thread t builds chain t -- round r
 * hashes keys[(t * rounds + r) * n ...] with data_key_hash and routing_filter_add's them
 * onto round r - 1 under value r -- keeping every filter in out[t * rounds + r]. Then each
 * thread looks up its nprobe probe keys (probe + t * nprobe * key_len) in its last filter,
 * synchronously (found_sync) and through routing_filter_lookup_async states it polls
 * (found_async). Each thread hashes its keys first; the threads then start their adds
 * together, and add_s[t] = thread t's time for its adds (hashing excluded).
 * Returns 0, or the first failing status.
 */
typedef struct rfr_mt {
   rfr_stack       *s;
   const uint8     *keys;
   const uint8     *probe;
   uint32           key_len, threads, rounds;
   uint64           n, nprobe;
   routing_filter  *out;
   uint64          *found_sync, *found_async;
   double          *add_s;
   _Atomic uint32   next_tid, arrived;
   _Atomic int      err;
} rfr_mt;

static void *
mt_worker(void *arg)
{
   rfr_mt      *m = arg;
   const uint32 t = atomic_fetch_add(&m->next_tid, 1);
   platform_register_thread();
   /* every round's fingerprints first (btree_pack's hashing is not what is timed) */
   uint32 *fpa = malloc(sizeof(uint32) * (m->n ? m->n : 1) * m->rounds);
   for (uint32 r = 0; r < m->rounds; r++) {
      const uint8 *kb = m->keys + ((uint64)t * m->rounds + r) * m->n * m->key_len;
      for (uint64 j = 0; j < m->n; j++) {
         fpa[(uint64)r * m->n + j] = data_key_hash(
            &m->s->data_cfg, key_create(FALSE, m->key_len, kb + j * m->key_len), m->s->rcfg.seed);
      }
   }
   uint32 *fps = malloc(sizeof(uint32) * (m->n ? m->n : 1));
   atomic_fetch_add(&m->arrived, 1);
   while (atomic_load(&m->arrived) < m->threads) {
      sched_yield();
   }
   double t0 = now_s();
   for (uint32 r = 0; r < m->rounds; r++) {
      memcpy(fps, fpa + (uint64)r * m->n, sizeof(uint32) * m->n); /* the reference sorts it in place */
      routing_filter  empty = NULL_ROUTING_FILTER;
      routing_filter *old   = r ? &m->out[(uint64)t * m->rounds + r - 1] : &empty;
      platform_status rc    = routing_filter_add((cache *)&m->s->cc, &m->s->rcfg, old,
                                              &m->out[(uint64)t * m->rounds + r], fps, m->n, (uint16)r);
      if (!SUCCESS(rc)) {
         atomic_store(&m->err, rc.r);
         break;
      }
   }
   m->add_s[t] = now_s() - t0;
   free(fps);
   free(fpa);
   if (atomic_load(&m->err) == 0) {
      routing_filter *last = &m->out[(uint64)t * m->rounds + m->rounds - 1];
      const uint8    *pb   = m->probe + (uint64)t * m->nprobe * m->key_len;
      uint64         *fs   = m->found_sync + (uint64)t * m->nprobe;
      uint64         *fa   = m->found_async + (uint64)t * m->nprobe;
      for (uint64 i = 0; i < m->nprobe; i++) {
         key             k  = key_create(FALSE, m->key_len, pb + i * m->key_len);
         platform_status rc = routing_filter_lookup((cache *)&m->s->cc, &m->s->rcfg, last, k, &fs[i]);
         if (!SUCCESS(rc)) {
            fs[i] = UINT64_MAX;
         }
      }
      routing_filter_lookup_async_state *st = calloc(m->nprobe ? m->nprobe : 1, sizeof(*st));
      for (uint64 i = 0; i < m->nprobe; i++) {
         key k = key_create(FALSE, m->key_len, pb + i * m->key_len);
         routing_filter_lookup_async_state_init(&st[i], (cache *)&m->s->cc, &m->s->rcfg, *last, k,
                                                &fa[i], NULL, NULL);
         routing_filter_lookup_async(&st[i]);
      }
      for (uint64 i = 0; i < m->nprobe; i++) {
         while (routing_filter_lookup_async(&st[i]) != ASYNC_STATUS_DONE) {
            cache_cleanup((cache *)&m->s->cc);
         }
         if (!SUCCESS(st[i].__async_result)) {
            fa[i] = UINT64_MAX;
         }
      }
      free(st);
   }
   platform_deregister_thread();
   return NULL;
}

int
rfr_mt_chains(rfr_stack      *s,
              const uint8    *keys,
              uint32          key_len,
              uint32          threads,
              uint32          rounds,
              uint64          n,
              const uint8    *probe,
              uint64          nprobe,
              routing_filter *out,
              uint64         *found_sync,
              uint64         *found_async,
              double         *add_s)
{
   rfr_mt m;
   memset(&m, 0, sizeof(m));
   m.s           = s;
   m.keys        = keys;
   m.probe       = probe;
   m.key_len     = key_len;
   m.threads     = threads;
   m.rounds      = rounds;
   m.n           = n;
   m.nprobe      = nprobe;
   m.out         = out;
   m.found_sync  = found_sync;
   m.found_async = found_async;
   m.add_s       = add_s;
   pthread_t *th = malloc(sizeof(pthread_t) * threads);
   for (uint32 t = 0; t < threads; t++) {
      pthread_create(&th[t], NULL, mt_worker, &m);
   }
   for (uint32 t = 0; t < threads; t++) {
      pthread_join(th[t], NULL);
   }
   free(th);
   return atomic_load(&m.err);
}
