// rf_engine.cpp -- host runtime of the MI355X routing-filter engine (C ABI: include/rf_amd.h).
//
// Owns device workspaces, builds the per-batch plan (geometry of src/routing_filter.c:
// 357-389 per filter, plus the coarse-bucket / page-bound bookkeeping of this engine) and
// issues the kernel sequence of rf_kernels.hip on one HIP stream. No compute happens on
// the host: there is no CPU fallback, and every entry point fails with ENODEV when no HIP
// device is present.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <math.h>
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <x86intrin.h>

#include <map>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rf_amd.h"
#include "../../include/rf_amd_diag.h"
#include "rf_plan.h"

using namespace rf;

extern "C" int rf_launch_build(const LaunchArgs* a);
extern "C" int rf_launch_place(void* stream, const uint8_t* img, const uint64_t* slots, uint32_t first_page,
                                uint32_t count, uint32_t num_pages, uint32_t num_indices, uint32_t page_size,
                                const uint64_t* table, uint32_t addrs_per_page);
extern "C" int rf_launch_old_decode(const LaunchArgs* a);
extern "C" int rf_launch_wave_tab(void* stream, const uint64_t* runs, uint32_t nf, uint64_t n, uint32_t* tab);
extern "C" int rf_launch_plines(const LaunchArgs* a);
extern "C" int rf_launch_seg_fill(void* stream, const uint32_t* pre, uint32_t nf, uint32_t n, uint32_t* fof,
                                  uint32_t* start, uint32_t mul);
extern "C" int rf_launch_build_init(void* stream, uint32_t* cb_count, uint32_t* cb_cursor, uint32_t num_cb,
                                    uint32_t* outs_words, uint32_t num_out_words, uint32_t* overflow,
                                    uint32_t* spill, uint32_t* plist);
extern "C" int rf_launch_probe(const LaunchArgs* a, int kind, const void* in0, const uint64_t* offs,
                               uint32_t key_len, const uint32_t* filter_id, uint64_t n, uint64_t* found);

static thread_local std::string g_err;
static int fail(int rc, const std::string& msg) {
  g_err = msg;
  return rc;
}
#define HIPCHK(x)                                                                     \
  do {                                                                                \
    hipError_t _e = (x);                                                              \
    if (_e != hipSuccess)                                                             \
      return fail(_e == hipErrorOutOfMemory ? RF_AMD_ENOMEM : RF_AMD_EINVAL,          \
                  std::string(#x) + ": " + hipGetErrorString(_e));                    \
  } while (0)

// Device allocations of an engine's batches are recycled through a pool: SplinterDB builds
// a new set of filters on every compaction, so in steady state rf_amd_batch_create finds
// its ~25 work buffers here instead of calling hipMalloc. Sizes are rounded up to classes
// of 1/8 of a power of two (at most 12.5 % slack); a block returns to the pool when its
// batch is destroyed unless the pool already holds RF_AMD_POOL_MIB MiB (default: a quarter
// of the device memory free at engine creation; rf_amd_engine_pool_trim
// hands blocks back).
// rf_amd_batch_destroy synchronises the device first; rf_amd_batch_destroy_on instead
// parks the blocks behind an event on the caller's stream (stream-ordered release, as
// hipFreeAsync): they become reusable once that event has completed.
// RF_AMD_POOL_TRACE=<ms>: diagnostics, every pool hipMalloc / hipFree slower than that
static uint64_t pool_trace_ns() {
  static const char* v = getenv("RF_AMD_POOL_TRACE");
  if (!v) return 0;
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
static void pool_trace(const char* what, size_t bytes, uint64_t t0) {
  if (!t0) return;
  static const double lim = atof(getenv("RF_AMD_POOL_TRACE"));
  const double ms = (pool_trace_ns() - t0) * 1e-6;
  fprintf(stderr, "rf_amd pool: %s %zu B %.3f ms%s\n", what, bytes, ms, ms >= lim ? " SLOW" : "");
}

struct DevPool {
  std::mutex mu;
  std::multimap<size_t, void*> free_blocks;
  struct Parked {
    hipEvent_t ev;
    std::vector<std::pair<void*, size_t>> blocks;  // size 0: not pooled, hipFree when released
  };
  std::vector<Parked> parked;
  size_t pooled = 0, limit = 0;
  uint64_t hits = 0, misses = 0;
  static size_t size_class(size_t bytes) {
    if (bytes <= 4096) return 4096;
    const int lg = 63 - __builtin_clzll((unsigned long long)bytes);
    const size_t step = (size_t)1 << (lg - 3);
    return (bytes + step - 1) / step * step;
  }
  void give_locked(void* p, size_t cls) {
    if (cls == 0 || pooled + cls > limit) {
      const uint64_t t0 = pool_trace_ns();
      (void)hipFree(p);
      pool_trace("hipFree", cls, t0);
      return;
    }
    free_blocks.emplace(cls, p);
    pooled += cls;
  }
  // parked blocks whose event has completed (wait: every parked block) go to free_blocks
  void reap_locked(bool wait) {
    for (size_t i = 0; i < parked.size();) {
      Parked& k = parked[i];
      if (wait) (void)hipEventSynchronize(k.ev);
      if (!wait && hipEventQuery(k.ev) != hipSuccess) {
        i++;
        continue;
      }
      for (auto& b : k.blocks) give_locked(b.first, b.second);
      (void)hipEventDestroy(k.ev);
      parked[i] = std::move(parked.back());
      parked.pop_back();
    }
  }
  // best fit: the smallest pooled block of at least `*cls` bytes and at most twice that
  // (compaction rounds grow from one round to the next, so exact classes rarely recur within
  // a chain); *cls becomes the block's size
  void* take(size_t* cls) {
    std::lock_guard<std::mutex> g(mu);
    if (!parked.empty()) reap_locked(false);
    auto it = free_blocks.lower_bound(*cls);
    if (it == free_blocks.end() || it->first > 2 * *cls) {
      misses++;
      return nullptr;
    }
    void* p = it->second;
    *cls = it->first;
    free_blocks.erase(it);
    pooled -= *cls;
    hits++;
    return p;
  }
  bool give(void* p, size_t cls) {
    std::lock_guard<std::mutex> g(mu);
    if (pooled + cls > limit) return false;
    free_blocks.emplace(cls, p);
    pooled += cls;
    return true;
  }
  void park(Parked&& k) {
    std::lock_guard<std::mutex> g(mu);
    parked.push_back(std::move(k));
  }
  void drain() {
    std::lock_guard<std::mutex> g(mu);
    reap_locked(true);
    for (auto& kv : free_blocks) (void)hipFree(kv.second);
    free_blocks.clear();
    pooled = 0;
  }
};

// host-buffer entry points stage through these (rf_amd_batch_*_host): pinned host memory
// and a device buffer per engine, grown on demand, one caller at a time
struct HostStage {
  std::mutex mu;
  void* h = nullptr;
  void* d = nullptr;
  size_t cap = 0;
};

// A lookup channel of the host-buffer probe entry points (rf_amd_probe_filters_host and the
// forms built on it). Callers on different threads take different slots, so their round
// trips -- stream, pinned buffers, completion word -- run concurrently. A round trip is ONE
// kernel launch: the kernel reads the probes from `h` (pinned, device-mapped) or, for large
// calls, from `d` after one H2D copy, writes every result straight into `h`, and its last
// workgroup stores the call's sequence number into `flag`, which the host polls.
struct ProbeSlot {
  hipStream_t st = nullptr;
  uint8_t* h = nullptr;  // pinned coherent host memory: [hashes | groups ids | group table | results]
  size_t hcap = 0;
  uint8_t* d = nullptr;  // device copy of the inputs (copy mode)
  size_t dcap = 0;
  uint32_t* flag = nullptr;       // pinned coherent: the kernel's completion word
  uint32_t* d_counter = nullptr;  // device: workgroups finished (k_probe_groups)
  uint32_t seq = 0;
};

// The engine's lookup server (k_lookup_server): rings in pinned coherent host memory, the
// persistent kernel's generation and state, and the host-side bookkeeping of tickets.
// Submitting threads and the reaping thread run on different cores (often different CCDs of
// the host, where moving a written cache line costs ~300 ns), so the words each side writes
// sit on lines of their own: the submitters' ticket counter, the reaper's lock and cursor, and
// the read-mostly server state each get a 128-byte block (round 5 had them on one line, and a
// reaper spinning on its lock cost each submit several such transfers: 0.7 us per submit,
// profiles/r06_async_submit.txt).
struct LookupServer {
  std::once_flag once;
  int init_rc = 0;
  SrvReq* ring = nullptr;  // device memory the host writes through the BAR (or pinned host memory)
  bool ring_dev = false;
  SrvRes* res = nullptr;   // pinned coherent host memory
  SrvCtl* ctl = nullptr;
  hipStream_t st = nullptr;             // its own HSA queue (CU-masked), so it never blocks other work
  std::atomic<uint64_t> idle_ticks{0}, life_ticks{0};  // of the next launch (rf_amd_lookup_server_set_times)
  std::atomic<bool> ready{false};  // rings allocated and initialised (srv_init done)
  // read-mostly: written when a server is launched or fails
  alignas(128) std::atomic<uint64_t> state{0};  // generation << 1 | running
  std::atomic<uint64_t> launches{0};
  // sticky: the first error of the server (a launch that failed, a faulted stream). Every
  // waiter then returns it, submits fail at once, and rf_amd_lookup_server_failed hands the
  // unanswered tickets' tags back, so no caller spins on an answer that cannot come
  std::atomic<int> dead{0};
  // the submitters'
  alignas(128) std::atomic<uint64_t> tail{0};  // the next ticket
  // the reaper's
  alignas(128) std::mutex reap_mu;
  uint64_t reap_next = 0;                      // the next ticket reap() looks at (under reap_mu)
  std::atomic<uint64_t> reap_hint{0};          // reap_next, for the lock-free look of an idle reap
  std::atomic<uint64_t> last_check_ns{0};      // the reaper's last look at the server stream
  // per slot, host-only: the slot's ticket (published after the tag) and the submitter's tag
  // (NULL: a waiter's) -- read by rf_amd_lookup_server_failed (tags of tickets a dead server
  // never answered) and by the next submitter of the slot; the reaper reads answer lines only
  struct Meta {
    std::atomic<uint64_t> ticket{~0ull};
    void* tag = nullptr;
  };
  alignas(128) Meta meta[SRV_RING];
  std::atomic<uint64_t> consumed[SRV_RING];  // per slot: 1 + the last ticket whose result was taken
  // per slot: a ticket whose submitter gave up before publishing it (the server died while it
  // waited for the slot): the reap and failure cursors step over it instead of waiting on it
  std::atomic<uint64_t> abandoned[SRV_RING];
};

struct rf_amd_engine {
  int device;
  uint64_t uid = 0;  // unique per engine created in this process (per-thread caches key on it)
  LookupServer srv;
  // completion points on the engine stream (rf_amd_engine_fence): recycled events
  std::mutex fence_mu;
  std::vector<hipEvent_t> fence_free;
  // host ranges registered for direct image placement (rf_amd_host_register): host base,
  // bytes, device address of the base
  struct HostReg {
    uintptr_t h;
    uint64_t bytes;
    uintptr_t d;
  };
  std::mutex reg_mu;
  std::vector<HostReg> regs;
  hipStream_t stream;
  DevPool pool;
  HostStage stage;
  std::mutex slot_mu;
  std::vector<ProbeSlot*> slots_all, slots_free;
  // builds issued on `stream` (do_build) and the count last seen finished: a lookup slot
  // queries the engine stream only when a build may still be in flight (a HIP call less on
  // the lookup round trip)
  std::atomic<uint64_t> builds_issued{0}, builds_seen_idle{0};
};

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  DevPool* pool = nullptr;
  ~DevBuf() { release(); }
  void release() {
    if (p && !(pool && pool->give(p, n))) (void)hipFree(p);
    p = nullptr;
  }
  int alloc(size_t bytes, DevPool* from = nullptr) {
    release();
    pool = from;
    n = from ? DevPool::size_class(bytes ? bytes : 16) : (bytes ? bytes : 16);
    if (from && (p = from->take(&n)) != nullptr) return 0;
    const uint64_t t0 = pool_trace_ns();
    hipError_t e = hipMalloc(&p, n);
    pool_trace("hipMalloc", n, t0);
    if (e != hipSuccess && from) {  // the pool may hold what this needs: give it back, retry
      from->drain();
      e = hipMalloc(&p, n);
    }
    if (e != hipSuccess) {
      p = nullptr;
      return fail(RF_AMD_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    return 0;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

struct rf_amd_batch {
  rf_amd_engine* eng = nullptr;
  rf_amd_config cfg{};
  uint32_t F = 0;
  bool wide = false;
  bool flag32 = false;      // wide build with 32-bit flagged entries (every fp_size + vs <= 31)
  uint64_t old_total = 0;   // flag32: decoded old entries reserved (sum of old num_fingerprints)
  std::vector<FilterPlan> plans;
  // per-filter prefix arrays (F + 1 each) of the batch's per-element maps: tiles, old tiles,
  // coarse buckets, pages, indices, decoded old indices. The maps themselves (element ->
  // filter, tile -> first key) are filled on the device (k_seg_fill), so creating a batch
  // uploads O(filters) bytes, not O(indices + pages)
  enum { PRE_TILE, PRE_OTILE, PRE_CB, PRE_PG, PRE_IDX, PRE_OIDX, NUM_PRE };
  std::vector<uint32_t> pre;  // NUM_PRE x (F + 1)
  uint32_t* pre_of(int k) { return pre.data() + (size_t)k * (F + 1); }
  uint32_t num_tiles = 0, num_old_tiles = 0, num_old_idx = 0;
  DevBuf d_pre;
  uint64_t E = 0, keys_total = 0;
  uint32_t CB = 0, I = 0, PS = 0, PF = 0;
  uint64_t NL = 0;         // probe lines (64 B each)
  bool plines_needed = false;  // some filter's lines come from k_plines
  uint32_t line_lmax = 0;  // max probe lines per index
  DevBuf d_runs, d_wave_tab;        // probe run bounds (rf_amd_batch_probe_*_runs), their wave table
  std::vector<uint64_t> runs_host;  // their last uploaded value
  DevBuf d_plans, d_outs, d_ent, d_part, d_sorted, d_cb_count, d_cb_start, d_cb_cursor, d_cb_filter,
      d_overflow, d_idx_cnt, d_idx_start, d_slots, d_page_first, d_pg_filter, d_pages, d_tile_filter,
      d_tile_start, d_old_tile_filter, d_old_tile_start, d_old_cnt, d_old_pos, d_first_old, d_has_old, d_pplans, d_lines, d_idx_filter, d_spill,
      d_old_idx_filter, d_old32, d_old_tot, d_ob_lo, d_ob_n, d_pg_noline, d_cb_out;
  bool built = false;
  bool has_entries = false;  // built here: its sorted entries (d_part / d_sorted) are current
  std::vector<uint32_t> err_host;  // per-filter build error bits once read back (err_ready)
  std::atomic<bool> err_ready{false};
  std::mutex err_mu;
  hipEvent_t built_ev = nullptr;   // recorded after the last build's kernels (on the stream it ran on)
  std::vector<hipEvent_t> events;  // per-stage timing: ev_sets rings of NUM_EVENTS (rf_amd_batch_set_timing)
  uint32_t ev_sets = 0, ev_set = 0;  // each build starts the next set; probes record into the current one
  uint32_t ev_mask = EV_MASK_ALL;     // EV_MASK_PROBE: the probe's two events only
  ~rf_amd_batch() {
    if (built_ev) (void)hipEventDestroy(built_ev);
    for (auto ev : events) (void)hipEventDestroy(ev);
  }
  std::vector<DevBuf*> bufs() {
    return {&d_runs, &d_wave_tab, &d_plans, &d_outs, &d_ent, &d_part, &d_sorted, &d_cb_count, &d_cb_start, &d_cb_cursor,
            &d_cb_filter, &d_overflow, &d_idx_cnt, &d_idx_start, &d_slots, &d_page_first, &d_pg_filter,
            &d_pages, &d_tile_filter, &d_tile_start, &d_old_tile_filter, &d_old_tile_start, &d_old_cnt,
            &d_old_pos, &d_first_old, &d_has_old, &d_pplans, &d_lines, &d_idx_filter, &d_spill,
            &d_old_idx_filter, &d_old32, &d_old_tot, &d_ob_lo, &d_ob_n, &d_pg_noline, &d_pre, &d_cb_out};
  }
};

extern "C" const char* rf_amd_last_error(void) { return g_err.c_str(); }

// ---- engines alive at process exit ---------------------------------------------------------
// The compiler-generated constructor of this library registers its kernels with HIP when the
// library loads and registers, with atexit, the destructor that unregisters them again. An
// engine still alive at exit then has a lookup-server wave that may be running, pinned rings
// the GPU writes, host registrations and streams -- and the process's other threads (a
// drop-in's completion threads) may still be inside HIP calls -- while HIP tears the code
// objects down (a free() of an invalid pointer in __hipUnregisterFatBinary at the
// exit of the two-stack latency tool). Every engine alive at exit is therefore destroyed by a
// handler registered at the first engine creation, i.e. after the library's own destructor,
// so it runs before it (atexit order): server waves stopped, streams drained, pinned memory
// freed, registrations dropped. A drop-in that owns threads stops them in its own handler,
// registered after its engine's creation, so that one runs first (shim/routing_filter_amd.c).
static std::mutex g_live_mu;
static std::vector<rf_amd_engine*>* g_live = nullptr;  // never destroyed: read by the exit handler
static bool engine_quiesce(rf_amd_engine* e, int budget_ms);
static void engine_destroy_now(rf_amd_engine* e, bool device_sync);
static void engines_at_exit() {
  std::vector<rf_amd_engine*> v;
  {
    std::lock_guard<std::mutex> g(g_live_mu);
    if (g_live) v.swap(*g_live);
  }
  for (rf_amd_engine* e : v) {
    // a stream that does not drain in time (a hung kernel) leaves the engine as it is: exit
    // must not wait forever
    if (engine_quiesce(e, 2000)) engine_destroy_now(e, false);
  }
}

extern "C" int rf_amd_engine_create(int device, rf_amd_engine** out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(RF_AMD_ENODEV, "no HIP device: the routing-filter engine has no CPU fallback");
  if (device < 0 || device >= n) return fail(RF_AMD_EINVAL, "bad device ordinal");
  HIPCHK(hipSetDevice(device));
  auto* e = new rf_amd_engine();
  static std::atomic<uint64_t> next_uid{1};
  e->uid = next_uid.fetch_add(1);
  e->device = device;
  {
    // default: a quarter of the memory free at engine creation (~62 GB on an idle MI355X);
    // other allocators of the process can reclaim it with rf_amd_engine_pool_trim. The
    // compaction chain of 64 x 8M-fingerprint filters keeps 7.4 GB pooled beside the ~10 GB
    // its last round parks; a cap below that (round 5 had 16 GiB) makes every chain free and
    // re-allocate blocks of up to 2.7 GB, and hipFree of those costs ~28 ms per GB once the
    // driver clears released memory (profiles/r06_pool_churn.txt)
    const char* lim = getenv("RF_AMD_POOL_MIB");
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    const size_t dflt = free_b / 4;
    e->pool.limit = lim ? (size_t)atoll(lim) << 20 : dflt;
  }
  // a BLOCKING stream: ordered with the legacy null stream that torch and most callers use
  if (hipStreamCreateWithFlags(&e->stream, hipStreamDefault) != hipSuccess) {
    delete e;
    return fail(RF_AMD_EINVAL, "hipStreamCreate failed");
  }
  {
    static std::once_flag at_exit_once;
    std::call_once(at_exit_once, [] { (void)atexit(engines_at_exit); });
    std::lock_guard<std::mutex> g(g_live_mu);
    if (!g_live) g_live = new std::vector<rf_amd_engine*>();
    g_live->push_back(e);
  }
  *out = e;
  return 0;
}

static void srv_stop(rf_amd_engine* e);
extern "C" void rf_amd_engine_destroy(rf_amd_engine* e) {
  if (!e) return;
  {
    std::lock_guard<std::mutex> g(g_live_mu);
    if (g_live) g_live->erase(std::remove(g_live->begin(), g_live->end(), e), g_live->end());
  }
  engine_destroy_now(e, true);
}

// device_sync false: the engine's own streams are known drained (engines_at_exit)
static void engine_destroy_now(rf_amd_engine* e, bool device_sync) {
  (void)hipSetDevice(e->device);
  srv_stop(e);
  if (device_sync) (void)hipDeviceSynchronize();
  (void)hipStreamDestroy(e->stream);
  for (ProbeSlot* s : e->slots_all) {
    if (s->st) (void)hipStreamDestroy(s->st);
    if (s->h) (void)hipHostFree(s->h);
    if (s->d) (void)hipFree(s->d);
    if (s->flag) (void)hipHostFree(s->flag);
    if (s->d_counter) (void)hipFree(s->d_counter);
    delete s;
  }
  e->pool.drain();
  for (hipEvent_t ev : e->fence_free) (void)hipEventDestroy(ev);
  for (const auto& r : e->regs) (void)hipHostUnregister((void*)r.h);
  if (e->stage.h) (void)hipHostFree(e->stage.h);
  if (e->stage.d) (void)hipFree(e->stage.d);
  delete e;
}

static int check_cfg(const rf_amd_config* cfg) {
  if (!cfg) return fail(RF_AMD_EINVAL, "null config");
  if (cfg->page_size != MAX_PAGE || cfg->pages_per_extent != 32)
    return fail(RF_AMD_EINVAL, "engine supports 4 KiB pages in 32-page extents");
  if (cfg->fingerprint_size == 0 || cfg->fingerprint_size > 32 || cfg->log_index_size > MAX_LIS ||
      cfg->log_index_size < 3)
    return fail(RF_AMD_EINVAL, "unsupported fingerprint_size / log_index_size");
  return 0;
}

static uint32_t vsize_of(uint32_t value) { return value == 0 ? 0 : 32 - __builtin_clz(value); }

// Probe-line group size (k_plines): the largest G = 2^g <= min(IS, 64) whose 64-byte line
// (128 encoding bits for n + G, 384 remainder bits for n * rvs) holds mean + SIGMA sd + 2
// entries, n ~ Poisson(lam*G) with lam = fingerprints per bucket (< 2 by the choice of
// log_num_buckets). Larger G = smaller line table but more overflowed lines (those probes
// walk the image). SIGMA: RF_AMD_LINE_SIGMA (tuning knob), default 3.5 (lam is an upper
// bound; table size measured not to matter for the probe, overflow rate does).
// Returns g + 1, or 0 = no lines (rvs > 32: probes walk the image).
// K6 cuts a filter's probe lines from its LDS page images when the per-page group table
// fits: each block needs IS/G + 1 entries. Returns 0: never (k_plines cuts every line),
// 1: always (even a page of the smallest blocks fits), 2: page by page -- K6 flags a page
// whose blocks do not fit and k_plines cuts those pages' lines.
static int lines_in_assembly(uint32_t lis, uint32_t lg_line, uint32_t page_size) {
  const uint32_t IS = 1u << lis, L = IS >> (lg_line - 1);
  const uint32_t min_block = 2 + (IS - 1) / 8 + 4 + 3;
  const uint32_t maxb = page_size / min_block + 1;
  if (maxb > ASM_MAXB_HOST || L + 1 > ASM_GT_HOST) return 0;
  return (uint64_t)maxb * (L + 1) <= ASM_GT_HOST ? 1 : 2;
}

static double line_sigma() {
  const char* e = getenv("RF_AMD_LINE_SIGMA");
  const double v = e ? atof(e) : 0.0;
  return v > 0.0 ? v : 3.5;
}
static uint32_t line_log_group(uint32_t lis, uint32_t rvs, double lam) {
  if (rvs > 32) return 0;
  const double sg = line_sigma();
  for (int g = (int)(lis < 6 ? lis : 6); g >= 0; g--) {
    const double G = (double)(1u << g), mean = lam * G;
    const double cap = rvs ? std::min(128.0 - G, 384.0 / rvs) : 128.0 - G;
    if (mean + sg * sqrt(mean) + 2.0 <= cap) return (uint32_t)g + 1;
  }
  return 0;
}

extern "C" int rf_amd_batch_create(rf_amd_engine* e, const rf_amd_config* cfg, uint32_t num_filters,
                                   const uint32_t* num_new, const uint16_t* value,
                                   rf_amd_batch* const* old_batch, const uint32_t* old_index,
                                   rf_amd_batch** out) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (int rc = check_cfg(cfg)) return rc;
  if (num_filters == 0 || !num_new || !out) return fail(RF_AMD_EINVAL, "empty batch");
  HIPCHK(hipSetDevice(e->device));
  auto* b = new rf_amd_batch();
  b->eng = e;
  b->cfg = *cfg;
  b->F = num_filters;
  b->plans.resize(num_filters);
  b->pre.assign((size_t)rf_amd_batch::NUM_PRE * (num_filters + 1), 0u);
  const uint32_t lis = cfg->log_index_size, fps = cfg->fingerprint_size, P = cfg->page_size;
  const uint32_t IS = 1u << lis;
  uint64_t e_first = 0, key_first = 0;
  uint32_t cb_base = 0, idx_base = 0, page_base = 0, pf_base = 0;
  uint64_t line_base = 0;
  std::vector<std::pair<const rf_amd_batch*, const FilterPlan*>> olds(num_filters, {nullptr, nullptr});
  for (uint32_t f = 0; f < num_filters; f++) {
    FilterPlan& p = b->plans[f];
    memset(&p, 0, sizeof(p));
    const rf_amd_batch* ob = (old_batch && old_batch[f]) ? old_batch[f] : nullptr;
    const FilterPlan* op = nullptr;
    if (ob) {
      const uint32_t oi = old_index ? old_index[f] : 0;
      if (oi >= ob->F || !ob->built || ob->eng->device != e->device) {
        delete b;
        return fail(RF_AMD_EINVAL, "bad old filter reference");
      }
      op = &ob->plans[oi];
      b->wide = true;
    }
    const uint32_t v = value ? value[f] : 0;
    p.num_new = num_new[f];
    p.old_region = op ? op->num_fp : 0;
    const uint64_t nfp = (uint64_t)p.num_new + p.old_region;
    if (nfp > rf_amd_max_fingerprints(cfg)) {  // checked before the u32 descriptor field can wrap
      delete b;
      return fail(RF_AMD_EINVAL, "num_fingerprints over routing_filter_max_fingerprints (reference: UB)");
    }
    p.num_fp = (uint32_t)nfp;
    if (p.num_fp == 0) {
      delete b;
      return fail(RF_AMD_EINVAL, "routing_filter_add with zero fingerprints (reference: UB)");
    }
    uint32_t lnb = 31 - __builtin_clz(p.num_fp);
    if (lnb < lis) lnb = lis;
    p.vs = vsize_of(v);
    if (lnb > fps || (1u << (lnb - lis)) > MAX_INDICES || fps + p.vs > 32 || (op && p.vs < op->vs)) {
      delete b;
      return fail(RF_AMD_EINVAL, "filter geometry out of range (over routing_filter_max_fingerprints, "
                                 "fp_size + value_size > 32, or value narrower than old filter)");
    }
    p.lnb = lnb;
    p.value = v;
    p.rem = fps - lnb;
    p.rvs = p.rem + p.vs;
    p.num_indices = 1u << (lnb - lis);
    int cb = (int)lnb - (int)CB_LOG_MEAN;
    if (cb < 0) cb = 0;
    if (cb > (int)(lnb - lis)) cb = (int)(lnb - lis);
    // load factor ~1 (nfp just over a power of two: C3/C4's 2^20 keys) leaves coarse buckets
    // of 2^12 buckets half full (~4K of SORT_CAP entries), and K4's cost is mostly per
    // workgroup: use coarse buckets of 2^13 buckets (~8K entries, still >= 9 sd under
    // SORT_CAP) with K4 bins of two buckets each (at most MAX_BINS bins, MAX_IPC indices)
    p.binsh = 0;
    if (cb >= 1 && lnb - cb == CB_LOG_MEAN && lis + 9 >= CB_LOG_MEAN + 1 /* ipc <= MAX_IPC */ &&
        nfp * 1000 <= (1026ull << lnb)) {
      cb -= 1;
      p.binsh = 1;
    }
    p.cbits = (uint32_t)cb;
    p.bbits = lnb - p.cbits;
    p.e_first = e_first;
    p.key_first = key_first;
    p.cb_base = cb_base;
    p.idx_base = idx_base;
    // page bound: sum of block sizes <= NI*(12 + IS/8) + E*(1+rvs)/8; next-fit <= 2x + 1
    const uint64_t bound = (uint64_t)p.num_indices * (12 + IS / 8) + (nfp * (1 + p.rvs) + 7) / 8;
    uint64_t cap = 2 * ((bound + P - 1) / P) + 2;
    if (cap > p.num_indices) cap = p.num_indices;
    p.page_cap = (uint32_t)cap;
    p.page_base = page_base;
    p.pf_base = pf_base;
    p.lg_line = line_log_group(lis, p.rvs, (double)nfp / (double)(1ull << lnb));
    p.line_base = (uint32_t)line_base;
    const int la = p.lg_line ? lines_in_assembly(lis, p.lg_line, P) : 0;
    p.lines_asm = la != 0;
    p.lines_flag = la == 2;
    if (p.lg_line && la != 1) b->plines_needed = true;
    if (p.lg_line) {
      line_base += (uint64_t)p.num_indices << (lis - (p.lg_line - 1));
      b->line_lmax = std::max(b->line_lmax, IS >> (p.lg_line - 1));
    }
    if (op) {
      p.old_num_indices = op->num_indices;
      p.old_vs = op->vs;
      p.old_rvs = op->rvs;
      p.npo = p.num_indices / op->num_indices;
      p.old_pages = ob->d_pages.as<uint8_t>() + (uint64_t)op->page_base * P;
      p.old_slots = ob->d_slots.as<uint64_t>() + op->idx_base;
      olds[f] = {ob, op};
    }
    {
      auto pre = [&](int k, uint32_t count) { b->pre_of(k)[f + 1] = b->pre_of(k)[f] + count; };
      pre(rf_amd_batch::PRE_TILE, (p.num_new + TILE_KEYS - 1) / TILE_KEYS);
      pre(rf_amd_batch::PRE_OTILE, (p.old_region + TILE_KEYS - 1) / TILE_KEYS);
      pre(rf_amd_batch::PRE_CB, 1u << p.cbits);
      pre(rf_amd_batch::PRE_PG, p.page_cap);
      pre(rf_amd_batch::PRE_IDX, p.num_indices);
    }
    e_first += nfp;
    key_first += p.num_new;
    cb_base += 1u << p.cbits;
    idx_base += p.num_indices;
    page_base += p.page_cap;
    pf_base += p.page_cap + 1;
  }
  if (b->wide) {
    // 32-bit entries when (e << 1) | flag fits: fp_size + value_size <= 31 in every filter
    b->flag32 = getenv("RF_AMD_WIDE64") == nullptr;
    for (const auto& p : b->plans) b->flag32 = b->flag32 && fps + p.vs <= 31;
  }
  if (!b->wide || b->flag32) {
    // fresh and 32-bit incremental builds: the fused kernel partitions the new keys straight
    // into SORT_CAP slots per coarse bucket (k_hash_scatter), so each filter's entry region is
    // its buckets' regions (>= its num_fingerprints: incremental builds' sorted entries, laid
    // out by the scan of new + old counts, fit in it too)
    e_first = 0;
    for (auto& p : b->plans) {
      p.e_first = e_first;
      e_first += (uint64_t)CB_REGION << p.cbits;
    }
  }
  if (b->wide) {
    // old filters: read in place from their batch's sorted entries when the geometry is the
    // same (32-bit pipeline; the old batch built here, not imported), else decoded from the
    // image -- only those join the batch's old-index list and old32
    const bool direct_ok = b->flag32 && getenv("RF_AMD_OLD_DECODE") == nullptr;
    for (uint32_t f = 0; f < num_filters; f++) {
      const rf_amd_batch* ob = olds[f].first;
      const FilterPlan* op = olds[f].second;
      if (!op) continue;
      FilterPlan& p = b->plans[f];
      // in place also across a geometry change (lnb grew: rounds 2, 3 and 5 of the compaction
      // chain), as long as each new coarse bucket lies inside one old one (cbits did not shrink)
      // (RF_AMD_OLD_RESPLIT_OFF: decode those, for A/B)
      const bool same_cfg = direct_ok && ob->has_entries && ob->cfg.fingerprint_size == fps &&
                            ob->cfg.log_index_size == lis;
      const bool same_geo = op->lnb == p.lnb && op->cbits == p.cbits;
      const bool resplit = p.cbits >= op->cbits && p.lnb >= op->lnb && getenv("RF_AMD_OLD_RESPLIT_OFF") == nullptr;
      if (same_cfg && (same_geo || resplit)) {
        const uint32_t* es = ob->wide ? ob->d_sorted.as<uint32_t>() : ob->d_part.as<uint32_t>();
        p.old_direct = 1;
        p.old_cbits = op->cbits;
        p.old_bbits = op->bbits;
        p.old_entries = es + op->e_first;
        p.old_idx_start = ob->d_idx_start.as<uint32_t>() + op->idx_base;
        p.old_idx_cnt = ob->d_idx_cnt.as<uint32_t>() + op->idx_base;
        continue;
      }
      p.old_idx_base = b->num_old_idx;
      p.old_first = b->old_total;
      b->old_total += p.old_region;
      b->num_old_idx += op->num_indices;
    }
    // decoded old indices per filter (0 for filters without an old filter or read in place)
    uint32_t* po = b->pre_of(rf_amd_batch::PRE_OIDX);
    for (uint32_t f = 0; f < num_filters; f++) {
      const FilterPlan& p = b->plans[f];
      po[f + 1] = po[f] + ((olds[f].second && !p.old_direct) ? p.old_num_indices : 0u);
    }
  }
  b->num_tiles = b->pre_of(rf_amd_batch::PRE_TILE)[num_filters];
  b->num_old_tiles = b->pre_of(rf_amd_batch::PRE_OTILE)[num_filters];
  b->E = e_first;
  b->keys_total = key_first;
  b->CB = cb_base;
  b->I = idx_base;
  b->PS = page_base;
  b->PF = pf_base;
  if (line_base > 0xffffffffull) {
    delete b;
    return fail(RF_AMD_EINVAL, "batch too large (probe lines > 2^32)");
  }
  b->NL = line_base;
  const size_t esz = (b->wide && !b->flag32) ? 8 : 4;
  int rc = 0;
  DevPool* pool = &e->pool;
  const uint64_t ta0 = pool_trace_ns();
  rc |= b->d_plans.alloc(sizeof(FilterPlan) * num_filters, pool);
  rc |= b->d_pplans.alloc(16ull * num_filters, pool);
  rc |= b->d_outs.alloc(sizeof(FilterOut) * num_filters, pool);
  rc |= b->d_ent.alloc(esz * b->E + 64, pool);
  rc |= b->d_part.alloc(esz * b->E + 64, pool);
  if (b->wide) rc |= b->d_sorted.alloc(4 * b->E + 64, pool);
  if (b->flag32) rc |= b->d_cb_out.alloc(4 * b->CB, pool);
  rc |= b->d_cb_count.alloc(4 * b->CB, pool);
  rc |= b->d_cb_start.alloc(4 * b->CB, pool);
  rc |= b->d_cb_cursor.alloc(4 * b->CB, pool);
  rc |= b->d_cb_filter.alloc(4 * b->CB, pool);
  rc |= b->d_overflow.alloc(4 * (b->CB + 1), pool);
  rc |= b->d_spill.alloc(4, pool);
  rc |= b->d_idx_cnt.alloc(4 * b->I, pool);
  rc |= b->d_idx_start.alloc(4 * b->I, pool);
  rc |= b->d_slots.alloc(8 * b->I, pool);
  rc |= b->d_lines.alloc(64ull * b->NL + 64, pool);
  rc |= b->d_idx_filter.alloc(4ull * b->I, pool);
  rc |= b->d_page_first.alloc(4 * b->PF, pool);
  rc |= b->d_pg_filter.alloc(4 * b->PS, pool);
  rc |= b->d_pg_noline.alloc(4 * b->PS + 4, pool);
  rc |= b->d_pages.alloc((size_t)b->PS * P + 256, pool);
  rc |= b->d_tile_filter.alloc(4ull * b->num_tiles, pool);
  rc |= b->d_tile_start.alloc(4ull * b->num_tiles, pool);
  rc |= b->d_old_tile_filter.alloc(4ull * b->num_old_tiles, pool);
  rc |= b->d_old_tile_start.alloc(4ull * b->num_old_tiles, pool);
  rc |= b->d_pre.alloc(4 * b->pre.size(), pool);
  if (b->wide) {
    rc |= b->d_old_cnt.alloc(4ull * b->num_old_idx, pool);
    rc |= b->d_old_pos.alloc(4ull * b->num_old_idx, pool);
    rc |= b->d_old_idx_filter.alloc(4ull * b->num_old_idx, pool);
    rc |= b->d_first_old.alloc(4 * b->I, pool);
    rc |= b->d_has_old.alloc(4 * b->I, pool);
    if (b->flag32) {
      rc |= b->d_old32.alloc(4 * b->old_total + 64, pool);
      rc |= b->d_old_tot.alloc(4 * b->F, pool);
      rc |= b->d_ob_lo.alloc(4 * b->CB, pool);
      rc |= b->d_ob_n.alloc(4 * b->CB, pool);
    }
  }
  pool_trace("create allocs", 0, ta0);
  if (rc) {
    delete b;
    return fail(RF_AMD_ENOMEM, "device allocation failed");
  }
  hipStream_t st = e->stream;
  // Page bytes the reference never writes are zero on a fresh cache page (SURVEY finding 4).
  // K6 writes every byte of every page it assembles (block bytes and the zero tail), and no
  // reader looks past a filter's num_pages, so the reserved pages a build does not use are
  // not cleared (page_cap reserves ~2x the pages: clearing them cost a compaction round
  // ~0.3 ms); only the tail pad that windowed reads of the last page may touch is zeroed.
  HIPCHK(hipMemsetAsync(b->d_pages.as<uint8_t>() + (size_t)b->PS * P, 0, 256, st));
  if (const char* pz = getenv("RF_AMD_POISON")) {
    // test hook: fill every work buffer -- the page images included -- with a pattern, so
    // that a kernel reading memory it did not write in this build, or leaving page bytes
    // unwritten, cannot pass the parity tests
    const int v = atoi(pz) & 0xff;
    for (DevBuf* d : {&b->d_ent, &b->d_part, &b->d_sorted, &b->d_cb_start, &b->d_idx_cnt, &b->d_idx_start,
                      &b->d_slots, &b->d_lines, &b->d_page_first, &b->d_pages, &b->d_first_old, &b->d_has_old,
                      &b->d_old32, &b->d_old_tot, &b->d_ob_lo, &b->d_ob_n})
      if (d->p) HIPCHK(hipMemsetAsync(d->p, v, d->n, st));
  }
#define UP(buf, vec) \
  if (!(vec).empty()) HIPCHK(hipMemcpyAsync(buf.p, (vec).data(), sizeof((vec)[0]) * (vec).size(), hipMemcpyHostToDevice, st))
  UP(b->d_plans, b->plans);
  std::vector<uint4> pp(num_filters);
  for (uint32_t f = 0; f < num_filters; f++) {
    const FilterPlan& q = b->plans[f];
    pp[f] = make_uint4(q.vs | (q.rem << 8) | (q.rvs << 16) | (q.lg_line << 24), q.line_base, q.idx_base, 0);
  }
  UP(b->d_pplans, pp);
  UP(b->d_pre, b->pre);
#undef UP
  {
    // element -> filter maps (and tile -> first key) from the prefix arrays, on the device
    const uint32_t F1 = num_filters + 1;
    const uint32_t* dp = b->d_pre.as<uint32_t>();
    struct M { int k; DevBuf* fof; DevBuf* start; };
    const M maps[] = {{rf_amd_batch::PRE_TILE, &b->d_tile_filter, &b->d_tile_start},
                      {rf_amd_batch::PRE_OTILE, &b->d_old_tile_filter, &b->d_old_tile_start},
                      {rf_amd_batch::PRE_CB, &b->d_cb_filter, nullptr},
                      {rf_amd_batch::PRE_PG, &b->d_pg_filter, nullptr},
                      {rf_amd_batch::PRE_IDX, &b->d_idx_filter, nullptr},
                      {rf_amd_batch::PRE_OIDX, &b->d_old_idx_filter, nullptr}};
    for (const M& m : maps) {
      const uint32_t n = b->pre_of(m.k)[num_filters];
      if (n == 0 || !m.fof->p) continue;
      if (rf_launch_seg_fill(st, dp + (size_t)m.k * F1, num_filters, n, m.fof->as<uint32_t>(),
                             m.start ? m.start->as<uint32_t>() : nullptr, TILE_KEYS)) {
        delete b;
        return fail(RF_AMD_EINVAL, "map fill launch failed");
      }
    }
  }
  const uint64_t ts0 = pool_trace_ns();
  HIPCHK(hipStreamSynchronize(st));
  pool_trace("create sync", 0, ts0);
  *out = b;
  return 0;
}

extern "C" void rf_amd_batch_destroy(rf_amd_batch* b) {
  if (!b) return;
  (void)hipSetDevice(b->eng->device);
  // work on a caller's stream may still read the batch: its blocks go back to the pool only
  // once the device is idle (what hipFree would have waited for)
  (void)hipDeviceSynchronize();
  delete b;
}

// stream-ordered destroy: every use of the batch is ordered before the current end of
// `stream`; its device blocks are parked behind an event recorded there and reused (or
// freed) once it completes. Returns without waiting.
extern "C" int rf_amd_batch_destroy_on(rf_amd_batch* b, void* stream) {
  if (!b) return 0;
  HIPCHK(hipSetDevice(b->eng->device));
  hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
  DevPool::Parked k{};
  hipError_t he = hipEventCreateWithFlags(&k.ev, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventRecord(k.ev, st);
  if (he != hipSuccess) {  // fall back to the synchronising destroy
    if (k.ev) (void)hipEventDestroy(k.ev);
    rf_amd_batch_destroy(b);
    return 0;
  }
  for (DevBuf* d : b->bufs()) {
    if (!d->p) continue;
    k.blocks.emplace_back(d->p, d->pool == &b->eng->pool ? d->n : 0);
    d->p = nullptr;
  }
  b->eng->pool.park(std::move(k));
  delete b;
  return 0;
}

// Drops a built batch's work buffers (entries, maps, counters), keeping what lookups, image
// reads, estimates and use as an old filter by image decode need: plans, outs, pages, slots,
// probe lines, index map, probe runs. Stream-ordered like rf_amd_batch_destroy_on. A trimmed
// batch no longer offers its entries in place to incremental adds (they decode its image).
extern "C" int rf_amd_batch_trim(rf_amd_batch* b, void* stream) {
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "trim of an unbuilt batch");
  HIPCHK(hipSetDevice(b->eng->device));
  DevBuf* keep[] = {&b->d_plans, &b->d_pplans, &b->d_outs, &b->d_pages, &b->d_slots, &b->d_lines,
                    &b->d_idx_filter, &b->d_runs, &b->d_wave_tab};
  DevPool::Parked k{};
  for (DevBuf* d : b->bufs()) {
    if (!d->p || std::find(std::begin(keep), std::end(keep), d) != std::end(keep)) continue;
    k.blocks.emplace_back(d->p, d->pool == &b->eng->pool ? d->n : 0);
    d->p = nullptr;
    d->n = 0;
  }
  b->has_entries = false;
  if (k.blocks.empty()) return 0;
  hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
  hipError_t he = hipEventCreateWithFlags(&k.ev, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventRecord(k.ev, st);
  if (he != hipSuccess) {  // cannot order the release: wait, then release
    if (k.ev) (void)hipEventDestroy(k.ev);
    (void)hipStreamSynchronize(st);
    std::lock_guard<std::mutex> g(b->eng->pool.mu);
    for (auto& blk : k.blocks) b->eng->pool.give_locked(blk.first, blk.second);
    return 0;
  }
  b->eng->pool.park(std::move(k));
  return 0;
}

// device bytes a batch holds (its buffers, pooled sizes)
extern "C" uint64_t rf_amd_batch_device_bytes(const rf_amd_batch* b) {
  if (!b) return 0;
  uint64_t s = 0;
  for (DevBuf* d : const_cast<rf_amd_batch*>(b)->bufs())
    if (d->p) s += d->n;
  return s;
}

// the engine's own stream (builds from host buffers, imports run there)
extern "C" void* rf_amd_engine_stream(rf_amd_engine* e) { return e ? (void*)e->stream : nullptr; }
extern "C" int rf_amd_engine_sync(rf_amd_engine* e) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

extern "C" int rf_amd_host_alloc(rf_amd_engine* e, uint64_t bytes, void** out) {
  if (!e || !out) return fail(RF_AMD_EINVAL, "null argument");
  HIPCHK(hipSetDevice(e->device));
  *out = nullptr;
  if (hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) {
    *out = nullptr;
    return fail(RF_AMD_ENOMEM, "hipHostMalloc failed");
  }
  return 0;
}

extern "C" void rf_amd_host_free(rf_amd_engine* e, void* p) {
  (void)e;
  if (p) (void)hipHostFree(p);
}

// a fence is an event recorded on the engine stream; its handle travels as a uint64
extern "C" int rf_amd_engine_fence(rf_amd_engine* e, uint64_t* fence) {
  if (!e || !fence) return fail(RF_AMD_EINVAL, "null argument");
  HIPCHK(hipSetDevice(e->device));
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> g(e->fence_mu);
    if (!e->fence_free.empty()) {
      ev = e->fence_free.back();
      e->fence_free.pop_back();
    }
  }
  if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ev, e->stream));
  *fence = (uint64_t)(uintptr_t)ev;
  return 0;
}

extern "C" int rf_amd_engine_fence_wait(rf_amd_engine* e, uint64_t fence) {
  if (!e || !fence) return fail(RF_AMD_EINVAL, "null argument");
  hipEvent_t ev = (hipEvent_t)(uintptr_t)fence;
  const hipError_t r = hipEventSynchronize(ev);
  {
    std::lock_guard<std::mutex> g(e->fence_mu);
    e->fence_free.push_back(ev);
  }
  if (r != hipSuccess) return fail(RF_AMD_EINVAL, std::string("fence: ") + hipGetErrorString(r));
  return 0;
}

static int batch_errors(rf_amd_batch* b);

extern "C" int rf_amd_host_register(rf_amd_engine* e, void* p, uint64_t bytes) {
  if (!e || !p || !bytes) return fail(RF_AMD_EINVAL, "null argument");
  HIPCHK(hipSetDevice(e->device));
  std::lock_guard<std::mutex> g(e->reg_mu);
  const uintptr_t h = (uintptr_t)p;
  for (const auto& r : e->regs)
    if (h < r.h + r.bytes && r.h < h + bytes) return fail(RF_AMD_EINVAL, "range overlaps a registered one");
  if (hipHostRegister(p, bytes, hipHostRegisterMapped) != hipSuccess) {
    (void)hipGetLastError();
    return fail(RF_AMD_ENOMEM, "hipHostRegister failed");
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
    (void)hipHostUnregister(p);
    return fail(RF_AMD_EINVAL, "no device address for the registered range");
  }
  e->regs.push_back({h, bytes, (uintptr_t)d});
  return 0;
}

extern "C" int rf_amd_host_unregister(rf_amd_engine* e, void* p) {
  if (!e || !p) return fail(RF_AMD_EINVAL, "null argument");
  std::lock_guard<std::mutex> g(e->reg_mu);
  for (size_t i = 0; i < e->regs.size(); i++) {
    if (e->regs[i].h == (uintptr_t)p) {
      HIPCHK(hipSetDevice(e->device));
      (void)hipHostUnregister(p);
      e->regs.erase(e->regs.begin() + i);
      return 0;
    }
  }
  return fail(RF_AMD_EINVAL, "not a registered range");
}

// Filter f's image pages [first_page, first_page + count) (and, with_index, its index slots)
// written straight into host pages (D2H by the kernel's own stores, no staging copy): table (rf_amd_host_alloc'd, 2 * num_pages + ceil(num_indices /
// addrs_per_page) words) = the destination of each image page (host addresses inside a
// registered range), each page's disk address, and each index page's destination. The
// destinations are checked against the registered ranges and replaced in place by their
// device addresses; index slot i becomes disk_addr[slot / page_size] + slot % page_size,
// written at word i % addrs_per_page of index page i / addrs_per_page (src/routing_filter.c
// :612-620). Stream-ordered; the caller waits (rf_amd_engine_fence) before using the pages.
extern "C" int rf_amd_batch_place_image(rf_amd_batch* b, uint32_t f, uint64_t* table, uint32_t num_pages,
                                        uint32_t first_page, uint32_t count, int with_index,
                                        uint32_t addrs_per_page, void* stream) {
  if (!b || f >= b->F || !table || !addrs_per_page) return fail(RF_AMD_EINVAL, "bad argument");
  if (int rc = batch_errors(b)) return rc;
  if (b->err_host[f]) return fail(RF_AMD_EINVAL, "the filter's build failed");
  const FilterPlan& p = b->plans[f];
  const uint32_t P = b->cfg.page_size;
  if (num_pages > p.page_cap || first_page > num_pages || count > num_pages - first_page)
    return fail(RF_AMD_EINVAL, "pages outside the filter's reservation");
  const uint32_t nidx = with_index ? p.num_indices : 0u, nip = (nidx + addrs_per_page - 1) / addrs_per_page;
  if ((uint64_t)addrs_per_page * 8 > P) return fail(RF_AMD_EINVAL, "index page overflow");
  rf_amd_engine* e = b->eng;
  {
    std::lock_guard<std::mutex> g(e->reg_mu);
    size_t hint = 0;
    auto xlate = [&](uint64_t& w, uint64_t len) -> bool {
      const uintptr_t h = (uintptr_t)w;
      for (size_t k = 0; k < e->regs.size(); k++) {
        const auto& r = e->regs[(hint + k) % e->regs.size()];
        if (h >= r.h && h + len <= r.h + r.bytes) {
          hint = (hint + k) % e->regs.size();
          w = r.d + (h - r.h);
          return true;
        }
      }
      return false;
    };
    for (uint32_t k = first_page; k < first_page + count; k++)
      if (!xlate(table[k], P)) return fail(RF_AMD_EINVAL, "page destination outside the registered ranges");
    for (uint32_t k = 0; k < nip; k++)
      if (!xlate(table[2ull * num_pages + k], P)) return fail(RF_AMD_EINVAL, "index page outside the registered ranges");
  }
  void* dt = nullptr;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipHostGetDevicePointer(&dt, table, 0));
  hipStream_t st = stream ? (hipStream_t)stream : e->stream;
  const int rc = rf_launch_place(st, b->d_pages.as<uint8_t>() + (uint64_t)p.page_base * P,
                                 b->d_slots.as<uint64_t>() + p.idx_base, first_page, count, num_pages, nidx, P,
                                 (const uint64_t*)dt, addrs_per_page);
  if (rc) return fail(RF_AMD_EINVAL, std::string("place launch: ") + hipGetErrorString((hipError_t)rc));
  return 0;
}

extern "C" int rf_amd_engine_pool_stats(rf_amd_engine* e, uint64_t* pooled_bytes, uint64_t* hits, uint64_t* misses) {
  if (!e) return fail(RF_AMD_EINVAL, "null engine");
  std::lock_guard<std::mutex> g(e->pool.mu);
  if (pooled_bytes) *pooled_bytes = e->pool.pooled;
  if (hits) *hits = e->pool.hits;
  if (misses) *misses = e->pool.misses;
  return 0;
}

// hands pooled device blocks back to the device until at most keep_bytes stay pooled (blocks
// parked behind stream events are released once those complete)
extern "C" int rf_amd_engine_pool_trim(rf_amd_engine* e, uint64_t keep_bytes) {
  if (!e) return fail(RF_AMD_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->device));
  std::lock_guard<std::mutex> g(e->pool.mu);
  e->pool.reap_locked(false);
  for (auto it = e->pool.free_blocks.begin(); it != e->pool.free_blocks.end() && e->pool.pooled > keep_bytes;) {
    (void)hipFree(it->second);
    e->pool.pooled -= it->first;
    it = e->pool.free_blocks.erase(it);
  }
  return 0;
}

// the most device memory the pool keeps parked for reuse (RF_AMD_POOL_MIB at creation), trimmed
// to it now
extern "C" int rf_amd_engine_set_pool_limit(rf_amd_engine* e, uint64_t bytes) {
  if (!e) return fail(RF_AMD_EINVAL, "null engine");
  {
    std::lock_guard<std::mutex> g(e->pool.mu);
    e->pool.limit = bytes;
  }
  return rf_amd_engine_pool_trim(e, bytes);
}

extern "C" uint32_t rf_amd_batch_num_filters(const rf_amd_batch* b) { return b ? b->F : 0; }

static LaunchArgs make_args(rf_amd_batch* b, hipStream_t st) {
  LaunchArgs a;
  memset(&a, 0, sizeof(a));
  a.stream = st;
  a.wide = b->wide;
  a.plans = b->d_plans.as<FilterPlan>();
  a.pplans = b->d_pplans.as<uint4>();
  a.pplans_mut = b->d_pplans.as<uint4>();
  a.num_filters = b->F;
  a.tile_filter = b->d_tile_filter.as<uint32_t>();
  a.tile_start = b->d_tile_start.as<uint32_t>();
  a.num_tiles = b->num_tiles;
  a.old_tile_filter = b->d_old_tile_filter.as<uint32_t>();
  a.old_tile_start = b->d_old_tile_start.as<uint32_t>();
  a.num_old_tiles = b->num_old_tiles;
  a.old_idx_filter = b->d_old_idx_filter.as<uint32_t>();
  a.num_old_idx = b->num_old_idx;
  a.old_cnt = b->d_old_cnt.as<uint32_t>();
  a.old_pos = b->d_old_pos.as<uint32_t>();
  a.flag32 = b->flag32 ? 1u : 0u;
  a.old32 = b->d_old32.as<uint32_t>();
  a.old_tot = b->d_old_tot.as<uint32_t>();
  a.ob_lo = b->d_ob_lo.as<uint32_t>();
  a.ob_n = b->d_ob_n.as<uint32_t>();
  a.fp_size = b->cfg.fingerprint_size;
  a.seed = b->cfg.seed;
  a.lis = b->cfg.log_index_size;
  a.page_size = b->cfg.page_size;
  a.ent = b->d_ent.p;
  a.part = b->d_part.p;
  a.sorted32 = b->wide ? b->d_sorted.as<uint32_t>() : b->d_part.as<uint32_t>();
  a.cb_count = b->d_cb_count.as<uint32_t>();
  a.cb_start = b->d_cb_start.as<uint32_t>();
  a.cb_cursor = b->d_cb_cursor.as<uint32_t>();
  a.cb_filter = b->d_cb_filter.as<uint32_t>();
  a.num_cb = b->CB;
  a.overflow = b->d_overflow.as<uint32_t>();
  a.spill = b->d_spill.p ? b->d_spill.as<uint32_t>() : nullptr;
  a.cb_outs = b->d_cb_out.p ? b->d_cb_out.as<uint32_t>() : nullptr;
  a.idx_cnt = b->d_idx_cnt.as<uint32_t>();
  a.idx_start = b->d_idx_start.as<uint32_t>();
  a.first_old = b->d_first_old.as<uint32_t>();
  a.has_old = b->d_has_old.as<uint32_t>();
  a.slots = b->d_slots.as<uint64_t>();
  a.lines = b->d_lines.as<uint4>();
  a.line_lmax = b->line_lmax;
  a.plines_needed = b->plines_needed ? 1u : 0u;
  a.pg_noline = b->d_pg_noline.as<uint32_t>();
  a.idx_filter = b->d_idx_filter.as<uint32_t>();
  a.num_idx = b->I;
  a.page_first = b->d_page_first.as<uint32_t>();
  a.pg_filter = b->d_pg_filter.as<uint32_t>();
  a.num_page_slots = b->PS;
  a.pages = b->d_pages.as<uint8_t>();
  a.outs = b->d_outs.p ? b->d_outs.as<FilterOut>() : nullptr;
  a.events = b->events.empty() ? nullptr : reinterpret_cast<void**>(b->events.data() + (size_t)b->ev_set * NUM_EVENTS);
  a.ev_mask = b->ev_mask;
  return a;
}

static int do_probe(rf_amd_batch* b, int kind, const void* in0, const uint64_t* offs, uint32_t key_len,
                    const uint32_t* fid, uint64_t n, uint64_t* found, void* stream,
                    const uint64_t* d_runs = nullptr);

// The build's completion point: host reads of the batch (info, images) wait for this event
// and then copy on the engine stream -- never a device-wide synchronisation or a null-stream
// copy, which would also wait for the lookup server's wave
static int note_built(rf_amd_batch* b, hipStream_t st) {
  if (!b->built_ev) HIPCHK(hipEventCreateWithFlags(&b->built_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(b->built_ev, st));
  return 0;
}
static int wait_built(rf_amd_batch* b) {
  if (b->built_ev) HIPCHK(hipEventSynchronize(b->built_ev));
  return 0;
}

static int do_build(rf_amd_batch* b, int kind, const void* in0, const uint64_t* offs, uint32_t key_len,
                    void* stream) {
  if (!b) return fail(RF_AMD_EINVAL, "null batch");
  if (b->keys_total && !in0) return fail(RF_AMD_EINVAL, "null input");
  HIPCHK(hipSetDevice(b->eng->device));
  hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
  (void)hipGetLastError();  // launch checks below must see only their own errors
  if (b->ev_sets) b->ev_set = (b->ev_set + 1) % b->ev_sets;
  LaunchArgs a = make_args(b, st);
  a.kind = kind;
  a.in0 = in0;
  a.offs = offs;
  a.key_len = key_len;
  if (a.events && (a.ev_mask >> EV_B_START & 1u)) HIPCHK(hipEventRecord(((hipEvent_t*)a.events)[EV_B_START], st));
  if (rf_launch_build_init(st, b->d_cb_count.as<uint32_t>(), (b->wide && !b->flag32) ? nullptr : b->d_cb_cursor.as<uint32_t>(),
                           b->CB, b->d_outs.as<uint32_t>(), (uint32_t)(sizeof(FilterOut) / 4 * b->F),
                           b->d_overflow.as<uint32_t>(), (b->wide && !b->flag32) ? nullptr : b->d_spill.as<uint32_t>(),
                           b->d_pg_noline.as<uint32_t>()))
    return fail(RF_AMD_EINVAL, "init kernel launch failed");
  if (b->wide) {
    // every old filter of the batch decoded by one launch sequence (which also marks the
    // unused tail of each old region); the new regions are written whole by the hashing pass
    int rc = rf_launch_old_decode(&a);
    if (rc) return fail(RF_AMD_EINVAL, std::string("old decode launch: ") + hipGetErrorString((hipError_t)rc));
  }
  b->err_ready.store(false, std::memory_order_release);  // a rebuild: read the new bits back
  int rc = rf_launch_build(&a);
  // counted once every kernel of the build is queued: a lookup that finds the stream idle
  // after reading this count cannot miss a build it covers
  if (st == b->eng->stream) b->eng->builds_issued.fetch_add(1, std::memory_order_acq_rel);
  if (rc) return fail(RF_AMD_EINVAL, std::string("build launch: ") + hipGetErrorString((hipError_t)rc));
  if (getenv("RF_AMD_DIAG_OVERFLOW") && b->d_overflow.p) {  // diagnostics: coarse buckets handed back by K4/K4m
    uint32_t nov = 0;
    if (hipMemcpyAsync(&nov, b->d_overflow.p, 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
        hipStreamSynchronize(st) == hipSuccess)
      fprintf(stderr, "rf_amd: %u of %u coarse buckets handed back (K4b / list mode)\n", nov, b->CB);
  }
  if (int erc = note_built(b, st)) return erc;
  b->built = true;
  b->has_entries = true;
  return 0;
}

static int fixed_kind(const void* p, uint32_t key_len) {
  const uintptr_t u = (uintptr_t)p;
  if (key_len == 24 && (u & 7) == 0) return IN_KEYS24;
  if ((key_len & 3) == 0 && (u & 3) == 0) return IN_KEYS_W;
  return IN_KEYS_B;
}

extern "C" int rf_amd_batch_build_keys(rf_amd_batch* b, const void* d_keys, uint32_t key_len, void* stream) {
  if (key_len == 0) return fail(RF_AMD_EINVAL, "key_len 0");
  return do_build(b, fixed_kind(d_keys, key_len), d_keys, nullptr, key_len, stream);
}
extern "C" int rf_amd_batch_build_var_keys(rf_amd_batch* b, const uint8_t* d_bytes, const uint64_t* d_offsets,
                                           void* stream) {
  if (!d_offsets) return fail(RF_AMD_EINVAL, "null offsets");
  return do_build(b, IN_VAR, d_bytes, d_offsets, 0, stream);
}
extern "C" int rf_amd_batch_build_hashes(rf_amd_batch* b, const uint32_t* d_hashes, void* stream) {
  return do_build(b, IN_HASH, d_hashes, nullptr, 4, stream);
}

// the engine's host staging area, grown to `bytes`; the caller holds e->stage.mu
static int stage_reserve(rf_amd_engine* e, size_t bytes) {
  HostStage& s = e->stage;
  if (s.cap >= bytes) return 0;
  if (s.h) (void)hipHostFree(s.h);
  if (s.d) (void)hipFree(s.d);
  s.h = s.d = nullptr;
  s.cap = 0;
  const size_t c = std::max<size_t>(bytes, (size_t)1 << 20);
  if (hipHostMalloc(&s.h, c, hipHostMallocDefault) != hipSuccess) {
    s.h = nullptr;
    return fail(RF_AMD_ENOMEM, "pinned staging allocation failed");
  }
  if (hipMalloc(&s.d, c) != hipSuccess) {
    (void)hipHostFree(s.h);
    s.h = nullptr;
    return fail(RF_AMD_ENOMEM, "device staging allocation failed");
  }
  s.cap = c;
  return 0;
}

// Host-buffer forms for callers that hold no device memory (the routing_filter.h shim,
// shim/routing_filter_amd.c): inputs are staged through the engine's pinned buffer on the
// engine stream, and the call returns once the results are complete.
// Two-step form of rf_amd_batch_build_hashes_host for callers that fill the staging buffer
// themselves, e.g. from several threads at once (the shim's coalesced adds: each adding
// thread copies its own fingerprints): stage_begin takes the engine's pinned staging buffer,
// sized for the batch's keys_total hashes (filter f's at its run offset), and returns it;
// stage_build uploads it, builds, waits, and releases the buffer. Every stage_begin must be
// followed by one stage_build (or stage_abort) on the same batch.
extern "C" int rf_amd_batch_stage_begin(rf_amd_batch* b, uint32_t** h_stage) {
  if (!b || !h_stage) return fail(RF_AMD_EINVAL, "null batch / out-param");
  rf_amd_engine* e = b->eng;
  HIPCHK(hipSetDevice(e->device));
  e->stage.mu.lock();
  if (int rc = stage_reserve(e, 4ull * b->keys_total + 16)) {
    e->stage.mu.unlock();
    return rc;
  }
  *h_stage = static_cast<uint32_t*>(e->stage.h);
  return 0;
}

extern "C" int rf_amd_batch_stage_build(rf_amd_batch* b) {
  rf_amd_engine* e = b->eng;
  std::lock_guard<std::mutex> g(e->stage.mu, std::adopt_lock);  // taken by stage_begin
  const size_t bytes = 4ull * b->keys_total;
  if (bytes) HIPCHK(hipMemcpyAsync(e->stage.d, e->stage.h, bytes, hipMemcpyHostToDevice, e->stream));
  if (int rc = do_build(b, IN_HASH, e->stage.d, nullptr, 4, e->stream)) return rc;
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

extern "C" void rf_amd_batch_stage_abort(rf_amd_batch* b) {
  if (b) b->eng->stage.mu.unlock();
}

extern "C" int rf_amd_batch_build_hashes_host(rf_amd_batch* b, const uint32_t* h_hashes) {
  if (!b) return fail(RF_AMD_EINVAL, "null batch");
  if (b->keys_total && !h_hashes) return fail(RF_AMD_EINVAL, "null hashes");
  rf_amd_engine* e = b->eng;
  HIPCHK(hipSetDevice(e->device));
  std::lock_guard<std::mutex> g(e->stage.mu);
  const size_t bytes = 4ull * b->keys_total;
  if (int rc = stage_reserve(e, bytes + 16)) return rc;
  if (bytes) {
    memcpy(e->stage.h, h_hashes, bytes);
    HIPCHK(hipMemcpyAsync(e->stage.d, e->stage.h, bytes, hipMemcpyHostToDevice, e->stream));
  }
  if (int rc = do_build(b, IN_HASH, e->stage.d, nullptr, 4, e->stream)) return rc;
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

// ---- host-buffer lookups over the engine's lookup slots (ProbeSlot) -----------------------
extern "C" int rf_launch_probe_groups(void* stream, const uint32_t* in, const ProbeGroup* groups, uint32_t ng,
                                      uint64_t n, uint64_t* found, uint32_t* counter, uint32_t* done_flag,
                                      uint32_t seq);
extern "C" int rf_launch_probe_small(void* stream, const SmallProbe* a);

static ProbeSlot* slot_take(rf_amd_engine* e) {
  {
    std::lock_guard<std::mutex> g(e->slot_mu);
    if (!e->slots_free.empty()) {
      ProbeSlot* s = e->slots_free.back();
      e->slots_free.pop_back();
      return s;
    }
  }
  auto* s = new ProbeSlot();
  // non-blocking: a lookup does not wait for unrelated work on the legacy null stream
  bool ok = hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) == hipSuccess &&
            hipHostMalloc((void**)&s->flag, 64, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
            hipMalloc((void**)&s->d_counter, 64) == hipSuccess &&
            hipMemsetAsync(s->d_counter, 0, 64, s->st) == hipSuccess && hipStreamSynchronize(s->st) == hipSuccess;
  if (!ok) {
    if (s->st) (void)hipStreamDestroy(s->st);
    if (s->flag) (void)hipHostFree(s->flag);
    if (s->d_counter) (void)hipFree(s->d_counter);
    delete s;
    fail(RF_AMD_ENOMEM, "lookup slot allocation failed");
    return nullptr;
  }
  *s->flag = 0;
  std::lock_guard<std::mutex> g(e->slot_mu);
  e->slots_all.push_back(s);
  return s;
}

static void slot_give(rf_amd_engine* e, ProbeSlot* s) {
  std::lock_guard<std::mutex> g(e->slot_mu);
  e->slots_free.push_back(s);
}

static int slot_reserve(ProbeSlot* s, size_t hbytes, size_t dbytes) {
  if (s->hcap < hbytes) {
    if (s->h) (void)hipHostFree(s->h);
    s->h = nullptr;
    s->hcap = 0;
    const size_t c = std::max<size_t>(hbytes, (size_t)1 << 16);
    if (hipHostMalloc((void**)&s->h, c, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
      s->h = nullptr;
      return fail(RF_AMD_ENOMEM, "pinned lookup buffer allocation failed");
    }
    s->hcap = c;
  }
  if (dbytes && s->dcap < dbytes) {
    if (s->d) (void)hipFree(s->d);
    s->d = nullptr;
    s->dcap = 0;
    const size_t c = std::max<size_t>(dbytes, (size_t)1 << 20);
    if (hipMalloc((void**)&s->d, c) != hipSuccess) {
      s->d = nullptr;
      return fail(RF_AMD_ENOMEM, "device lookup buffer allocation failed");
    }
    s->dcap = c;
  }
  return 0;
}

// per-filter build error bits of a built batch, read back once (a batch is immutable once
// built; a filter whose build failed finds nothing, as k_probe does through pplans.w)
static int batch_errors(rf_amd_batch* b) {
  // concurrent lookups of one batch may both get here first (rf_amd.h: host lookups are
  // thread-safe): the read-back happens once, under the batch's lock, and err_host is
  // published (err_ready) only once filled
  if (b->err_ready.load(std::memory_order_acquire)) return 0;
  std::lock_guard<std::mutex> lk(b->err_mu);
  if (b->err_ready.load(std::memory_order_relaxed)) return 0;
  std::vector<FilterOut> o(b->F);
  HIPCHK(hipMemcpyAsync(o.data(), b->d_outs.p, sizeof(FilterOut) * b->F, hipMemcpyDeviceToHost, b->eng->stream));
  HIPCHK(hipStreamSynchronize(b->eng->stream));
  b->err_host.resize(b->F);
  for (uint32_t f = 0; f < b->F; f++) b->err_host[f] = o[f].error;
  b->err_ready.store(true, std::memory_order_release);
  return 0;
}

static ProbeGroup probe_group_of(const rf_amd_batch* b, uint32_t f) {
  const FilterPlan& p = b->plans[f];
  ProbeGroup g;
  g.x = p.vs | (p.rem << 8) | (p.rvs << 16) | (p.lg_line << 24);
  g.err = b->err_host[f];
  g.fpl = b->cfg.fingerprint_size | (b->cfg.log_index_size << 8);
  g.pad = 0;
  g.lines = b->d_lines.as<uint4>() + 4ull * p.line_base;
  g.pages = b->d_pages.as<uint8_t>() + (uint64_t)p.page_base * b->cfg.page_size;
  g.slots = b->d_slots.as<uint64_t>() + p.idx_base;
  return g;
}

// Probe modes of a round trip: inputs read by the kernel from pinned host memory (small
// calls: no copy command) or copied to the device with one H2D first; results always written
// by the kernel into pinned host memory; completion by polling the slot's flag word (or, with
// RF_AMD_PROBE_WAIT=sync, hipStreamSynchronize). RF_AMD_PROBE_MODE=mapped|copy forces a mode.
static int env_mode(const char* name, const char* a, const char* b) {
  const char* v = getenv(name);
  if (!v) return 0;
  return !strcmp(v, a) ? 1 : (!strcmp(v, b) ? 2 : 0);
}
// measured on MI355X (profiles/r03_probe_latency.txt): reading the inputs over PCIe from the
// kernel beats one H2D copy first up to at least 8,192 probes (17.7 vs 34.9 us per round trip)
static const uint64_t MAPPED_MAX_PROBES = 32768;

// The common body: n probes, probe i in group h_group[i] (NULL: group 0) of the ng-entry group
// table, results into h_found. Waits for any work still queued on the engine stream (builds
// issued there), then runs on a lookup slot of its own.
// waits for a slot's kernel to publish `seq` (or fails if the stream errored without it)
static int slot_wait(ProbeSlot* s, uint32_t seq, bool sync) {
  if (sync) {
    HIPCHK(hipStreamSynchronize(s->st));
    return 0;
  }
  for (uint32_t spin = 1;; spin++) {
    if (__atomic_load_n(s->flag, __ATOMIC_ACQUIRE) == seq) return 0;
    __builtin_ia32_pause();
    if ((spin & 4095) == 0) {  // a kernel that faulted never stores the flag
      const hipError_t q = hipStreamQuery(s->st);
      if (q == hipErrorNotReady) continue;
      if (q != hipSuccess) return fail(RF_AMD_EINVAL, std::string("probe kernel: ") + hipGetErrorString(q));
      if (__atomic_load_n(s->flag, __ATOMIC_ACQUIRE) != seq)
        return fail(RF_AMD_EINVAL, "probe kernel finished without its completion flag");
      return 0;
    }
  }
}

// ---- the lookup server (host side) --------------------------------------------------------
extern "C" int rf_launch_lookup_server(void* stream, const SrvReq* ring, SrvRes* res, SrvCtl* ctl, uint64_t head,
                                       uint64_t gen, uint64_t idle_ticks, uint64_t life_ticks);
static const uint64_t SRV_UNPUBLISHED = ~0ull, SRV_BUSY = ~0ull - 1;
static_assert(SRV_RING == RF_AMD_SERVER_RING, "rf_amd.h and the kernels agree on the ring size");

// the host's stop word, after the request ring (the wave polls it with the requests)
static inline volatile uint64_t* srv_stop_word(SrvReq* ring) { return reinterpret_cast<volatile uint64_t*>(ring + SRV_RING); }
static void srv_set_stop(LookupServer& v) {
  if (!v.ring) return;
  *srv_stop_word(v.ring) = 1;
  _mm_sfence();  // out of the write-combining buffer now
}
// answer of ticket t in its slot: 1 = all four words carry t's check (found/tag filled in),
// -1 = the slot holds a later ticket's answer (a waiter took t and the slot moved on), 0 = not yet
static inline int srv_answer(const SrvRes* r, uint64_t t, uint64_t* found, uint64_t* tag) {
  const uint32_t c = srv_check(t);
  uint64_t w[4];
  for (int k = 0; k < 4; k++) w[k] = __atomic_load_n(&r->w[k], __ATOMIC_ACQUIRE);
  const uint32_t c0 = (uint32_t)(w[0] >> 32);
  if (c0 != c) return (c0 != 0 && (int32_t)(c0 - c) > 0) ? -1 : 0;
  for (int k = 1; k < 4; k++)
    if ((uint32_t)(w[k] >> 32) != c) return 0;  // still arriving
  if (found) *found = (w[0] & 0xffffffffull) | (w[1] << 32);
  if (tag) *tag = (w[2] & 0xffffffffull) | (w[3] << 32);
  return 1;
}
// RF_AMD_SRV_RING=host puts the request ring in pinned host memory (the round-6 layout's
// placement); default: fine-grained device memory, written by the host through the BAR
static bool srv_ring_on_device() {
  const char* s = getenv("RF_AMD_SRV_RING");
  return !(s && !strcmp(s, "host"));
}

static int srv_init(rf_amd_engine* e) {
  LookupServer& v = e->srv;
  // once initialised, one load (std::call_once's own fast path measured ~900 TSC cycles per
  // submit, profiles/r06_async_submit.txt)
  if (v.ready.load(std::memory_order_acquire)) return 0;
  std::call_once(v.once, [&] {
    const size_t ring_bytes = sizeof(SrvReq) * SRV_RING + 128;  // + the stop word's line
    if (hipSetDevice(e->device) != hipSuccess) {
      v.init_rc = RF_AMD_ENOMEM;
      return;
    }
    v.ring_dev = srv_ring_on_device() &&
                 hipExtMallocWithFlags((void**)&v.ring, ring_bytes, hipDeviceMallocFinegrained) == hipSuccess;
    if (v.ring_dev) {
      // the host writes it through its mapping of device memory: zero it there, then check on
      // the device that a host store landed (a box whose BAR does not reach it falls back)
      if (hipMemset(v.ring, 0, ring_bytes) != hipSuccess || hipStreamSynchronize(nullptr) != hipSuccess) {
        (void)hipFree(v.ring);
        v.ring = nullptr;
        v.ring_dev = false;
      } else {
        volatile uint64_t* w = &v.ring[SRV_RING - 1].w[SRV_REQ_WORDS - 1];
        *w = 0x5EEDF00Dull;
        _mm_sfence();
        uint64_t back = 0;
        const bool ok = hipMemcpy(&back, (const void*)w, 8, hipMemcpyDeviceToHost) == hipSuccess && back == 0x5EEDF00Dull;
        *w = 0;
        _mm_sfence();
        if (!ok) {
          (void)hipFree(v.ring);
          v.ring = nullptr;
          v.ring_dev = false;
        }
      }
    }
    if (!v.ring_dev) {
      if (hipHostMalloc((void**)&v.ring, ring_bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        v.ring = nullptr;
        v.init_rc = RF_AMD_ENOMEM;
        return;
      }
      memset((void*)v.ring, 0, ring_bytes);
    }
    if (hipHostMalloc((void**)&v.res, sizeof(SrvRes) * SRV_RING, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc((void**)&v.ctl, sizeof(SrvCtl), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
      v.init_rc = RF_AMD_ENOMEM;
      return;
    }
    memset(v.res, 0, sizeof(SrvRes) * SRV_RING);  // check 0: no answer yet
    for (uint32_t s = 0; s < SRV_RING; s++) {
      v.consumed[s].store(0, std::memory_order_relaxed);
      v.abandoned[s].store(~0ull, std::memory_order_relaxed);
    }
    memset(v.ctl, 0, sizeof(SrvCtl));
    // a CU-masked stream is a queue of its own: the persistent wave never sits in front of
    // another stream's work (one CU is enough for one wave); without it, a plain stream
    // and a short lifetime bound the wait of whatever shares its queue
    uint32_t mask[8] = {1u, 0, 0, 0, 0, 0, 0, 0};
    const bool masked = hipExtStreamCreateWithCUMask(&v.st, 8, mask) == hipSuccess;
    if (!masked && hipStreamCreateWithFlags(&v.st, hipStreamNonBlocking) != hipSuccess) {
      v.init_rc = RF_AMD_EINVAL;
      return;
    }
    // s_memrealtime runs at 100 MHz. Idle exit 400 us, lifetime 800 us (busy or not; waiters
    // relaunch it, a few us per relaunch): the masked stream synchronises with the legacy null
    // stream and hipDeviceSynchronize waits for every stream, so a device-wide sync or a
    // null-stream op waits at most one lifetime, under 1 ms, for a running wave.
    // rf_amd_lookup_server_set_times (or RF_AMD_SERVER_IDLE_US / _LIFE_US) sets others.
    const char* idle = getenv("RF_AMD_SERVER_IDLE_US");
    const char* life = getenv("RF_AMD_SERVER_LIFE_US");
    if (!v.idle_ticks.load()) v.idle_ticks = (idle ? strtoull(idle, nullptr, 10) : 400) * 100;
    if (!v.life_ticks.load()) v.life_ticks = (life ? strtoull(life, nullptr, 10) : 800) * 100;
    v.ready.store(true, std::memory_order_release);  // reapers on other threads may look now
  });
  return v.init_rc ? fail(v.init_rc, "lookup server allocation failed") : 0;
}

// make sure a server wave is running (or queued): the first submit launches one; a server that
// exited (idle, lifetime, stop) while tickets wait is relaunched from the first ticket it did
// not serve. The generation CAS makes exactly one caller launch.
static int srv_dead(rf_amd_engine* e);
static int srv_ensure(rf_amd_engine* e) {
  LookupServer& v = e->srv;
  if (int rc = srv_dead(e)) return rc;  // a dead server is never relaunched
  uint64_t s = v.state.load(std::memory_order_acquire);
  const uint64_t gen = s >> 1;
  if (s & 1) {
    if (__atomic_load_n(&v.ctl->exit_gen, __ATOMIC_ACQUIRE) != gen) return 0;  // running
  }
  const uint64_t next = ((gen + 1) << 1) | 1;
  if (!v.state.compare_exchange_strong(s, next, std::memory_order_acq_rel)) return 0;  // another launched
  const uint64_t head = __atomic_load_n(&v.ctl->exit_head, __ATOMIC_ACQUIRE);
  (void)hipSetDevice(e->device);
  if (int rc = rf_launch_lookup_server(v.st, v.ring, v.res, v.ctl, head, gen + 1, v.idle_ticks.load(),
                                       v.life_ticks.load())) {
    int z = 0;
    v.dead.compare_exchange_strong(z, RF_AMD_EINVAL);
    return fail(RF_AMD_EINVAL, std::string("lookup server launch: ") + hipGetErrorString((hipError_t)rc));
  }
  v.launches.fetch_add(1, std::memory_order_relaxed);
  return 0;
}

static void srv_stop(rf_amd_engine* e) {
  LookupServer& v = e->srv;
  if (!v.ctl || !v.st) return;
  v.ready.store(false, std::memory_order_release);
  srv_set_stop(v);
  (void)hipStreamSynchronize(v.st);
  (void)hipStreamDestroy(v.st);
  if (v.ring_dev)
    (void)hipFree(v.ring);
  else
    (void)hipHostFree(v.ring);
  v.ring = nullptr;
  (void)hipHostFree(v.res);
  (void)hipHostFree(v.ctl);
  v.st = nullptr;
  v.ctl = nullptr;
}

// stops the server wave and waits, at most budget_ms, for the engine's streams to drain (no
// device-wide wait: other streams of the process are not the engine's)
static bool stream_drained(hipStream_t st, uint64_t deadline_ns);
static bool engine_quiesce(rf_amd_engine* e, int budget_ms) {
  (void)hipSetDevice(e->device);
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  const uint64_t deadline = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec + (uint64_t)budget_ms * 1000000ull;
  LookupServer& v = e->srv;
  if (v.ctl) srv_set_stop(v);
  if (v.st && !stream_drained(v.st, deadline)) return false;
  if (!stream_drained(e->stream, deadline)) return false;
  std::lock_guard<std::mutex> g(e->slot_mu);
  for (ProbeSlot* s : e->slots_all)
    if (s->st && !stream_drained(s->st, deadline)) return false;
  return true;
}
static bool stream_drained(hipStream_t st, uint64_t deadline_ns) {
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q != hipErrorNotReady) return true;  // idle, or faulted: nothing more will run on it
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    if ((uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec > deadline_ns) return false;
    struct timespec nap = {0, 100000};
    nanosleep(&nap, nullptr);
  }
}

// the server stream's error, if its kernel faulted (checked while waiting)
static int srv_check(rf_amd_engine* e) {
  const hipError_t q = hipStreamQuery(e->srv.st);
  if (q == hipSuccess || q == hipErrorNotReady) return 0;
  int z = 0;
  e->srv.dead.compare_exchange_strong(z, RF_AMD_EINVAL);
  return fail(RF_AMD_EINVAL, std::string("lookup server: ") + hipGetErrorString(q));
}
static int srv_dead(rf_amd_engine* e) {
  const int d = e->srv.dead.load(std::memory_order_acquire);
  return d ? fail(d, "lookup server failed earlier") : 0;
}

static ProbeGroup probe_group_of(const rf_amd_batch* b, uint32_t f);
static int batch_errors(rf_amd_batch* b);

// RF_AMD_REAP_TAIL=1: the reap loop bounded by the ticket counter (A/B switch; by default the
// answers' checks bound it and the submitters' counter line is not read)
static bool srv_reap_tail() {
  static const bool on = [] {
    const char* s = getenv("RF_AMD_REAP_TAIL");
    return s && atoi(s) > 0;
  }();
  return on;
}
// the request's 16 words (payload | check << 32) into its slot. Each 8-byte word is valid on
// its own, so wider stores are as safe as 8-byte ones: RF_AMD_SRV_STORE = 8 (eight-byte
// stores), 16 (SSE, the default) or 32 (AVX) -- an A/B switch
static int srv_store_width() {
  static const int w = [] {
    const char* s = getenv("RF_AMD_SRV_STORE");
    const int v = s ? atoi(s) : 16;
    return v == 8 || v == 32 ? v : 16;
  }();
  return w;
}
__attribute__((target("avx2"))) static void srv_write_request_avx(uint64_t* dst, const uint64_t* src) {
  for (uint32_t k = 0; k < SRV_REQ_WORDS; k += 4)
    _mm256_store_si256(reinterpret_cast<__m256i*>(dst + k), _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + k)));
}
static inline void srv_write_request(uint64_t* dst, const uint32_t* p, uint64_t ck) {
  alignas(32) uint64_t w[SRV_REQ_WORDS];
  for (uint32_t k = 0; k < SRV_REQ_WORDS; k++) w[k] = (uint64_t)p[k] | ck;
  const int width = srv_store_width();
  if (width == 8) {
    volatile uint64_t* d = dst;
    for (uint32_t k = 0; k < SRV_REQ_WORDS; k++) d[k] = w[k];
  } else if (width == 16) {
    for (uint32_t k = 0; k < SRV_REQ_WORDS; k += 2)
      _mm_store_si128(reinterpret_cast<__m128i*>(dst + k), _mm_load_si128(reinterpret_cast<const __m128i*>(w + k)));
  } else {
    srv_write_request_avx(dst, w);
  }
}
// RF_AMD_SRV_SFENCE=1: an sfence after each request (A/B switch: whole lines leave the
// write-combining buffers without one)
static bool srv_sfence() {
  static const bool on = [] {
    const char* s = getenv("RF_AMD_SRV_SFENCE");
    return s && atoi(s) > 0;
  }();
  return on;
}

// RF_AMD_SUBMIT_PROFILE=1 (diagnostics): TSC cycles of the steps of rf_amd_lookup_submit --
// checks, ticket + slot wait, request write, server check -- printed to stderr at exit
static int g_subprof = -1;
static uint64_t g_subprof_cyc[7], g_subprof_n;
// a TSC stamp that waits for the loads before it (lfence on both sides): each step's misses
// land in its own interval
static inline uint64_t tsc_ser() {
  _mm_lfence();
  const uint64_t t = __rdtsc();
  _mm_lfence();
  return t;
}
// the reaper's side (one completion thread in the profiled runs): TSC cycles of reaps that
// returned states -- the idle look at the next answer, lock + cursor, the answer loop -- and
// the states they returned
static uint64_t g_reapprof_cyc[3], g_reapprof_n, g_reapprof_states;
static rf_amd_engine* g_subprof_eng = nullptr;
static void subprof_print() {
  if (g_subprof_eng && g_subprof_eng->srv.ctl && g_subprof_eng->srv.ctl->prof[5]) {
    const uint64_t* q = g_subprof_eng->srv.ctl->prof;
    const double np = (double)q[5];
    fprintf(stderr, "rf_amd server passes (RF_SRV_PROF build): %llu served, us each: poll %.2f payloads %.2f "
            "probe+answers %.2f; %.1f requests per pass, %llu passes cut by a request still arriving\n",
            (unsigned long long)q[5], q[0] / np / 100, q[1] / np / 100, q[2] / np / 100, q[4] / np,
            (unsigned long long)q[3]);
  }
  if (g_reapprof_n)
    fprintf(stderr, "rf_amd reap profile: %llu reaps with answers, %.1f states each, TSC cycles each: idle look %.0f "
            "lock+cursor %.0f answers %.0f\n", (unsigned long long)g_reapprof_n, (double)g_reapprof_states / g_reapprof_n,
            (double)g_reapprof_cyc[0] / g_reapprof_n, (double)g_reapprof_cyc[1] / g_reapprof_n,
            (double)g_reapprof_cyc[2] / g_reapprof_n);
  if (g_subprof_n)
    fprintf(stderr, "rf_amd submit profile: %llu submissions, TSC cycles each: checks %.0f (args %.0f init %.0f "
            "errors %.0f) ticket %.0f write %.0f ensure %.0f\n",
            (unsigned long long)g_subprof_n, (double)g_subprof_cyc[0] / g_subprof_n, (double)g_subprof_cyc[4] / g_subprof_n,
            (double)g_subprof_cyc[5] / g_subprof_n, (double)g_subprof_cyc[6] / g_subprof_n,
            (double)g_subprof_cyc[1] / g_subprof_n, (double)g_subprof_cyc[2] / g_subprof_n,
            (double)g_subprof_cyc[3] / g_subprof_n);
}

extern "C" int rf_amd_lookup_submit(rf_amd_engine* e, rf_amd_batch* b, uint32_t filter_index, uint32_t hash,
                                    void* tag, uint64_t* ticket) {
  if (g_subprof < 0) {
    const char* pv = getenv("RF_AMD_SUBMIT_PROFILE");
    g_subprof = pv && atoi(pv) > 0;
    if (g_subprof) atexit(subprof_print);
  }
  const uint64_t c0 = g_subprof > 0 ? tsc_ser() : 0;
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (g_subprof > 0) g_subprof_eng = e;
  if (!b || !b->built || b->eng != e) return fail(RF_AMD_EINVAL, "lookup on an unbuilt or foreign batch");
  if (filter_index >= b->F) return fail(RF_AMD_EINVAL, "bad filter index");
  if (!ticket) return fail(RF_AMD_EINVAL, "null ticket");
  const uint64_t c0a = g_subprof > 0 ? tsc_ser() : 0;
  if (__builtin_expect(!e->srv.ready.load(std::memory_order_acquire), 0))
    if (int rc = srv_init(e)) return rc;
  const uint64_t c0b = g_subprof > 0 ? tsc_ser() : 0;
  if (int rc = batch_errors(b)) return rc;
  const uint64_t c0c = g_subprof > 0 ? tsc_ser() : 0;
  if (int rc = srv_dead(e)) return rc;
  LookupServer& v = e->srv;
  const uint64_t c1 = g_subprof > 0 ? tsc_ser() : 0;
  const uint64_t t = v.tail.fetch_add(1, std::memory_order_acq_rel);
  const uint32_t slot = (uint32_t)(t & (SRV_RING - 1));
  if (t >= SRV_RING) {
    // the slot's previous ticket p must have been taken: by the reaper (a tagged ticket: the
    // reap cursor passed it, having copied its answer out), by its waiter (consumed), or never
    // published (abandoned)
    const uint64_t p = t - SRV_RING;
    // the reap cursor only moves forward, and it is usually ~64 tickets behind the tail, far
    // past p = t - SRV_RING: a submitting thread re-reads it (a line the reaper writes on every
    // reap) only when its last look does not already show p reaped
    static thread_local uint64_t hint_uid = 0, hint_seen = 0;
    if (hint_uid != e->uid) {
      hint_uid = e->uid;
      hint_seen = 0;
    }
    auto reaped = [&] {
      if (hint_seen > p) return true;
      hint_seen = v.reap_hint.load(std::memory_order_acquire);
      return hint_seen > p;
    };
    auto taken = [&] {
      if (v.consumed[slot].load(std::memory_order_acquire) == p + 1) return true;
      if (!reaped()) return false;
      if (v.abandoned[slot].load(std::memory_order_acquire) == p) return true;
      return v.meta[slot].ticket.load(std::memory_order_acquire) == p && v.meta[slot].tag != nullptr;
    };
    for (uint32_t spin = 1; !taken(); spin++) {
      __builtin_ia32_pause();
      if ((spin & 1023) == 0) {  // ticket t stays unpublished only on a server that is dead
        int rc = srv_ensure(e);
        if (!rc) rc = srv_check(e);
        if (!rc) rc = srv_dead(e);
        if (rc) {  // ticket t is never published: the cursors step over it
          v.abandoned[slot].store(t, std::memory_order_release);
          return rc;
        }
      }
    }
    // the slot is being rewritten: readers that see this do not trust its tag (the server
    // reads the request only after its new ticket is published)
    v.meta[slot].ticket.store(SRV_BUSY, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);  // BUSY before the new tag (a seqlock)
  }
  const uint64_t c2 = g_subprof > 0 ? tsc_ser() : 0;
  {
    // 16 words, each with t's check in its high half; plain 8-byte stores in any order (two
    // whole 64-byte lines: through the write-combining BAR mapping they leave as two bursts)
    const ProbeGroup g = probe_group_of(b, filter_index);
    const uint64_t tg = (uint64_t)(uintptr_t)tag;
    const uint64_t lp = (uint64_t)(uintptr_t)g.lines, pp = (uint64_t)(uintptr_t)g.pages, sp = (uint64_t)(uintptr_t)g.slots;
    const uint32_t p[SRV_REQ_WORDS] = {g.x, g.err, g.fpl, hash, (uint32_t)lp, (uint32_t)(lp >> 32), (uint32_t)pp, (uint32_t)(pp >> 32),
                                       (uint32_t)sp, (uint32_t)(sp >> 32), (uint32_t)tg, (uint32_t)(tg >> 32), 0u, 0u, 0u, 0u};
    v.meta[slot].tag = tag;
    v.meta[slot].ticket.store(t, std::memory_order_release);
    const uint64_t ck = (uint64_t)srv_check(t) << 32;
    srv_write_request(v.ring[slot].w, p, ck);
    if (srv_sfence()) _mm_sfence();
  }
  *ticket = t;
  const uint64_t c3 = g_subprof > 0 ? tsc_ser() : 0;
  // published: from here the ticket's tag comes back through rf_amd_lookup_reap or, if the
  // server is (or now becomes) dead, rf_amd_lookup_server_failed -- so a launch failure here is
  // not the submit's error (the caller would complete the state a second time)
  (void)srv_ensure(e);
  if (g_subprof > 0) {  // one submitting thread in the profiled runs: plain sums
    const uint64_t c4 = tsc_ser();
    g_subprof_cyc[0] += c1 - c0;
    g_subprof_cyc[4] += c0a - c0;
    g_subprof_cyc[5] += c0b - c0a;
    g_subprof_cyc[6] += c0c - c0b;
    g_subprof_cyc[1] += c2 - c1;
    g_subprof_cyc[2] += c3 - c2;
    g_subprof_cyc[3] += c4 - c3;
    g_subprof_n++;
  }
  return 0;
}

extern "C" int rf_amd_lookup_wait(rf_amd_engine* e, uint64_t ticket, uint64_t* found_values) {
  if (!e || !e->srv.ready.load(std::memory_order_acquire)) return fail(RF_AMD_EINVAL, "no lookup server");
  LookupServer& v = e->srv;
  const uint32_t slot = (uint32_t)(ticket & (SRV_RING - 1));
  for (uint32_t spin = 1;; spin++) {
    if (srv_answer(&v.res[slot], ticket, found_values, nullptr) == 1) {
      v.consumed[slot].store(ticket + 1, std::memory_order_release);
      return 0;
    }
    __builtin_ia32_pause();
    if ((spin & 255) == 0) {
      if (int rc = srv_dead(e)) return rc;
      if (int rc = srv_ensure(e)) return rc;
      if ((spin & 65535) == 0)
        if (int rc = srv_check(e)) return rc;
    }
  }
}

extern "C" uint64_t rf_amd_lookup_reap(rf_amd_engine* e, void** tags, uint64_t* found_values, uint64_t max) {
  // (ready, not ring: another thread's srv_init may have allocated the request ring only)
  if (!e || !e->srv.ready.load(std::memory_order_acquire) || !tags || !found_values) return 0;
  LookupServer& v = e->srv;
  const bool prof = g_subprof > 0;
  const uint64_t r0 = prof ? __rdtsc() : 0;
  {
    // an idle reap (callers spin on this) looks only at the next ticket's answer line, which
    // only the GPU writes: no lock taken, no line the submitters write read. The full pass
    // below runs once that ticket is answered (or its slot moved on: answered later tickets
    // mean a waiter took it), when it was abandoned, and every few microseconds regardless --
    // it relaunches a server that exited with tickets waiting and notices a faulted one.
    const uint64_t t = v.reap_hint.load(std::memory_order_relaxed);
    const uint32_t slot = (uint32_t)(t & (SRV_RING - 1));
    if (srv_answer(&v.res[slot], t, nullptr, nullptr) == 0 && v.abandoned[slot].load(std::memory_order_relaxed) != t) {
      static thread_local uint64_t last_full = 0;
      const uint64_t now = __rdtsc();
      if (now - last_full < 8192) return 0;  // a few microseconds at the hosts' TSC rates
      last_full = now;
    }
  }
  const uint64_t r1 = prof ? __rdtsc() : 0;
  std::unique_lock<std::mutex> lk(v.reap_mu, std::try_to_lock);
  if (!lk.owns_lock()) return 0;  // another thread is reaping
  uint64_t n = 0, t = v.reap_next;
  // Only the answer lines are read: written by the GPU over PCIe (a miss each, fetched ahead so
  // the misses of consecutive tickets overlap), they carry the request's tag and check -- no line
  // of the submitting threads is touched per state, not even the ticket counter: a slot past
  // the last ticket holds an older check and stops the loop like an unanswered one. Ticket t is
  // done when its answer is there (a waiter's, tag 0, is left to its waiter), when its slot
  // already holds a later answer (a waiter took t and the slot was reused), or when it was
  // abandoned unpublished.
  const uint64_t tail = srv_reap_tail() ? v.tail.load(std::memory_order_acquire) : ~0ull;
  const uint64_t r2 = prof ? __rdtsc() : 0;
  for (uint64_t q = t; q < tail && q < t + 16; q += 2) __builtin_prefetch(&v.res[q & (SRV_RING - 1)], 0, 0);
  while (n < max && t < tail) {
    const uint32_t slot = (uint32_t)(t & (SRV_RING - 1));
    if ((t & 1) == 0) __builtin_prefetch(&v.res[(t + 16) & (SRV_RING - 1)], 0, 0);
    uint64_t found = 0, tag = 0;
    const int a = srv_answer(&v.res[slot], t, &found, &tag);
    if (a == 1) {
      if (tag) {
        tags[n] = (void*)(uintptr_t)tag;
        found_values[n] = found;
        n++;
      }
      t++;
      continue;
    }
    if (a < 0 || v.abandoned[slot].load(std::memory_order_acquire) == t) {
      t++;
      continue;
    }
    break;  // not answered yet (or past the last ticket)
  }
  v.reap_next = t;
  v.reap_hint.store(t, std::memory_order_release);  // the answers before t are copied out
  lk.unlock();
  if (prof && n) {
    const uint64_t r3 = __rdtsc();
    g_reapprof_cyc[0] += r1 - r0;
    g_reapprof_cyc[1] += r2 - r1;
    g_reapprof_cyc[2] += r3 - r2;
    g_reapprof_n++;
    g_reapprof_states += n;
  }
  if (n == 0 && t < v.tail.load(std::memory_order_acquire)) {
    (void)srv_ensure(e);
    // a faulted server stream never answers and nothing else would notice with only tagged
    // tickets outstanding: look at it about once a millisecond, so `dead` gets set and the
    // caller's rf_amd_lookup_server_error / _failed path completes the waiting states
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const uint64_t now = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    uint64_t last = v.last_check_ns.load(std::memory_order_relaxed);
    if (now - last > 1000000 && v.last_check_ns.compare_exchange_strong(last, now)) (void)srv_check(e);
  }
  return n;
}

// a dead server's unanswered tickets: the tags of the published ones from the reap cursor on
// (waiters' tickets skipped: rf_amd_lookup_wait returns the error to them), consumed here
extern "C" uint64_t rf_amd_lookup_server_failed(rf_amd_engine* e, void** tags, uint64_t max) {
  if (!e || !e->srv.ready.load(std::memory_order_acquire) || !tags || !e->srv.dead.load(std::memory_order_acquire)) return 0;
  LookupServer& v = e->srv;
  std::lock_guard<std::mutex> lk(v.reap_mu);
  uint64_t n = 0, t = v.reap_next;
  const uint64_t tail = v.tail.load(std::memory_order_acquire);
  // Stops at the first ticket not yet published: a submitter that passed the dead
  // check before `dead` was set publishes it later, and the next call hands its tag back. A
  // ticket its submitter abandoned is stepped over; a slot already holding a later ticket means
  // a waiter took ticket t (waiters' tickets are not tagged).
  for (; n < max && t < tail; t++) {
    const uint32_t slot = (uint32_t)(t & (SRV_RING - 1));
    const uint64_t tk = v.meta[slot].ticket.load(std::memory_order_acquire);
    if (tk != t) {
      if (v.abandoned[slot].load(std::memory_order_acquire) == t) continue;
      if (tk == SRV_UNPUBLISHED || tk == SRV_BUSY || tk < t) break;
      continue;  // reused: a waiter's ticket, already taken
    }
    void* tag = v.meta[slot].tag;
    std::atomic_thread_fence(std::memory_order_acquire);
    if (v.meta[slot].ticket.load(std::memory_order_relaxed) != t) break;  // being rewritten: next call
    if (!tag) continue;
    if (srv_answer(&v.res[slot], t, nullptr, nullptr) == 1) break;  // answered: reap takes it
    tags[n++] = tag;
    v.consumed[slot].store(t + 1, std::memory_order_release);
  }
  v.reap_next = t;
  v.reap_hint.store(t, std::memory_order_release);
  return n;
}

// diagnostics (rf_amd_diag.h): the server stops answering (its wave told to exit; a relaunched
// wave exits at once), then, after `gap_us`, is marked dead as a failed launch or a faulted
// stream marks it: tickets published in the gap are never answered
extern "C" int rf_amd_diag_lookup_server_kill(rf_amd_engine* e, int err, uint32_t gap_us) {
  if (!e || !err) return fail(RF_AMD_EINVAL, "bad argument");
  if (int rc = srv_init(e)) return rc;
  srv_set_stop(e->srv);
  if (gap_us) {
    struct timespec nap = {(time_t)(gap_us / 1000000), (long)(gap_us % 1000000) * 1000};
    nanosleep(&nap, nullptr);
  }
  int z = 0;
  e->srv.dead.compare_exchange_strong(z, err);
  return 0;
}

extern "C" int rf_amd_lookup_server_error(rf_amd_engine* e) { return e ? e->srv.dead.load() : RF_AMD_ENODEV; }

// the idle exit and lifetime (microseconds) of the server waves launched from now on (a
// host-controlled keep-alive: a caller that needs one wave across a long stretch raises them)
extern "C" int rf_amd_lookup_server_set_times(rf_amd_engine* e, uint64_t idle_us, uint64_t life_us) {
  if (!e || !idle_us || !life_us) return fail(RF_AMD_EINVAL, "bad server times");
  e->srv.idle_ticks = idle_us * 100;
  e->srv.life_ticks = life_us * 100;
  return 0;
}

extern "C" int rf_amd_diag_lookup_ring(rf_amd_engine* e) {
  if (!e || !e->srv.ready.load(std::memory_order_acquire)) return -1;
  return e->srv.ring_dev ? 1 : 0;
}

extern "C" int rf_amd_lookup_server_stats(rf_amd_engine* e, uint64_t* out) {
  if (!e || !out) return fail(RF_AMD_EINVAL, "null argument");
  out[0] = e->srv.tail.load();
  out[1] = e->srv.launches.load();
  out[2] = e->srv.ctl ? __atomic_load_n(&e->srv.ctl->exit_head, __ATOMIC_ACQUIRE) : 0;
  return 0;
}

// where a host-buffer lookup round trip spends its time (rf_amd_diag_lookup_stats): calls,
// ns before the launch (slot, buffers, build ordering, argument packing), ns in the launch
// call, ns waiting for the completion word (and copying the results out)
static std::atomic<uint64_t> g_lk_calls{0}, g_lk_prep_ns{0}, g_lk_launch_ns{0}, g_lk_wait_ns{0};
static inline uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
struct LookupClock {
  uint64_t t0 = mono_ns(), t1 = 0, t2 = 0;
  void launching() { t1 = mono_ns(); }
  void launched() { t2 = mono_ns(); }
  ~LookupClock() {
    if (!t2) return;  // failed before the launch
    const uint64_t t3 = mono_ns();
    g_lk_calls.fetch_add(1, std::memory_order_relaxed);
    g_lk_prep_ns.fetch_add(t1 - t0, std::memory_order_relaxed);
    g_lk_launch_ns.fetch_add(t2 - t1, std::memory_order_relaxed);
    g_lk_wait_ns.fetch_add(t3 - t2, std::memory_order_relaxed);
  }
};
#ifndef RF_AMD_SRC_ID
#define RF_AMD_SRC_ID "unknown"
#endif
extern "C" const char* rf_amd_build_id(void) { return RF_AMD_SRC_ID; }

extern "C" int rf_amd_diag_lookup_stats(uint64_t* out, int reset) {
  if (!out) return fail(RF_AMD_EINVAL, "null output");
  std::atomic<uint64_t>* c[4] = {&g_lk_calls, &g_lk_prep_ns, &g_lk_launch_ns, &g_lk_wait_ns};
  for (int k = 0; k < 4; k++) out[k] = reset ? c[k]->exchange(0) : c[k]->load();
  return 0;
}

static int probe_groups_host(rf_amd_engine* e, const std::vector<ProbeGroup>& groups,
                             const uint32_t* h_hashes, const uint32_t* h_group, uint64_t n, uint64_t* h_found) {
  if (n == 0) return 0;
  LookupClock clk;
  static const int mode = env_mode("RF_AMD_PROBE_MODE", "mapped", "copy");
  static const int wait = env_mode("RF_AMD_PROBE_WAIT", "flag", "sync");
  static const bool small_ok = !getenv("RF_AMD_PROBE_SMALL") || atoi(getenv("RF_AMD_PROBE_SMALL")) != 0;
  const uint32_t ng = (uint32_t)groups.size();
  const size_t o_g = (8 * n + 15) & ~15ull, o_f = (o_g + sizeof(ProbeGroup) * ng + 63) & ~63ull;
  const bool small = small_ok && wait != 2 && n <= SMALL_PROBES && ng <= SMALL_GROUPS;
  const bool mapped = mode == 1 || (mode == 0 && n <= MAPPED_MAX_PROBES);
  ProbeSlot* s = slot_take(e);
  if (!s) return RF_AMD_ENOMEM;
  struct Give {
    rf_amd_engine* e;
    ProbeSlot* s;
    ~Give() { slot_give(e, s); }
  } give{e, s};
  if (int rc = slot_reserve(s, small ? 8 * n : o_f + 8 * n, (small || mapped) ? 0 : o_f)) return rc;
  const uint64_t issued = e->builds_issued.load(std::memory_order_acquire);
  if (issued != e->builds_seen_idle.load(std::memory_order_acquire)) {
    if (hipStreamQuery(e->stream) == hipErrorNotReady) {  // order after builds still in flight
      hipEvent_t ev;
      HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      HIPCHK(hipEventRecord(ev, e->stream));
      HIPCHK(hipStreamWaitEvent(s->st, ev, 0));
      (void)hipEventDestroy(ev);
    } else {
      e->builds_seen_idle.store(issued, std::memory_order_release);  // every build up to `issued` is done
    }
  }
  const uint32_t seq = ++s->seq ? s->seq : ++s->seq;  // never 0 (the flag's initial value)
  (void)hipGetLastError();
  if (small) {  // everything in the kernel arguments: no host-memory read before the probe
    SmallProbe sp;
    memset(&sp, 0, sizeof(sp));
    sp.n = (uint32_t)n;
    sp.ng = ng;
    sp.seq = seq;
    for (uint64_t i = 0; i < n; i++) {
      sp.h[i] = h_hashes[i];
      const uint32_t g = h_group ? h_group[i] : 0u;
      sp.g[i] = (uint8_t)(g < ng ? g : 255u);
    }
    for (uint32_t g = 0; g < ng; g++) sp.groups[g] = groups[g];
    sp.found = reinterpret_cast<uint64_t*>(s->h);
    sp.done_flag = s->flag;
    clk.launching();
    if (int rc = rf_launch_probe_small(s->st, &sp))
      return fail(RF_AMD_EINVAL, std::string("probe launch: ") + hipGetErrorString((hipError_t)rc));
    clk.launched();
    if (int rc = slot_wait(s, seq, false)) return rc;
    memcpy(h_found, s->h, 8 * n);
    return 0;
  }
  memcpy(s->h, h_hashes, 4 * n);
  uint32_t* hg = reinterpret_cast<uint32_t*>(s->h + 4 * n);
  if (h_group) memcpy(hg, h_group, 4 * n);
  else memset(hg, 0, 4 * n);
  memcpy(s->h + o_g, groups.data(), sizeof(ProbeGroup) * ng);
  const uint8_t* in = s->h;
  if (!mapped) {
    HIPCHK(hipMemcpyAsync(s->d, s->h, o_f, hipMemcpyHostToDevice, s->st));
    in = s->d;
  }
  uint64_t* found = reinterpret_cast<uint64_t*>(s->h + o_f);
  clk.launching();
  if (int rc = rf_launch_probe_groups(s->st, reinterpret_cast<const uint32_t*>(in),
                                      reinterpret_cast<const ProbeGroup*>(in + o_g), ng, n, found,
                                      s->d_counter, wait == 2 ? nullptr : s->flag, seq))
    return fail(RF_AMD_EINVAL, std::string("probe launch: ") + hipGetErrorString((hipError_t)rc));
  clk.launched();
  if (int rc = slot_wait(s, seq, wait == 2)) return rc;
  memcpy(h_found, found, 8 * n);
  return 0;
}

extern "C" int rf_amd_batch_probe_hashes_host(rf_amd_batch* b, const uint32_t* h_hashes, const uint32_t* h_filter_id,
                                              uint64_t n, uint64_t* h_found) {
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "probe on an unbuilt batch");
  if (n == 0) return 0;
  if (!h_hashes || !h_found) return fail(RF_AMD_EINVAL, "null probe buffer");
  rf_amd_engine* e = b->eng;
  HIPCHK(hipSetDevice(e->device));
  if (int rc = batch_errors(b)) return rc;
  std::vector<ProbeGroup> groups(h_filter_id ? b->F : 1);  // group = filter id (ids >= F find nothing)
  for (uint32_t f = 0; f < groups.size(); f++) groups[f] = probe_group_of(b, f);
  return probe_groups_host(e, groups, h_hashes, h_filter_id, n, h_found);
}

extern "C" int rf_amd_probe_filters_host(rf_amd_engine* e, rf_amd_batch* const* batches, const uint32_t* filter_index,
                                         uint32_t num_groups, const uint32_t* h_hashes, const uint32_t* h_group,
                                         uint64_t n, uint64_t* h_found) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (num_groups && !batches) return fail(RF_AMD_EINVAL, "null group arrays");
  if (n == 0) return 0;
  if (!h_hashes || !h_found) return fail(RF_AMD_EINVAL, "null probe buffer");
  HIPCHK(hipSetDevice(e->device));
  // each group carries its own batch's routing config: filters of kvstores with different
  // fingerprint or index sizes go out in the same launch
  std::vector<ProbeGroup> groups(num_groups);
  for (uint32_t g = 0; g < num_groups; g++) {
    rf_amd_batch* b = batches[g];
    const uint32_t f = filter_index ? filter_index[g] : 0u;
    if (!b || !b->built || b->eng != e) return fail(RF_AMD_EINVAL, "group on an unbuilt or foreign batch");
    if (f >= b->F) return fail(RF_AMD_EINVAL, "bad filter index");
    if (int rc = batch_errors(b)) return rc;
    groups[g] = probe_group_of(b, f);
  }
  if (!num_groups) {  // no filters: nothing found
    memset(h_found, 0, 8 * n);
    return 0;
  }
  return probe_groups_host(e, groups, h_hashes, h_group, n, h_found);
}

// Lookups against many resident filters in ONE launch: group g probes counts[g] hashes
// (consecutive in h_hashes) against filter filter_index[g] of batches[g] -- the batch form of
// trunk_merge_lookup's per-bundle routing_filter_lookup calls (src/trunk.c:6008-6075) and of
// a flush of queued routing_filter_lookup_async states.
extern "C" int rf_amd_probe_many_hashes_host(rf_amd_engine* e, rf_amd_batch* const* batches,
                                             const uint32_t* filter_index, const uint64_t* counts,
                                             uint32_t num_groups, const uint32_t* h_hashes, uint64_t* h_found) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (num_groups && (!batches || !counts)) return fail(RF_AMD_EINVAL, "null group arrays");
  uint64_t n = 0;
  for (uint32_t g = 0; g < num_groups; g++) n += counts[g];
  if (n == 0) return 0;
  std::vector<uint32_t> gid(n);
  for (uint32_t g = 0, at = 0; g < num_groups; at += (uint32_t)counts[g], g++)
    std::fill(gid.begin() + at, gid.begin() + at + counts[g], g);
  return rf_amd_probe_filters_host(e, batches, filter_index, num_groups, h_hashes, gid.data(), n, h_found);
}

static int do_probe(rf_amd_batch* b, int kind, const void* in0, const uint64_t* offs, uint32_t key_len,
                    const uint32_t* fid, uint64_t n, uint64_t* found, void* stream,
                    const uint64_t* d_runs) {
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "probe on an unbuilt batch");
  if (n && (!in0 || !(fid || d_runs) || !found)) return fail(RF_AMD_EINVAL, "null probe buffer");
  HIPCHK(hipSetDevice(b->eng->device));
  hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
  (void)hipGetLastError();
  LaunchArgs a = make_args(b, st);
  a.probe_runs = d_runs;
  a.wave_tab = d_runs ? b->d_wave_tab.as<uint32_t>() : nullptr;
  int rc = rf_launch_probe(&a, kind, in0, offs, key_len, fid, n, found);
  if (rc) return fail(RF_AMD_EINVAL, std::string("probe launch: ") + hipGetErrorString((hipError_t)rc));
  return 0;
}

extern "C" int rf_amd_batch_probe_keys(rf_amd_batch* b, const void* d_keys, uint32_t key_len,
                                       const uint32_t* d_filter_id, uint64_t n, uint64_t* d_found, void* stream) {
  if (key_len == 0) return fail(RF_AMD_EINVAL, "key_len 0");
  return do_probe(b, fixed_kind(d_keys, key_len), d_keys, nullptr, key_len, d_filter_id, n, d_found, stream);
}
extern "C" int rf_amd_batch_probe_var_keys(rf_amd_batch* b, const uint8_t* d_bytes, const uint64_t* d_offsets,
                                           const uint32_t* d_filter_id, uint64_t n, uint64_t* d_found,
                                           void* stream) {
  return do_probe(b, IN_VAR, d_bytes, d_offsets, 0, d_filter_id, n, d_found, stream);
}
extern "C" int rf_amd_batch_probe_hashes(rf_amd_batch* b, const uint32_t* d_hashes, const uint32_t* d_filter_id,
                                         uint64_t n, uint64_t* d_found, void* stream) {
  return do_probe(b, IN_HASH, d_hashes, nullptr, 4, d_filter_id, n, d_found, stream);
}

// Probes grouped by filter (filter f's h_counts[f] probes follow filter f-1's): the filter of
// a probe comes from its position, so no per-probe filter id is read. The run bounds are
// uploaded when they change.
static int upload_runs(rf_amd_batch* b, const uint64_t* h_counts, void* stream, uint64_t* n_out) {
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "probe on an unbuilt batch");
  if (!h_counts) return fail(RF_AMD_EINVAL, "null counts");
  std::vector<uint64_t> runs(b->F + 1, 0);
  for (uint32_t f = 0; f < b->F; f++) runs[f + 1] = runs[f] + h_counts[f];
  const uint64_t n = runs[b->F];
  *n_out = n;
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(b->eng->device));
  if (runs != b->runs_host) {
    if (!b->d_runs.p && b->d_runs.alloc(8ull * (b->F + 1), &b->eng->pool)) return RF_AMD_ENOMEM;
    hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
    HIPCHK(hipStreamSynchronize(st));  // earlier probes may still read the old bounds
    const uint64_t nw = (n + 63) / 64;
    if (b->d_wave_tab.n < 4 * nw && b->d_wave_tab.alloc(4 * nw, &b->eng->pool)) return RF_AMD_ENOMEM;
    HIPCHK(hipMemcpyAsync(b->d_runs.p, runs.data(), 8ull * (b->F + 1), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    if (rf_launch_wave_tab(st, b->d_runs.as<uint64_t>(), b->F, n, b->d_wave_tab.as<uint32_t>()))
      return fail(RF_AMD_EINVAL, "wave table launch failed");
    b->runs_host = runs;
  }
  return 0;
}

static int probe_runs(rf_amd_batch* b, int kind, const void* in0, uint32_t key_len, const uint64_t* h_counts,
                      uint64_t* d_found, void* stream) {
  uint64_t n = 0;
  if (int rc = upload_runs(b, h_counts, stream, &n)) return rc;
  if (n == 0) return 0;
  return do_probe(b, kind, in0, nullptr, key_len, nullptr, n, d_found, stream, b->d_runs.as<uint64_t>());
}

// bench.py's measured probe floor: k_probe_floor over the same runs (rf_amd_diag.h)
extern "C" int rf_launch_probe_floor(const LaunchArgs* pa, int kind, const void* in0, uint64_t n, uint64_t* found);
extern "C" int rf_amd_debug_probe_floor(rf_amd_batch* b, const void* d_in, uint32_t key_len, const uint64_t* h_counts,
                                        uint64_t* d_out, void* stream) {
  if (key_len != 24 && key_len != 4) return fail(RF_AMD_EINVAL, "probe floor: 24-byte keys or 4-byte hashes");
  if (!d_in || !d_out) return fail(RF_AMD_EINVAL, "null probe buffer");
  if (key_len == 24 && ((uintptr_t)d_in & 15)) return fail(RF_AMD_EINVAL, "probe floor: keys 16-byte aligned");
  uint64_t n = 0;
  if (int rc = upload_runs(b, h_counts, stream, &n)) return rc;
  if (n == 0) return 0;
  hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
  (void)hipGetLastError();
  LaunchArgs a = make_args(b, st);
  a.probe_runs = b->d_runs.as<uint64_t>();
  a.wave_tab = b->d_wave_tab.as<uint32_t>();
  int rc = rf_launch_probe_floor(&a, key_len == 24 ? IN_KEYS24 : IN_HASH, d_in, n, d_out);
  if (rc) return fail(RF_AMD_EINVAL, std::string("probe floor launch: ") + hipGetErrorString((hipError_t)rc));
  return 0;
}

extern "C" int rf_amd_batch_probe_keys_runs(rf_amd_batch* b, const void* d_keys, uint32_t key_len,
                                            const uint64_t* h_counts, uint64_t* d_found, void* stream) {
  if (key_len == 0) return fail(RF_AMD_EINVAL, "key_len 0");
  return probe_runs(b, fixed_kind(d_keys, key_len), d_keys, key_len, h_counts, d_found, stream);
}
extern "C" int rf_amd_batch_probe_hashes_runs(rf_amd_batch* b, const uint32_t* d_hashes, const uint64_t* h_counts,
                                              uint64_t* d_found, void* stream) {
  return probe_runs(b, IN_HASH, d_hashes, 4, h_counts, d_found, stream);
}

extern "C" int rf_debug_set_phase_buffer(uint64_t* d_buf, uint32_t kid);
extern "C" int rf_amd_debug_phase_buffer(void* d_buf, uint32_t kernel) {
#ifdef RF_PHASE_STAMPS
  return rf_debug_set_phase_buffer(static_cast<uint64_t*>(d_buf), kernel) ? fail(RF_AMD_EINVAL, "phase buffer") : 0;
#else
  (void)kernel;
  return d_buf ? fail(RF_AMD_EINVAL, "phase stamps exist only in the diagnostics library") : 0;
#endif
}

extern "C" int rf_amd_debug_read_lines(rf_amd_batch* b, uint8_t* h_lines, uint64_t bytes, uint64_t* num_lines) {
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "unbuilt batch");
  if (num_lines) *num_lines = b->NL;
  if (!h_lines) return 0;
  if (bytes < 64ull * b->NL) return fail(RF_AMD_EINVAL, "lines buffer too small");
  HIPCHK(hipSetDevice(b->eng->device));
  if (int rc = wait_built(b)) return rc;
  HIPCHK(hipMemcpyAsync(h_lines, b->d_lines.p, 64ull * b->NL, hipMemcpyDeviceToHost, b->eng->stream));
  HIPCHK(hipStreamSynchronize(b->eng->stream));
  return 0;
}

extern "C" int rf_amd_debug_rebuild_lines(rf_amd_batch* b) {
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "unbuilt batch");
  HIPCHK(hipSetDevice(b->eng->device));
  if (int rc = wait_built(b)) return rc;
  (void)hipGetLastError();
  LaunchArgs a = make_args(b, b->eng->stream);
  a.plines_force = 1;  // every filter, also those whose lines K6 cut
  if (int rc = rf_launch_plines(&a)) return fail(RF_AMD_EINVAL, std::string("probe-line launch: ") + hipGetErrorString((hipError_t)rc));
  HIPCHK(hipStreamSynchronize(b->eng->stream));
  return 0;
}

extern "C" int rf_amd_batch_set_timing(rf_amd_batch* b, int enable) {
  if (!b) return fail(RF_AMD_EINVAL, "null batch");
  HIPCHK(hipSetDevice(b->eng->device));
  for (auto ev : b->events) (void)hipEventDestroy(ev);
  b->events.clear();
  b->ev_sets = b->ev_set = 0;
  b->ev_mask = enable < 0 ? EV_MASK_PROBE : EV_MASK_ALL;
  if (enable < 0) enable = -enable;
  if (enable > 0) {
    b->events.resize((size_t)NUM_EVENTS * enable);
    for (auto& ev : b->events) HIPCHK(hipEventCreate(&ev));
    b->ev_sets = (uint32_t)enable;
  }
  return 0;
}
extern "C" int rf_amd_batch_timings_back(rf_amd_batch* b, uint32_t back, float* ms, uint32_t n) {
  if (!b || b->events.empty() || !ms || n < RF_AMD_NUM_TIMINGS) return fail(RF_AMD_EINVAL, "timing not enabled");
  if (back >= b->ev_sets) return fail(RF_AMD_EINVAL, "timing set out of range");
  HIPCHK(hipSetDevice(b->eng->device));
  const hipEvent_t* ev = b->events.data() + (size_t)((b->ev_set + b->ev_sets - back) % b->ev_sets) * NUM_EVENTS;
  static const int pairs[RF_AMD_NUM_TIMINGS][2] = {
      {EV_B_START, EV_B_HASH},    {EV_B_HASH, EV_B_SCAN},     {EV_B_SCAN, EV_B_SCATTER},
      {EV_B_SCATTER, EV_B_SORT},  {EV_B_SORT, EV_B_SORT_BIG}, {EV_B_SORT_BIG, EV_B_LAYOUT},
      {EV_B_LAYOUT, EV_B_ASSEMBLE}, {EV_B_START, EV_B_ASSEMBLE}, {EV_P_START, EV_P_END}};
  for (uint32_t i = 0; i < RF_AMD_NUM_TIMINGS; i++) {
    ms[i] = -1.f;
    if (!(b->ev_mask >> pairs[i][0] & 1u) || !(b->ev_mask >> pairs[i][1] & 1u)) continue;  // not recorded
    if (hipEventSynchronize(ev[pairs[i][1]]) != hipSuccess) continue;
    float t = 0;
    if (hipEventElapsedTime(&t, ev[pairs[i][0]], ev[pairs[i][1]]) == hipSuccess) ms[i] = t;
  }
  (void)hipGetLastError();  // a stage not run yet (e.g. no probe) must not poison later launches
  return 0;
}
extern "C" int rf_amd_batch_timings(rf_amd_batch* b, float* ms, uint32_t n) {
  return rf_amd_batch_timings_back(b, 0, ms, n);
}

extern "C" int rf_amd_batch_info(rf_amd_batch* b, uint32_t f, rf_amd_filter_info* out) {
  if (!b || f >= b->F || !out) return fail(RF_AMD_EINVAL, "bad batch/filter");
  HIPCHK(hipSetDevice(b->eng->device));
  FilterOut o;
  if (int rc = wait_built(b)) return rc;
  hipStream_t st = b->eng->stream;
  HIPCHK(hipMemcpyAsync(&o, b->d_outs.as<FilterOut>() + f, sizeof(o), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const FilterPlan& p = b->plans[f];
  out->num_fingerprints = p.num_fp;
  out->num_unique = o.num_unique;
  out->value_size = p.vs;
  out->num_indices = p.num_indices;
  out->num_pages = o.num_pages;
  out->error = o.error;
  return 0;
}

// every filter's info with one copy (rf_amd_batch_info per filter synchronises F times)
extern "C" int rf_amd_batch_infos(rf_amd_batch* b, rf_amd_filter_info* out, void* stream) {
  if (!b || !out) return fail(RF_AMD_EINVAL, "bad batch");
  HIPCHK(hipSetDevice(b->eng->device));
  std::vector<FilterOut> o(b->F);
  if (stream) {  // the build was issued on `stream`: wait for it alone
    HIPCHK(hipMemcpyAsync(o.data(), b->d_outs.p, sizeof(FilterOut) * b->F, hipMemcpyDeviceToHost,
                          (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  } else {  // wherever the build ran: its event, then a copy on the engine stream
    if (int rc = wait_built(b)) return rc;
    HIPCHK(hipMemcpyAsync(o.data(), b->d_outs.p, sizeof(FilterOut) * b->F, hipMemcpyDeviceToHost, b->eng->stream));
    HIPCHK(hipStreamSynchronize(b->eng->stream));
  }
  {
    std::lock_guard<std::mutex> lk(b->err_mu);
    b->err_host.resize(b->F);
    for (uint32_t f = 0; f < b->F; f++) b->err_host[f] = o[f].error;
    b->err_ready.store(true, std::memory_order_release);
  }
  for (uint32_t f = 0; f < b->F; f++) {
    const FilterPlan& p = b->plans[f];
    out[f].num_fingerprints = p.num_fp;
    out[f].num_unique = o[f].num_unique;
    out[f].value_size = p.vs;
    out[f].num_indices = p.num_indices;
    out[f].num_pages = o[f].num_pages;
    out[f].error = o[f].error;
  }
  return 0;
}

extern "C" int rf_amd_batch_read_image(rf_amd_batch* b, uint32_t f, uint8_t* h_pages, uint64_t pages_bytes,
                                       uint64_t* h_slots, uint32_t num_slots) {
  rf_amd_filter_info info;
  if (int rc = rf_amd_batch_info(b, f, &info)) return rc;
  if (info.error) return fail(RF_AMD_EINVAL, "filter build reported error bits");
  const FilterPlan& p = b->plans[f];
  const uint64_t need = (uint64_t)info.num_pages * b->cfg.page_size;
  hipStream_t st = b->eng->stream;  // after rf_amd_batch_info waited for the build
  if (h_pages) {
    if (pages_bytes < need) return fail(RF_AMD_EINVAL, "pages buffer too small");
    HIPCHK(hipMemcpyAsync(h_pages, b->d_pages.as<uint8_t>() + (uint64_t)p.page_base * b->cfg.page_size, need,
                          hipMemcpyDeviceToHost, st));
  }
  if (h_slots) {
    if (num_slots < p.num_indices) return fail(RF_AMD_EINVAL, "slots buffer too small");
    HIPCHK(hipMemcpyAsync(h_slots, b->d_slots.as<uint64_t>() + p.idx_base, 8ull * p.num_indices,
                          hipMemcpyDeviceToHost, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

extern "C" int rf_amd_batch_read_image_async(rf_amd_batch* b, uint32_t f, void* h_pages, uint64_t pages_bytes,
                                             void* h_slots, uint32_t num_slots, void* stream) {
  if (!b || f >= b->F) return fail(RF_AMD_EINVAL, "bad batch/filter");
  const FilterPlan& p = b->plans[f];
  if (pages_bytes > (uint64_t)p.page_cap * b->cfg.page_size || num_slots > p.num_indices)
    return fail(RF_AMD_EINVAL, "copy larger than the filter's reservation");
  HIPCHK(hipSetDevice(b->eng->device));
  hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
  if (h_pages && pages_bytes)
    HIPCHK(hipMemcpyAsync(h_pages, b->d_pages.as<uint8_t>() + (uint64_t)p.page_base * b->cfg.page_size,
                          pages_bytes, hipMemcpyDeviceToHost, st));
  if (h_slots && num_slots)
    HIPCHK(hipMemcpyAsync(h_slots, b->d_slots.as<uint64_t>() + p.idx_base, 8ull * num_slots,
                          hipMemcpyDeviceToHost, st));
  return 0;
}

extern "C" int rf_amd_batch_image_ptrs(rf_amd_batch* b, uint32_t f, void** d_pages, void** d_slots) {
  if (!b || f >= b->F) return fail(RF_AMD_EINVAL, "bad batch/filter");
  const FilterPlan& p = b->plans[f];
  if (d_pages) *d_pages = b->d_pages.as<uint8_t>() + (uint64_t)p.page_base * b->cfg.page_size;
  if (d_slots) *d_slots = b->d_slots.as<uint64_t>() + p.idx_base;
  return 0;
}

// ---- image batches: images (host or device) imported as a built, probe-only batch --------
// Filter f's pages are the num_pages[f] * page_size bytes after those of filters < f in
// `pages`, its index slots (relocatable, filter-relative) the num_indices[f] u64 after
// those of filters < f in `slots`. Probe lines are cut from the images by k_plines.
static int batch_import(rf_amd_engine* e, const rf_amd_config* cfg, uint32_t F, const rf_amd_filter_info* infos,
                        const void* pages, const uint64_t* slots, hipMemcpyKind kind, rf_amd_batch** out) {
  if (int rc = check_cfg(cfg)) return rc;
  if (F == 0 || !infos || !pages || !slots) return fail(RF_AMD_EINVAL, "bad image");
  HIPCHK(hipSetDevice(e->device));
  auto* b = new rf_amd_batch();
  b->eng = e;
  b->cfg = *cfg;
  b->F = F;
  b->plans.resize(F);
  const uint32_t lis = cfg->log_index_size;
  std::vector<uint4> pp(F);
  std::vector<uint32_t> idx_filter;
  uint64_t pages_total = 0, idx_total = 0, lines_total = 0;
  for (uint32_t f = 0; f < F; f++) {
    const rf_amd_filter_info& in = infos[f];
    FilterPlan& p = b->plans[f];
    memset(&p, 0, sizeof(p));
    uint32_t lnb = in.num_fingerprints ? 31 - __builtin_clz(in.num_fingerprints) : 0;
    if (lnb < lis) lnb = lis;
    if (in.num_fingerprints == 0 || lnb > cfg->fingerprint_size || (1u << (lnb - lis)) > MAX_INDICES ||
        in.num_indices != (1u << (lnb - lis)) || in.value_size > 32 - cfg->fingerprint_size || in.error ||
        in.num_pages == 0) {
      delete b;
      return fail(RF_AMD_EINVAL, "image geometry out of range (filter " + std::to_string(f) + ")");
    }
    p.num_fp = in.num_fingerprints;
    p.lnb = lnb;
    p.vs = in.value_size;
    p.rem = cfg->fingerprint_size - lnb;
    p.rvs = p.rem + p.vs;
    p.num_indices = in.num_indices;
    p.page_cap = in.num_pages;
    p.page_base = (uint32_t)pages_total;
    p.idx_base = (uint32_t)idx_total;
    p.lg_line = line_log_group(lis, p.rvs, (double)in.num_fingerprints / (double)(1ull << lnb));
    p.line_base = (uint32_t)lines_total;
    pp[f] = make_uint4(p.vs | (p.rem << 8) | (p.rvs << 16) | (p.lg_line << 24), p.line_base, p.idx_base, 0);
    if (p.lg_line) {
      lines_total += (uint64_t)p.num_indices << (lis - (p.lg_line - 1));
      b->line_lmax = std::max(b->line_lmax, (1u << lis) >> (p.lg_line - 1));
      b->plines_needed = true;
    }
    idx_filter.insert(idx_filter.end(), p.num_indices, f);
    pages_total += in.num_pages;
    idx_total += p.num_indices;
  }
  if (lines_total >= (1ull << 32) || pages_total >= (1ull << 32)) {
    delete b;
    return fail(RF_AMD_EINVAL, "import too large");
  }
  b->PS = (uint32_t)pages_total;
  b->I = (uint32_t)idx_total;
  b->NL = lines_total;
  const size_t page_bytes = (size_t)pages_total * cfg->page_size;
  DevPool* pool = &e->pool;
  int rc = b->d_plans.alloc(sizeof(FilterPlan) * F, pool);
  rc |= b->d_pplans.alloc(16ull * F, pool);
  rc |= b->d_pages.alloc(page_bytes + 256, pool);
  rc |= b->d_slots.alloc(8ull * idx_total, pool);
  rc |= b->d_lines.alloc(64ull * b->NL + 64, pool);
  rc |= b->d_idx_filter.alloc(4ull * idx_total, pool);
  rc |= b->d_outs.alloc(sizeof(FilterOut) * F, pool);
  if (rc) {
    delete b;
    return fail(RF_AMD_ENOMEM, "device allocation failed");
  }
  std::vector<FilterOut> outs(F);
  for (uint32_t f = 0; f < F; f++) outs[f] = FilterOut{infos[f].num_unique, infos[f].num_pages, 0u, 0u};
  hipStream_t st = e->stream;
  HIPCHK(hipMemcpyAsync(b->d_outs.p, outs.data(), sizeof(FilterOut) * F, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(b->d_pages.as<uint8_t>() + page_bytes, 0, 256, st));
  HIPCHK(hipMemcpyAsync(b->d_pages.p, pages, page_bytes, kind, st));
  HIPCHK(hipMemcpyAsync(b->d_slots.p, slots, 8ull * idx_total, kind, st));
  HIPCHK(hipMemcpyAsync(b->d_idx_filter.p, idx_filter.data(), 4ull * idx_total, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(b->d_plans.p, b->plans.data(), sizeof(FilterPlan) * F, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(b->d_pplans.p, pp.data(), 16ull * F, hipMemcpyHostToDevice, st));
  {
    LaunchArgs a = make_args(b, st);
    if (int lrc = rf_launch_plines(&a)) {
      delete b;
      return fail(RF_AMD_EINVAL, std::string("probe-line launch: ") + hipGetErrorString((hipError_t)lrc));
    }
  }
  HIPCHK(hipStreamSynchronize(st));  // host vectors above are released on return
  if (int erc = note_built(b, st)) {
    delete b;
    return erc;
  }
  b->err_host.assign(F, 0u);  // imports carry no error bits (checked above)
  b->err_ready.store(true, std::memory_order_release);
  b->built = true;
  *out = b;
  return 0;
}

static int batch_from_image(rf_amd_engine* e, const rf_amd_config* cfg, const rf_amd_image* img,
                            rf_amd_batch** out) {
  if (!img || !img->pages || !img->slots || img->info.num_fingerprints == 0)
    return fail(RF_AMD_EINVAL, "bad image");
  return batch_import(e, cfg, 1, &img->info, img->pages, img->slots, hipMemcpyHostToDevice, out);
}

extern "C" int rf_amd_batch_export(rf_amd_batch* b, void* d_pages, uint64_t pages_bytes, uint64_t* d_slots,
                                   uint64_t num_slots, void* stream) {
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "export of an unbuilt batch");
  uint64_t po = 0, so = 0;
  std::vector<rf_amd_filter_info> inf(b->F);
  for (uint32_t f = 0; f < b->F; f++) {
    if (int rc = rf_amd_batch_info(b, f, &inf[f])) return rc;
    if (inf[f].error) return fail(RF_AMD_EINVAL, "filter build reported error bits");
    po += (uint64_t)inf[f].num_pages * b->cfg.page_size;
    so += inf[f].num_indices;
  }
  if (!d_pages || !d_slots || pages_bytes < po || num_slots < so) return fail(RF_AMD_EINVAL, "export buffers too small");
  hipStream_t st = stream ? (hipStream_t)stream : b->eng->stream;
  po = so = 0;
  for (uint32_t f = 0; f < b->F; f++) {
    const FilterPlan& p = b->plans[f];
    const uint64_t pb = (uint64_t)inf[f].num_pages * b->cfg.page_size;
    HIPCHK(hipMemcpyAsync(static_cast<uint8_t*>(d_pages) + po,
                          b->d_pages.as<uint8_t>() + (uint64_t)p.page_base * b->cfg.page_size, pb,
                          hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(d_slots + so, b->d_slots.as<uint64_t>() + p.idx_base, 8ull * p.num_indices,
                          hipMemcpyDeviceToDevice, st));
    po += pb;
    so += p.num_indices;
  }
  return 0;
}

extern "C" int rf_amd_batch_import(rf_amd_engine* e, const rf_amd_config* cfg, uint32_t num_filters,
                                   const rf_amd_filter_info* infos, const void* pages, const uint64_t* slots,
                                   int device_resident, rf_amd_batch** out) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (!out) return fail(RF_AMD_EINVAL, "null out-param");
  *out = nullptr;
  return batch_import(e, cfg, num_filters, infos, pages, slots,
                      device_resident ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, out);
}

extern "C" int rf_amd_filter_add(rf_amd_engine* e, const rf_amd_config* cfg, const rf_amd_image* old_filter,
                                 rf_amd_image* filter, const uint32_t* new_fp_arr, uint64_t num_new_fp,
                                 uint16_t value) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (!filter) return fail(RF_AMD_EINVAL, "null filter out-param");
  memset(filter, 0, sizeof(*filter));
  if (num_new_fp && !new_fp_arr) return fail(RF_AMD_EINVAL, "null fingerprint array");
  if (num_new_fp > 0xffffffffull) return fail(RF_AMD_EINVAL, "too many fingerprints");
  rf_amd_batch* ob = nullptr;
  const bool has_old = old_filter && old_filter->pages && old_filter->info.num_fingerprints;
  if (has_old)
    if (int rc = batch_from_image(e, cfg, old_filter, &ob)) return rc;
  rf_amd_batch* b = nullptr;
  const uint32_t n32 = (uint32_t)num_new_fp;
  uint32_t zero = 0;
  int rc = rf_amd_batch_create(e, cfg, 1, &n32, &value, has_old ? &ob : nullptr, has_old ? &zero : nullptr, &b);
  if (rc) {
    rf_amd_batch_destroy(ob);
    return rc;
  }
  DevBuf d_h;
  if ((rc = d_h.alloc(4ull * num_new_fp + 16)) == 0) {
    hipError_t he = hipMemcpyAsync(d_h.p, new_fp_arr, 4ull * num_new_fp, hipMemcpyHostToDevice, e->stream);
    if (he != hipSuccess) rc = fail(RF_AMD_EINVAL, "H2D failed");
  }
  if (!rc) rc = rf_amd_batch_build_hashes(b, d_h.as<uint32_t>(), nullptr);
  rf_amd_filter_info info{};
  if (!rc) rc = rf_amd_batch_info(b, 0, &info);
  if (!rc && info.error) rc = fail(RF_AMD_EINVAL, "filter exceeds the on-disk format (error bits set)");
  if (!rc) {
    filter->info = info;
    filter->pages = (uint8_t*)calloc((size_t)info.num_pages * cfg->page_size + 16, 1);
    filter->slots = (uint64_t*)calloc(info.num_indices, 8);
    if (!filter->pages || !filter->slots) rc = fail(RF_AMD_ENOMEM, "host allocation failed");
  }
  if (!rc) rc = rf_amd_batch_read_image(b, 0, filter->pages, (uint64_t)info.num_pages * cfg->page_size,
                                        filter->slots, info.num_indices);
  if (rc) rf_amd_image_free(filter);
  rf_amd_batch_destroy(b);
  rf_amd_batch_destroy(ob);
  return rc;
}

extern "C" int rf_amd_filter_lookup_hashes(rf_amd_engine* e, const rf_amd_config* cfg, const rf_amd_image* filter,
                                           const uint32_t* hashes, uint64_t n, uint64_t* found_values) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (!filter || !filter->pages) {  // NULL filter finds nothing (src/routing_filter.c:1003-1006)
    if (found_values) memset(found_values, 0, 8 * n);
    return 0;
  }
  if (n == 0) return 0;
  rf_amd_batch* b = nullptr;
  if (int rc = batch_from_image(e, cfg, filter, &b)) return rc;
  DevBuf d_h, d_f, d_id;
  int rc = d_h.alloc(4 * n) | d_f.alloc(8 * n) | d_id.alloc(4 * n);
  if (!rc) {
    hipStream_t st = e->stream;
    if (hipMemcpyAsync(d_h.p, hashes, 4 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemsetAsync(d_id.p, 0, 4 * n, st) != hipSuccess)
      rc = fail(RF_AMD_EINVAL, "H2D failed");
    if (!rc) rc = rf_amd_batch_probe_hashes(b, d_h.as<uint32_t>(), d_id.as<uint32_t>(), n, d_f.as<uint64_t>(), st);
    if (!rc && (hipMemcpyAsync(found_values, d_f.p, 8 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess))
      rc = fail(RF_AMD_EINVAL, "D2H failed");
  }
  rf_amd_batch_destroy(b);
  return rc;
}

extern "C" int rf_amd_filter_lookup_keys(rf_amd_engine* e, const rf_amd_config* cfg, const rf_amd_image* filter,
                                         const void* keys, uint32_t key_len, uint64_t n, uint64_t* found_values) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (!filter || !filter->pages) {
    if (found_values) memset(found_values, 0, 8 * n);
    return 0;
  }
  if (n == 0) return 0;
  if (!keys || key_len == 0) return fail(RF_AMD_EINVAL, "null keys");
  rf_amd_batch* b = nullptr;
  if (int rc = batch_from_image(e, cfg, filter, &b)) return rc;
  DevBuf d_k, d_f, d_id;
  int rc = d_k.alloc((size_t)key_len * n + 16) | d_f.alloc(8 * n) | d_id.alloc(4 * n);
  if (!rc) {
    hipStream_t st = e->stream;
    if (hipMemcpyAsync(d_k.p, keys, (size_t)key_len * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemsetAsync(d_id.p, 0, 4 * n, st) != hipSuccess)
      rc = fail(RF_AMD_EINVAL, "H2D failed");
    if (!rc) rc = rf_amd_batch_probe_keys(b, d_k.p, key_len, d_id.as<uint32_t>(), n, d_f.as<uint64_t>(), st);
    if (!rc && (hipMemcpyAsync(found_values, d_f.p, 8 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess))
      rc = fail(RF_AMD_EINVAL, "D2H failed");
  }
  rf_amd_batch_destroy(b);
  return rc;
}

extern "C" void rf_amd_image_free(rf_amd_image* img) {
  if (!img) return;
  free(img->pages);
  free(img->slots);
  img->pages = nullptr;
  img->slots = nullptr;
}

extern "C" uint64_t rf_amd_max_fingerprints(const rf_amd_config* cfg) {
  const uint64_t addrs_per_extent = (uint64_t)cfg->page_size * cfg->pages_per_extent / 8;
  return 2ull * addrs_per_extent * (1ull << cfg->log_index_size) - 1;
}

// src/routing_filter.c:1119-1139 as the reference's release build evaluates it (-O3
// -ffast-math, Makefile:89,123-124: GCC reassociates the sum into two fused multiply-adds and
// truncates through 64 bits). The order decides the result where the exact value is an
// integer (num_unique = 1: exactly 1 there, 0 in source order); oracle/rf_oracle.c holds the
// same restatement, pinned against the reference for fingerprint sizes 8-32.
extern "C" uint32_t rf_amd_estimate_unique_keys_from_count(const rf_amd_config* cfg, uint64_t num_unique) {
#pragma clang fp contract(off)
  const double U = (double)(1ull << cfg->fingerprint_size);
  const double s = U - (double)num_unique;
  const double U2 = U * U, s2 = s * s;
  const double lU = log(U), ls = log(s);
  const double a = fma(1.0 / U - 1.0 / s, 0.5, (1.0 / s2 - 1.0 / U2) * (1.0 / 12.0));
  const double b = fma(1.0 / (U2 * U2) - 1.0 / (s2 * s2), 1.0 / 120.0, lU);
  return (uint32_t)(int64_t)(U * ((a + b) - ls));
}

extern "C" uint64_t rf_amd_space_use_bytes(const rf_amd_config* cfg, uint32_t num_pages) {
  const uint64_t extent = (uint64_t)cfg->page_size * cfg->pages_per_extent;
  return cfg->page_size + extent * (1 + (num_pages + cfg->pages_per_extent - 1) / cfg->pages_per_extent);
}

// ---- routing_filter_estimate_unique_fp (src/routing_filter.c:702-848) --------------------
extern "C" int rf_launch_estimate(void* stream, const EstFilter* fl, uint32_t num_filters, uint32_t total_idx,
                                  uint32_t lis, uint32_t* bitmap, uint64_t bitmap_words, uint32_t* counters);
constexpr uint64_t EST_MAX_FILTERS = 32;  // MAX_FILTERS, src/routing_filter.h:25

// fl: the filters to decode (pages/slots already device pointers, idx_first unset);
// total_num_fp: the reference's uint32 sum of num_fingerprints over ALL filters (:719-722)
static int estimate_run(rf_amd_engine* e, hipStream_t st, const rf_amd_config* cfg, std::vector<EstFilter>& fl,
                        uint32_t total_num_fp, uint32_t* num_unique_fp) {
  uint32_t total_idx = 0;
  for (auto& f : fl) {
    f.idx_first = total_idx;
    total_idx += f.num_idx;
  }
  const uint32_t ubits = cfg->fingerprint_size > 4 ? cfg->fingerprint_size - 4 : 0;  // fps < 2^(fp_size-4)
  uint64_t words = ((1ull << ubits) + 31) / 32;
  words = (words + 3) & ~3ull;
  DevBuf d_fl, d_bm, d_cnt;
  if (d_fl.alloc(sizeof(EstFilter) * (fl.size() + 1)) || d_bm.alloc(4 * words) || d_cnt.alloc(16))
    return fail(RF_AMD_ENOMEM, "device allocation failed");
  if (!fl.empty())
    HIPCHK(hipMemcpyAsync(d_fl.p, fl.data(), sizeof(EstFilter) * fl.size(), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(d_bm.p, 0, 4 * words, st));
  HIPCHK(hipMemsetAsync(d_cnt.p, 0, 16, st));
  if (rf_launch_estimate(st, d_fl.as<EstFilter>(), (uint32_t)fl.size(), total_idx, cfg->log_index_size,
                         d_bm.as<uint32_t>(), words, d_cnt.as<uint32_t>()))
    return fail(RF_AMD_EINVAL, "estimate kernel launch failed");
  uint32_t cnt[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(cnt, d_cnt.p, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  (void)e;
  // the reference unpacks every decoded entry into a total_num_fp / 12 buffer and asserts
  // it fits (:776-780); the running count only grows, so this is the same condition
  if (cnt[0] > total_num_fp / 12)
    return fail(RF_AMD_EINVAL, "decoded fingerprints exceed num_fingerprints / 12 (reference asserts, :776)");
  *num_unique_fp = cnt[1] * 16;
  return 0;
}

static uint32_t est_lnb(const rf_amd_config* cfg, uint32_t num_fp) {
  uint32_t lnb = num_fp ? 31 - __builtin_clz(num_fp) : 0;
  return lnb < cfg->log_index_size ? cfg->log_index_size : lnb;
}

extern "C" int rf_amd_estimate_unique_fp(rf_amd_engine* e, const rf_amd_config* cfg, const rf_amd_image* filters,
                                         uint64_t num_filters, uint32_t* num_unique_fp) {
  if (!num_unique_fp) return fail(RF_AMD_EINVAL, "num_unique_fp must not be NULL");  // :710-714
  *num_unique_fp = 0;
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (int rc = check_cfg(cfg)) return rc;
  if (num_filters > EST_MAX_FILTERS) return fail(RF_AMD_EINVAL, "more than MAX_FILTERS filters (:717)");
  if (num_filters && !filters) return fail(RF_AMD_EINVAL, "null filters");
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = e->stream;
  uint32_t total_num_fp = 0;
  std::vector<EstFilter> fl;
  std::vector<DevBuf> bufs(2 * num_filters);
  for (uint64_t i = 0; i < num_filters; i++) {
    const rf_amd_image& im = filters[i];
    total_num_fp += im.info.num_fingerprints;
    if (!im.pages || !im.slots) continue;  // filter.addr == 0 (:739-742)
    const uint32_t lnb = est_lnb(cfg, im.info.num_fingerprints);
    if (lnb > cfg->fingerprint_size || lnb - cfg->log_index_size > 14)
      return fail(RF_AMD_EINVAL, "image geometry out of range");
    const uint32_t num_indices = 1u << (lnb - cfg->log_index_size);
    if (num_indices < 16) continue;  // "the filter is too small forget it" (:755)
    if (cfg->fingerprint_size + im.info.value_size > 32) return fail(RF_AMD_EINVAL, "fp_size + value_size > 32");
    const uint32_t nidx = num_indices / 16;
    uint64_t last_page = 0;  // upload only the pages the decoded indices live on
    for (uint32_t k = 0; k < nidx; k++) last_page = std::max<uint64_t>(last_page, im.slots[k] / cfg->page_size);
    if (last_page >= im.info.num_pages) return fail(RF_AMD_EINVAL, "index slot outside the image");
    const uint64_t pbytes = (last_page + 1) * cfg->page_size;
    DevBuf& dp = bufs[2 * i];
    DevBuf& ds = bufs[2 * i + 1];
    if (dp.alloc(pbytes + 256) || ds.alloc(8ull * nidx)) return fail(RF_AMD_ENOMEM, "device allocation failed");
    HIPCHK(hipMemsetAsync(dp.as<uint8_t>() + pbytes, 0, 256, st));
    HIPCHK(hipMemcpyAsync(dp.p, im.pages, pbytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(ds.p, im.slots, 8ull * nidx, hipMemcpyHostToDevice, st));
    const uint32_t rem = cfg->fingerprint_size - lnb;
    fl.push_back(EstFilter{dp.as<uint8_t>(), ds.as<uint64_t>(), im.info.value_size, rem + im.info.value_size, nidx, 0});
  }
  return estimate_run(e, st, cfg, fl, total_num_fp, num_unique_fp);
}

extern "C" int rf_amd_batch_estimate_unique_fp(rf_amd_batch* const* batches, const uint32_t* filter_index,
                                               uint64_t num_filters, uint32_t* num_unique_fp) {
  if (!num_unique_fp) return fail(RF_AMD_EINVAL, "num_unique_fp must not be NULL");
  *num_unique_fp = 0;
  if (num_filters > EST_MAX_FILTERS) return fail(RF_AMD_EINVAL, "more than MAX_FILTERS filters (:717)");
  if (num_filters == 0) return 0;
  if (!batches || !filter_index) return fail(RF_AMD_EINVAL, "null batch list");
  rf_amd_engine* e = nullptr;
  const rf_amd_config* cfg = nullptr;
  uint32_t total_num_fp = 0;
  std::vector<EstFilter> fl;
  for (uint64_t i = 0; i < num_filters; i++) {
    rf_amd_batch* b = batches[i];
    if (!b) continue;  // NULL_ROUTING_FILTER
    const uint32_t f = filter_index[i];
    if (f >= b->F || !b->built) return fail(RF_AMD_EINVAL, "bad batch/filter (not built)");
    if (!e) {
      e = b->eng;
      cfg = &b->cfg;
    } else if (b->eng != e || memcmp(&b->cfg, cfg, sizeof(*cfg)) != 0) {
      return fail(RF_AMD_EINVAL, "filters of one estimate must share an engine and a routing config");
    }
    const FilterPlan& p = b->plans[f];
    total_num_fp += p.num_fp;
    if (p.num_indices < 16) continue;
    fl.push_back(EstFilter{b->d_pages.as<uint8_t>() + (uint64_t)p.page_base * b->cfg.page_size,
                           b->d_slots.as<uint64_t>() + p.idx_base, p.vs, p.rvs, p.num_indices / 16, 0});
  }
  if (!e) return 0;
  HIPCHK(hipSetDevice(e->device));
  // the images must be complete (and error-free) before they are decoded
  for (uint64_t i = 0; i < num_filters; i++) {
    if (!batches[i]) continue;
    rf_amd_filter_info info;
    if (int rc = rf_amd_batch_info(batches[i], filter_index[i], &info)) return rc;
    if (info.error) return fail(RF_AMD_EINVAL, "filter build reported error bits");
  }
  return estimate_run(e, e->stream, cfg, fl, total_num_fp, num_unique_fp);
}

extern "C" uint32_t rf_amd_estimate_unique_keys(const rf_amd_filter_info* filter, const rf_amd_config* cfg) {
  return rf_amd_estimate_unique_keys_from_count(cfg, filter->num_unique);  // .c:1141-1146
}

// ---- asynchronous batched lookup (routing_filter_lookup_async, src/routing_filter.h:130-155,
// .c:895-972) ---------------------------------------------------------------------------
// The reference's coroutine yields while a filter page is read and calls `callback` when it
// can be resumed; here one call stages a whole batch of lookups (H2D, probe, D2H) on a
// stream and the callback fires from a HIP host function once the results are in h_found.
struct rf_amd_lookup_async_state {
  rf_amd_batch* b = nullptr;
  hipStream_t st = nullptr;
  uint64_t n = 0;
  uint64_t* h_found = nullptr;
  void* h_stage = nullptr;  // pinned: keys in, found values out
  size_t stage_bytes = 0;
  DevBuf d_keys, d_fid, d_found;
  hipEvent_t done_ev = nullptr;
  rf_amd_callback_fn cb = nullptr;
  void* cb_arg = nullptr;
  volatile int done = 0;
  ~rf_amd_lookup_async_state() {
    if (done_ev) (void)hipEventSynchronize(done_ev);
    if (done_ev) (void)hipEventDestroy(done_ev);
    if (h_stage) (void)hipHostFree(h_stage);
  }
};

static void lookup_async_finish(void* arg) {  // HIP host function: no HIP calls in here
  auto* s = static_cast<rf_amd_lookup_async_state*>(arg);
  memcpy(s->h_found, s->h_stage, 8 * s->n);
  __atomic_store_n(&s->done, 1, __ATOMIC_RELEASE);
  if (s->cb) s->cb(s->cb_arg);
}

extern "C" int rf_amd_lookup_async(rf_amd_batch* b, const void* h_keys, uint32_t key_len,
                                   const uint32_t* h_filter_id, uint64_t n, uint64_t* h_found,
                                   rf_amd_callback_fn callback, void* callback_arg, void* stream,
                                   rf_amd_lookup_async_state** out) {
  if (!out) return fail(RF_AMD_EINVAL, "null state out-param");
  *out = nullptr;
  if (!b || !b->built) return fail(RF_AMD_EINVAL, "batch not built");
  if (n && (!h_keys || !h_found || key_len == 0)) return fail(RF_AMD_EINVAL, "null keys / results");
  HIPCHK(hipSetDevice(b->eng->device));
  auto* s = new rf_amd_lookup_async_state();
  s->b = b;
  s->st = stream ? (hipStream_t)stream : b->eng->stream;
  s->n = n;
  s->h_found = h_found;
  s->cb = callback;
  s->cb_arg = callback_arg;
  const size_t kbytes = (size_t)key_len * n;
  s->stage_bytes = std::max<size_t>(std::max<size_t>(kbytes, 8 * n), 16);
  int rc = 0;
  if (hipHostMalloc(&s->h_stage, s->stage_bytes, hipHostMallocDefault) != hipSuccess) {
    s->h_stage = nullptr;
    rc = fail(RF_AMD_ENOMEM, "pinned staging allocation failed");
  }
  if (!rc) rc = s->d_keys.alloc(kbytes + 16) | s->d_fid.alloc(4 * n + 16) | s->d_found.alloc(8 * n + 16);
  if (!rc && hipEventCreateWithFlags(&s->done_ev, hipEventDisableTiming) != hipSuccess)
    rc = fail(RF_AMD_EINVAL, "event creation failed");
  if (rc) {
    delete s;
    return rc;
  }
  if (n) {
    memcpy(s->h_stage, h_keys, kbytes);
    if (hipMemcpyAsync(s->d_keys.p, s->h_stage, kbytes, hipMemcpyHostToDevice, s->st) != hipSuccess ||
        (h_filter_id ? hipMemcpyAsync(s->d_fid.p, h_filter_id, 4 * n, hipMemcpyHostToDevice, s->st)
                     : hipMemsetAsync(s->d_fid.p, 0, 4 * n, s->st)) != hipSuccess)
      rc = fail(RF_AMD_EINVAL, "H2D failed");
    if (!rc) rc = rf_amd_batch_probe_keys(b, s->d_keys.p, key_len, s->d_fid.as<uint32_t>(), n,
                                          s->d_found.as<uint64_t>(), s->st);
    // the keys' staging copy has been consumed once the probe ran: reuse it for the results
    if (!rc && hipMemcpyAsync(s->h_stage, s->d_found.p, 8 * n, hipMemcpyDeviceToHost, s->st) != hipSuccess)
      rc = fail(RF_AMD_EINVAL, "D2H failed");
  }
  if (!rc && hipLaunchHostFunc(s->st, lookup_async_finish, s) != hipSuccess)
    rc = fail(RF_AMD_EINVAL, "host function launch failed");
  if (!rc && hipEventRecord(s->done_ev, s->st) != hipSuccess) rc = fail(RF_AMD_EINVAL, "event record failed");
  if (rc) {
    (void)hipStreamSynchronize(s->st);
    delete s;
    return rc;
  }
  *out = s;
  return 0;
}

extern "C" int rf_amd_lookup_async_poll(rf_amd_lookup_async_state* s) {
  if (!s) return RF_AMD_ASYNC_DONE;
  return __atomic_load_n(&s->done, __ATOMIC_ACQUIRE) ? RF_AMD_ASYNC_DONE : RF_AMD_ASYNC_RUNNING;
}

extern "C" int rf_amd_lookup_async_wait(rf_amd_lookup_async_state* s) {
  if (!s) return 0;
  HIPCHK(hipEventSynchronize(s->done_ev));
  while (!__atomic_load_n(&s->done, __ATOMIC_ACQUIRE)) {
  }
  return 0;
}

extern "C" void rf_amd_lookup_async_free(rf_amd_lookup_async_state* s) {
  if (!s) return;
  (void)rf_amd_lookup_async_wait(s);
  delete s;
}

// ---- batch hashing (data_key_hash, btree_pack's fingerprint loop) -------------------------
extern "C" int rf_launch_hash(void* stream, int kind, const void* in0, const uint64_t* offs, uint32_t key_len,
                              uint32_t seed, uint64_t n, uint32_t* out);

extern "C" int rf_amd_hash_keys(rf_amd_engine* e, const rf_amd_config* cfg, const void* d_keys, uint32_t key_len,
                                uint64_t n, uint32_t* d_hashes, void* stream) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (int rc = check_cfg(cfg)) return rc;
  if (n && (!d_keys || !d_hashes || key_len == 0)) return fail(RF_AMD_EINVAL, "null keys / output");
  HIPCHK(hipSetDevice(e->device));
  if (rf_launch_hash(stream ? stream : e->stream, fixed_kind(d_keys, key_len), d_keys, nullptr, key_len, cfg->seed,
                     n, d_hashes))
    return fail(RF_AMD_EINVAL, "hash kernel launch failed");
  return 0;
}

extern "C" int rf_amd_hash_var_keys(rf_amd_engine* e, const rf_amd_config* cfg, const uint8_t* d_bytes,
                                    const uint64_t* d_offsets, uint64_t n, uint32_t* d_hashes, void* stream) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (int rc = check_cfg(cfg)) return rc;
  if (n && (!d_bytes || !d_offsets || !d_hashes)) return fail(RF_AMD_EINVAL, "null keys / output");
  HIPCHK(hipSetDevice(e->device));
  if (rf_launch_hash(stream ? stream : e->stream, IN_VAR, d_bytes, d_offsets, 0, cfg->seed, n, d_hashes))
    return fail(RF_AMD_EINVAL, "hash kernel launch failed");
  return 0;
}

// ---- routed probes across ranks --------------------------------------------
extern "C" uint64_t rf_route_scratch_words(uint64_t n, uint32_t world);
extern "C" int rf_launch_route(void* stream, const uint32_t* hashes, const uint32_t* gfid, uint64_t n,
                               const uint32_t* route, uint32_t num_g, uint32_t world, uint64_t* pairs,
                               uint32_t* perm, uint32_t* scratch, uint64_t* totals);
extern "C" int rf_launch_unroute(void* stream, const uint64_t* back, const uint32_t* perm, uint64_t n,
                                 uint64_t* found);

extern "C" uint64_t rf_amd_route_scratch_bytes(uint64_t n, uint32_t world) {
  return 4 * rf_route_scratch_words(n, world) + 8 + 8 * (uint64_t)RF_AMD_ROUTE_MAX_WORLD;
}

extern "C" int rf_amd_route_probes(rf_amd_engine* e, const uint32_t* d_hashes, const uint32_t* d_filter_id,
                                   uint64_t n, const uint32_t* d_route, uint32_t num_filters, uint32_t world,
                                   uint64_t* d_pairs, uint32_t* d_perm, void* d_scratch, uint64_t* h_counts,
                                   void* stream) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (world == 0 || world > RF_AMD_ROUTE_MAX_WORLD) return fail(RF_AMD_EINVAL, "world out of range");
  if (!h_counts) return fail(RF_AMD_EINVAL, "null counts");
  for (uint32_t d = 0; d < world; d++) h_counts[d] = 0;
  if (n == 0) return 0;
  if (n >= (1ull << 32)) return fail(RF_AMD_EINVAL, "more than 2^32 - 1 probes");
  if (!d_hashes || !d_filter_id || !d_route || !d_pairs || !d_perm || !d_scratch)
    return fail(RF_AMD_EINVAL, "null route buffer");
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = stream ? (hipStream_t)stream : e->stream;
  uint32_t* scratch = static_cast<uint32_t*>(d_scratch);
  const uint64_t words = rf_route_scratch_words(n, world);
  uint64_t* d_tot = reinterpret_cast<uint64_t*>(scratch + ((words + 1) & ~1ull));
  if (rf_launch_route(st, d_hashes, d_filter_id, n, d_route, num_filters, world, d_pairs, d_perm, scratch, d_tot))
    return fail(RF_AMD_EINVAL, "route kernel launch failed");
  uint32_t err = 0;
  HIPCHK(hipMemcpyAsync(h_counts, d_tot, 8 * world, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&err, scratch + words - 4, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (err & 1u) return fail(RF_AMD_EINVAL, "probe filter id out of range");
  if (err & 2u) return fail(RF_AMD_EINVAL, "route table names a rank >= world");
  return 0;
}

extern "C" int rf_amd_unroute_found(rf_amd_engine* e, const uint64_t* d_back, const uint32_t* d_perm, uint64_t n,
                                    uint64_t* d_found, void* stream) {
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (n && (!d_back || !d_perm || !d_found)) return fail(RF_AMD_EINVAL, "null unroute buffer");
  HIPCHK(hipSetDevice(e->device));
  if (rf_launch_unroute(stream ? stream : e->stream, d_back, d_perm, n, d_found))
    return fail(RF_AMD_EINVAL, "unroute kernel launch failed");
  return 0;
}

extern "C" int rf_amd_batch_probe_pairs(rf_amd_batch* b, const uint64_t* d_pairs, uint64_t n, uint64_t* d_found,
                                        void* stream) {
  return do_probe(b, IN_PAIR, d_pairs, nullptr, 8, reinterpret_cast<const uint32_t*>(d_pairs), n, d_found, stream);
}

// ---- routing_filter_verify (src/routing_filter.c:1163-1183) ------------------------------
extern "C" int rf_launch_count_missing(void* stream, const uint64_t* found, uint64_t n, uint32_t value,
                                       unsigned long long* missing);

extern "C" int rf_amd_filter_verify(rf_amd_engine* e, const rf_amd_config* cfg, const rf_amd_image* filter,
                                    const void* keys, uint32_t key_len, uint64_t n, uint16_t value,
                                    uint64_t* num_missing) {
  if (num_missing) *num_missing = 0;
  if (!e) return fail(RF_AMD_ENODEV, "no engine");
  if (value >= 64) return fail(RF_AMD_EINVAL, "value >= 64");
  if (n == 0) return 0;
  if (!keys || key_len == 0) return fail(RF_AMD_EINVAL, "null keys");
  if (!filter || !filter->pages) {  // a NULL filter finds nothing: every key is missing
    if (num_missing) *num_missing = n;
    return fail(RF_AMD_EINVAL, "verify: key not found in a NULL filter");
  }
  rf_amd_batch* b = nullptr;
  if (int rc = batch_from_image(e, cfg, filter, &b)) return rc;
  DevBuf d_k, d_f, d_id, d_m;
  int rc = d_k.alloc((size_t)key_len * n + 16) | d_f.alloc(8 * n) | d_id.alloc(4 * n) | d_m.alloc(8);
  unsigned long long missing = 0;
  if (!rc) {
    hipStream_t st = e->stream;
    if (hipMemcpyAsync(d_k.p, keys, (size_t)key_len * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemsetAsync(d_id.p, 0, 4 * n, st) != hipSuccess || hipMemsetAsync(d_m.p, 0, 8, st) != hipSuccess)
      rc = fail(RF_AMD_EINVAL, "H2D failed");
    if (!rc) rc = rf_amd_batch_probe_keys(b, d_k.p, key_len, d_id.as<uint32_t>(), n, d_f.as<uint64_t>(), st);
    if (!rc && rf_launch_count_missing(st, d_f.as<uint64_t>(), n, value, d_m.as<unsigned long long>()))
      rc = fail(RF_AMD_EINVAL, "verify kernel launch failed");
    if (!rc && (hipMemcpyAsync(&missing, d_m.p, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess))
      rc = fail(RF_AMD_EINVAL, "D2H failed");
  }
  rf_amd_batch_destroy(b);
  if (rc) return rc;
  if (num_missing) *num_missing = missing;
  // the reference asserts routing_filter_is_value_found for every key (:1177)
  return missing ? fail(RF_AMD_EINVAL, "verify: " + std::to_string(missing) + " keys not found") : 0;
}

// ---- routing_filter_print (src/routing_filter.c:1185-1286): debug text, host only ----------
static int print_filter(const rf_amd_config* cfg, const rf_amd_image* filter, uint64_t filter_addr,
                        const uint64_t* abs_slots, void* out_file);

extern "C" int rf_amd_filter_print(const rf_amd_config* cfg, const rf_amd_image* filter, void* out_file) {
  return print_filter(cfg, filter, 0, nullptr, out_file);
}

extern "C" int rf_amd_filter_print_abs(const rf_amd_config* cfg, const rf_amd_image* filter, uint64_t filter_addr,
                                       const uint64_t* abs_slots, void* out_file) {
  if (!abs_slots) return fail(RF_AMD_EINVAL, "null absolute slots");
  return print_filter(cfg, filter, filter_addr, abs_slots, out_file);
}

static int print_filter(const rf_amd_config* cfg, const rf_amd_image* filter, uint64_t filter_addr,
                        const uint64_t* abs_slots, void* out_file) {
  if (int rc = check_cfg(cfg)) return rc;
  if (!filter || !filter->pages || !filter->slots) return fail(RF_AMD_EINVAL, "null filter");
  FILE* fo = out_file ? (FILE*)out_file : stdout;
  const uint32_t lis = cfg->log_index_size, index_size = 1u << lis;
  const uint32_t lnb = est_lnb(cfg, filter->info.num_fingerprints);
  const uint32_t num_indices = 1u << (lnb - lis);
  const uint32_t rem = cfg->fingerprint_size - lnb, vs = filter->info.value_size, rvs = rem + vs;
  const uint8_t* pg = filter->pages;
  auto bit = [&](uint64_t bp) { return (pg[bp >> 3] >> (bp & 7)) & 1u; };
  fprintf(fo, "********************************************************************************\n");
  fprintf(fo, "***   filter INDEX\n");
  fprintf(fo, "***   filter_addr: %lu\n", (unsigned long)filter_addr);
  fprintf(fo, "--------------------------------------------------------------------------------\n");
  for (uint32_t i = 0; i < num_indices; i++)
    fprintf(fo, "index 0x%x: %lu\n", i, (unsigned long)(abs_slots ? abs_slots[i] : filter->slots[i]));
  for (uint32_t i = 0; i < num_indices; i++) {
    const uint64_t h = filter->slots[i];
    const uint32_t c = (uint32_t)pg[h] | ((uint32_t)pg[h + 1] << 8);
    fprintf(fo, "----------------------------------------\n");
    fprintf(fo, "--- Index 0x%x\n", i);
    fprintf(fo, "--- Encoding: %u\n", c);
    const uint64_t eb = (h + 2) * 8;
    for (uint32_t k = 0; k < c + index_size; k++) {
      if (k != 0 && k % 16 == 0) fprintf(fo, " | ");
      fputc(bit(eb + k) ? '1' : '0', fo);
    }
    fputc('\n', fo);
    fprintf(fo, "--- Remainders\n");
    // print_remainders' header_length uses (c + index_size - 1) / 8 + 1 encoding bytes, not
    // the block's + 4 (:1234-1236 vs :207-211): the reference prints from that offset, so do we
    const uint64_t hl = (c + index_size - 1) / 8 + 1 + 2;
    const uint64_t rb = (h + hl) * 8;
    // bucket bounds by walking the unary encoding (routing_get_bucket_bounds, :230-279)
    uint32_t pos = 0, start = 0;
    for (uint32_t bo = 0; bo < index_size; bo++) {
      uint32_t cnt = 0;
      while (pos < c + index_size && !bit(eb + pos)) { pos++; cnt++; }
      pos++;  // the bucket's terminating 1
      fprintf(fo, "0x%x remainders:", bo);
      for (uint32_t j = start; j < start + cnt; j++) {
        uint32_t rv = 0;
        for (uint32_t t = 0; t < rvs; t++) rv |= bit(rb + (uint64_t)j * rvs + t) << t;
        fprintf(fo, " 0x%x:%u", vs >= 32 ? 0u : rv >> vs, rv & (uint32_t)((1ull << vs) - 1));
      }
      fputc('\n', fo);
      start += cnt;
    }
  }
  fflush(fo);
  return 0;
}
