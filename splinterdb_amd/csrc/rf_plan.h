// rf_plan.h -- host/device shared batch plan of the routing-filter engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rf {

// geometry limits (page 4096 B, 32-page extents: 16384 index slots, src/routing_filter.h:120-127)
constexpr uint32_t MAX_PAGE = 4096;
constexpr uint32_t MAX_INDICES = 16384;
constexpr uint32_t MAX_LIS = 12;
constexpr uint32_t CB_LOG_MEAN = 12;  // coarse bucket ~ 2^12..2^13 entries
constexpr uint32_t MAX_CB = 2048;     // coarse buckets per filter (lnb <= 23)
constexpr uint32_t MAX_BINS = 4096;   // filter buckets per coarse bucket
constexpr uint32_t MAX_IPC = 512;     // indices per coarse bucket (2^(12-3))

// kernel shapes
constexpr int TILE_NT = 256;
#ifndef RF_TILE_KEYS
#define RF_TILE_KEYS 16384
#endif
constexpr int TILE_KEYS = RF_TILE_KEYS;  // keys per K1/K3 tile
constexpr int SCAT_NT = 512;
constexpr int SORT_NT = 512;
constexpr int SORT_CAP = 9216;   // entries per coarse bucket held in LDS (means 4096..8192, sd < 91)
#ifndef RF_REGION_PAD
#define RF_REGION_PAD 0
#endif
// fused build: each coarse bucket's region in `part` (SORT_CAP slots, spaced CB_REGION apart)
constexpr uint32_t CB_REGION = SORT_CAP + RF_REGION_PAD;
constexpr int BIG_NT = 1024;
constexpr int BIG_GRID = 64;
constexpr int LAYOUT_NT = 1024;
constexpr int ASM_NT = 128;
constexpr uint32_t ASM_MAXB_HOST = 128;  // = ASM_MAXB in rf_kernels.hip (blocks per page in LDS)
constexpr uint32_t ASM_GT_HOST = 1024;   // = ASM_GT (group-start table entries per page)

enum InputKind { IN_KEYS24 = 0, IN_KEYS_W = 1, IN_KEYS_B = 2, IN_VAR = 3, IN_HASH = 4, IN_PAIR = 5 };

constexpr uint32_t ERR_INDEX_OVERFLOW = 1u, ERR_BLOCK_TOO_BIG = 2u, ERR_PAGE_CAP = 4u,
                   ERR_GEOMETRY = 8u;

struct FilterPlan {
  uint64_t e_first;    // first entry slot of this filter in the entry arrays
  uint64_t key_first;  // first input (key / hash) of this filter's new fingerprints
  uint64_t old_first;  // 32-bit incremental builds: first of its decoded old entries in old32
  uint32_t num_new;    // new fingerprints
  uint32_t old_region; // entry slots reserved for decoded old entries (old num_fingerprints)
  uint32_t num_fp;     // routing_filter.num_fingerprints (new + old)
  uint32_t value;
  uint32_t vs, rem, rvs, lnb;
  uint32_t num_indices;
  uint32_t cbits, bbits;  // coarse-bucket bits, bucket-in-coarse-bucket bits (sum = lnb)
  uint32_t binsh;         // K4 bins = buckets >> binsh (1: coarse buckets of 2^13 buckets at
                          // load factor ~1, so a workgroup sorts ~8K entries, not ~4K)
  uint32_t cb_base, idx_base, page_base, page_cap, pf_base;
  // probe lines (device-only, 64 B per group of 2^(lg_line-1) buckets; lg_line 0 = none)
  uint32_t lg_line, line_base;
  uint32_t lines_asm;  // 1: K6 cuts this filter's lines from its LDS page images; 0: k_plines
  // old filter (incremental add)
  uint32_t old_num_indices, old_vs, old_rvs, npo;  // npo = new indices per old index
  uint32_t old_idx_base;  // first of this filter's old indices in the batch's old-index list
  uint32_t lines_flag;    // lines_asm, but a page's group table may not fit K6's LDS: such pages
                          // are flagged in pg_noline and k_plines cuts their indices' lines
  const uint8_t* old_pages;
  const uint64_t* old_slots;
  // 32-bit incremental builds whose old filter was built by this engine: its entries are read
  // in place from the old batch's sorted entry array (old_entries, old_idx_start / old_idx_cnt
  // relative to it) -- no decode of its image. Value bits are re-widened (old_vs -> vs) as K4
  // loads them. The old filter may have fewer coarse buckets (old_cbits <= cbits: a chain round
  // whose num_fingerprints crossed a power of two): each new coarse bucket's run is then a
  // sub-range of one old coarse bucket's, found by binary search (entries are sorted by
  // fingerprint in either geometry).
  uint32_t old_direct;
  uint32_t old_cbits, old_bbits;
  const uint32_t* old_entries;
  const uint32_t* old_idx_start;
  const uint32_t* old_idx_cnt;
};

// one filter of routing_filter_estimate_unique_fp (src/routing_filter.c:702-848): the first
// num_indices/16 indices of its image are decoded into a fingerprint bitmap
struct EstFilter {
  const uint8_t* pages;   // the filter's data pages (relocatable slots index into them)
  const uint64_t* slots;  // index slots
  uint32_t vs, rvs;       // value_size, remainder + value bits
  uint32_t num_idx;       // indices to decode (num_indices / 16)
  uint32_t idx_first;     // prefix sum of num_idx over the filters before this one
};

// one resident filter of a multi-filter probe (k_probe_groups): the lookups of many batches'
// filters -- the shim's queued routing_filter_lookup_async states, routing_filter_lookup
// calls of different bundles -- go to the GPU in ONE launch; each probe names its group
struct ProbeGroup {
  uint32_t x;             // vs | rem << 8 | rvs << 16 | lg_line << 24 (the filter's pplans[f].x)
  uint32_t err;           // nonzero: the filter's build failed, nothing is found
  uint32_t fpl;           // fingerprint_size | log_index_size << 8 (its batch's routing config)
  uint32_t pad;
  const uint4* lines;     // the filter's first probe line (lg_line != 0)
  const uint8_t* pages;   // the filter's data pages
  const uint64_t* slots;  // the filter's (relocatable) index slots
};

// The lookup server (k_lookup_server): single lookups travel through a ring of requests that a
// persistent wave polls, instead of one kernel launch per call. The ring lives in fine-grained
// device memory that the host writes through its BAR mapping (posted writes; the wave polls its
// own HBM: 0.09 us per 64-slot poll against 1.1-4.3 us for pinned host memory,
// profiles/r06_ring_placement.txt), or in pinned host memory (RF_AMD_SRV_RING=host). The
// host's stores reach the device in no particular order (a write-combining mapping), so every
// 8-byte word of a request carries the request's check value in its high half and the server
// serves a request only when all of its words do; answers are written the same way, so
// neither side waits for the other's stores to complete before publishing.
// Request t sits in slot t % SRV_RING; its check is t / SRV_RING + 1 (0: never written).
constexpr uint32_t SRV_RING = 4096;
constexpr uint32_t SRV_REQ_WORDS = 16;
// payload u32 of word i: 0 x, 1 err, 2 fpl (ProbeGroup), 3 the key's hash, 4-5 lines, 6-7 pages,
// 8-9 slots, 10-11 the submitter's tag (0: a waiter's ticket), 12-15 zero (two whole 64-byte
// lines: a full write-combining buffer leaves the host at once)
struct SrvReq {
  uint64_t w[SRV_REQ_WORDS];
};
static_assert(sizeof(SrvReq) == 128, "one request per two 64-byte lines");
// found lo, found hi, tag lo, tag hi (each | check << 32): an answer carries its request's tag,
// so the reaping thread reads only answer lines (written by the GPU)
struct SrvRes {
  uint64_t w[4];
};
static_assert(sizeof(SrvRes) == 32, "two answers per 64-byte line");
__host__ __device__ inline uint32_t srv_check(uint64_t t) { return (uint32_t)(t / SRV_RING) + 1u; }
// control block (pinned coherent host memory): the server writes the first ticket it did not
// serve, then its generation, when it exits. (The host's stop word sits after the request ring,
// where the wave polls it with the requests.)
struct SrvCtl {
  uint64_t unused;
  uint64_t exit_head;
  uint64_t exit_gen;
  uint64_t served;
  // diagnostics builds (RF_SRV_PROF): over every served pass of every launch, 10-ns ticks
  // polling the tickets, loading the payloads, probing + storing the answers, waiting for those
  // stores, storing the tickets; then the served passes
  uint64_t prof[6];
};

// a lookup call small enough to travel in the kernel arguments (k_probe_small)
constexpr uint32_t SMALL_PROBES = 64, SMALL_GROUPS = 8;
struct SmallProbe {
  uint32_t n, ng, seq;
  uint32_t h[SMALL_PROBES];
  uint8_t g[SMALL_PROBES];
  ProbeGroup groups[SMALL_GROUPS];
  uint64_t* found;      // pinned host memory
  uint32_t* done_flag;  // pinned host memory: seq once every result is visible
};

struct FilterOut {
  uint32_t num_unique;
  uint32_t num_pages;
  uint32_t error;
  uint32_t pad;
};

struct LaunchArgs {
  void* stream;
  int kind;
  int wide;  // 64-bit entries (old/new flag) -- only for incremental adds
  const FilterPlan* plans;
  const uint4* pplans;  // packed probe plan per filter {vs|rem<<8|rvs<<16|lg_line<<24, line_base, idx_base, error}
  uint4* pplans_mut;
  uint32_t num_filters;
  const uint32_t* tile_filter;
  const uint32_t* tile_start;
  uint32_t num_tiles;
  const uint32_t* old_tile_filter;
  const uint32_t* old_tile_start;
  uint32_t num_old_tiles;
  const uint32_t* old_idx_filter;  // incremental adds: filter of each old index of the batch
  uint32_t num_old_idx;
  uint32_t* old_cnt;  // per old index: entries (num_remainders), then their start
  uint32_t* old_pos;
  uint32_t flag32;     // incremental build with 32-bit flagged entries (fp_size + value_size <= 31)
  uint32_t* old32;     // flag32: every filter's decoded old entries, in order (P.old_first ..)
  uint32_t* old_tot;   // flag32: decoded old entries per filter
  uint32_t* ob_lo;     // flag32: per coarse bucket, its run of old entries (start, length)
  uint32_t* ob_n;
  const void* in0;
  const uint64_t* offs;
  uint32_t key_len, fp_size, seed, lis, page_size;
  void* ent;
  void* part;
  uint32_t* sorted32;
  uint32_t* cb_count;
  uint32_t* cb_start;
  uint32_t* cb_cursor;
  const uint32_t* cb_filter;
  uint32_t num_cb;
  uint32_t* overflow;
  uint32_t* spill;  // fused build: a coarse bucket exceeded its SORT_CAP region
  uint32_t* idx_cnt;
  uint32_t* idx_start;
  uint32_t* first_old;  // wide mode: per index, smallest old entry (valid if has_old)
  uint32_t* has_old;
  uint64_t* slots;
  uint4* lines;             // device-only probe lines (64 B = 4 x uint4 each)
  uint32_t line_lmax;       // max lines per index over the batch (k_plines LDS sizing)
  uint32_t plines_needed;   // some filter's lines come from k_plines
  uint32_t plines_force;    // k_plines over every filter (diagnostics)
  const uint32_t* idx_filter;
  uint32_t num_idx;
  uint32_t* page_first;
  uint32_t* pg_noline;      // [0] = count, then the page slots whose probe lines K6 left to k_plines_list
  uint32_t* cb_outs;        // 32-bit incremental builds: per coarse bucket, where K4 writes its sorted entries
  const uint32_t* pg_filter;
  uint32_t num_page_slots;
  uint8_t* pages;
  FilterOut* outs;
  const uint64_t* probe_runs;  // probes grouped by filter: runs[f] <= i < runs[f+1] (nullptr: per-probe ids)
  const uint32_t* wave_tab;    // with probe_runs: per 64-probe wave, filter << 7 | leading probes in it
  void** events;  // optional hipEvent_t[NUM_EVENTS] for per-stage timing (nullptr = off)
  uint32_t ev_mask;  // slots recorded (bit per EventSlot): all, or only the probe's two
};

// per-stage timing events: build = [B_START .. B_ASSEMBLE], probe = [P_START, P_END]
enum EventSlot { EV_B_START = 0, EV_B_HASH, EV_B_SCAN, EV_B_SCATTER, EV_B_SORT, EV_B_SORT_BIG,
                 EV_B_LAYOUT, EV_B_ASSEMBLE, EV_P_START, EV_P_END, NUM_EVENTS };
// probe-only timing: just the probe's start/end events, so a timed loop pays for 2 event
// records per step instead of one between every kernel (10 records cost a C2 step 42 us)
constexpr uint32_t EV_MASK_ALL = (1u << NUM_EVENTS) - 1;
constexpr uint32_t EV_MASK_PROBE = 1u << EV_P_START | 1u << EV_P_END;

}  // namespace rf
