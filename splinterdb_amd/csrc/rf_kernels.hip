// rf_kernels.hip -- MI355X (gfx950) kernels of the routing-filter engine.
//
// Build pipeline for a batch of F filters (each a SplinterDB routing_filter_add,
// reference src/routing_filter.c:337-656), one launch each, all on one stream:
//
//   K1 k_hash_count   keys/hashes -> entry e = (fp << value_size) | value  (+ coarse-bucket
//                     histogram in LDS, one global atomic per non-empty bin per tile)
//   K2 k_cb_scan      per filter: exclusive scan of coarse-bucket counts
//   K3 k_scatter      entries -> coarse buckets (LDS ranks + per-tile range reservation)
//   K4 k_cb_sort      one workgroup per coarse bucket (~4-8K entries, held in LDS):
//                     counting sort by filter bucket, per-bucket insertion sort, dedupe
//                     (src/routing_filter.c:471-482), per-index counts (:484-494),
//                     num_unique (:572-574)
//   K4b k_cb_sort_big same for coarse buckets over LDS capacity (duplicate-heavy input)
//   K5 k_layout       per filter: block sizes (:599-602) and the greedy page placement
//                     (:603-610) as a parallel pointer-jumping scan; index slots (:612-620)
//   K6 k_assemble     one workgroup per 4 KiB page: header, unary encoding with 0xFF
//                     padding (:622-626), PackedArray remainders (:627-633) built in LDS,
//                     written with 16-byte stores
//   K0 k_old_*        incremental add: decode the old filter (:496-544) into entries
//
// Probe lines: k_plines, one wave per index: device-only 64-byte lines per bucket group
//                     cut from the image (see "probe lines" below)
// Probe: k_probe, one lane per probe (routing_filter_lookup, :986-1073).
//
// The coarse bucket of an entry is its top `cbits` bits; K4 sorts the low bits, so the
// result depends only on the multiset of entries, exactly like the reference's sort.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rf_device.h"
#include "rf_plan.h"

using namespace rf;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

// XXH32 of input k (btree_pack / routing_filter_lookup hashing, src/btree.c:4020-4024,
// src/routing_filter.c:1004-1005). NT = non-temporal streaming loads (probe key stream).
template <int KIND, bool NT = false>
__device__ __forceinline__ uint32_t hash_key(const void* __restrict__ in0, const uint64_t* __restrict__ offs,
                                             uint32_t key_len, uint32_t seed, uint64_t k) {
  if constexpr (KIND == IN_KEYS24) {
    const v2u* kp = reinterpret_cast<const v2u*>(static_cast<const uint8_t*>(in0) + k * 24);
    v2u a, b, c;
    if constexpr (NT) {
      a = __builtin_nontemporal_load(kp);
      b = __builtin_nontemporal_load(kp + 1);
      c = __builtin_nontemporal_load(kp + 2);
    } else {
      a = kp[0];
      b = kp[1];
      c = kp[2];
    }
    uint32_t w[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
    return xxh32_24(w, seed);
  } else if constexpr (KIND == IN_KEYS_W) {
    return xxh32_words(reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(in0) + k * key_len),
                       key_len, seed);
  } else if constexpr (KIND == IN_KEYS_B) {
    const uint8_t* kp = static_cast<const uint8_t*>(in0) + k * key_len;
    return NT ? xxh32_unaligned_prefetch(kp, key_len, seed) : xxh32_unaligned(kp, key_len, seed);
  } else if constexpr (KIND == IN_VAR) {
    const uint64_t o0 = offs[k], o1 = offs[k + 1];
    const uint8_t* kp = static_cast<const uint8_t*>(in0) + o0;
    return NT ? xxh32_unaligned_prefetch(kp, (uint32_t)(o1 - o0), seed) : xxh32_unaligned(kp, (uint32_t)(o1 - o0), seed);
  } else {  // IN_HASH
    if constexpr (NT) return __builtin_nontemporal_load(static_cast<const uint32_t*>(in0) + k);
    else return static_cast<const uint32_t*>(in0)[k];
  }
}

// position of the r-th (0-based) set bit of x (exists)
__device__ __forceinline__ uint32_t select64_fast(uint64_t x, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 32; w >= 1; w >>= 1) {
    const uint32_t c = __popcll(x & ((1ull << w) - 1));
    if (r >= c) { r -= c; x >>= w; pos += w; }
  }
  return pos;
}
__device__ __forceinline__ uint64_t lowmask64(uint32_t k) { return k >= 64 ? ~0ull : ((1ull << k) - 1); }

// XCD-aware block -> work-item remap (bijective for any grid): the blocks that share an XCD
// (b % 8, round-robin dispatch) take one contiguous eighth of the work items, so one XCD's
// L2 sees one range of tiles / coarse buckets / pages / probes (MI355X_MICROARCH.md, XCD
// L2): partial lines written by neighbouring items merge in that L2 instead of reaching
// HBM as separate partial writes, and the next kernel finds the same range in the same L2.
__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t nb) {
  const uint32_t q = nb / 8, r = nb % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// ======================================================================================
// K1: hash + coarse-bucket histogram
// ======================================================================================
template <int KIND, typename EntT, bool FL = (sizeof(EntT) == 8)>
__global__ __launch_bounds__(TILE_NT) void k_hash_count(const FilterPlan* __restrict__ plans,
                                                        const uint32_t* __restrict__ tile_filter,
                                                        const uint32_t* __restrict__ tile_start,
                                                        const void* __restrict__ in0,
                                                        const uint64_t* __restrict__ offs,
                                                        uint32_t key_len, uint32_t fp_size,
                                                        uint32_t seed, EntT* __restrict__ ent,
                                                        uint32_t* __restrict__ cb_count,
                                                        const uint32_t* __restrict__ gate, uint32_t num_tiles) {
  __shared__ uint32_t s_hist[MAX_CB];
  if (gate && *gate == 0) return;  // fallback pass of the fused build: not needed
  // tiles grid-strided: the gated fallback launches a small grid (it is rarely needed)
  for (uint32_t t = blockIdx.x; t < num_tiles; t += gridDim.x) {
  const FilterPlan& P = plans[tile_filter[t]];
  const uint32_t start = tile_start[t];
  const uint32_t count = min((uint32_t)TILE_KEYS, P.num_new - start);
  const uint32_t num_cb = 1u << P.cbits;
  __syncthreads();  // the previous tile's histogram has been flushed
  for (uint32_t i = threadIdx.x; i < num_cb; i += TILE_NT) s_hist[i] = 0;
  __syncthreads();
  const uint32_t esh = fp_size + P.vs - P.cbits;  // entry >> esh = coarse bucket
  for (uint32_t j = threadIdx.x; j < count; j += TILE_NT) {
    const uint32_t h = hash_key<KIND>(in0, offs, key_len, seed, P.key_first + start + j);
    const uint32_t e = ((h >> (32 - fp_size)) << P.vs) | P.value;
    if constexpr (FL) {
      ent[P.e_first + start + j] = (EntT)(((EntT)e << 1) | EntT(1));  // new entry: flag 1
    } else {
      ent[P.e_first + start + j] = e;
    }
    const uint32_t cb = P.cbits ? (e >> esh) : 0u;
    atomicAdd(&s_hist[cb], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < num_cb; i += TILE_NT) {
    const uint32_t c = s_hist[i];
    if (c) atomicAdd(&cb_count[P.cb_base + i], c);
  }
  }
}

// Histogram of the old-entry region (K0 output); sentinel (~0) slots are skipped.
__global__ __launch_bounds__(TILE_NT) void k_old_count(const FilterPlan* __restrict__ plans,
                                                       const uint32_t* __restrict__ tile_filter,
                                                       const uint32_t* __restrict__ tile_start,
                                                       uint32_t fp_size,
                                                       const uint64_t* __restrict__ ent,
                                                       uint32_t* __restrict__ cb_count) {
  __shared__ uint32_t s_hist[MAX_CB];
  const uint32_t t = blockIdx.x;
  const FilterPlan& P = plans[tile_filter[t]];
  const uint32_t start = tile_start[t];
  const uint32_t count = min((uint32_t)TILE_KEYS, P.old_region - start);
  const uint32_t num_cb = 1u << P.cbits;
  for (uint32_t i = threadIdx.x; i < num_cb; i += TILE_NT) s_hist[i] = 0;
  __syncthreads();
  const uint32_t esh = fp_size + P.vs - P.cbits;
  for (uint32_t j = threadIdx.x; j < count; j += TILE_NT) {
    const uint64_t x = ent[P.e_first + P.num_new + start + j];
    if (x == ~0ull) continue;
    const uint32_t e = (uint32_t)(x >> 1);
    atomicAdd(&s_hist[P.cbits ? (e >> esh) : 0u], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < num_cb; i += TILE_NT) {
    const uint32_t c = s_hist[i];
    if (c) atomicAdd(&cb_count[P.cb_base + i], c);
  }
}

// ======================================================================================
// K2: per-filter exclusive scan of coarse-bucket counts
// ======================================================================================
__global__ __launch_bounds__(256) void k_cb_scan(const FilterPlan* __restrict__ plans,
                                                 const uint32_t* counts,  // may alias cb_count / cb_cursor
                                                 uint32_t* cb_count,
                                                 uint32_t* __restrict__ cb_start,
                                                 uint32_t* cb_cursor,
                                                 const uint32_t* __restrict__ gate) {
  __shared__ uint32_t s_tmp[256 / WAVE + 1];
  if (gate && *gate == 0) return;
  const FilterPlan& P = plans[blockIdx.x];
  const uint32_t num_cb = 1u << P.cbits;
  constexpr uint32_t PER = MAX_CB / 256;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < PER; k++) {
    const uint32_t i = threadIdx.x * PER + k;
    v[k] = i < num_cb ? counts[P.cb_base + i] : 0u;
    sum += v[k];
  }
  uint32_t total;
  uint32_t run = block_excl_scan<256>(sum, s_tmp, &total);
#pragma unroll
  for (uint32_t k = 0; k < PER; k++) {
    const uint32_t i = threadIdx.x * PER + k;
    if (i < num_cb) {
      cb_count[P.cb_base + i] = v[k];
      cb_start[P.cb_base + i] = run;
      cb_cursor[P.cb_base + i] = run;
    }
    run += v[k];
  }
}

// ======================================================================================
// K3: scatter entries into coarse buckets
// ======================================================================================
template <typename EntT, bool FL = (sizeof(EntT) == 8)>
__global__ __launch_bounds__(SCAT_NT) void k_scatter(const FilterPlan* __restrict__ plans,
                                                     const uint32_t* __restrict__ tile_filter,
                                                     const uint32_t* __restrict__ tile_start,
                                                     uint32_t region_is_old, uint32_t fp_size,
                                                     const EntT* __restrict__ ent,
                                                     EntT* __restrict__ part,
                                                     uint32_t* __restrict__ cb_cursor,
                                                     const uint32_t* __restrict__ gate, uint32_t num_tiles) {
  // The tile is sorted by coarse bucket in LDS, then each bucket's run is written by
  // consecutive lanes: whole 64-byte granules instead of scattered 4-byte stores.
  __shared__ EntT s_stage[TILE_KEYS];
  __shared__ uint32_t s_off[MAX_CB];  // local offsets, then (global base - local offset)
  __shared__ uint32_t s_tmp[SCAT_NT / WAVE + 1];
  if (gate && *gate == 0) return;
  constexpr int PER = TILE_KEYS / SCAT_NT;
  constexpr int BPT = MAX_CB / SCAT_NT;
  // tiles grid-strided: the gated fallback launches a small grid (it is rarely needed)
  for (uint32_t t = blockIdx.x; t < num_tiles; t += gridDim.x) {
  __syncthreads();  // the previous tile's staging has been written out
  const FilterPlan& P = plans[tile_filter[t]];
  const uint32_t start = tile_start[t];
  const uint32_t region = region_is_old ? P.old_region : P.num_new;
  const uint64_t base = P.e_first + (region_is_old ? P.num_new : 0u) + start;
  const uint32_t count = min((uint32_t)TILE_KEYS, region - start);
  const uint32_t num_cb = 1u << P.cbits;
  for (uint32_t i = threadIdx.x; i < num_cb; i += SCAT_NT) s_off[i] = 0;
  __syncthreads();
  const uint32_t esh = fp_size + P.vs - P.cbits;
  auto cb_of = [&](EntT x) -> uint32_t {
    uint32_t e;
    if constexpr (FL) e = (uint32_t)(x >> 1);
    else e = x;
    return P.cbits ? (e >> esh) : 0u;
  };
  EntT v[PER];
  uint32_t cbv[PER], rank[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) v[k] = ent[base + min(threadIdx.x + k * SCAT_NT, count - 1)];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t j = threadIdx.x + k * SCAT_NT;
    cbv[k] = ~0u;
    if (j < count) {
      bool valid = true;
      if constexpr (sizeof(EntT) == 8) valid = v[k] != ~0ull;
      if (valid) {
        cbv[k] = cb_of(v[k]);
        rank[k] = atomicAdd(&s_off[cbv[k]], 1u);
      }
    }
  }
  __syncthreads();
  // local exclusive offsets + one global reservation per non-empty bucket
  uint32_t cnt[BPT], sum = 0;
#pragma unroll
  for (int k = 0; k < BPT; k++) {
    const uint32_t b = threadIdx.x * BPT + k;
    cnt[k] = b < num_cb ? s_off[b] : 0u;
    sum += cnt[k];
  }
  uint32_t valid_total;
  uint32_t run = block_excl_scan<SCAT_NT>(sum, s_tmp, &valid_total);
  uint32_t gbase[BPT];
#pragma unroll
  for (int k = 0; k < BPT; k++) {
    const uint32_t b = threadIdx.x * BPT + k;
    gbase[k] = 0;
    if (b < num_cb) {
      s_off[b] = run;
      if (cnt[k]) gbase[k] = atomicAdd(&cb_cursor[P.cb_base + b], cnt[k]) - run;
      run += cnt[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; k++) {
    if (cbv[k] != ~0u) s_stage[s_off[cbv[k]] + rank[k]] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < BPT; k++) {
    const uint32_t b = threadIdx.x * BPT + k;
    if (b < num_cb) s_off[b] = gbase[k];
  }
  __syncthreads();
  EntT* dst = part + P.e_first;
  for (uint32_t j = threadIdx.x; j < valid_total; j += SCAT_NT) {
    const EntT x = s_stage[j];
    dst[s_off[cb_of(x)] + j] = x;
  }
  }
}

// Diagnostics: with g_dbg_ts set (rf_amd_debug_phase_buffer), workgroup b's thread 0
// stamps the shader clock at phase k of a kernel into g_dbg_ts[b * 16 + k] (phase timing).
// g_dbg_kid selects the kernel: 1 = bucket sort (K4), 2 = fused partition (K1+K3),
// 3 = page assembly (K6), 4 = layout (K5).
__device__ uint64_t* g_dbg_ts = nullptr;
__device__ uint32_t g_dbg_kid = 0;
// Compiled in only for the diagnostics library (RF_PHASE_STAMPS, build.py stamps=True):
// reading the stamp buffer pointer is a vector load whose wait (vmcnt(0)) would also wait
// for every load or atomic the kernel has in flight at that point.
#ifdef RF_PHASE_STAMPS
#define DBG_PHASE_K(kid, k)                                                  \
  do {                                                                       \
    uint64_t* _ts = g_dbg_ts;                                                \
    if (_ts && g_dbg_kid == (kid) && threadIdx.x == 0)                       \
      _ts[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime();             \
  } while (0)
#else
#define DBG_PHASE_K(kid, k) \
  do {                      \
  } while (0)
#endif
#define DBG_PHASE(k) DBG_PHASE_K(1, k)

extern "C" int rf_debug_set_phase_buffer(uint64_t* d_buf, uint32_t kid) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_kid), &kid, sizeof(kid)) != hipSuccess) return 1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_ts), &d_buf, sizeof(d_buf)) == hipSuccess ? 0 : 1;
}

// ======================================================================================
// K1+K3 fused (fresh builds, 32-bit entries): hash a tile, rank its entries by coarse
// bucket in LDS, reserve each bucket's run with one atomic, and write the runs straight
// into the bucket's fixed region of SORT_CAP slots at part[e_first + cb * SORT_CAP] --
// no entry array round trip and no separate count/scan pass. A bucket that would exceed
// SORT_CAP (duplicate-heavy or adversarial input) raises *spill; the exact count -> scan
// -> scatter pipeline (K1, K2, K3 gated on *spill) then rebuilds the partition.
// ======================================================================================
#ifndef RF_SCAT_WPE
#define RF_SCAT_WPE 4
#endif
#ifndef RF_SCAT_X3
#define RF_SCAT_X3 1
#endif
// FL (32-bit incremental builds): the entries are written flagged new, (e << 1) | 1.
template <int KIND, bool FL = false>
__global__ __launch_bounds__(SCAT_NT) __attribute__((amdgpu_waves_per_eu(RF_SCAT_WPE))) void k_hash_scatter(const FilterPlan* __restrict__ plans,
                                                          const uint32_t* __restrict__ tile_filter,
                                                          const uint32_t* __restrict__ tile_start,
                                                          const void* __restrict__ in0,
                                                          const uint64_t* __restrict__ offs,
                                                          uint32_t key_len, uint32_t fp_size, uint32_t seed,
                                                          uint32_t* __restrict__ part,
                                                          uint32_t* __restrict__ cb_fill,
                                                          uint32_t* __restrict__ spill) {
  __shared__ __attribute__((aligned(16))) uint32_t s_stage[TILE_KEYS];
  __shared__ uint32_t s_off[MAX_CB];  // local counts -> local starts -> (global slot - local start)
  __shared__ uint32_t s_tmp[SCAT_NT / WAVE + 1];
  constexpr int PER = TILE_KEYS / SCAT_NT;
  constexpr int BPT = MAX_CB / SCAT_NT;
  DBG_PHASE_K(2, 15);
  const uint32_t t = xcd_chunk(blockIdx.x, gridDim.x);  // a filter's tiles share an XCD
  const FilterPlan& P = plans[tile_filter[t]];
  const uint32_t start = tile_start[t];
  const uint32_t count = min((uint32_t)TILE_KEYS, P.num_new - start);
  const uint32_t num_cb = 1u << P.cbits;
  for (uint32_t i = threadIdx.x; i < num_cb; i += SCAT_NT) s_off[i] = 0;
  __syncthreads();
  DBG_PHASE_K(2, 0);
  const uint32_t esh = fp_size + P.vs - P.cbits + (FL ? 1u : 0u);  // entry >> esh = coarse bucket
  auto cb_of = [&](uint32_t e) -> uint32_t { return P.cbits ? (e >> esh) : 0u; };
  const uint32_t flag = FL ? 1u : 0u;
  uint32_t v[PER], rank[PER];
  // all key loads first (clamped index: no branch, every load in flight at once), then the
  // LDS ranking -- interleaving them serialises one HBM round trip per key
  // in chunks of HASH_CHUNK keys: a chunk's loads are all in flight together; the next
  // chunk's addresses take an opaque zero computed from this chunk's last hash, so the
  // compiler cannot hoist every key of the tile into registers (236 VGPRs, 2 waves/SIMD)
  constexpr int HASH_CHUNK = 8;
  uint32_t dep = 0;
  // key j of the tile handled by this thread's k-th slot: strided across the block, except
  // for variable-length keys, where a wave takes 64 * PER consecutive keys (one byte stream)
  // 24-byte keys (X3): a wave's 64 keys of slot k are one 1,536-byte range, read as two
  // contiguous 768-byte dwordx3 loads; lane 2i holds key i, lane 2i + 1 key 32 + i
  constexpr bool X3 = KIND == IN_KEYS24 && RF_SCAT_X3;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  auto key_of = [&](int k) -> uint32_t {
    if constexpr (KIND == IN_VAR) return (threadIdx.x & ~(WAVE - 1)) * PER + k * WAVE + lane;
    else if constexpr (X3) return (threadIdx.x & ~(WAVE - 1)) + k * SCAT_NT + (lane >> 1) + (lane & 1) * 32;
    else return threadIdx.x + k * SCAT_NT;
  };
  constexpr uint32_t VWIN = (TILE_KEYS / (SCAT_NT / WAVE)) * 4 - 16;  // bytes (s_stage slice - pad)
  uint32_t* s_vwin = s_stage + (threadIdx.x / WAVE) * (TILE_KEYS / (SCAT_NT / WAVE));
  uint64_t vw0 = 0, vw1 = 0, vo0 = 0, vo1 = 0;
  if constexpr (KIND == IN_VAR) {
    const uint32_t j = min(key_of(0), count - 1);
    vo0 = offs[P.key_first + start + j];
    vo1 = offs[P.key_first + start + j + 1];
  }
#pragma unroll
  for (int k0 = 0; k0 < PER; k0 += HASH_CHUNK) {
    if constexpr (X3) {
      // lane l reads bytes [12 (l & 1), +12) of key (l >> 1) and of key 32 + (l >> 1): two
      // wave loads cover the slot's 64 keys with 12 cache lines, where three 8-byte loads per
      // lane strided by the key touch 36. A DPP swap of the lane pair completes each key:
      // the even lane sends its half of key 32 + i and receives the odd lane's of key i.
      const uint32_t half = lane & 1, ki = lane >> 1;
      const uint8_t* kbase = static_cast<const uint8_t*>(in0) + (uint64_t)(P.key_first + start) * 24 + 12 * half;
      uint32_t a[HASH_CHUNK][3], b[HASH_CHUNK][3];
#pragma unroll
      for (int k = 0; k < HASH_CHUNK; k++) {
        const uint32_t c0 = (threadIdx.x & ~(WAVE - 1)) + (k0 + k) * SCAT_NT;
        const uint32_t ja = min(c0 + ki, count - 1) + dep, jb = min(c0 + 32 + ki, count - 1) + dep;
        const uint32_t* pa = reinterpret_cast<const uint32_t*>(kbase + (uint64_t)ja * 24);
        const uint32_t* pb = reinterpret_cast<const uint32_t*>(kbase + (uint64_t)jb * 24);
        a[k][0] = pa[0]; a[k][1] = pa[1]; a[k][2] = pa[2];
        b[k][0] = pb[0]; b[k][1] = pb[1]; b[k][2] = pb[2];
      }
#pragma unroll
      for (int k = 0; k < HASH_CHUNK; k++) {
        uint32_t w[6];
#pragma unroll
        for (int q = 0; q < 3; q++) {
          const uint32_t send = half ? a[k][q] : b[k][q];
          const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
          w[q] = half ? recv : a[k][q];
          w[3 + q] = half ? b[k][q] : recv;
        }
        const uint32_t h = xxh32_24(w, seed);
        v[k0 + k] = ((((h >> (32 - fp_size)) << P.vs) | P.value) << flag) | flag;
      }
    } else if constexpr (KIND == IN_KEYS24) {
      // 24-byte keys: issue all of the chunk's loads, then hash (z depends on every loaded
      // word, so no hash starts before the last load is issued)
      v2u ka[HASH_CHUNK], kb[HASH_CHUNK], kc[HASH_CHUNK];
#pragma unroll
      for (int k = 0; k < HASH_CHUNK; k++) {
        const uint32_t j = min(threadIdx.x + (k0 + k) * SCAT_NT, count - 1) + dep;
        const v2u* kp = reinterpret_cast<const v2u*>(static_cast<const uint8_t*>(in0) +
                                                     (P.key_first + start + j) * 24);
        ka[k] = kp[0];
        kb[k] = kp[1];
        kc[k] = kp[2];
      }
      uint32_t z;
      asm volatile("v_mov_b32 %0, 0" : "=v"(z)
                   : "v"(ka[0].x), "v"(ka[1].x), "v"(ka[2].x), "v"(ka[3].x), "v"(ka[4].x), "v"(ka[5].x),
                     "v"(ka[6].x), "v"(ka[7].x), "v"(kb[0].x), "v"(kb[1].x), "v"(kb[2].x), "v"(kb[3].x),
                     "v"(kb[4].x), "v"(kb[5].x), "v"(kb[6].x), "v"(kb[7].x), "v"(kc[0].x), "v"(kc[1].x),
                     "v"(kc[2].x), "v"(kc[3].x), "v"(kc[4].x), "v"(kc[5].x), "v"(kc[6].x), "v"(kc[7].x));
#pragma unroll
      for (int k = 0; k < HASH_CHUNK; k++) {
        uint32_t w[6] = {ka[k].x + z, ka[k].y, kb[k].x, kb[k].y, kc[k].x, kc[k].y};
        const uint32_t h = xxh32_24(w, seed);
        v[k0 + k] = ((((h >> (32 - fp_size)) << P.vs) | P.value) << flag) | flag;
      }
    } else if constexpr (KIND == IN_VAR) {
      // variable-length keys: this wave's keys [wave * 64 * PER, +64 * PER) are one
      // contiguous byte stream, read into the wave's 8 KiB slice of s_stage (unused until
      // the ranking) with coalesced 16-byte loads and hashed from LDS (wave_hash_var).
      // The window persists across k: a key already staged is hashed without a reload.
      // the next key's offsets load while this key's window is staged and hashed
#pragma unroll
      for (int k = 0; k < HASH_CHUNK; k++) {
        const uint64_t o0 = vo0, o1 = vo1;
        if (k0 + k + 1 < PER) {
          const uint32_t j = min(key_of(k0 + k + 1), count - 1);
          vo0 = offs[P.key_first + start + j];
          vo1 = offs[P.key_first + start + j + 1];
        }
        const uint32_t h = wave_hash_var<VWIN, false>(static_cast<const uint8_t*>(in0), o0, o1,
                                                      key_of(k0 + k) < count, s_vwin, seed, &vw0, &vw1);
        v[k0 + k] = ((((h >> (32 - fp_size)) << P.vs) | P.value) << flag) | flag;
      }
    } else {
#pragma unroll
      for (int k = k0; k < k0 + HASH_CHUNK; k++) {
        const uint32_t j = min(threadIdx.x + k * SCAT_NT, count - 1) + dep;
        const uint32_t h = hash_key<KIND>(in0, offs, key_len, seed, P.key_first + start + j);
        v[k] = ((((h >> (32 - fp_size)) << P.vs) | P.value) << flag) | flag;
      }
    }
    static_assert(HASH_CHUNK == 8, "opaque dependency below takes 8 hashes");
    asm volatile("v_mov_b32 %0, 0" : "=v"(dep)
                 : "v"(v[k0]), "v"(v[k0 + 1]), "v"(v[k0 + 2]), "v"(v[k0 + 3]), "v"(v[k0 + 4]),
                   "v"(v[k0 + 5]), "v"(v[k0 + 6]), "v"(v[k0 + 7]));
  }
  DBG_PHASE_K(2, 5);  // thread 0's keys loaded and hashed (no barrier)
#pragma unroll
  for (int k = 0; k < PER; k++) {
    if (key_of(k) < count) rank[k] = atomicAdd(&s_off[cb_of(v[k])], 1u);
  }
  __syncthreads();
  DBG_PHASE_K(2, 1);
  uint32_t cnt[BPT], sum = 0;
#pragma unroll
  for (int k = 0; k < BPT; k++) {
    const uint32_t b = threadIdx.x * BPT + k;
    cnt[k] = b < num_cb ? s_off[b] : 0u;
    sum += cnt[k];
  }
  uint32_t total;
  uint32_t run = block_excl_scan<SCAT_NT>(sum, s_tmp, &total);
  // reserve each bucket's run in its region (global atomics), then stage the tile in LDS
  // while the reservations are in flight; their results are first needed after staging
  uint32_t g[BPT], lstart[BPT];
#pragma unroll
  for (int k = 0; k < BPT; k++) {
    const uint32_t b = threadIdx.x * BPT + k;
    g[k] = 0;
    lstart[k] = run;
    if (b < num_cb) {
      if (cnt[k]) g[k] = atomicAdd(&cb_fill[P.cb_base + b], cnt[k]);
      s_off[b] = run;
      run += cnt[k];
    }
  }
  __syncthreads();
  DBG_PHASE_K(2, 2);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    if (key_of(k) < count) s_stage[s_off[cb_of(v[k])] + rank[k]] = v[k];
  }
  __syncthreads();
  DBG_PHASE_K(2, 3);
  bool over = false;
#pragma unroll
  for (int k = 0; k < BPT; k++) {
    const uint32_t b = threadIdx.x * BPT + k;
    if (b < num_cb) {
      over |= cnt[k] && g[k] + cnt[k] > (uint32_t)SORT_CAP;
      s_off[b] = g[k] - lstart[k];
    }
  }
  if (over) atomicOr(spill, 1u);
  __syncthreads();
  DBG_PHASE_K(2, 4);
  uint32_t* dst = part + P.e_first;
  for (uint32_t j = threadIdx.x; j < total; j += SCAT_NT) {
    const uint32_t x = s_stage[j];
    const uint32_t cb = cb_of(x);
    const uint32_t slot = s_off[cb] + j;  // position inside the bucket's region
    if (slot < (uint32_t)SORT_CAP) dst[(uint64_t)cb * CB_REGION + slot] = x;
  }
  DBG_PHASE_K(2, 8);
}

// ======================================================================================
// K4: per coarse bucket sort / dedupe / index counts
// ======================================================================================
// Entries: e = (fp << vs) | value, or, in incremental builds (FL), (e << 1) | new-flag --
// 64-bit, or 32-bit when fp_size + value_size <= 31 leaves room for the flag.
template <typename EntT, bool FL = (sizeof(EntT) == 8)>
__device__ __forceinline__ uint32_t ent_e(EntT x) {
  if constexpr (FL) return (uint32_t)(x >> 1);
  else return x;
}
// dedupe rule (src/routing_filter.c:471-482 for new entries; old entries are never
// deduplicated, :559-597): drop x if it equals its predecessor and is a new entry.
template <typename EntT, bool FL = (sizeof(EntT) == 8)>
__device__ __forceinline__ bool ent_drop(EntT x, EntT prev) {
  if constexpr (FL) return x == prev && (x & EntT(1));
  else return x == prev;
}

// 8-input sorting network (Batcher odd-even merge, 19 compare-exchanges)
template <typename T>
__device__ __forceinline__ void sort8(T (&x)[8]) {
#define CE(a, b) { const T lo = x[a] < x[b] ? x[a] : x[b], hi = x[a] < x[b] ? x[b] : x[a]; x[a] = lo; x[b] = hi; }
  CE(0, 1) CE(2, 3) CE(4, 5) CE(6, 7) CE(0, 2) CE(1, 3) CE(4, 6) CE(5, 7) CE(1, 2) CE(5, 6)
  CE(0, 4) CE(1, 5) CE(2, 6) CE(3, 7) CE(2, 4) CE(3, 5) CE(1, 2) CE(3, 4) CE(5, 6)
#undef CE
}
template <typename T>
__device__ __forceinline__ void sort16(T (&x)[16]) {  // Batcher odd-even merge, 63 CEs
#define CE(a, b) { const T lo = x[a] < x[b] ? x[a] : x[b], hi = x[a] < x[b] ? x[b] : x[a]; x[a] = lo; x[b] = hi; }
  CE(0, 1) CE(2, 3) CE(0, 2) CE(1, 3) CE(1, 2) CE(4, 5) CE(6, 7) CE(4, 6) CE(5, 7) CE(5, 6) CE(0, 4)
  CE(2, 6) CE(2, 4) CE(1, 5) CE(3, 7) CE(3, 5) CE(1, 2) CE(3, 4) CE(5, 6) CE(8, 9) CE(10, 11) CE(8, 10)
  CE(9, 11) CE(9, 10) CE(12, 13) CE(14, 15) CE(12, 14) CE(13, 15) CE(13, 14) CE(8, 12) CE(10, 14)
  CE(10, 12) CE(9, 13) CE(11, 15) CE(11, 13) CE(9, 10) CE(11, 12) CE(13, 14) CE(0, 8) CE(4, 12)
  CE(4, 8) CE(2, 10) CE(6, 14) CE(6, 10) CE(2, 4) CE(6, 8) CE(10, 12) CE(1, 9) CE(5, 13) CE(5, 9)
  CE(3, 11) CE(7, 15) CE(7, 11) CE(3, 5) CE(7, 9) CE(11, 13) CE(1, 2) CE(3, 4) CE(5, 6) CE(7, 8)
  CE(9, 10) CE(11, 12) CE(13, 14)
#undef CE
}

// Sorts a[0, cnt) with the whole workgroup (NT threads; a in LDS or global memory): Batcher's
// odd-even merge sort network over the next power of two, the elements past cnt taken as +inf
// (every comparator is ascending, so those never swap and are skipped). O(cnt log^2 cnt)
// comparisons in log(n)(log(n)+1)/2 barrier-separated stages: a bucket of 12K duplicates of a
// few distinct (fingerprint, value) entries -- quadratic for the per-bin insertion sort this
// replaces -- sorts in 105 stages.
template <typename T, int NT>
__device__ void oe_sort_group(T* a, uint32_t cnt) {
  uint32_t n = 1;
  while (n < cnt) n <<= 1;
  for (uint32_t p = 1; p < n; p <<= 1) {
    for (uint32_t k = p; k >= 1; k >>= 1) {
      const uint32_t r = k & (p - 1);
      for (uint32_t L = threadIdx.x; L + k < cnt; L += NT) {
        if (L >= r && ((L - r) & (2 * k - 1)) < k && (L / (2 * p)) == ((L + k) / (2 * p))) {
          const T x = a[L], y = a[L + k];
          if (y < x) {
            a[L] = y;
            a[L + k] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Finish a sorted coarse bucket held in `B` (LDS or global): write per-index counts and
// starts, the compacted entries, and the num_unique contribution. Shared by K4 and K4b.
struct CbCtx {
  uint32_t rvs, vs, lis, bbits, idx0;  // idx0 = global index id of the cb's first index
  uint32_t cb_rel;                     // cb start relative to the filter's e_first
  uint64_t e_first;
};

__device__ __forceinline__ void write_index_bounds(const CbCtx& c, const uint32_t* sorted, uint32_t kept,
                                                   uint32_t* idx_cnt, uint32_t* idx_start,
                                                   uint32_t* uniq_out) {
  // sorted: compacted e values (u32). Index-in-cb of e = (e >> (lis + rvs)) & (ipc - 1)
  const uint32_t ipc = 1u << (c.bbits - c.lis);
  const uint32_t ish = c.lis + c.rvs;
  for (uint32_t li = threadIdx.x; li < ipc; li += blockDim.x) {
    auto lb = [&](uint32_t key) {
      uint32_t lo = 0, hi = kept;
      while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        uint32_t m = ish >= 32 ? 0u : ((sorted[mid] >> ish) & (ipc - 1));
        if (m < key) lo = mid + 1; else hi = mid;
      }
      return lo;
    };
    const uint32_t lo = lb(li);
    const uint32_t hi = (li + 1 < ipc) ? lb(li + 1) : kept;
    idx_cnt[c.idx0 + li] = hi - lo;
    idx_start[c.idx0 + li] = c.cb_rel + lo;
  }
  // num_unique (:558, :572-574): per index, count entries whose fingerprint differs from the
  // previous entry's; the first entry of an index compares against UINT32_MAX >> value_size.
  // Equal fingerprints share an index, so "previous entry in the coarse bucket" suffices
  // except at an index's first entry.
  uint32_t uniq = 0;
  for (uint32_t i = threadIdx.x; i < kept; i += blockDim.x) {
    const uint32_t fp = sorted[i] >> c.vs;
    const bool first = (i == 0) || (ish < 32 && ((sorted[i] >> ish) != (sorted[i - 1] >> ish)));
    const uint32_t prev = first ? (0xffffffffu >> c.vs) : (sorted[i - 1] >> c.vs);
    uniq += (fp != prev) ? 1u : 0u;
  }
  *uniq_out = uniq;
}

// DUAL (32-bit incremental builds): a coarse bucket's entries come from two places -- its
// new entries, scattered into part, and its run of the old filter's decoded entries
// (already in order: old32 + P.old_first + ob_lo[cb], ob_n[cb] of them), loaded as (e << 1).
// Only the new entries are ranked and sorted (s_b[0, nn)); the old run is stored as it comes
// (s_b[nn, n)), and the dedupe pass reads the two sorted runs through a merge path. Old
// flagged values are even and new ones odd, so no old value equals a new one and the merge
// yields exactly the order a sort of all n would (old first on equal e).
template <typename EntT, bool FL = (sizeof(EntT) == 8), bool DUAL = false, bool LIST = false>
__global__ __launch_bounds__(SORT_NT, 6) void k_cb_sort(const FilterPlan* __restrict__ plans,
                                                     const uint32_t* __restrict__ cb_filter,
                                                     const uint32_t* __restrict__ cb_count,
                                                     const uint32_t* __restrict__ cb_start,
                                                     const EntT* __restrict__ part,
                                                     const uint32_t* __restrict__ old32,
                                                     const uint32_t* __restrict__ ob_lo,
                                                     const uint32_t* __restrict__ ob_n,
                                                     uint32_t* __restrict__ sorted32,
                                                     uint32_t* __restrict__ idx_cnt,
                                                     uint32_t* __restrict__ idx_start,
                                                     FilterOut* __restrict__ outs,
                                                     uint32_t* __restrict__ overflow,
                                                     uint32_t lis, uint32_t* __restrict__ first_old,
                                                     uint32_t* __restrict__ has_old,
                                                     const uint32_t* __restrict__ spill,
                                                     const uint32_t* __restrict__ cb_outs,
                                                     const uint32_t* __restrict__ cb_list) {
  constexpr int PER = SORT_CAP / SORT_NT;
  DBG_PHASE(15);
  __shared__ EntT s_b[SORT_CAP];
  __shared__ __attribute__((aligned(16))) uint32_t s_bin[MAX_BINS + 1];
  __shared__ uint32_t s_tmp[SORT_NT / WAVE + 1];
  // incremental builds: per index, its smallest old entry and whether it has one; they live
  // in s_bin past s_first's ipc + 1 words, initialised once the bins are no longer read (no
  // LDS beyond the fresh build's, so the same 3 workgroups per CU)
  static_assert(MAX_BINS + 1 >= 2048 + 2 * MAX_IPC && MAX_IPC + 1 <= 2048, "s_fo / s_ho inside s_bin");
  constexpr uint32_t BIG_LIST = 64;
  __shared__ uint32_t s_big[BIG_LIST];  // bins over 8 entries (s_nbig may exceed the list)
  __shared__ uint32_t s_nbig;
  uint32_t* s_first = s_bin;  // compacted start of each index: reuses s_bin once bins are sorted
  uint32_t* s_fo = s_bin + 2048;
  uint32_t* s_ho = s_bin + 2048 + MAX_IPC;
  // LIST (K4m's fallback, 32-bit incremental builds): the coarse buckets K4m listed in cb_list
  // with bit 31 set (more new entries than it takes, or a bin of duplicates), one after
  // another; otherwise one coarse bucket per workgroup (the loop runs once: a compile-time
  // trip count, so the fresh build's kernel is the same code as without it)
  const uint32_t nit = LIST ? cb_list[0] : 1u;
  for (uint32_t it = LIST ? blockIdx.x : 0u; it < nit; it += LIST ? gridDim.x : 1u) {
  uint32_t cb;
  if constexpr (LIST) {
    cb = cb_list[1 + it];
    if (!(cb >> 31)) continue;  // K4b's (over SORT_CAP)
    cb &= 0x7fffffffu;
  } else {
    cb = xcd_chunk(blockIdx.x, gridDim.x);  // a filter's buckets share an XCD (its partition's L2)
  }
  const uint32_t f = cb_filter[cb];
  const FilterPlan& P = plans[f];
  const uint32_t n = cb_count[cb];
  const uint32_t cbl = cb - P.cb_base;
  // fused build without spill: fixed SORT_CAP regions; otherwise the scanned starts
  const uint32_t cb_rel = (spill && *spill == 0) ? cbl * CB_REGION : cb_start[cb];
  // where the sorted entries go: in place, or (32-bit incremental builds with the fused
  // partition) at the scan of the coarse buckets' new + old counts (cb_outs)
  const uint32_t cb_out = (DUAL && spill) ? cb_outs[cb] : cb_rel;
  CbCtx c{P.rvs, P.vs, lis, P.bbits, P.idx_base + (cbl << (P.bbits - lis)), cb_out, P.e_first};
  if (n > SORT_CAP) {  // handled by k_cb_sort_big
    if (threadIdx.x == 0 && !LIST) overflow[1 + atomicAdd(&overflow[0], 1u)] = cb;
    continue;
  }
  const uint32_t nbins = 1u << (P.bbits - P.binsh);  // a bin = 2^binsh filter buckets
  const uint32_t bmask = nbins - 1, bsh = P.rvs + P.binsh;
  const uint32_t ipc = 1u << (P.bbits - lis), ish = lis + P.rvs;
  // the bucket's entry loads go out first (clamped, branch-free) and land while the bin
  // counters are cleared; the barrier after the clearing orders only LDS (a full
  // __syncthreads would also wait for the loads)
  EntT v[PER];
  // ranks within a bin (< SORT_CAP): two 16-bit ranks per register -- the DUAL variant spilled
  // with one register per rank
  static_assert(SORT_CAP <= 65536 && PER % 2 == 0, "16-bit ranks, packed in pairs");
  uint32_t rp[PER / 2];
#pragma unroll
  for (int k = 0; k < PER / 2; k++) rp[k] = 0;
  const EntT* src = part + P.e_first + cb_rel;
  const uint32_t nm1 = n ? n - 1 : 0u;
  if constexpr (DUAL) {
    // new entries first, then the old run, loaded raw (one load per element from a selected
    // address: nothing computed on the data before the barrier below, so it does not wait
    // for the loads); old values get their flag (<< 1) when stored into s_b
    const uint32_t nn = n - ob_n[cb];
    const uint32_t* osrc = (P.old_direct ? P.old_entries : old32 + P.old_first) + ob_lo[cb];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t j = min(threadIdx.x + k * SORT_NT, nm1);
      v[k] = *(j < nn ? reinterpret_cast<const uint32_t*>(src) + j : osrc + (j - nn));
    }
  } else {
#pragma unroll
    for (int k = 0; k < PER; k++) v[k] = src[min(threadIdx.x + k * SORT_NT, nm1)];
  }
  for (uint32_t i = threadIdx.x; i <= nbins; i += SORT_NT) s_bin[i] = 0;
  if (threadIdx.x == 0) s_nbig = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  DBG_PHASE(0);
  // the entries ranked and sorted here: all of them, or (DUAL) the new ones
  uint32_t nsort = n;
  if constexpr (DUAL) nsort = n - ob_n[cb];
  // per-bin rank (bin = filter bucket within the coarse bucket)
#pragma unroll
  for (int k = 0; k < PER; k++) {
    if (threadIdx.x + k * SORT_NT < nsort) {
      const uint32_t e = ent_e<EntT, FL>(v[k]);
      const uint32_t b = bsh >= 32 ? 0u : ((e >> bsh) & bmask);
      rp[k / 2] |= atomicAdd(&s_bin[b], 1u) << (16 * (k & 1));
    }
  }
  __syncthreads();
  DBG_PHASE(1);
  // exclusive scan of bin counts (nbins <= MAX_BINS = 8 * SORT_NT): thread t owns bins
  // [8t, 8t + 8), read and written as two 16-byte LDS accesses (8 scalar accesses strided
  // by 8 words were 16-way bank conflicts)
  {
    constexpr int BPT = MAX_BINS / SORT_NT;
    static_assert(BPT == 8, "two 16-byte accesses per thread");
    v4u* sb4 = reinterpret_cast<v4u*>(s_bin) + 2 * threadIdx.x;
    const bool own = threadIdx.x * BPT < nbins;  // nbins is a power of two >= 8 or < 8
    v4u a = own ? sb4[0] : v4u{0u, 0u, 0u, 0u}, b = own ? sb4[1] : v4u{0u, 0u, 0u, 0u};
    if (own && nbins < BPT) {  // fewer than 8 bins: only the first nbins words are counts
      uint32_t t8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int k = 0; k < 8; k++) if ((uint32_t)k >= nbins) t8[k] = 0;
      a = v4u{t8[0], t8[1], t8[2], t8[3]};
      b = v4u{t8[4], t8[5], t8[6], t8[7]};
    }
    const uint32_t sum = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
    uint32_t total;
    uint32_t run = block_excl_scan<SORT_NT>(sum, s_tmp, &total);
    v4u ea, eb;
    ea.x = run; run += a.x; ea.y = run; run += a.y; ea.z = run; run += a.z; ea.w = run; run += a.w;
    eb.x = run; run += b.x; eb.y = run; run += b.y; eb.z = run; run += b.z; eb.w = run;
    if (own && nbins >= BPT) {
      sb4[0] = ea;
      sb4[1] = eb;
    } else if (own) {
      const uint32_t e8[8] = {ea.x, ea.y, ea.z, ea.w, eb.x, eb.y, eb.z, eb.w};
      for (uint32_t k = 0; k < nbins; k++) s_bin[k] = e8[k];
    }
    if (threadIdx.x == 0) s_bin[nbins] = nsort;
  }
  __syncthreads();
  DBG_PHASE(2);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t i = threadIdx.x + k * SORT_NT;
    if (i < nsort) {
      const uint32_t e = ent_e<EntT, FL>(v[k]);
      const uint32_t b = bsh >= 32 ? 0u : ((e >> bsh) & bmask);
      s_b[s_bin[b] + ((rp[k / 2] >> (16 * (k & 1))) & 0xffffu)] = v[k];
    } else if (i < n) {
      // DUAL: the old run, already in order, flagged old (read in place: value bits re-widened
      // to this filter's value_size, src/routing_filter.c:536-543; order is unchanged)
      const uint32_t eo = (uint32_t)v[k];
      const uint32_t e = P.old_direct ? ((eo >> P.old_vs) << P.vs) | (eo & ((1u << P.old_vs) - 1u)) : eo;
      s_b[i] = (EntT)e << 1;
    }
  }
  __syncthreads();
  DBG_PHASE(3);
  // order inside each bin. The entries of S consecutive bins are one contiguous segment of
  // s_b, and sorting a segment by value orders its bins (a bin is the value's high part)
  // and every bin's entries at once. S makes a segment hold ~8 entries on average; one
  // thread sorts it in registers with a 16-input network. A segment over 16 entries falls
  // back to an 8-input network per bin; bins over 8 entries are listed and ranked
  // afterwards by a whole wave each (lane j's entry goes to the bin start + the number of
  // entries that sort before it: smaller, or equal and earlier).
  {
    constexpr EntT EMAX = ~EntT(0);
    uint32_t S = 8;  // largest power of two <= 8 with S * nsort / nbins <= 8
    while (S > 1 && (uint64_t)S * nsort > 8ull * nbins) S >>= 1;
    if (S > nbins) S = nbins;
    const uint32_t nseg = nbins / S;
    for (uint32_t sg = threadIdx.x; sg < nseg; sg += SORT_NT) {
      const uint32_t b0 = sg * S, st = s_bin[b0], c = s_bin[b0 + S] - st;
      if (c <= 16) {
        EntT x[16];
#pragma unroll
        for (int j = 0; j < 16; j++) x[j] = (uint32_t)j < c ? s_b[st + j] : EMAX;
        sort16(x);
        if (c >= 2) {
#pragma unroll
          for (int j = 0; j < 16; j++)
            if ((uint32_t)j < c) s_b[st + j] = x[j];
        }
      } else {
        for (uint32_t b = b0; b < b0 + S; b++) {
          const uint32_t bs = s_bin[b], bc = s_bin[b + 1] - bs;
          if (bc <= 1) continue;
          if (bc <= 8) {
            EntT y[8];
#pragma unroll
            for (int j = 0; j < 8; j++) y[j] = (uint32_t)j < bc ? s_b[bs + j] : EMAX;
            sort8(y);
#pragma unroll
            for (int j = 0; j < 8; j++)
              if ((uint32_t)j < bc) s_b[bs + j] = y[j];
          } else {
            const uint32_t q = atomicAdd(&s_nbig, 1u);
            if (q < BIG_LIST) s_big[q] = b;
          }
        }
      }
    }
  }
  __syncthreads();
  if (s_nbig) {
    // bins over 8 entries: those of at most 64 ranked by one wave each; larger ones
    // (duplicate-heavy input) sorted one after another by the whole workgroup. More than
    // BIG_LIST of them: every bin is visited (the list holds only the first BIG_LIST)
    const uint32_t nb = s_nbig;
    const bool listed = nb <= BIG_LIST;
    const uint32_t nq = listed ? nb : nbins;
    const uint32_t wv = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
    for (uint32_t q = wv; q < nq; q += SORT_NT / WAVE) {
      const uint32_t b = listed ? s_big[q] : q, st = s_bin[b], cnt = s_bin[b + 1] - st;
      if (cnt > 8 && cnt <= WAVE) {
        EntT mine = lane < cnt ? s_b[st + lane] : EntT(0);
        uint32_t before = 0;
        for (uint32_t j = 0; j < cnt; j++) {
          const EntT y = s_b[st + j];  // same address in every lane: a broadcast
          before += (y < mine || (y == mine && j < lane)) ? 1u : 0u;
        }
        __builtin_amdgcn_wave_barrier();  // all reads of the bin before any write
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        if (lane < cnt) s_b[st + before] = mine;
      }
    }
    __syncthreads();
    for (uint32_t q = 0; q < nq; q++) {  // workgroup-uniform
      const uint32_t b = listed ? s_big[q] : q, st = s_bin[b], cnt = s_bin[b + 1] - st;
      if (cnt > WAVE) oe_sort_group<EntT, SORT_NT>(s_b + st, cnt);
    }
    __syncthreads();
  }
  // incremental builds that split old indices (npo > 1) need each index's smallest old entry
  // for K5's num_unique put-back quirk; with one new index per old index nothing reads it
  const bool track_old = FL && P.npo > 1;
  if (track_old) {  // s_bin is no longer read; the scan below orders these before use
    for (uint32_t i = threadIdx.x; i < ipc; i += SORT_NT) { s_fo[i] = 0xffffffffu; s_ho[i] = 0; }
  }
  DBG_PHASE(4);
  // dedupe + compaction: thread t owns the contiguous run [t*drun, t*drun + drun), drun =
  // ceil(n / SORT_NT) made odd (lanes drun words apart fall on distinct LDS banks) and
  // capped at PER: every thread takes a share of a small bucket, not half of them PER each
  const uint32_t drun = min((uint32_t)PER, ((n + SORT_NT - 1) / SORT_NT) | 1u);
  uint32_t keep_mask = 0, cnt = 0;
  EntT w[PER];
  const uint32_t i0 = threadIdx.x * drun;
  EntT prev0 = (!DUAL && i0 > 0 && i0 <= n) ? s_b[i0 - 1] : EntT(0);
  // DUAL: element i of the merged order of A = s_b[0, nsort) and B = s_b[nsort, n). The
  // split of the first i0 - 1 elements (ia of them from A) by binary search; this thread's
  // prev0 and run are the next drun + 1 elements of the merge.
  uint32_t ia = 0, ib = 0;
  if constexpr (DUAL) {
    const uint32_t na = nsort, nbo = n - nsort;
    const EntT* A = s_b;
    const EntT* B = s_b + nsort;
    const uint32_t d = i0 > 0 ? min(i0 - 1, n) : 0u;
    uint32_t lo = d > nbo ? d - nbo : 0u, hi = min(d, na);
    while (lo < hi) {  // ia = number of A elements among the first d merged ones
      const uint32_t mid = (lo + hi) >> 1;
      if (A[mid] < B[d - mid - 1]) lo = mid + 1; else hi = mid;
    }
    ia = lo;
    ib = d - lo;
    if (i0 > 0 && i0 <= n) {  // merged element i0 - 1
      const bool ta = ib >= nbo || (ia < na && A[ia] < B[ib]);
      prev0 = ta ? A[ia++] : B[ib++];
    }
  }
  DBG_PHASE(9);  // (thread 0) merge-path split found
  {
    EntT prev = prev0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t i = i0 + k;
      if ((uint32_t)k < drun && i < n) {
        if constexpr (DUAL) {
          const bool ta = ib >= n - nsort || (ia < nsort && s_b[ia] < s_b[nsort + ib]);
          w[k] = ta ? s_b[ia++] : s_b[nsort + ib++];
        } else {
          w[k] = s_b[i];
        }
        const bool drop = (i > 0) && ent_drop<EntT, FL>(w[k], prev);
        if (!drop) { keep_mask |= 1u << k; cnt++; }
        prev = w[k];
      }
    }
  }
  DBG_PHASE(10);  // (thread 0) its run merged and flagged
  uint32_t kept;
  uint32_t pos = block_excl_scan<SORT_NT>(cnt, s_tmp, &kept);  // has barriers: reads done
  uint32_t* s_sorted = reinterpret_cast<uint32_t*>(s_b);        // compacted e values (u32)
  // Index bounds and num_unique in the same pass. A dropped entry equals its sorted
  // predecessor, so the previous SORTED entry has the index and fingerprint of the previous
  // KEPT one. Indices (index of previous entry, index of this kept entry] start here.
  // num_unique (:558, :572-574): per index, entries whose fingerprint differs from the
  // previous entry's; an index's first entry compares against UINT32_MAX >> value_size.
  const uint32_t NONE = 0xffffffffu;
  auto index_of = [&](uint32_t e) -> uint32_t { return ish >= 32 ? 0u : ((e >> ish) & (ipc - 1)); };
  uint32_t lprev = (i0 > 0 && i0 <= n) ? index_of(ent_e<EntT, FL>(prev0)) : NONE;
  uint32_t fprev = (i0 > 0 && i0 <= n) ? (ent_e<EntT, FL>(prev0) >> P.vs) : 0u;
  uint32_t uniq = 0;
  uint32_t fo_li = NONE;  // index of this run's last recorded old entry
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t i = i0 + k;
    if ((uint32_t)k < drun && i < n) {
      const uint32_t e = ent_e<EntT, FL>(w[k]);
      const uint32_t li = index_of(e), fp = e >> P.vs;
      if (keep_mask & (1u << k)) {
        s_sorted[pos] = e;
        for (uint32_t l = lprev + 1; l <= li; l++) s_first[l] = pos;  // lprev NONE: from 0
        uniq += (fp != (li != lprev ? (0xffffffffu >> P.vs) : fprev)) ? 1u : 0u;
        pos++;
        if constexpr (FL) {
          // old entry: remember each index's smallest (num_unique quirk). The run is in
          // order, so its first old entry of an index is its smallest there: one LDS atomic
          // per (run, index) instead of one per old entry (all of an index's entries would
          // otherwise contend for one address)
          if (track_old && !(w[k] & EntT(1)) && li != fo_li) {
            atomicMin(&s_fo[li], e);
            s_ho[li] = 1;
            fo_li = li;
          }
        }
      }
      lprev = li;
      fprev = fp;
    }
  }
  __syncthreads();
  DBG_PHASE(5);
  {  // indices after the last entry's start at `kept`
    const uint32_t llast = kept ? index_of(s_sorted[kept - 1]) : NONE;
    for (uint32_t l = threadIdx.x; l < ipc; l += SORT_NT)
      if (llast == NONE || l > llast) s_first[l] = kept;
    if (threadIdx.x == 0) s_first[ipc] = kept;
  }
  if (track_old) {
    for (uint32_t i = threadIdx.x; i < ipc; i += SORT_NT) {
      first_old[c.idx0 + i] = s_fo[i];
      has_old[c.idx0 + i] = s_ho[i];
    }
  }
  uint32_t* dst = sorted32 + P.e_first + c.cb_rel;
  for (uint32_t i = threadIdx.x; i < kept; i += SORT_NT) dst[i] = s_sorted[i];
  __syncthreads();
  DBG_PHASE(6);
  for (uint32_t l = threadIdx.x; l < ipc; l += SORT_NT) {
    idx_cnt[c.idx0 + l] = s_first[l + 1] - s_first[l];
    idx_start[c.idx0 + l] = c.cb_rel + s_first[l];
  }
  DBG_PHASE(7);
  uint32_t tot_uniq;
  block_excl_scan<SORT_NT>(uniq, s_tmp, &tot_uniq);
  if (threadIdx.x == 0) atomicAdd(&outs[f].num_unique, tot_uniq);
  DBG_PHASE(8);
  if constexpr (LIST) __syncthreads();  // the next bucket reuses the LDS
  }
}

// K4m: the bucket sort of 32-bit incremental builds (routing_filter_add with an old filter,
// src/routing_filter.c:496-597). A coarse bucket's entries are its old run -- the old filter's
// entries, already in order -- and a small share of new ones (an eighth in round 8 of a
// compaction chain). Only the new entries are sorted (bins over their top bits sized to their
// count, then sorting networks); a new entry is dropped if it equals the previous new one
// (duplicates are dropped only among the new entries; one equal to an old entry is kept after
// it, src/routing_filter.c:559-597). The old run reaches LDS by LDS-DMA while the new entries
// sort, and is never sorted, scattered or compacted (the K4 DUAL path did all three). The
// merge (old first on equal entries) gives each thread a contiguous share of the output (a
// merge-path split of both runs, merged into registers); the merged run is staged in place
// over the old run and copied out with coalesced stores, num_unique and the index starts
// computed on the way.
// Buckets with more new entries than MRG_NEW_CAP, or a bin of more than 64 equal-bin new
// entries, go to k_cb_sort in list mode (bit 31 on their overflow-list entry); buckets over
// SORT_CAP to K4b as before.
constexpr uint32_t MRG_NEW_CAP = 2048;
constexpr uint32_t MRG_LNB_MAX = 9;  // at most 512 bins
constexpr uint32_t MRG_RUN = (SORT_CAP + SORT_NT - 1) / SORT_NT + 1;  // output slots per thread (odd)
__global__ __launch_bounds__(SORT_NT, 6) void k_cb_merge(const FilterPlan* __restrict__ plans,
                                                      const uint32_t* __restrict__ cb_filter,
                                                      const uint32_t* __restrict__ cb_count,
                                                      const uint32_t* __restrict__ cb_start,
                                                      const uint32_t* __restrict__ part,
                                                      const uint32_t* __restrict__ old32,
                                                      const uint32_t* __restrict__ ob_lo,
                                                      const uint32_t* __restrict__ ob_n,
                                                      uint32_t* __restrict__ sorted32,
                                                      uint32_t* __restrict__ idx_cnt,
                                                      uint32_t* __restrict__ idx_start,
                                                      FilterOut* __restrict__ outs,
                                                      uint32_t* __restrict__ overflow,
                                                      uint32_t lis, uint32_t* __restrict__ first_old,
                                                      uint32_t* __restrict__ has_old,
                                                      const uint32_t* __restrict__ spill,
                                                      const uint32_t* __restrict__ cb_outs) {
  constexpr int NPER = MRG_NEW_CAP / SORT_NT;
  __shared__ uint32_t s_old[SORT_CAP + 1];      // + a sentinel past the last old entry
  __shared__ uint32_t s_new[MRG_NEW_CAP + 1];   // + a sentinel past the last kept new entry
  static_assert((1u << MRG_LNB_MAX) >= MAX_IPC, "s_start (MAX_IPC + 1 words) over s_bin");
  __shared__ uint32_t s_bin[(1u << MRG_LNB_MAX) + 1];
  __shared__ uint32_t s_fo[MAX_IPC];
  __shared__ uint32_t s_tmp[SORT_NT / WAVE + 1];
  __shared__ uint32_t s_big;
  __shared__ uint32_t s_uniq;
  DBG_PHASE_K(5, 15);
  const uint32_t cb = xcd_chunk(blockIdx.x, gridDim.x);
  const uint32_t f = cb_filter[cb];
  const FilterPlan& P = plans[f];
  const uint32_t n = cb_count[cb];
  if (n > SORT_CAP) {  // K4b
    if (threadIdx.x == 0) overflow[1 + atomicAdd(&overflow[0], 1u)] = cb;
    return;
  }
  const uint32_t no = ob_n[cb], nn = n - no;
  if (nn > MRG_NEW_CAP) {  // k_cb_sort, list mode
    if (threadIdx.x == 0) overflow[1 + atomicAdd(&overflow[0], 1u)] = cb | 0x80000000u;
    return;
  }
  const uint32_t cbl = cb - P.cb_base;
  const uint32_t cb_rel = (spill && *spill == 0) ? cbl * CB_REGION : cb_start[cb];
  const uint32_t cb_out = cb_outs[cb];
  const uint32_t vs = P.vs, rvs = P.rvs, ovs = P.old_vs, bbits = P.bbits;
  const bool od = P.old_direct != 0;
  const uint32_t ipc = 1u << (bbits - lis), ish = lis + rvs;
  const uint32_t idx0 = P.idx_base + (cbl << (bbits - lis));
  // an old entry as this filter sees it (read in place from an engine-built old batch: value
  // bits re-widened to the new value_size, src/routing_filter.c:536-543; the order is unchanged)
  auto okey = [&](uint32_t raw) -> uint32_t { return od ? ((raw >> ovs) << vs) | (raw & ((1u << ovs) - 1u)) : raw; };
  auto index_of = [&](uint32_t e) -> uint32_t { return ish >= 32 ? 0u : ((e >> ish) & (ipc - 1)); };
  const uint32_t lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  // a barrier ordering this workgroup's LDS accesses only: the old run's LDS-DMA stays in
  // flight across it (__syncthreads, and even a release fence on LDS, wait for every
  // outstanding load -- LDS-DMA writes LDS and is counted as a load)
  auto lds_sync = [] {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // compiler-only ordering: no hardware wait implied
    __builtin_amdgcn_s_waitcnt(0xc07f);       // lgkmcnt(0): this wave's LDS accesses done
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  };
  // 1. the new entries ((e << 1) | 1 in the partition region): bins over their top bits,
  //    about four entries per bin
  uint32_t lnb = 0;
  while (lnb < MRG_LNB_MAX && lnb < bbits && (8u << lnb) <= nn) lnb++;
  const uint32_t nb = 1u << lnb, bsh = rvs + bbits - lnb;
  auto bin_of = [&](uint32_t e) -> uint32_t { return lnb ? (e >> bsh) & (nb - 1) : 0u; };
  const uint32_t* nsrc = part + P.e_first + cb_rel;
  uint32_t v[NPER], rk[NPER];
  const uint32_t nm1 = nn ? nn - 1 : 0u;  // clamped, branch-free: the loads go out together
#pragma unroll
  for (int k = 0; k < NPER; k++) v[k] = nsrc[min(threadIdx.x + k * SORT_NT, nm1)] >> 1;
  static_assert((1u << MRG_LNB_MAX) <= SORT_NT, "one bin counter per thread (+ the last)");
  if (threadIdx.x <= nb) s_bin[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    s_bin[nb] = 0;
    s_big = 0;
  }
  lds_sync();
  DBG_PHASE_K(5, 0);
#pragma unroll
  for (int k = 0; k < NPER; k++)
    if (threadIdx.x + k * SORT_NT < nn) rk[k] = atomicAdd(&s_bin[bin_of(v[k])], 1u);
  // 2. the old run into LDS (LDS-DMA, a dword per lane), in flight while the new entries sort:
  //    issued once the new entries have landed (a wave with plain loads and LDS-DMA both
  //    outstanding can only wait for all of them; splitting the two over different waves
  //    measured slower: the new entries then land behind the old run's traffic)
  {
    const uint32_t* osrc = (od ? P.old_entries : old32 + P.old_first) + ob_lo[cb];
    for (uint32_t i0 = wv * WAVE; i0 < no; i0 += SORT_NT)
      if (i0 + lane < no)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(osrc + i0 + lane),
                                         (__attribute__((address_space(3))) void*)(s_old + i0), 4, 0, 0);
  }
  lds_sync();
  DBG_PHASE_K(5, 1);
  if (wv == 0) {  // exclusive scan of the nb <= 512 counts: 8 per lane
    uint32_t c8[8], sum = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t b = lane * 8 + q;
      c8[q] = b < nb ? s_bin[b] : 0u;
      sum += c8[q];
    }
    uint32_t run = wave_incl_scan(sum) - sum;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t b = lane * 8 + q;
      if (b < nb) s_bin[b] = run;
      run += c8[q];
    }
    if (lane == WAVE - 1) s_bin[nb] = run;
  }
  lds_sync();
  DBG_PHASE_K(5, 2);
#pragma unroll
  for (int k = 0; k < NPER; k++)
    if (threadIdx.x + k * SORT_NT < nn) s_new[s_bin[bin_of(v[k])] + rk[k]] = v[k];
  lds_sync();
  DBG_PHASE_K(5, 3);
  {  // order inside the bins: segments of S bins (about 8 entries) sorted by one thread each
    uint32_t S = 8;
    while (S > 1 && S * nn > 8 * nb) S >>= 1;
    if (S > nb) S = nb;
    const uint32_t nseg = nb / S;
    for (uint32_t sg = threadIdx.x; sg < nseg; sg += SORT_NT) {
      const uint32_t b0 = sg * S, st = s_bin[b0], c = s_bin[b0 + S] - st;
      if (c <= 16) {
        uint32_t x[16];
#pragma unroll
        for (int j = 0; j < 16; j++) x[j] = (uint32_t)j < c ? s_new[st + j] : 0xffffffffu;
        sort16(x);
        if (c >= 2) {
#pragma unroll
          for (int j = 0; j < 16; j++)
            if ((uint32_t)j < c) s_new[st + j] = x[j];
        }
      } else {
        for (uint32_t b = b0; b < b0 + S; b++) {
          const uint32_t bs = s_bin[b], bc = s_bin[b + 1] - bs;
          if (bc > WAVE) {
            s_big = 1;  // duplicate-heavy input: k_cb_sort takes the bucket
          } else {
            for (uint32_t i = bs + 1; i < bs + bc; i++) {  // insertion sort, at most 64
              const uint32_t x = s_new[i];
              uint32_t q = i;
              while (q > bs && s_new[q - 1] > x) {
                s_new[q] = s_new[q - 1];
                q--;
              }
              s_new[q] = x;
            }
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of the old run has landed
  __syncthreads();                                   // ... and every wave's
  DBG_PHASE_K(5, 4);
  if (s_big) {
    if (threadIdx.x == 0) overflow[1 + atomicAdd(&overflow[0], 1u)] = cb | 0x80000000u;
    return;
  }
  // 3. drop new duplicates of the previous new entry (only among the new ones: a new entry
  //    equal to an old one is kept, after it -- src/routing_filter.c:559-597) and compact the
  //    kept ones to s_new[0, kn). Thread t takes new entries [t NPER, t NPER + NPER).
  uint32_t kv[NPER], kc = 0;
  bool keep[NPER];
#pragma unroll
  for (int k = 0; k < NPER; k++) {
    const uint32_t j = threadIdx.x * NPER + k;
    kv[k] = j < nn ? s_new[j] : 0u;
    keep[k] = j < nn && (j == 0 || s_new[j - 1] != kv[k]);
    kc += keep[k] ? 1u : 0u;
  }
  // (skipping the compaction when there are no duplicates, behind a __syncthreads_or, measured
  // slower: 3.9K -> 4.9K cycles for this phase)
  uint32_t kn;
  uint32_t r = block_excl_scan<SORT_NT>(kc, s_tmp, &kn);  // its barriers: every s_new read done
#pragma unroll
  for (int k = 0; k < NPER; k++)
    if (keep[k]) s_new[r++] = kv[k];
  if (threadIdx.x == 0) s_uniq = 0;
  // the old run as this filter sees it, once (value bits re-widened when the old filter's
  // value_size differs), and the sentinels the merge reads past each side's end (entries are
  // < 2^31: the sentinel sorts after every entry)
  if (od && ovs != vs)
    for (uint32_t i = threadIdx.x; i < no; i += SORT_NT) s_old[i] = okey(s_old[i]);
  if (threadIdx.x == 0) {
    s_old[no] = 0xffffffffu;
    s_new[kn] = 0xffffffffu;
  }
  for (uint32_t l = threadIdx.x; l < ipc; l += SORT_NT) {
    s_fo[l] = 0xffffffffu;
    s_bin[l] = 0xffffffffu;  // s_start below: the start of each non-empty index
  }
  __syncthreads();
  DBG_PHASE_K(5, 5);
  // 4. the merge (old first on equal entries), each thread a contiguous range of output slots
  //    (merge-path split by binary search) merged into registers, branch-free: one LDS read per
  //    step from the side just consumed. num_unique, the start of each non-empty index (s_start,
  //    over s_bin) and each index's smallest old entry (s_fo, for builds that split old indices:
  //    npo > 1) from each entry and its predecessor. After a barrier the merged run is staged in
  //    place over s_old (slot sl holds merged entry sl; every input was read before the
  //    barrier) and copied out with coalesced stores.
  const uint32_t tot = no + kn;
  uint32_t* dst = sorted32 + P.e_first + cb_out;
  uint32_t* s_start = s_bin;  // MAX_IPC + 1 words
  const bool track_old = P.npo > 1;
  const uint32_t NONE = 0xffffffffu;
  const uint32_t run = min((uint32_t)MRG_RUN, ((tot + SORT_NT - 1) / SORT_NT) | 1u);
  const uint32_t d = threadIdx.x * run;
  uint32_t uniq = 0;
  uint32_t mv[MRG_RUN];
  if (d < tot) {
    uint32_t lo = d > kn ? d - kn : 0u, hi = min(d, no);
    while (lo < hi) {  // ia = old entries among the first d merged ones
      const uint32_t mid = (lo + hi) >> 1;
      if (s_old[mid] <= s_new[d - mid - 1]) lo = mid + 1; else hi = mid;
    }
    uint32_t ia = lo, ib = d - lo;
    // the merged predecessor of slot d (new after old on equal entries), its index and
    // fingerprint; the last old entry before slot d (its index): NONE = none
    uint32_t prev = NONE, pold = NONE;
    if (d > 0) {
      const uint32_t po = ia > 0 ? s_old[ia - 1] : 0u;
      const uint32_t pn = ib > 0 ? s_new[ib - 1] : 0u;
      prev = (ib > 0 && (ia == 0 || pn >= po)) ? pn : po;
      if (ia > 0) pold = index_of(po);
    }
    uint32_t pli = prev == NONE ? NONE : index_of(prev);
    uint32_t pfp = prev == NONE ? 0u : prev >> vs;
    uint32_t onext = s_old[ia], nnext = s_new[ib];  // sentinels past the ends
    const uint32_t end = min(tot, d + run);
#pragma unroll
    for (uint32_t k = 0; k < MRG_RUN; k++) {
      const uint32_t sl = d + k;
      if (sl < end) {
        const bool take_old = onext <= nnext;  // old first on equal entries; a side's sentinel never wins
        const uint32_t e = take_old ? onext : nnext;
        ia += take_old ? 1u : 0u;
        ib += take_old ? 0u : 1u;
        const uint32_t x = take_old ? s_old[ia] : s_new[ib];
        onext = take_old ? x : onext;
        nnext = take_old ? nnext : x;
        mv[k] = e;
        const uint32_t li = index_of(e), fp = e >> vs;
        const bool first = li != pli;  // pli NONE: no predecessor
        uniq += fp != (first ? (0xffffffffu >> vs) : pfp) ? 1u : 0u;
        if (first) s_start[li] = sl;
        if (track_old && take_old) {
          if (li != pold) s_fo[li] = e;
          pold = li;
        }
        pli = li;
        pfp = fp;
      }
    }
  }
  __syncthreads();  // every input read
  if (d < tot) {
#pragma unroll
    for (uint32_t k = 0; k < MRG_RUN; k++)
      if (k < run && d + k < tot) s_old[d + k] = mv[k];
  }
  // 5. per index: start (an empty index starts where the next non-empty one does: a suffix
  //    minimum over the indices, tot past the last) and count; its smallest old entry (npo > 1)
  static_assert(MAX_IPC <= SORT_NT, "one index per thread");
  uint32_t st = threadIdx.x < ipc ? s_start[threadIdx.x] : NONE;
#pragma unroll
  for (uint32_t off = 1; off < WAVE; off <<= 1) {
    const uint32_t y = __shfl_down(st, off, WAVE);
    if (lane + off < WAVE) st = min(st, y);
  }
  if (lane == 0) s_tmp[wv] = st;
  __syncthreads();  // also: the merged run staged in s_old
  for (uint32_t w2 = wv + 1; w2 < SORT_NT / WAVE; w2++) st = min(st, s_tmp[w2]);
  st = min(st, tot);
  for (uint32_t i = threadIdx.x; i < tot; i += SORT_NT) dst[i] = s_old[i];
  __syncthreads();  // every s_tmp and s_start read
  if (threadIdx.x < ipc) s_start[threadIdx.x] = st;
  if (threadIdx.x == 0) s_start[ipc] = tot;
  __syncthreads();
  DBG_PHASE_K(5, 6);
  if (threadIdx.x < ipc) {
    const uint32_t l = threadIdx.x;
    idx_cnt[idx0 + l] = s_start[l + 1] - st;
    idx_start[idx0 + l] = cb_out + st;
    if (track_old) {
      first_old[idx0 + l] = s_fo[l];
      has_old[idx0 + l] = s_fo[l] != NONE ? 1u : 0u;
    }
  }
  DBG_PHASE_K(5, 7);
  // num_unique: a wave sum, one LDS atomic per wave, one global atomic per workgroup
  const uint32_t wsum = __builtin_amdgcn_readlane((int)wave_incl_scan(uniq), WAVE - 1);
  if (lane == 0 && wsum) atomicAdd(&s_uniq, wsum);
  __syncthreads();
  if (threadIdx.x == 0 && s_uniq) atomicAdd(&outs[f].num_unique, s_uniq);
  DBG_PHASE_K(5, 8);
}

// K4b: coarse buckets larger than LDS (duplicate-heavy inputs). One workgroup per listed
// bucket, working in global memory: `scratch` is the K1 entry array (free after K3).
template <typename EntT, bool FL = (sizeof(EntT) == 8), bool DUAL = false>
__global__ __launch_bounds__(BIG_NT) void k_cb_sort_big(const FilterPlan* __restrict__ plans,
                                                        const uint32_t* __restrict__ cb_filter,
                                                        const uint32_t* __restrict__ cb_count,
                                                        const uint32_t* __restrict__ cb_start,
                                                        const EntT* __restrict__ part,
                                                        const uint32_t* __restrict__ old32,
                                                        const uint32_t* __restrict__ ob_lo,
                                                        const uint32_t* __restrict__ ob_n,
                                                        EntT* __restrict__ scratch,
                                                        uint32_t* __restrict__ sorted32,
                                                        uint32_t* __restrict__ idx_cnt,
                                                        uint32_t* __restrict__ idx_start,
                                                        FilterOut* __restrict__ outs,
                                                        const uint32_t* __restrict__ overflow,
                                                        uint32_t lis, uint32_t* __restrict__ first_old,
                                                        uint32_t* __restrict__ has_old,
                                                        const uint32_t* __restrict__ spill,
                                                        const uint32_t* __restrict__ cb_outs) {
  __shared__ uint32_t s_bin[MAX_BINS + 1];
  __shared__ uint32_t s_fo[MAX_IPC];
  __shared__ uint32_t s_ho[MAX_IPC];
  __shared__ uint32_t s_cur[MAX_BINS];
  __shared__ uint32_t s_tmp[BIG_NT / WAVE + 1];
  __shared__ uint32_t s_run;
  const uint32_t nover = overflow[0];
  for (uint32_t it = blockIdx.x; it < nover; it += gridDim.x) {
    const uint32_t cb = overflow[1 + it];
    if (cb >> 31) continue;  // K4m's fallback entries: k_cb_sort in list mode
    const uint32_t f = cb_filter[cb];
    const FilterPlan& P = plans[f];
    const uint32_t n = cb_count[cb];
    const uint32_t cbl = cb - P.cb_base;
    const uint32_t in_rel = (spill && *spill == 0) ? cbl * CB_REGION : cb_start[cb];
    // fused 32-bit incremental builds: the sorted (and scratch) layout is the scan of the
    // coarse buckets' new + old counts (cb_outs), the new entries' layout is the partition's
    const uint32_t out_rel = (DUAL && spill) ? cb_outs[cb] : in_rel;
    CbCtx c{P.rvs, P.vs, lis, P.bbits, P.idx_base + (cbl << (P.bbits - lis)), out_rel, P.e_first};
    const uint32_t nbins = 1u << (P.bbits - P.binsh), bmask = nbins - 1, bsh = P.rvs + P.binsh;
    const EntT* srcp = part + P.e_first + in_rel;
    const uint32_t nn = DUAL ? n - ob_n[cb] : n;
    const uint32_t* osrc = DUAL ? (P.old_direct ? P.old_entries : old32 + P.old_first) + ob_lo[cb] : nullptr;
    auto src = [&](uint32_t i) -> EntT {
      if (!DUAL || i < nn) return srcp[i];
      const uint32_t eo = osrc[i - nn];  // read in place: re-widen the value bits
      const uint32_t e = P.old_direct ? ((eo >> P.old_vs) << P.vs) | (eo & ((1u << P.old_vs) - 1u)) : eo;
      return (EntT)(e << 1);
    };
    EntT* tmp = scratch + P.e_first + c.cb_rel;
    uint32_t* dst = sorted32 + P.e_first + c.cb_rel;
    const uint32_t ipc = 1u << (P.bbits - lis), ish = lis + P.rvs;
    for (uint32_t i = threadIdx.x; i <= nbins; i += BIG_NT) s_bin[i] = 0;
    for (uint32_t i = threadIdx.x; i < ipc; i += BIG_NT) { s_fo[i] = 0xffffffffu; s_ho[i] = 0; }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += BIG_NT) {
      const uint32_t e = ent_e<EntT, FL>(src(i));
      atomicAdd(&s_bin[bsh >= 32 ? 0u : ((e >> bsh) & bmask)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t run = 0;
      for (uint32_t b = 0; b < nbins; b++) {
        const uint32_t x = s_bin[b];
        s_bin[b] = run;
        s_cur[b] = run;
        run += x;
      }
      s_bin[nbins] = run;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += BIG_NT) {
      const EntT x = src(i);
      const uint32_t e = ent_e<EntT, FL>(x);
      tmp[atomicAdd(&s_cur[bsh >= 32 ? 0u : ((e >> bsh) & bmask)], 1u)] = x;
    }
    __syncthreads();
    // order inside each bin: small bins by one thread each (insertion sort of at most 64),
    // larger ones (duplicate-heavy) by the whole workgroup, one after another
    for (uint32_t b = threadIdx.x; b < nbins; b += BIG_NT) {
      const uint32_t s = s_bin[b], e = s_bin[b + 1];
      if (e - s > WAVE) continue;
      for (uint32_t i = s + 1; i < e; i++) {
        const EntT x = tmp[i];
        uint32_t j = i;
        while (j > s && tmp[j - 1] > x) {
          tmp[j] = tmp[j - 1];
          j--;
        }
        tmp[j] = x;
      }
    }
    __syncthreads();
    for (uint32_t b = 0; b < nbins; b++) {  // workgroup-uniform
      const uint32_t s = s_bin[b], cnt = s_bin[b + 1] - s;
      if (cnt > WAVE) oe_sort_group<EntT, BIG_NT>(tmp + s, cnt);
    }
    __syncthreads();
    if (threadIdx.x == 0) s_run = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += BIG_NT) {
      const uint32_t i = base + threadIdx.x;
      uint32_t keep = 0;
      EntT x = 0;
      if (i < n) {
        x = tmp[i];
        keep = (i == 0 || !ent_drop<EntT, FL>(x, tmp[i - 1])) ? 1u : 0u;
      }
      uint32_t tot;
      const uint32_t p = block_excl_scan<BIG_NT>(keep, s_tmp, &tot);
      const uint32_t run = s_run;
      if (keep) {
        dst[run + p] = ent_e<EntT, FL>(x);
        if constexpr (FL) {
          if (!(x & EntT(1))) {
            const uint32_t e = ent_e<EntT, FL>(x);
            const uint32_t li = ish >= 32 ? 0u : ((e >> ish) & (ipc - 1));
            atomicMin(&s_fo[li], e);
            s_ho[li] = 1;
          }
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) s_run = run + tot;
      __syncthreads();
    }
    const uint32_t kept = s_run;
    if constexpr (FL) {
      for (uint32_t i = threadIdx.x; i < ipc; i += BIG_NT) {
        first_old[c.idx0 + i] = s_fo[i];
        has_old[c.idx0 + i] = s_ho[i];
      }
    }
    uint32_t uniq, tot_uniq;
    write_index_bounds(c, dst, kept, idx_cnt, idx_start, &uniq);
    block_excl_scan<BIG_NT>(uniq, s_tmp, &tot_uniq);
    if (threadIdx.x == 0) atomicAdd(&outs[f].num_unique, tot_uniq);
    __syncthreads();
  }
}

// ======================================================================================
// K5: block sizes + greedy page placement (src/routing_filter.c:599-620)
//
// next(j) = the block that starts the page after a page starting at block j
// (first q with excl[q+1] - excl[j] > page_size). Page starts are the orbit of block 0
// under next(); it is marked in ceil(log2(n+1)) pointer-doubling rounds.
// ======================================================================================
__device__ __forceinline__ uint32_t block_size(uint32_t c, uint32_t index_size, uint32_t rvs) {
  const uint32_t enc = (c + index_size - 1) / 8 + 4;
  const uint64_t bits = (uint64_t)c * rvs;
  const uint32_t rbs = bits == 0 ? 3u : (uint32_t)((bits - 1) / 8 + 4);  // u32 wrap quirk
  return enc + 2 + rbs;
}

constexpr uint32_t LAYOUT_LIST = 520;
__global__ __launch_bounds__(LAYOUT_NT) void k_layout(const FilterPlan* __restrict__ plans,
                                                      const uint32_t* __restrict__ idx_cnt,
                                                      const uint32_t* __restrict__ idx_start,
                                                      const uint32_t* __restrict__ sorted32,
                                                      const uint32_t* __restrict__ first_old,
                                                      const uint32_t* __restrict__ has_old,
                                                      uint4* __restrict__ pplans,
                                                      uint64_t* __restrict__ slots,
                                                      uint32_t* __restrict__ page_first,
                                                      FilterOut* __restrict__ outs,
                                                      uint32_t lis, uint32_t page_size) {
  __shared__ uint32_t s_excl[MAX_INDICES + 1];
  __shared__ uint16_t s_jA[MAX_INDICES + 1];
  __shared__ uint16_t s_jB[MAX_INDICES + 1];
  __shared__ uint8_t s_mark[MAX_INDICES + 1];
  __shared__ uint32_t s_tmp[LAYOUT_NT / WAVE + 1];
  __shared__ uint32_t s_err;
  __shared__ uint16_t s_list[LAYOUT_LIST];  // every 2^R-th page start (<= 2 est / 2^R + 1 <= 257 of them)
  __shared__ uint32_t s_wt[MAX_INDICES / LAYOUT_NT * (LAYOUT_NT / WAVE) + 1];  // k-major scan totals
  __shared__ uint32_t s_nlist;
  const uint32_t f = blockIdx.x;
  const FilterPlan& P = plans[f];
  const uint32_t n = P.num_indices;
  const uint32_t index_size = 1u << lis;
  constexpr int PER = MAX_INDICES / LAYOUT_NT;
  DBG_PHASE_K(4, 15);
  if (threadIdx.x == 0) s_err = 0;
  __syncthreads();
  // sizes -> exclusive prefix (element j = k * LAYOUT_NT + thread: coalesced loads)
  // every count load first, from a clamped index (no branch around a load: each branch
  // ended in its own wait, 16 serialised round trips per thread), then the sizes
  uint32_t sz[PER], err = 0;
#pragma unroll
  for (int k = 0; k < PER; k++) sz[k] = idx_cnt[P.idx_base + min((uint32_t)(k * LAYOUT_NT) + threadIdx.x, n - 1)];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t j = k * LAYOUT_NT + threadIdx.x;
    const uint32_t c = sz[k];
    sz[k] = 0;
    if (j < n) {
      if (c > 4096) err |= ERR_INDEX_OVERFLOW;
      sz[k] = block_size(c, index_size, P.rvs);
      if (sz[k] > page_size) err |= ERR_BLOCK_TOO_BIG;
    }
  }
  if (err) atomicOr(&s_err, err);
  DBG_PHASE_K(4, 5);  // thread 0's sizes loaded (no barrier)
  uint32_t total;
  block_excl_scan_kmajor<LAYOUT_NT, PER>(sz, s_wt, &total);  // sz becomes the exclusive prefix
  DBG_PHASE_K(4, 6);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t j = k * LAYOUT_NT + threadIdx.x;
    if (j < n) s_excl[j] = sz[k];
  }
  // the total at j == n: no thread owns it when n == MAX_INDICES
  if (threadIdx.x == 0) s_excl[n] = total;
  __syncthreads();
  if (s_err) {
    if (threadIdx.x == 0) {
      outs[f].error |= s_err;
      pplans[f].w = s_err;  // probes of a failed filter find nothing
    }
    return;
  }
  DBG_PHASE_K(4, 0);
  if (threadIdx.x == 0) pplans[f].w = 0;
  // next(j) = first block that does not fit on a page opened at block j. next() is
  // non-decreasing in j, so each thread takes a run of `run` consecutive blocks: the first
  // is found by galloping from j + 1 then bisecting, the rest by advancing that pointer
  // (about one LDS read per block instead of a gallop + bisect each). An odd run length
  // (17 at 16,384 indices) keeps a wave's reads on distinct LDS banks.
  {
    const uint32_t run = ((n + LAYOUT_NT - 1) / LAYOUT_NT) | 1u;  // run * LAYOUT_NT >= n
    const uint32_t j0 = threadIdx.x * run, j1 = min(j0 + run, n);
    uint32_t qp = 0;
#pragma unroll 1
    for (uint32_t j = j0; j < j1; j++) {
      const uint32_t lim = s_excl[j] + page_size;
      if (j == j0) {
        qp = j + 1;  // first q' > j with excl[q'] > lim (n + 1: none)
        if (qp <= n && s_excl[qp] <= lim) {
          uint32_t lo = qp, hi = qp + 1, step = 1;  // excl[lo] <= lim
          while (hi <= n && s_excl[hi] <= lim) {
            lo = hi;
            step <<= 1;
            hi = lo + step;
          }
          if (hi > n + 1) hi = n + 1;
          while (hi - lo > 1) {  // excl[lo] <= lim < excl[hi] (hi == n + 1: past the end)
            const uint32_t mid = (lo + hi) >> 1;
            if (s_excl[mid] <= lim) lo = mid; else hi = mid;
          }
          qp = hi;
        }
      } else {
        // blocks in [j, next(j - 1)) fit under lim(j - 1) <= lim(j): start there
        qp = max(qp, j + 1);
        while (qp <= n && s_excl[qp] <= lim) qp++;
      }
      s_jA[j] = (uint16_t)(qp - 1);  // block qp-1 is the first that does not fit (n: none)
    }
    if (threadIdx.x == 0) s_jA[n] = (uint16_t)n;
  }
  __syncthreads();
  DBG_PHASE_K(4, 1);
  // Mark the orbit of block 0 under next() (the page starts). R rounds of in-place pointer
  // doubling give J = next^(2^R) in s_jB; one lane walks the orbit with J (every 2^R-th
  // page start), then each of those points walks up to 2^R - 1 steps of next() marking the
  // page starts in between. A doubling round (every index, a barrier) costs about as much as
  // ~100 dependent LDS reads of the single-lane walk, so R = log2(pages) - 7 (C2: 1,366
  // pages, R = 4: 85 + 15 dependent reads; R = 6 took 41 % of K5, 17 us).
  {
    const uint32_t est = s_excl[n] / page_size + 1;  // pages >= est - 1, and <= 2 est
    const uint32_t lg = 32u - __clz(est);
    const uint32_t R = min(8u, lg > 8 ? lg - 7 : 1u);
    for (uint32_t j = threadIdx.x; j <= n; j += LAYOUT_NT) s_jB[j] = s_jA[j];
    __syncthreads();
    for (uint32_t r = 0; r < R; r++) {
      uint16_t c1[PER + 1];
#pragma unroll
      for (int k = 0; k <= PER; k++) {
        const uint32_t j = threadIdx.x + k * LAYOUT_NT;
        c1[k] = j <= n ? s_jB[j] : (uint16_t)0;
      }
#pragma unroll
      for (int k = 0; k <= PER; k++) {
        const uint32_t j = threadIdx.x + k * LAYOUT_NT;
        if (j <= n) c1[k] = s_jB[c1[k]];
      }
      __syncthreads();  // every read of this round before any write
#pragma unroll
      for (int k = 0; k <= PER; k++) {
        const uint32_t j = threadIdx.x + k * LAYOUT_NT;
        if (j <= n) s_jB[j] = c1[k];
      }
      __syncthreads();
    }
    // one lane walks the coarse orbit 0, J(0), J(J(0)), ... up to the end marker n
    if (threadIdx.x == 0) {
      uint32_t m = 0, x = 0;
      while (x != n && m < LAYOUT_LIST) {
        s_list[m++] = (uint16_t)x;
        x = s_jB[x];
      }
      s_nlist = m;
      if (x != n) {  // cannot happen (m <= 257); reported, never silently wrong
        outs[f].error |= ERR_PAGE_CAP;
        pplans[f].w = ERR_PAGE_CAP;
      }
    }
    for (uint32_t j = threadIdx.x; j <= n; j += LAYOUT_NT) s_mark[j] = 0;
    __syncthreads();
    const uint32_t m = s_nlist;
    for (uint32_t i = threadIdx.x; i < m; i += LAYOUT_NT) {
      uint32_t x = s_list[i];
      s_mark[x] = 1;
      for (uint32_t st = 1; st < (1u << R); st++) {
        x = s_jA[x];
        if (x == n) break;
        s_mark[x] = 1;
      }
    }
    __syncthreads();
  }
  DBG_PHASE_K(4, 2);
  // page numbers: inclusive scan of marks over [0, n)
  uint32_t mk[PER], pg[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t j = k * LAYOUT_NT + threadIdx.x;
    mk[k] = j < n ? s_mark[j] : 0u;
    pg[k] = mk[k];
  }
  uint32_t npages;
  block_excl_scan_kmajor<LAYOUT_NT, PER>(pg, s_wt, &npages);
  uint16_t* s_pstart = s_jB;  // reuse: page -> first block
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t j = k * LAYOUT_NT + threadIdx.x;
    pg[k] += mk[k] - 1;  // inclusive count - 1
    if (j < n && mk[k]) s_pstart[pg[k]] = (uint16_t)j;
  }
  __syncthreads();
  uint32_t* pf = page_first + P.pf_base;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t j = k * LAYOUT_NT + threadIdx.x;
    if (j < n) {
      const uint32_t ps = s_pstart[pg[k]];
      slots[P.idx_base + j] = (uint64_t)pg[k] * page_size + (s_excl[j] - s_excl[ps]);
      if (mk[k] && pg[k] < P.page_cap) pf[pg[k]] = j;
    }
  }
  DBG_PHASE_K(4, 3);
  // num_unique quirk of the old/new merge (src/routing_filter.c:572-590): when index j runs
  // out of entries while its old index still holds entries of a later new index, the first
  // of those is counted before the bucket check puts it back, and counted again later.
  if (P.npo > 1) {
    __syncthreads();
    uint32_t* s_next = s_excl;  // reuse: next index with an old entry (suffix min)
    uint32_t loc[PER], m = 0xffffffffu;
#pragma unroll
    for (int k = PER - 1; k >= 0; k--) {
      const uint32_t j = threadIdx.x * PER + k;
      loc[k] = m;  // exclusive suffix min within this thread's chunk
      if (j < n && has_old[P.idx_base + j]) m = j;
    }
    // exclusive suffix-min across threads: thread t needs min over threads > t
    uint32_t x = m;
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const uint32_t y = __shfl_down(x, d, WAVE);
      if (lane + d < WAVE) x = min(x, y);
    }
    if (lane == 0) s_tmp[wv] = x;  // wave-inclusive suffix min at lane 0
    __syncthreads();
    uint32_t after_wave = 0xffffffffu;
    for (int w2 = wv + 1; w2 < LAYOUT_NT / WAVE; w2++) after_wave = min(after_wave, s_tmp[w2]);
    __syncthreads();  // every wave has read s_tmp before block_excl_scan below rewrites it
    uint32_t xn = __shfl_down(x, 1, WAVE);
    if (lane == WAVE - 1) xn = 0xffffffffu;
    const uint32_t beyond = min(xn, after_wave);  // min over threads > t
    uint32_t extra = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t j = threadIdx.x * PER + k;
      const uint32_t nx = min(loc[k], beyond);
      if (j < n && (j + 1) % P.npo != 0 && nx < (j / P.npo + 1) * P.npo) {
        const uint32_t c = idx_cnt[P.idx_base + j];
        const uint32_t last = c ? sorted32[P.e_first + idx_start[P.idx_base + j] + c - 1] : 0xffffffffu;
        const uint32_t peek = first_old[P.idx_base + nx];
        if ((peek >> P.vs) != (last >> P.vs)) extra++;
      }
    }
    (void)s_next;
    uint32_t tot_extra;
    block_excl_scan<LAYOUT_NT>(extra, s_tmp, &tot_extra);
    if (threadIdx.x == 0 && tot_extra) atomicAdd(&outs[f].num_unique, tot_extra);
  }
  if (threadIdx.x == 0) {
    if (npages <= P.page_cap) pf[npages] = n;
    outs[f].num_pages = npages;
    if (npages > P.page_cap) {
      outs[f].error |= ERR_PAGE_CAP;
      pplans[f].w = ERR_PAGE_CAP;
    }
  }
  DBG_PHASE_K(4, 8);
}

// ======================================================================================
// K6: page assembly in LDS, 16-byte stores (src/routing_filter.c:612-633)
// ======================================================================================
__device__ __forceinline__ void lds_or_bits(uint32_t* s, uint64_t bitpos, uint32_t val, uint32_t nbits) {
  if (nbits == 0) return;
  const uint32_t w = (uint32_t)(bitpos >> 5), sh = (uint32_t)(bitpos & 31);
  const uint64_t v = (uint64_t)(nbits >= 32 ? val : (val & ((1u << nbits) - 1))) << sh;
  if ((uint32_t)v) atomicOr(&s[w], (uint32_t)v);
  if ((uint32_t)(v >> 32)) atomicOr(&s[w + 1], (uint32_t)(v >> 32));
}

// Fallback for pages with more blocks / entries than the word-parallel path stages in LDS
// (tiny index_size or rvs): bits OR-ed into the LDS page image s_pg with atomics (the
// caller stores it).
__device__ __forceinline__ void assemble_atomic(const FilterPlan& P, uint32_t p, uint32_t slot, uint32_t b0,
                                                uint32_t b1, const uint32_t* __restrict__ idx_cnt,
                                                const uint32_t* __restrict__ idx_start,
                                                const uint32_t* __restrict__ sorted32,
                                                const uint64_t* __restrict__ slots, uint8_t* __restrict__ pages,
                                                uint32_t lis, uint32_t page_size, uint32_t* s_pg) {
  const uint32_t nwords = page_size / 4;
  for (uint32_t i = threadIdx.x; i < nwords + 4; i += ASM_NT) s_pg[i] = 0;
  const uint32_t index_size = 1u << lis;
  __syncthreads();
  // phase 1: header count + 0xFF encoding fill
  for (uint32_t b = b0; b < b1; b++) {
    const uint32_t g = P.idx_base + b;
    const uint32_t off = (uint32_t)(slots[g] - (uint64_t)p * page_size);
    const uint32_t c = idx_cnt[g];
    const uint32_t enc = (c + index_size - 1) / 8 + 4;
    if (threadIdx.x == 0) lds_or_bits(s_pg, (uint64_t)off * 8, c & 0xffffu, 16);
    const uint32_t e0 = off + 2, e1 = off + 2 + enc;
    for (uint32_t w = (e0 >> 2) + threadIdx.x; w <= ((e1 - 1) >> 2); w += ASM_NT) {
      const uint32_t lo = max(e0, w * 4), hi = min(e1, w * 4 + 4);
      const uint32_t m = (hi - lo == 4) ? 0xffffffffu : (((1u << ((hi - lo) * 8)) - 1) << ((lo & 3) * 8));
      atomicOr(&s_pg[w], m);
    }
  }
  __syncthreads();
  // phase 2: clear encoding bits of entries, OR packed remainders
  const uint32_t remmask = P.rem >= 32 ? 0xffffffffu : ((1u << P.rem) - 1);
  for (uint32_t b = b0; b < b1; b++) {
    const uint32_t g = P.idx_base + b;
    const uint32_t off = (uint32_t)(slots[g] - (uint64_t)p * page_size);
    const uint32_t c = idx_cnt[g];
    const uint32_t enc = (c + index_size - 1) / 8 + 4;
    const uint32_t* ent = sorted32 + P.e_first + idx_start[g];
    const uint64_t ebit = (uint64_t)(off + 2) * 8;
    const uint64_t rbit = (uint64_t)(off + 2 + enc) * 8;
    for (uint32_t k = threadIdx.x; k < c; k += ASM_NT) {
      const uint32_t e = ent[k];
      const uint32_t fp = e >> P.vs;
      const uint32_t bucket_off = (P.rem >= 32 ? 0u : (fp >> P.rem)) & (index_size - 1);
      const uint64_t hb = ebit + k + bucket_off;
      atomicAnd(&s_pg[hb >> 5], ~(1u << (hb & 31)));
      const uint32_t rv = ((fp & remmask) << P.vs) | (e & ((1u << P.vs) - 1));
      lds_or_bits(s_pg, rbit + (uint64_t)k * P.rvs, rv, P.rvs);
    }
  }
}

constexpr uint32_t ASM_MAXB = 128;  // blocks per page held in LDS (more: assemble_atomic)
constexpr uint32_t ASM_RUN = 16;    // entries per thread-run in phase C
constexpr uint32_t ASM_MAXE = 16384;  // entries per page covered by the run table
constexpr uint32_t ASM_GT = 1024;     // group-start table entries per page (lines_asm bound)

// 64 bits of the LDS page image from bit `bitpos` (the image has 4 words of tail padding)
__device__ __forceinline__ uint64_t lds_bits64(const uint32_t* s_pg, uint32_t bitpos) {
  const uint32_t w = bitpos >> 5, sh = bitpos & 31;
  const uint64_t lo = ((uint64_t)s_pg[w + 1] << 32) | s_pg[w];
  return (lo >> sh) | (sh ? (uint64_t)s_pg[w + 2] << (64 - sh) : 0ull);
}

// One workgroup per page. (A) block metadata in LDS. (B) word-parallel fill of the LDS page
// image: header counts, 0xFF encodings, zeros -- plain stores. (C) entry runs: a thread
// takes ASM_RUN consecutive entries of the page, accumulates their encoding-clear bits
// (entry k at encoding bit k + bucket_off) and packed remainder bits (e & (2^rvs - 1) ==
// the reference's remainder|value) in 64-bit registers and flushes each 64-bit window
// with one atomic: adjacent lanes share at most a window edge. (D) 16-byte stores.
// Measured before: entry-parallel single-bit atomics (~19 LDS conflict cycles per LDS
// instruction), and a byte-serial gather per 16-byte chunk (3.6x slower again).
__global__ __launch_bounds__(ASM_NT) __attribute__((amdgpu_waves_per_eu(8))) void k_assemble(const FilterPlan* __restrict__ plans,
                                                     const uint32_t* __restrict__ pg_filter,
                                                     const uint32_t* __restrict__ idx_cnt,
                                                     const uint32_t* __restrict__ idx_start,
                                                     const uint32_t* __restrict__ sorted32,
                                                     const uint64_t* __restrict__ slots,
                                                     const uint32_t* __restrict__ page_first,
                                                     const FilterOut* __restrict__ outs,
                                                     uint8_t* __restrict__ pages, uint4* __restrict__ lines,
                                                     uint32_t* __restrict__ pg_noline,
                                                     uint32_t lis, uint32_t page_size) {
  __shared__ __attribute__((aligned(16))) uint32_t s_pg[MAX_PAGE / 4 + 4];
  __shared__ uint32_t s_wpre[ASM_MAXB];
  __shared__ uint32_t s_off[ASM_MAXB + 1];
  __shared__ uint32_t s_c[ASM_MAXB];
  __shared__ uint32_t s_est[ASM_MAXB + 1];
  __shared__ uint32_t s_src[ASM_MAXB];
  // block of each run (phases A-C; < ASM_MAXB blocks: one byte each)
  __shared__ uint8_t s_rblk[ASM_MAXE / ASM_RUN + ASM_MAXB];
  // s_wm (phases A-B; byte w: a block j >= 1 starts in word w) and s_gs (phases C-E; per
  // block: bit after each line group's last terminator) share one array: 16 pages per CU
  __shared__ __attribute__((aligned(16))) uint32_t s_wmgs[MAX_PAGE / 16 > ASM_GT / 2 ? MAX_PAGE / 16 : ASM_GT / 2];
  uint32_t* const s_wm = s_wmgs;
  uint16_t* const s_gs = reinterpret_cast<uint16_t*>(s_wmgs);
  __shared__ uint32_t s_tmp[ASM_NT / WAVE + 1];
  DBG_PHASE_K(3, 15);
  const uint32_t slot = xcd_chunk(blockIdx.x, gridDim.x);  // a filter's pages share an XCD
  const uint32_t f = pg_filter[slot];
  const FilterPlan& P = plans[f];
  const uint32_t p = slot - P.page_base;
  if (outs[f].error || p >= outs[f].num_pages) return;
  // a filter whose lines K6 never cuts: its pages go to k_plines_list
  if (!P.lines_asm && P.lg_line && threadIdx.x == 0) pg_noline[1 + atomicAdd(&pg_noline[0], 1u)] = slot;
  const uint32_t* pf = page_first + P.pf_base;
  const uint32_t b0 = pf[p], b1 = pf[p + 1], nb = b1 - b0;
  uint4* dst = reinterpret_cast<uint4*>(pages + (uint64_t)slot * page_size);
  if (nb > ASM_MAXB) {  // (never with lines_asm: the host bounds blocks per page for it)
    assemble_atomic(P, p, slot, b0, b1, idx_cnt, idx_start, sorted32, slots, pages, lis, page_size, s_pg);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < page_size / 16; i += ASM_NT) dst[i] = reinterpret_cast<const uint4*>(s_pg)[i];
    return;
  }
  const uint32_t IS = 1u << lis, rvs = P.rvs;
  // probe lines cut from this page (phase E): line groups of G buckets, L per block; a page
  // whose group table would not fit s_gs has its lines cut by k_plines_list
  const uint32_t lgG = P.lines_asm ? P.lg_line - 1 : 0u, G = 1u << lgG, L = IS >> lgG;
  const bool cut = P.lines_asm && !(P.lines_flag && nb * (L + 1) > ASM_GT);
  // (A) metadata + entry offsets (2 blocks per thread)
  uint32_t cj[2], oj[2], sj[2], sum = 0;
  uint64_t sl[2];
  // both blocks' metadata loads first (clamped index, no branch around a load: each branch
  // waited for its own loads)
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t g = P.idx_base + b0 + min(threadIdx.x * 2 + q, nb - 1);
    cj[q] = idx_cnt[g];
    sl[q] = slots[g];
    sj[q] = idx_start[g];
  }
  for (uint32_t i = threadIdx.x; i < MAX_PAGE / 16; i += ASM_NT) s_wm[i] = 0;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t j = threadIdx.x * 2 + q;
    oj[q] = 0;
    if (j < nb) {
      oj[q] = (uint32_t)(sl[q] - (uint64_t)p * page_size);
      s_off[j] = oj[q];
      s_c[j] = cj[q];
      s_src[j] = sj[q];
    } else {
      cj[q] = 0;
    }
    sum += cj[q];
  }
  // runs of ASM_RUN entries start at each block's first entry (a block's last run may be
  // short), so no run spans two blocks. One scan gives both prefixes: entries in the low 20
  // bits (< 128 blocks * 4096), runs above them (exact whenever ne <= ASM_MAXE)
  uint32_t tot;
  uint32_t run = block_excl_scan<ASM_NT>(sum + (((cj[0] + ASM_RUN - 1) / ASM_RUN + (cj[1] + ASM_RUN - 1) / ASM_RUN) << 20),
                                         s_tmp, &tot);
  const uint32_t ne = tot & 0xfffffu, nruns = tot >> 20;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t j = threadIdx.x * 2 + q;
    if (j < nb) s_est[j] = run >> 20;  // block j's first run
    run += cj[q] + (((cj[q] + ASM_RUN - 1) / ASM_RUN) << 20);
  }
  if (threadIdx.x == 0) { s_est[nb] = nruns; s_off[nb] = page_size; }
  DBG_PHASE_K(3, 0);
  if (ne > ASM_MAXE) {  // uniform (scan total)
    __syncthreads();
    assemble_atomic(P, p, slot, b0, b1, idx_cnt, idx_start, sorted32, slots, pages, lis, page_size, s_pg);
  } else {
  __syncthreads();
  // run table: block of each run; word marks of the block starts
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t j = threadIdx.x * 2 + q;
    if (j < nb) {
      for (uint32_t r = s_est[j]; r < s_est[j + 1]; r++) s_rblk[r] = (uint8_t)j;
    }
    if (j < nb && j > 0) reinterpret_cast<uint8_t*>(s_wm)[(oj[q] + 3) / 4] = 1;  // blocks >= 9 B apart
  }
  __syncthreads();
  // block of word w (the block holding byte 4w) = block starts in words <= w: thread t
  // owns the QPT 16-byte quads t*QPT.. (words 4 * quad ..), so one exclusive scan of the
  // per-thread mark counts
  const uint32_t nwp = page_size / 4;
  constexpr uint32_t QPT = (MAX_PAGE / 16 + ASM_NT - 1) / ASM_NT;
  uint32_t mwq[QPT], msum = 0;
#pragma unroll
  for (uint32_t q = 0; q < QPT; q++) {
    const uint32_t qd = threadIdx.x * QPT + q;
    mwq[q] = 4 * qd < nwp ? s_wm[qd] : 0u;
    msum += (mwq[q] & 0xffu) + ((mwq[q] >> 8) & 0xffu) + ((mwq[q] >> 16) & 0xffu) + (mwq[q] >> 24);
  }
  uint32_t mtot;
  const uint32_t jw0 = block_excl_scan<ASM_NT>(msum, s_tmp, &mtot);
  const uint32_t* base = sorted32 + P.e_first;
  // run r: block j, its entries [k0, k0 + len) of the block; independent loads, all in flight
  // together (a full run: four 16-byte loads -- gfx950 accepts unaligned global addresses; a
  // short one: clamped dword loads)
  // (pv: the block's entry before the run, or 0)
  auto load_run = [&](uint32_t r, uint32_t (&ev)[ASM_RUN], uint32_t& pv) {
    const uint32_t j = s_rblk[r], k0 = (r - s_est[j]) * ASM_RUN, c = s_c[j];
    const uint32_t* src = base + s_src[j] + k0;
    pv = k0 ? src[-1] : 0u;
    if (k0 + ASM_RUN <= c) {
      static_assert(ASM_RUN % 4 == 0, "runs of whole 16-byte loads");
#pragma unroll
      for (uint32_t i = 0; i < ASM_RUN; i += 4) {
        v4u x;
        __builtin_memcpy(&x, src + i, 16);
        ev[i] = x.x; ev[i + 1] = x.y; ev[i + 2] = x.z; ev[i + 3] = x.w;
      }
    } else {
      const uint32_t last = c - k0 - 1;
#pragma unroll
      for (uint32_t i = 0; i < ASM_RUN; i++) ev[i] = src[min(i, last)];
    }
  };
  // the first run's loads are issued before the fill, so they land while it runs
  uint32_t ev0[ASM_RUN], pv0 = 0;
  if (threadIdx.x < nruns) load_run(threadIdx.x, ev0, pv0);
  // (B) fill: thread t builds its quads' words (16 bytes each) and stores each quad at once
  uint32_t jw = jw0;
#pragma unroll
  for (uint32_t q = 0; q < QPT; q++) {
  const uint32_t qd = threadIdx.x * QPT + q;
  const uint32_t mw = mwq[q];
  if (4 * qd < nwp) {
    // blocks are >= 9 bytes: the quad's 16 bytes lie in blocks ja, ja + 1 and ja + 2, whose
    // metadata is read once (independent LDS reads) instead of per byte
    const uint32_t ja = jw + (mw & 0xffu);  // the block holding the quad's first byte
    jw += (mw & 0xffu) + ((mw >> 8) & 0xffu) + ((mw >> 16) & 0xffu) + (mw >> 24);
    const uint32_t jb = min(ja + 1, nb - 1), jc = min(ja + 2, nb - 1);
    const uint32_t o0 = s_off[ja], c0 = s_c[ja];
    const uint32_t o1 = ja + 1 < nb ? s_off[jb] : 0xffffffffu, c1 = s_c[jb];
    const uint32_t o2 = ja + 2 < nb ? s_off[jc] : 0xffffffffu, c2 = s_c[jc];
    const uint32_t n0 = o0 + 2 + (c0 + IS - 1) / 8 + 4;  // end of block ja's encoding bytes
    const uint32_t n1 = o1 + 2 + (c1 + IS - 1) / 8 + 4;
    const uint32_t n2 = o2 + 2 + (c2 + IS - 1) / 8 + 4;
    uint32_t x4[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t B = 16 * qd + 4 * k + i;
        const bool s2 = B >= o2, s1 = B >= o1;
        const uint32_t o = s2 ? o2 : (s1 ? o1 : o0), c = s2 ? c2 : (s1 ? c1 : c0);
        const uint32_t en = s2 ? n2 : (s1 ? n1 : n0);
        const uint32_t rel = B - o;
        const uint32_t byte = rel < 2 ? ((c >> (8 * rel)) & 0xffu) : (B < en ? 0xffu : 0u);
        x |= byte << (8 * i);
      }
      x4[k] = x;
    }
    reinterpret_cast<v4u*>(s_pg)[qd] = v4u{x4[0], x4[1], x4[2], x4[3]};
  }
  }
  if (threadIdx.x < 4) s_pg[page_size / 4 + threadIdx.x] = 0;
  __syncthreads();  // (also: s_wm read, s_gs free)
  DBG_PHASE_K(3, 1);
  // (C) entry runs, unrolled: entry k of block j clears encoding bit (j's encoding start) + k
  // + its bucket offset, and ORs its rvs remainder|value bits at (j's remainder start) + k rvs.
  // Encoding bits go into a 64-bit mask over two words (flushed, with two atomics, when an
  // entry lands past it); remainder bits stream through a 64-bit accumulator that emits a word
  // each time 32 bits have filled (an OR: a run's first and last words may be shared with its
  // neighbours). Entries past a short run's end contribute nothing.
  // Probe-line group boundaries come from the same entries (phase E's table s_gs): bucket
  // b's terminator is encoding bit b + (entries in buckets <= b), so the bit after group g's
  // last terminator (bucket gG - 1) is gG + (entries in groups < g). The run holding a block's
  // first entry of group >= g writes it (its predecessor, pv, tells whether the group starts
  // here); the run holding the block's last entry writes the groups past it.
  const uint32_t rmask = rvs >= 32 ? 0xffffffffu : ((1u << rvs) - 1);
  const uint32_t bsh = rvs >= 32 ? 0u : rvs, bmask = rvs >= 32 ? 0u : IS - 1;  // bucket offset
  for (uint32_t r = threadIdx.x; r < nruns; r += ASM_NT) {
    const uint32_t j = s_rblk[r], k0 = (r - s_est[j]) * ASM_RUN, c = s_c[j];
    const uint32_t len = min((uint32_t)ASM_RUN, c - k0);
    uint32_t (&ev)[ASM_RUN] = ev0;  // one register buffer: the first run's entries were loaded before the fill
    uint32_t& pv = pv0;
    if (r != threadIdx.x) load_run(r, ev, pv);
    if (cut) {
      const uint32_t gb = j * (L + 1);
      const uint32_t gp = k0 ? ((pv >> bsh) & bmask) >> lgG : 0u;  // group of the entry before the run
      uint32_t last = ev[0];
#pragma unroll
      for (uint32_t i = 1; i < ASM_RUN; i++) last = i < len ? ev[i] : last;
      const uint32_t gl = ((last >> bsh) & bmask) >> lgG;  // group of the run's last entry
      // groups (gp, gl] start in this run (usually none or one), at the entry after those of
      // smaller groups: entries below hi | (gG << bsh), hi = the index bits all entries share
      const uint32_t hi = bsh + lis >= 32 ? 0u : ev[0] & ~((IS << bsh) - 1u);
#pragma unroll 1
      for (uint32_t g = gp + 1; g <= gl; g++) {
        const uint32_t lim = hi | ((g * G) << bsh);
        uint32_t before = 0;
#pragma unroll
        for (uint32_t i = 0; i < ASM_RUN; i++) before += (i < len && ev[i] < lim) ? 1u : 0u;
        s_gs[gb + g] = (uint16_t)(g * G + k0 + before);
      }
      if (k0 + len == c)
#pragma unroll 1
        for (uint32_t g = gl + 1; g < L; g++) s_gs[gb + g] = (uint16_t)(g * G + c);
    }
    const uint32_t eb0 = (s_off[j] + 2) * 8 + k0;  // encoding bit of entry k0 at bucket offset 0
    const uint32_t rb0 = (s_off[j] + 2 + (c + IS - 1) / 8 + 4) * 8 + k0 * rvs;
    uint32_t wb = (eb0 + ((ev[0] >> bsh) & bmask)) & ~31u;
    uint64_t m = 0;
#pragma unroll
    for (uint32_t i = 0; i < ASM_RUN; i++) {
      const uint32_t hb = eb0 + i + ((ev[i] >> bsh) & bmask);
      const bool live = i < len;
      if (live && hb - wb >= 64) {
        if ((uint32_t)m) atomicAnd(&s_pg[wb >> 5], ~(uint32_t)m);
        if ((uint32_t)(m >> 32)) atomicAnd(&s_pg[(wb >> 5) + 1], ~(uint32_t)(m >> 32));
        m = 0;
        wb = hb & ~31u;
      }
      m |= (uint64_t)(live ? 1u : 0u) << ((hb - wb) & 63);
    }
    if ((uint32_t)m) atomicAnd(&s_pg[wb >> 5], ~(uint32_t)m);
    if ((uint32_t)(m >> 32)) atomicAnd(&s_pg[(wb >> 5) + 1], ~(uint32_t)(m >> 32));
    if (rvs >= 32) {  // (32-bit entries: rvs == 32) one whole word per entry, at a bit offset
#pragma unroll
      for (uint32_t i = 0; i < ASM_RUN; i++)
        if (i < len) lds_or_bits(s_pg, rb0 + i * rvs, ev[i], rvs);
    } else if (rvs) {
      // a word can only have filled after every 32 / rvs entries (uniform check points: the
      // accumulator then holds < 64 bits)
      const uint32_t per = 32u / rvs;
      uint32_t w = rb0 >> 5, nbit = rb0 & 31, since = 0;
      uint64_t acc = 0;
#pragma unroll
      for (uint32_t i = 0; i < ASM_RUN; i++) {
        const bool live = i < len;
        acc |= (uint64_t)(live ? ev[i] & rmask : 0u) << nbit;
        nbit += live ? rvs : 0u;
        if (++since == per) {
          since = 0;
          if (nbit >= 32) {
            atomicOr(&s_pg[w], (uint32_t)acc);
            acc >>= 32;
            nbit -= 32;
            w++;
          }
        }
      }
      if (nbit >= 32) {
        atomicOr(&s_pg[w], (uint32_t)acc);
        acc >>= 32;
        nbit -= 32;
        w++;
      }
      if (nbit) atomicOr(&s_pg[w], (uint32_t)acc);
    }
  }
  }  // word-parallel path
  __syncthreads();
  DBG_PHASE_K(3, 2);
  // (D) store
  const uint4* srcp = reinterpret_cast<const uint4*>(s_pg);
  for (uint32_t i = threadIdx.x; i < page_size / 16; i += ASM_NT) dst[i] = srcp[i];
  DBG_PHASE_K(3, 3);
  if (!P.lines_asm) return;
  // (E) probe lines of the page's blocks, cut from the LDS image (format: "probe lines").
  if (!cut) {  // this page's group table does not fit s_gs: k_plines cuts its lines
    if (threadIdx.x == 0) pg_noline[1 + atomicAdd(&pg_noline[0], 1u)] = slot;  // k_plines_list
    return;
  }
  if (ne <= ASM_MAXE) {
    // the entry runs wrote every group boundary of blocks with entries; the first and end
    // entries of each block and the boundaries of empty blocks here
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint32_t j = threadIdx.x * 2 + q;
      if (j < nb) {
        const uint32_t c = s_c[j];
        s_gs[j * (L + 1)] = 0;
        s_gs[j * (L + 1) + L] = (uint16_t)(c + IS);
        if (c == 0)
          for (uint32_t g = 1; g < L; g++) s_gs[j * (L + 1) + g] = (uint16_t)(g * G);
      }
    }
    __syncthreads();
  } else {
  // E1 (pages assembled by atomics): popcount scan over the blocks' encoding words -> group
  // boundaries in s_gs.
  uint32_t wc[2], wsum = 0;  // encoding words per block (2 blocks per thread)
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t j = threadIdx.x * 2 + q;
    wc[q] = j < nb ? (s_c[j] + IS + 63) / 64 : 0u;
    wsum += wc[q];
  }
  uint32_t nw;
  uint32_t wrun = block_excl_scan<ASM_NT>(wsum, s_tmp, &nw);
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t j = threadIdx.x * 2 + q;
    if (j < nb) {
      s_est[j] = wrun;  // reused: first encoding word item of block j
      s_gs[j * (L + 1)] = 0;
      s_gs[j * (L + 1) + L] = (uint16_t)(s_c[j] + IS);
    }
    wrun += wc[q];
  }
  if (threadIdx.x == 0) s_est[nb] = nw;
  __syncthreads();
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nw; base += ASM_NT) {
    const uint32_t it = base + threadIdx.x;
    uint32_t j = 0, w = 0, ones = 0;
    uint64_t x = 0;
    if (it < nw) {
      uint32_t lo = 0, hi = nb;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_est[mid] <= it) lo = mid; else hi = mid;
      }
      j = lo;
      w = it - s_est[j];
      const uint32_t nbits = s_c[j] + IS, b = w * 64;
      x = lds_bits64(s_pg, (s_off[j] + 2) * 8 + b);
      if (nbits - b < 64) x &= (1ull << (nbits - b)) - 1;
      ones = __popcll(x);
    }
    uint32_t tot;
    const uint32_t ex_all = block_excl_scan<ASM_NT>(ones, s_tmp, &tot) + carry;
    carry += tot;
    // prefix inside block j = ex_all - ex_all of the block's first word (this pass or earlier)
    if (it < nw && w == 0) s_wpre[j] = ex_all;
    __syncthreads();
    if (it < nw) {
      const uint32_t ex = ex_all - s_wpre[j];
      for (uint32_t k = (ex + G) >> lgG; k < L && k * G - 1 < ex + ones; k++)
        s_gs[j * (L + 1) + k] = (uint16_t)(w * 64 + select64_fast(x, k * G - 1 - ex) + 1);
    }
    __syncthreads();
  }
  }  // E1
  DBG_PHASE_K(3, 4);
  // E2: 4 lanes per line, 16 bytes each
  const uint32_t nt = nb * L * 4;
  for (uint32_t u = threadIdx.x; u < nt; u += ASM_NT) {
    const uint32_t j = u >> (lis - lgG + 2), rest = u & (4 * L - 1), gl = rest >> 2, qq = rest & 3;  // L = 2^(lis - lgG)
    const uint32_t c = s_c[j];
    const uint32_t ebit = (s_off[j] + 2) * 8, rbit = (s_off[j] + 2 + (c + IS - 1) / 8 + 4) * 8;
    const uint32_t a = s_gs[j * (L + 1) + gl], ne2 = s_gs[j * (L + 1) + gl + 1] - a;
    const uint32_t n = ne2 - G, E = a - gl * G;
    const bool ovf = ne2 > 128 || n * rvs > 384;
    uint64_t wv[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t o = qq * 128 + h * 64;
      uint64_t x = 0;
      if (ovf) {
        x = o < 128 ? ~0ull : 0ull;
      } else if (o < 128) {
        const uint32_t hi = min(o + 64, ne2);
        if (o < hi) x = lds_bits64(s_pg, ebit + a + o) & lowmask64(hi - o);
      } else {
        const uint32_t ro = o - 128, hi = min(ro + 64, n * rvs);
        if (ro < hi) x = lds_bits64(s_pg, rbit + E * rvs + ro) & lowmask64(hi - ro);
      }
      wv[h] = x;
    }
    const uint64_t line = (uint64_t)P.line_base + (uint64_t)(b0 + j) * L + gl;
    lines[line * 4 + qq] = make_uint4((uint32_t)wv[0], (uint32_t)(wv[0] >> 32), (uint32_t)wv[1], (uint32_t)(wv[1] >> 32));
  }
  DBG_PHASE_K(3, 8);
}

// ======================================================================================
// K0: incremental add -- decode an old filter into entries (src/routing_filter.c:496-544)
// ======================================================================================
// Every old index of the batch in one list (filter f's at P.old_idx_base ..): the decode of
// all old filters is three launches, whatever the number of filters.
// k_old_counts: per old index, num_remainders from its header -> cnt
__global__ void k_old_counts(const FilterPlan* __restrict__ plans, const uint32_t* __restrict__ old_idx_filter,
                             uint32_t num_old_idx, uint32_t* __restrict__ cnt) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= num_old_idx) return;
  const FilterPlan& P = plans[old_idx_filter[g]];
  const uint64_t s = P.old_slots[g - P.old_idx_base];
  cnt[g] = (uint32_t)P.old_pages[s] | ((uint32_t)P.old_pages[s + 1] << 8);
}

// one workgroup per filter: exclusive scan of its old indices' counts -> pos (filter-relative),
// and the sentinel (~0) on the entry slots past the decoded entries (old_region counts the old
// filter's num_fingerprints, duplicates included; k_old_count / k_scatter skip sentinels)
// (32-bit incremental builds: ent is null -- no sentinels -- and old_tot[f] gets the total)
__global__ __launch_bounds__(LAYOUT_NT) void k_old_scan(const FilterPlan* __restrict__ plans,
                                                        const uint32_t* __restrict__ cnt,
                                                        uint32_t* __restrict__ pos, uint64_t* __restrict__ ent,
                                                        uint32_t* __restrict__ old_tot) {
  __shared__ uint32_t s_tmp[LAYOUT_NT / WAVE + 1];
  const FilterPlan& P = plans[blockIdx.x];
  const uint32_t n = P.old_direct ? 0u : P.old_num_indices;  // direct: read in place, no decode
  if (n == 0) return;
  constexpr int PER = MAX_INDICES / LAYOUT_NT;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t i = threadIdx.x * PER + k;
    v[k] = i < n ? cnt[P.old_idx_base + i] : 0u;
    sum += v[k];
  }
  uint32_t total;
  uint32_t run = block_excl_scan<LAYOUT_NT>(sum, s_tmp, &total);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t i = threadIdx.x * PER + k;
    if (i < n) pos[P.old_idx_base + i] = run;
    run += v[k];
  }
  if (old_tot && threadIdx.x == 0) old_tot[blockIdx.x] = total;
  if (!ent) return;
  uint64_t* tail = ent + P.e_first + P.num_new;
  for (uint32_t j = total + threadIdx.x; j < P.old_region; j += LAYOUT_NT) tail[j] = ~0ull;
}

// k_old_decode: one wave per old index. Entry k of the block: bucket offset = number of
// 1-bits before its 0-bit in the encoding (routing_get_bucket_counts, :281-306); value
// bits re-widened to the new value_size (:536-543). Written as (e << 1) | 0 (old flag) into
// the 64-bit entry array, or (32-bit incremental builds, old32 set) as e into the filter's
// run of old32 -- in order, since the old image holds its entries sorted.
__global__ __launch_bounds__(256) void k_old_decode(const FilterPlan* __restrict__ plans,
                                                    const uint32_t* __restrict__ old_idx_filter,
                                                    uint32_t num_old_idx, const uint32_t* __restrict__ pos,
                                                    uint64_t* __restrict__ ent, uint32_t* __restrict__ old32,
                                                    uint32_t lis, uint32_t fp_size) {
  // Entry k sits at the k-th zero bit of the encoding; its bucket offset = 1-bits before it
  // = position - k (routing_get_bucket_counts, :281-306). One lane per encoding byte lists
  // its zero positions (at most 8) at the byte's zero prefix in a small LDS list, then one
  // lane per entry reads its position and its remainder. Consecutive lanes read consecutive
  // bytes and bit ranges (coalesced), and no lane walks a chain of entries. An index with
  // more entries than the list holds is decoded in CAP-entry chunks.
  constexpr uint32_t CAP = 1024;
  __shared__ uint16_t s_pos[256 / WAVE][CAP];
  const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  if (g >= num_old_idx) return;  // uniform per wave
  const FilterPlan& P = plans[old_idx_filter[g]];
  const uint32_t wid = g - P.old_idx_base;  // old index within its filter
  const uint32_t index_size = 1u << lis;
  const uint64_t hdr = P.old_slots[wid];
  const uint8_t* pg = P.old_pages;
  const uint32_t c = (uint32_t)pg[hdr] | ((uint32_t)pg[hdr + 1] << 8);
  const uint32_t enc = (c + index_size - 1) / 8 + 4;
  const uint64_t rbit = (hdr + 2 + enc) * 8;
  const uint32_t total_bits = c + index_size;
  uint64_t* out = old32 ? nullptr : ent + P.e_first + P.num_new + pos[g];
  uint32_t* out32 = old32 ? old32 + P.old_first + pos[g] : nullptr;
  const uint32_t old_vmask = (uint32_t)((1ull << P.old_vs) - 1);
  uint16_t* zpos = s_pos[threadIdx.x / WAVE];
  const uint32_t nbytes = (total_bits + 7) / 8;
  const uint8_t* encb = pg + hdr + 2;  // the encoding is byte aligned
  for (uint32_t k0 = 0; k0 < c; k0 += CAP) {
    uint32_t zeros_before = 0;
    for (uint32_t b0 = 0; b0 < nbytes && zeros_before < k0 + CAP; b0 += WAVE) {
      const uint32_t bb = b0 + lane;
      uint32_t z = 0;
      if (bb < nbytes) {
        const uint32_t nb = min(8u, total_bits - 8 * bb);
        z = ~(uint32_t)encb[bb] & ((1u << nb) - 1);  // bits past the end are not entries
      }
      const uint32_t cnt = __popc(z);
      const uint32_t inc = wave_incl_scan(cnt);
      uint32_t at = zeros_before + inc - cnt;
      while (z) {
        if (at >= k0 && at < k0 + CAP) zpos[at - k0] = (uint16_t)(8 * bb + __builtin_ctz(z));
        at++;
        z &= z - 1;
      }
      zeros_before += __shfl(inc, WAVE - 1, WAVE);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t k1 = min(c, k0 + CAP);
    for (uint32_t k = k0 + lane; k < k1; k += WAVE) {
      const uint32_t bo = (uint32_t)zpos[k - k0] - k;
      const uint32_t rv = ld_bits(pg, rbit + (uint64_t)k * P.old_rvs, P.old_rvs);
      const uint32_t bucket = wid * index_size + bo;
      const uint32_t e_old = (P.old_rvs >= 32 ? 0u : (bucket << P.old_rvs)) | rv;
      const uint32_t old_value = e_old & old_vmask;
      const uint32_t fpv = e_old >> P.old_vs;
      const uint32_t e = (fpv << P.vs) | old_value;
      if (out32) out32[k] = e;
      else out[k] = (uint64_t)e << 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the list is rewritten next chunk
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// 32-bit incremental builds: each coarse bucket's run of the filter's old entries. The old
// entries are sorted, so the run of coarse bucket c starts at the first entry >= c << esh;
// one thread per coarse bucket, then cb_count (the new entries' histogram) += run length.
__global__ __launch_bounds__(256) void k_old_cb_bounds(const FilterPlan* __restrict__ plans,
                                                       const uint32_t* __restrict__ cb_filter, uint32_t num_cb,
                                                       const uint32_t* __restrict__ old32,
                                                       const uint32_t* __restrict__ old_tot, uint32_t fp_size,
                                                       uint32_t lis, uint32_t* __restrict__ ob_lo,
                                                       uint32_t* __restrict__ ob_n, uint32_t* __restrict__ cb_count) {
  const uint32_t cb = blockIdx.x * blockDim.x + threadIdx.x;
  if (cb >= num_cb) return;
  const uint32_t f = cb_filter[cb];
  const FilterPlan& P = plans[f];
  const uint32_t cl = cb - P.cb_base, ncb = 1u << P.cbits;
  if (P.old_direct) {
    // new coarse bucket cl lies in the old filter's coarse bucket cl >> (cbits - old_cbits), whose
    // entries are those of its indices [c_old * ipc, (c_old + 1) * ipc), consecutive in its entry
    // array (K4 compacts a coarse bucket's indices in order); with the same geometry that is the
    // run, else the run is the sub-range of entries in cl (binary searches: the entries are sorted
    // by fingerprint, and re-widening the value bits keeps their order)
    const uint32_t c_old = cl >> (P.cbits - P.old_cbits);
    const uint32_t ipc = 1u << (P.old_bbits - lis), i0 = c_old * ipc, i1 = i0 + ipc - 1;
    uint32_t lo = P.old_idx_start[i0], hi = P.old_idx_start[i1] + P.old_idx_cnt[i1];
    if (P.cbits != P.old_cbits) {
      const uint32_t* o = P.old_entries;
      const uint32_t ovs = P.old_vs, vs = P.vs, esh = fp_size + vs - P.cbits;
      auto key = [&](uint32_t raw) -> uint32_t { return (((raw >> ovs) << vs) | (raw & ((1u << ovs) - 1u))) >> esh; };
      auto lb = [&](uint32_t c, uint32_t a, uint32_t b) -> uint32_t {  // first entry in [a, b) of coarse bucket >= c
        while (a < b) {
          const uint32_t mid = (a + b) >> 1;
          if (key(o[mid]) < c) a = mid + 1; else b = mid;
        }
        return a;
      };
      const uint32_t nlo = lb(cl, lo, hi);
      hi = lb(cl + 1, nlo, hi);
      lo = nlo;
    }
    ob_lo[cb] = lo;
    ob_n[cb] = hi - lo;
    cb_count[cb] += hi - lo;
    return;
  }
  const uint32_t tot = P.old_num_indices ? old_tot[f] : 0u;
  const uint32_t* o = old32 + P.old_first;
  const uint32_t esh = fp_size + P.vs - P.cbits;
  auto lb = [&](uint32_t c) -> uint32_t {  // first entry whose coarse bucket >= c
    uint32_t lo = 0, hi = tot;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((o[mid] >> esh) < c) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  const uint32_t lo = (P.cbits == 0 || cl == 0) ? 0u : lb(cl);
  const uint32_t hi = cl + 1 == ncb ? tot : lb(cl + 1);
  ob_lo[cb] = lo;
  ob_n[cb] = hi - lo;
  cb_count[cb] += hi - lo;
}

// ======================================================================================
// routing_filter_estimate_unique_fp (src/routing_filter.c:702-848)
//
// The reference decodes the first num_indices/16 indices of up to 32 filters (each list
// sorted, duplicates dropped) and k-way merges them, counting distinct fingerprints; the
// result is that count * 16. Those indices hold exactly the fingerprints below
// 2^(fp_size-4), so the distinct count of the union is the population of a bitmap over
// that range: one wave per decoded index sets its fingerprints' bits (bit-exact with the
// merge count; no sort, no k-way merge), one pass counts them.
// ======================================================================================
__global__ __launch_bounds__(256) void k_est_decode(const EstFilter* __restrict__ fl, uint32_t num_filters,
                                                    uint32_t total_idx, uint32_t lis,
                                                    uint32_t* __restrict__ bitmap,
                                                    uint32_t* __restrict__ num_entries) {
  const uint32_t wid = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  if (wid >= total_idx) return;
  uint32_t f = 0;
  while (f + 1 < num_filters && fl[f + 1].idx_first <= wid) f++;
  const EstFilter& F = fl[f];
  const uint32_t index_no = wid - F.idx_first;
  const uint32_t index_size = 1u << lis;
  const uint64_t hdr = F.slots[index_no];
  const uint8_t* pg = F.pages;
  const uint32_t c = (uint32_t)pg[hdr] | ((uint32_t)pg[hdr + 1] << 8);
  if (lane == 0 && c) atomicAdd(num_entries, c);
  const uint32_t enc = (c + index_size - 1) / 8 + 4;
  const uint64_t ebit = (hdr + 2) * 8;
  const uint64_t rbit = (hdr + 2 + enc) * 8;
  const uint32_t total_bits = c + index_size;
  uint32_t zeros_before = 0, ones_before = 0;
  for (uint32_t base = 0; base < total_bits; base += 64 * WAVE) {
    const uint32_t bit0 = base + lane * 64;
    uint64_t x = 0;
    uint32_t nb = 0;
    if (bit0 < total_bits) {
      nb = min(64u, total_bits - bit0);
      const uint64_t bp = ebit + bit0;
      const uint32_t sh = (uint32_t)(bp & 7);
      x = ld_u64_unaligned(pg, bp >> 3) >> sh;
      if (sh) x |= (uint64_t)pg[(bp >> 3) + 8] << (64 - sh);
      if (nb < 64) x &= (1ull << nb) - 1;
    }
    const uint32_t ones = __popcll(x);
    const uint32_t zer = nb - ones;
    const uint32_t ones_ex = wave_incl_scan(ones) - ones + ones_before;
    const uint32_t zer_ex = wave_incl_scan(zer) - zer + zeros_before;
    uint64_t z = ~x & (nb == 64 ? ~0ull : ((1ull << nb) - 1));
    uint32_t k = zer_ex;
    while (z) {  // every 0-bit is an entry; its bucket offset = 1-bits before it
      const uint32_t b = __builtin_ctzll(z);
      z &= z - 1;
      const uint32_t bo = ones_ex + (b - (k - zer_ex));
      const uint32_t rv = ld_bits(pg, rbit + (uint64_t)k * F.rvs, F.rvs);
      const uint32_t bucket = index_no * index_size + bo;
      const uint32_t fp = (((F.rvs >= 32 ? 0u : (bucket << F.rvs)) | rv) >> F.vs);  // :786-787
      atomicOr(&bitmap[fp >> 5], 1u << (fp & 31));
      k++;
    }
    ones_before = __shfl(ones_ex + ones, WAVE - 1, WAVE);
    zeros_before = __shfl(zer_ex + zer, WAVE - 1, WAVE);
  }
}

__global__ __launch_bounds__(256) void k_popcount(const uint4* __restrict__ words, uint64_t n4,
                                                  uint32_t* __restrict__ total) {
  __shared__ uint32_t s_tmp[256 / WAVE + 1];
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
    const uint4 w = words[i];
    c += __popc(w.x) + __popc(w.y) + __popc(w.z) + __popc(w.w);
  }
  uint32_t tot;
  block_excl_scan<256>(c, s_tmp, &tot);
  if (threadIdx.x == 0 && tot) atomicAdd(total, tot);
}

// bitmap (zeroed by the caller, bitmap_words a multiple of 4) -> counters[0] = entries
// decoded, counters[1] = distinct fingerprints
extern "C" int rf_launch_estimate(void* stream, const EstFilter* fl, uint32_t num_filters, uint32_t total_idx,
                                  uint32_t lis, uint32_t* bitmap, uint64_t bitmap_words, uint32_t* counters) {
  if (total_idx) {
    hipLaunchKernelGGL(k_est_decode, dim3((total_idx + 3) / 4), dim3(256), 0, (hipStream_t)stream, fl, num_filters,
                       total_idx, lis, bitmap, counters);
    if (hipGetLastError() != hipSuccess) return 1;
  }
  const uint64_t n4 = bitmap_words / 4;
  const uint64_t want = (n4 + 255) / 256 + 1;
  const uint32_t grid = (uint32_t)(want < 2048 ? want : 2048);
  hipLaunchKernelGGL(k_popcount, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)bitmap, n4,
                     counters + 1);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// per-build counters zeroed in one launch (instead of one memset each)
__global__ __launch_bounds__(256) void k_build_init(uint32_t* __restrict__ cb_count, uint32_t* __restrict__ cb_cursor,
                                                    uint32_t num_cb, uint32_t* __restrict__ outs_words,
                                                    uint32_t num_out_words, uint32_t* __restrict__ overflow,
                                                    uint32_t* __restrict__ spill, uint32_t* __restrict__ plist) {
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < num_cb; i += stride) {
    cb_count[i] = 0;
    if (cb_cursor) cb_cursor[i] = 0;
  }
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < num_out_words; i += stride) outs_words[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    overflow[0] = 0;
    if (spill) spill[0] = 0;
    if (plist) plist[0] = 0;  // k_plines_list's page count
  }
}

extern "C" int rf_launch_build_init(void* stream, uint32_t* cb_count, uint32_t* cb_cursor, uint32_t num_cb,
                                    uint32_t* outs_words, uint32_t num_out_words, uint32_t* overflow,
                                    uint32_t* spill, uint32_t* plist) {
  const uint32_t want = (num_cb > num_out_words ? num_cb : num_out_words) / 256 + 1;
  hipLaunchKernelGGL(k_build_init, dim3(want < 1024 ? want : 1024), dim3(256), 0, (hipStream_t)stream, cb_count,
                     cb_cursor, num_cb, outs_words, num_out_words, overflow, spill, plist);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// data_key_hash over a batch (btree_pack's fingerprint loop, src/btree.c:4020-4024)
template <int KIND>
__global__ __launch_bounds__(256) void k_hash(const void* __restrict__ in0, const uint64_t* __restrict__ offs,
                                              uint32_t key_len, uint32_t seed, uint64_t n,
                                              uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if constexpr (KIND == IN_VAR) {  // the wave's keys through a 4 KiB LDS window (wave_hash_var)
    constexpr uint32_t VCAP = 4096;
    __shared__ __attribute__((aligned(16))) uint32_t s_vk[256 / WAVE][VCAP / 4 + 4];
    uint64_t o0 = 0, o1 = 0, w0 = 0, w1 = 0;
    if (i < n) {
      o0 = offs[i];
      o1 = offs[i + 1];
    }
    const uint32_t h = wave_hash_var<VCAP, true>(static_cast<const uint8_t*>(in0), o0, o1, i < n,
                                                 s_vk[threadIdx.x / WAVE], seed, &w0, &w1);
    if (i < n) out[i] = h;
  } else {
    if (i < n) out[i] = hash_key<KIND, true>(in0, offs, key_len, seed, i);
  }
}

extern "C" int rf_launch_hash(void* stream, int kind, const void* in0, const uint64_t* offs, uint32_t key_len,
                              uint32_t seed, uint64_t n, uint32_t* out) {
  if (n == 0) return 0;
  const dim3 g((uint32_t)((n + 255) / 256)), b(256);
#define L(K) hipLaunchKernelGGL((k_hash<K>), g, b, 0, (hipStream_t)stream, in0, offs, key_len, seed, n, out)
  switch (kind) {
    case IN_KEYS24: L(IN_KEYS24); break;
    case IN_KEYS_W: L(IN_KEYS_W); break;
    case IN_KEYS_B: L(IN_KEYS_B); break;
    default: L(IN_VAR); break;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ======================================================================================
// Routed probes across ranks: probes arrive on any rank with a global
// filter id; each is sent to the rank that owns the filter's key range. k_route_count /
// k_route_scan / k_route_scatter form a stable partition of the probes by destination
// rank, packed as (local filter id << 32 | hash) pairs for one all-to-all; k_unroute puts
// the returned found_values back in the caller's order. route[g] = local_id << 8 | rank.
// ======================================================================================
constexpr uint32_t ROUTE_NT = 256;
constexpr uint32_t ROUTE_TILE = 16384;  // probes per workgroup
constexpr uint32_t ROUTE_MAX_WORLD = 16;

__device__ __forceinline__ uint32_t route_dest(const uint32_t* __restrict__ gfid, const uint32_t* __restrict__ route,
                                               uint32_t num_g, uint32_t world, uint64_t i, uint32_t* err) {
  const uint32_t g = gfid[i];
  if (g >= num_g) { atomicOr(err, 1u); return 0; }
  const uint32_t d = route[g] & 0xffu;
  if (d >= world) { atomicOr(err, 2u); return 0; }
  return d;
}

__global__ __launch_bounds__(ROUTE_NT) void k_route_count(const uint32_t* __restrict__ gfid, uint64_t n,
                                                          const uint32_t* __restrict__ route, uint32_t num_g,
                                                          uint32_t world, uint32_t* __restrict__ cnt,
                                                          uint32_t* __restrict__ err) {
  __shared__ uint32_t s_h[ROUTE_MAX_WORLD];
  if (threadIdx.x < ROUTE_MAX_WORLD) s_h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * ROUTE_TILE;
  const uint64_t b1 = min(b0 + ROUTE_TILE, n);
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += ROUTE_NT)
    atomicAdd(&s_h[route_dest(gfid, route, num_g, world, i, err)], 1u);
  __syncthreads();
  if (threadIdx.x < world) cnt[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = s_h[threadIdx.x];
}

// exclusive scan of cnt[world * nblk] (destination-major) into off; totals[d] = probes to d
__global__ __launch_bounds__(1024) void k_route_scan(const uint32_t* __restrict__ cnt, uint32_t m,
                                                     uint32_t nblk, uint32_t world, uint32_t* __restrict__ off,
                                                     uint64_t* __restrict__ totals) {
  __shared__ uint32_t s_tmp[1024 / WAVE + 1];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < m; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t x = i < m ? cnt[i] : 0u;
    uint32_t tot;
    const uint32_t r = block_excl_scan<1024>(x, s_tmp, &tot);
    if (i < m) off[i] = carry + r;
    carry += tot;
  }
  __syncthreads();
  if (threadIdx.x < world) {
    const uint32_t d = threadIdx.x;
    const uint32_t lo = off[d * nblk], hi = d + 1 < world ? off[(d + 1) * nblk] : carry;
    totals[d] = hi - lo;
  }
}

__global__ __launch_bounds__(ROUTE_NT) void k_route_scatter(const uint32_t* __restrict__ hashes,
                                                            const uint32_t* __restrict__ gfid, uint64_t n,
                                                            const uint32_t* __restrict__ route, uint32_t num_g,
                                                            uint32_t world, const uint32_t* __restrict__ off,
                                                            uint64_t* __restrict__ pairs,
                                                            uint32_t* __restrict__ perm, uint32_t* __restrict__ err) {
  constexpr uint32_t NW = ROUTE_NT / WAVE;
  __shared__ uint32_t s_base[ROUTE_MAX_WORLD];
  __shared__ uint32_t s_wc[NW][ROUTE_MAX_WORLD];
  if (threadIdx.x < world) s_base[threadIdx.x] = off[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x];
  const uint32_t w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const uint64_t lt = (1ull << lane) - 1;
  const uint64_t b0 = (uint64_t)blockIdx.x * ROUTE_TILE;
  const uint64_t b1 = min(b0 + ROUTE_TILE, n);
  __syncthreads();
  // chunks of ROUTE_NT consecutive probes: rank inside the chunk from per-destination
  // ballots, so the partition keeps the input order within each destination
  for (uint64_t c = b0; c < b1; c += ROUTE_NT) {
    const uint64_t i = c + threadIdx.x;
    const bool ok = i < b1;
    const uint32_t d = ok ? route_dest(gfid, route, num_g, world, i, err) : 0xffffffffu;
    uint32_t rank = 0;
    for (uint32_t q = 0; q < world; q++) {
      const uint64_t m = __ballot(d == q);
      if (d == q) rank = __popcll(m & lt);
      if (lane == 0) s_wc[w][q] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (ok) {
      uint32_t pos = s_base[d] + rank;
      for (uint32_t w2 = 0; w2 < w; w2++) pos += s_wc[w2][d];
      const uint32_t g = gfid[i];
      const uint32_t lid = g < num_g ? route[g] >> 8 : 0u;  // bad ids: reported through err
      pairs[pos] = ((uint64_t)lid << 32) | hashes[i];
      perm[pos] = (uint32_t)i;
    }
    __syncthreads();
    if (threadIdx.x < world) {
      uint32_t t = 0;
      for (uint32_t w2 = 0; w2 < NW; w2++) t += s_wc[w2][threadIdx.x];
      s_base[threadIdx.x] += t;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_unroute(const uint64_t* __restrict__ back, const uint32_t* __restrict__ perm,
                                                 uint64_t n, uint64_t* __restrict__ found) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < n) found[perm[j]] = back[j];
}

extern "C" uint64_t rf_route_scratch_words(uint64_t n, uint32_t world) {
  const uint64_t nblk = (n + ROUTE_TILE - 1) / ROUTE_TILE;
  return 2 * nblk * world + 4;  // cnt + off + err
}

// scratch: rf_route_scratch_words(n, world) u32 words; totals: world u64 (device)
extern "C" int rf_launch_route(void* stream, const uint32_t* hashes, const uint32_t* gfid, uint64_t n,
                               const uint32_t* route, uint32_t num_g, uint32_t world, uint64_t* pairs,
                               uint32_t* perm, uint32_t* scratch, uint64_t* totals) {
  if (world == 0 || world > ROUTE_MAX_WORLD) return 1;
  const uint64_t nblk64 = (n + ROUTE_TILE - 1) / ROUTE_TILE;
  if (nblk64 * world >= (1ull << 31) || n >= (1ull << 32)) return 1;
  const uint32_t nblk = (uint32_t)nblk64, m = nblk * world;
  uint32_t* cnt = scratch;
  uint32_t* off = scratch + m;
  uint32_t* err = scratch + 2 * (uint64_t)m;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(err, 0, 4, st) != hipSuccess) return 1;
  if (nblk) hipLaunchKernelGGL(k_route_count, dim3(nblk), dim3(ROUTE_NT), 0, st, gfid, n, route, num_g, world, cnt, err);
  hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, st, cnt, m, nblk, world, off, totals);
  if (nblk)
    hipLaunchKernelGGL(k_route_scatter, dim3(nblk), dim3(ROUTE_NT), 0, st, hashes, gfid, n, route, num_g, world, off,
                       pairs, perm, err);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int rf_launch_unroute(void* stream, const uint64_t* back, const uint32_t* perm, uint64_t n,
                                 uint64_t* found) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_unroute, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, back, perm, n,
                     found);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// routing_filter_verify (src/routing_filter.c:1163-1183): keys whose found_values lacks `value`
__global__ __launch_bounds__(256) void k_count_missing(const uint64_t* __restrict__ found, uint64_t n,
                                                       uint32_t value, unsigned long long* __restrict__ missing) {
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    c += ((found[i] >> value) & 1ull) ? 0u : 1u;
  c = wave_incl_scan(c);
  if ((threadIdx.x & (WAVE - 1)) == WAVE - 1 && c) atomicAdd(missing, (unsigned long long)c);
}

extern "C" int rf_launch_count_missing(void* stream, const uint64_t* found, uint64_t n, uint32_t value,
                                       unsigned long long* missing) {
  const uint64_t want = (n + 255) / 256;
  hipLaunchKernelGGL(k_count_missing, dim3((uint32_t)(want < 4096 ? (want ? want : 1) : 4096)), dim3(256), 0,
                     (hipStream_t)stream, found, n, value, missing);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ======================================================================================
// Probe: routing_filter_lookup (src/routing_filter.c:985-1073), one lane per probe
// ======================================================================================
// position of the r-th (0-based) set bit of the 128-bit value hi:lo
__device__ __forceinline__ uint32_t select128(uint64_t lo, uint64_t hi, uint32_t r) {
  const uint32_t c = __popcll(lo);
  return r < c ? select64_fast(lo, r) : 64 + select64_fast(hi, r - c);
}

// one 16-byte aligned window of the page bytes as two little-endian u64
__device__ __forceinline__ void ld_win(const uint8_t* pg, uint64_t a16, uint64_t& lo, uint64_t& hi) {
  const v4u v = *reinterpret_cast<const v4u*>(pg + a16);
  lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
}
__device__ __forceinline__ uint64_t pick4(uint32_t j, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  return j == 0 ? a : (j == 1 ? b : (j == 2 ? c : d));
}

// Probe = routing_filter_lookup (src/routing_filter.c:986-1073) on a built image, given
// the key's 32-bit hash. The common path reads one 64-byte probe line (below); the rare
// rest (overflowed lines, filters without lines) walks the image itself via the index slot.
// Full-scan fallback on the image (line overflowed, or the filter has no lines): 128-bit
// windows streamed from the index header, then per-entry bit reads.
// Kept lean (no large register arrays) so it does not cost the common path occupancy.
__device__ __forceinline__ uint64_t probe_stream(uint32_t bo, uint32_t remainder, uint32_t vs, uint32_t rvs,
                                                 const uint8_t* pg, uint64_t hdr, uint32_t lis) {
  const uint32_t index_size = 1u << lis;
  const uint32_t c = (uint32_t)pg[hdr] | ((uint32_t)pg[hdr + 1] << 8);
  const uint32_t enc = (c + index_size - 1) / 8 + 4;
  const uint64_t a0 = (hdr + 2) & ~15ull;
  const uint32_t e0 = (uint32_t)((hdr + 2 - a0) * 8);  // encoding bit 0 in window coordinates
  const uint32_t target_lo = bo ? bo - 1 : 0;
  uint32_t start = 0, end = 0, cum = 0;
  bool have_start = (bo == 0);
  const uint32_t nwin = (e0 + c + index_size + 127) / 128 + 1;
  for (uint32_t k = 0;; k++) {
    if (k > nwin) return 0;  // corrupt image: never hang
    uint64_t lo, hi;
    ld_win(pg, a0 + 16ull * k, lo, hi);
    if (k == 0 && e0) {
      if (e0 >= 64) { lo = 0; hi = (hi >> (e0 - 64)) << (e0 - 64); }
      else { lo = (lo >> e0) << e0; }
    }
    const uint32_t pc = __popcll(lo) + __popcll(hi);
    const uint32_t base = 128u * k - e0;
    if (!have_start && cum + pc > target_lo) {
      start = base + select128(lo, hi, target_lo - cum) + 1 - bo;
      have_start = true;
    }
    if (cum + pc > bo) {
      end = base + select128(lo, hi, bo - cum) - bo;
      break;
    }
    cum += pc;
  }
  if (start >= end) return 0;
  const uint64_t rbit0 = (hdr + 2 + enc) * 8;
  const uint32_t vmask = (uint32_t)((1ull << vs) - 1);
  uint64_t found = 0;
  for (uint32_t pos = start; pos < end; pos++) {
    const uint32_t rv = ld_bits(pg, rbit0 + (uint64_t)pos * rvs, rvs);
    if ((rv >> vs) == remainder) {
      const uint32_t v = rv & vmask;
      if (v < 64) found |= 1ull << v;
    }
  }
  return found;
}

// ---- probe lines ---------------------------------------------------------------------
// Device-only, not part of the on-disk image. An index's block is cut into groups of
// G = 2^(lg_line-1) consecutive buckets; group k of the filter (buckets [kG, kG+G)) gets a
// 64-byte line at line_base + k:
//   bits [0,128)    the group's slice of the unary encoding (0 = entry, 1 = bucket end),
//                   n + G bits, zero padded; all ones = overflow (probes use the image)
//   bits [128,512)  the group's n packed remainder|value entries, rvs bits each (LSB-first)
// Both slices are contiguous bit ranges of the reference block (layout written at
// src/routing_filter.c:622-633), so a probe touches ONE random 64-byte line instead of the
// index slot, header, encoding window and remainder run; and because the encoding and the
// remainders start at fixed offsets, decoding is one 128-bit select, one count of
// trailing zeros and one 96-bit window. G is chosen on the host so that n + G <= 128 and
// n * rvs <= 384 hold with margin for random fingerprints (engine: line_log_group).
__device__ __forceinline__ uint64_t bits64_at(const uint8_t* pg, uint64_t bitpos) {
  const uint64_t by = bitpos >> 3;
  const uint32_t sh = (uint32_t)(bitpos & 7);
  uint64_t x = ld_u64_unaligned(pg, by) >> sh;
  if (sh) x |= (uint64_t)pg[by + 8] << (64 - sh);
  return x;
}

// One wave per index (4 per workgroup). Phase 1: popcount-prefix over the encoding, the
// position after each group's last bucket terminator -> LDS. Phase 2: 4 lanes per line,
// 16 bytes each, bit-copied from the image.
// One index's probe lines, cut by one wave from its block in the image: the block (at most
// one page) is first copied into the wave's LDS slice `blk` with coalesced 16-byte loads;
// both phases then read their bits from LDS. s_a: the wave's group-start table (L + 1).
__device__ __forceinline__ void plines_index(const FilterPlan& P, uint32_t g, const uint64_t* __restrict__ slots,
                                             const uint8_t* __restrict__ pages, uint4* __restrict__ lines,
                                             uint8_t* blk, uint32_t* s_a, uint32_t lane, uint32_t lis,
                                             uint32_t page_size) {
  constexpr uint32_t SLICE = MAX_PAGE + 64;
  const uint32_t IS = 1u << lis;
  const uint32_t lgG = P.lg_line - 1, G = 1u << lgG, L = IS >> lgG;
  const uint8_t* pg = blk;
  const uint8_t* gp = pages + (uint64_t)P.page_base * page_size;
  const uint64_t rel_g = slots[g];
  const uint32_t c = (uint32_t)gp[rel_g] | ((uint32_t)gp[rel_g + 1] << 8);
  const uint64_t a0 = rel_g & ~15ull;
  const uint32_t used = (uint32_t)(rel_g - a0) + 2 + (c + IS - 1) / 8 + 4 +
                        (uint32_t)(((uint64_t)c * P.rvs + 7) / 8) + 12;
  const uint32_t nq = min((used + 15) / 16, SLICE / 16);
  for (uint32_t q = lane; q < nq; q += WAVE)
    reinterpret_cast<v4u*>(blk)[q] = *reinterpret_cast<const v4u*>(gp + a0 + 16ull * q);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint64_t rel = rel_g - a0;
  {
    const uint64_t ebit = (rel + 2) * 8;
    const uint32_t nbits = c + IS;
    if (lane == 0) { s_a[0] = 0; s_a[L] = nbits; }
    uint32_t ones_before = 0;
    for (uint32_t base = 0; base < nbits; base += 64 * WAVE) {
      const uint32_t b0 = base + lane * 64;
      uint64_t x = 0;
      if (b0 < nbits) {
        x = bits64_at(pg, ebit + b0);
        const uint32_t nb = min(64u, nbits - b0);
        x &= lowmask64(nb);
      }
      const uint32_t ones = __popcll(x);
      const uint32_t ex = wave_incl_scan(ones) - ones + ones_before;
      // terminators t = kG - 1 (k = 1..L-1) inside [ex, ex + ones): group k starts after t
      for (uint32_t k = (ex + G) >> lgG; k < L && k * G - 1 < ex + ones; k++)
        s_a[k] = b0 + select64_fast(x, k * G - 1 - ex) + 1;
      ones_before = __shfl(ex + ones, WAVE - 1, WAVE);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t rvs = P.rvs;
  const uint64_t ebit = (rel + 2) * 8;
  const uint32_t enc = (c + IS - 1) / 8 + 4;
  const uint64_t rbit0 = (rel + 2 + enc) * 8;
  const uint64_t line0 = (uint64_t)P.line_base + (uint64_t)(g - P.idx_base) * L;
  for (uint32_t u = lane; u < 4 * L; u += WAVE) {
    const uint32_t gl = u >> 2, qq = u & 3;
    const uint32_t a = s_a[gl], ne = s_a[gl + 1] - a;  // encoding bits of the group = n + G
    const uint32_t n = ne - G, E = a - gl * G;         // entries, first entry of the group
    const bool ovf = ne > 128 || (uint64_t)n * rvs > 384;
    uint64_t w[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t o = qq * 128 + h * 64;
      uint64_t x = 0;
      if (ovf) {
        x = o < 128 ? ~0ull : 0ull;
      } else if (o < 128) {
        const uint32_t hi = min(o + 64, ne);
        if (o < hi) x = bits64_at(pg, ebit + a + o) & lowmask64(hi - o);
      } else {
        const uint32_t ro = o - 128, hi = min(ro + 64, n * rvs);
        if (ro < hi) x = bits64_at(pg, rbit0 + (uint64_t)E * rvs + ro) & lowmask64(hi - ro);
      }
      w[h] = x;
    }
    lines[(line0 + gl) * 4 + qq] =
        make_uint4((uint32_t)w[0], (uint32_t)(w[0] >> 32), (uint32_t)w[1], (uint32_t)(w[1] >> 32));
  }
}


// Probe lines K6 did not cut, per index (rf_amd_batch_import's images and the diagnostics
// rebuild, force = 1: every filter): one wave per index.
__global__ __launch_bounds__(256) void k_plines(const FilterPlan* __restrict__ plans,
                                                const uint32_t* __restrict__ idx_filter,
                                                const uint64_t* __restrict__ slots,
                                                const uint8_t* __restrict__ pages,
                                                const FilterOut* __restrict__ outs,
                                                uint4* __restrict__ lines, uint32_t num_idx,
                                                uint32_t lmax, uint32_t lis, uint32_t page_size,
                                                uint32_t force) {
  constexpr uint32_t SLICE = MAX_PAGE + 64;
  __shared__ __attribute__((aligned(16))) uint8_t s_blk[256 / WAVE][SLICE];
  extern __shared__ uint32_t s_dyn[];
  const uint32_t wv = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const uint32_t g = blockIdx.x * (blockDim.x / WAVE) + wv;
  if (g >= num_idx) return;  // uniform per wave
  const uint32_t f = idx_filter[g];
  const FilterPlan& P = plans[f];
  if (P.lg_line == 0 || (outs && outs[f].error) || g - P.idx_base >= P.num_indices) return;
  if (!force && P.lines_asm) return;  // K6 cuts (or lists) this filter's lines
  plines_index(P, g, slots, pages, lines, s_blk[wv], s_dyn + wv * (lmax + 1), lane, lis, page_size);
}

// Builds: the pages whose lines K6 left (filters it never cuts, and pages whose group table
// does not fit its LDS) are listed by K6 in plist (plist[0] = count, then page slots); a small
// grid walks the list, one wave per index of a listed page. An empty list costs one load per
// workgroup (a grid over every index of the batch cost a compaction round 0.18 ms).
__global__ __launch_bounds__(256) void k_plines_list(const FilterPlan* __restrict__ plans,
                                                     const uint32_t* __restrict__ pg_filter,
                                                     const uint32_t* __restrict__ page_first,
                                                     const uint64_t* __restrict__ slots,
                                                     const uint8_t* __restrict__ pages,
                                                     const uint32_t* __restrict__ plist,
                                                     uint4* __restrict__ lines, uint32_t lmax, uint32_t lis,
                                                     uint32_t page_size) {
  constexpr uint32_t SLICE = MAX_PAGE + 64;
  __shared__ __attribute__((aligned(16))) uint8_t s_blk[256 / WAVE][SLICE];
  extern __shared__ uint32_t s_dyn[];
  const uint32_t wv = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const uint32_t n = plist[0];
  for (uint32_t e = blockIdx.x; e < n; e += gridDim.x) {
    const uint32_t slot = plist[1 + e];
    const FilterPlan& P = plans[pg_filter[slot]];
    const uint32_t* pf = page_first + P.pf_base;
    const uint32_t p = slot - P.page_base, b1 = pf[p + 1];
    for (uint32_t b = pf[p] + wv; b < b1; b += 256 / WAVE)
      plines_index(P, P.idx_base + b, slots, pages, lines, s_blk[wv], s_dyn + wv * (lmax + 1), lane, lis,
                   page_size);
  }
}

// position of the r-th (0-based) set bit of x (exists)
__device__ __forceinline__ uint32_t select32(uint32_t x, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 16; w >= 1; w >>= 1) {
    const uint32_t c = __popc(x & ((1u << w) - 1));
    const bool up = r >= c;
    r = up ? r - c : r;
    x = up ? x >> w : x;
    pos = up ? pos + w : pos;
  }
  return pos;
}

// bit 0 of every rvs-bit field of a 64-bit word (rvs in [1, 32]): sum of 2^(k rvs) for
// k < 64 / rvs, by doubling the pattern
__device__ __forceinline__ uint64_t field_ones64(uint32_t rvs) {
  uint64_t L = 1;
  uint32_t w = rvs;  // width covered so far
#pragma unroll
  for (int i = 0; i < 6; i++) {
    if (w < 64) {
      L |= L << w;
      w <<= 1;
    }
  }
  return L;
}

// Line probe, decode half (format above): bucket j of the line's group, its encoding dwords
// in E (line bytes [0, 16)); win(wi, w0, w1, w2) fetches dwords wi, wi + 1, wi + 2 of the
// remainder area (line dwords 4 + wi ..; past the line: 0). Returns false when the image must
// be walked instead (overflowed line, or a bucket too large for the 96-bit remainder window).
template <typename Win>
__device__ __forceinline__ bool line_decode_w(const v4u& E, Win win, uint32_t j, uint32_t remainder, uint32_t vs,
                                              uint32_t rvs, uint64_t& found) {
  const uint32_t d0 = E.x, d1 = E.y, d2 = E.z, d3 = E.w;
  if ((d0 & d1 & d2 & d3) == 0xffffffffu) return false;  // overflow marker
  // p1 = first bit after terminator j-1 (0 for bucket 0); entries before bucket j = p1 - j
  uint32_t p1 = 0;
  if (j) {
    const uint32_t r = j - 1, c0 = __popc(d0), c1 = c0 + __popc(d1), c2 = c1 + __popc(d2);
    const uint32_t x = r >= c2 ? d3 : (r >= c1 ? d2 : (r >= c0 ? d1 : d0));
    const uint32_t base = r >= c2 ? 96u : (r >= c1 ? 64u : (r >= c0 ? 32u : 0u));
    const uint32_t rr = r - (r >= c2 ? c2 : (r >= c1 ? c1 : (r >= c0 ? c0 : 0u)));
    p1 = base + select32(x, rr) + 1;
  }
  const uint32_t s = p1 - j;
  // c = entries of bucket j = zeros from p1 up to terminator j
  // (p1 <= 128: the encoding has j + 1 <= G terminators in 128 bits)
  const uint64_t e0 = (uint64_t)d1 << 32 | d0, e1 = (uint64_t)d3 << 32 | d2;
  const uint64_t y = p1 >= 128 ? 0ull
                     : (p1 >= 64 ? e1 >> (p1 - 64) : (e0 >> p1) | (p1 ? e1 << (64 - p1) : 0ull));
  if (y == 0) return false;
  const uint32_t c = (uint32_t)__builtin_ctzll(y);
  found = 0;
  if (c == 0 || rvs == 0) {
    if (c && remainder == 0) found = 1;  // rvs == 0: every entry matches, value 0
    return true;
  }
  // the bucket's remainders: bits [s*rvs, (s+c)*rvs) of the 384-bit remainder area
  const uint32_t b = s * rvs, wi = b >> 5, off = b & 31;
  if (off + c * rvs > 96 || b + c * rvs > 384) return false;
  uint32_t w0, w1, w2;
  win(wi, w0, w1, w2);
  const uint64_t wl = (uint64_t)w1 << 32 | w0;
  const uint32_t vmask = (uint32_t)((1ull << vs) - 1);
  const uint32_t nb = c * rvs, rem = rvs - vs;
  if (nb <= 64 && rem > 0) {
    // all c entries at once (SWAR): W holds them as c fields of rvs bits, remainder part
    // [vs, rvs) of each. Y keeps each field's remainder part XOR the probe's; a field
    // matches iff its part of Y is zero: adding the all-ones low part MH carries into the
    // part's top bit H exactly when the low bits are nonzero (no carry leaves a field).
    const uint64_t W = off ? (wl >> off) | ((uint64_t)w2 << (64 - off)) : wl;
    const uint64_t L = field_ones64(rvs);  // bit 0 of every rvs-bit field
    const uint64_t valid = nb == 64 ? ~0ull : (1ull << nb) - 1;
    const uint64_t M = ((L << rvs) - (L << vs)) & valid;  // remainder part of each field
    const uint64_t H = (L << (rvs - 1)) & valid;          // top bit of each remainder part
    const uint64_t MH = M & ~H;
    const uint64_t Y = (W ^ ((uint64_t)(remainder << vs) * L)) & M;
    uint64_t Z = H & ~((((Y & MH) + MH) | Y) & H);  // top bits of the matching fields
    if (vs == 0) {
      found = Z ? 1ull : 0ull;
    } else {
      while (Z) {  // one pass per match (usually 0 or 1)
        const uint32_t p = (uint32_t)__builtin_ctzll(Z) + 1 - rvs;  // the field's first bit
        const uint32_t val = (uint32_t)(W >> p) & vmask;
        if (val < 64) found |= 1ull << val;
        Z &= Z - 1;
      }
    }
    return true;
  }
  const uint32_t rvmask = rvs >= 32 ? 0xffffffffu : ((1u << rvs) - 1);
  for (uint32_t k = 0; k < c; k++) {
    const uint32_t qb = off + k * rvs;  // < 96
    const uint64_t v = qb < 64 ? ((wl >> qb) | (qb ? (uint64_t)w2 << (64 - qb) : 0ull)) : (uint64_t)(w2 >> (qb - 64));
    const uint32_t rv = (uint32_t)v & rvmask;
    if ((rv >> vs) == remainder) {
      const uint32_t val = rv & vmask;
      if (val < 64) found |= 1ull << val;
    }
  }
  return true;
}

// the window from the line held in registers (Q[1..3]: the 384-bit remainder area): 96 bits at
// dword wi (wi <= 9) -- pick the 4-dword group g = wi / 4, then dwords o..o+2 (o = wi % 4) of
// that group's 6-dword span (21 selects instead of 36)
__device__ __forceinline__ bool line_decode(const v4u (&Q)[4], uint32_t j, uint32_t remainder, uint32_t vs,
                                            uint32_t rvs, uint64_t& found) {
  auto win = [&](uint32_t wi, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
    const uint32_t R[14] = {Q[1].x, Q[1].y, Q[1].z, Q[1].w, Q[2].x, Q[2].y, Q[2].z,
                            Q[2].w, Q[3].x, Q[3].y, Q[3].z, Q[3].w, 0u, 0u};
    const uint32_t g = wi >> 2, o = wi & 3;
    uint32_t W[6];
#pragma unroll
    for (int k = 0; k < 6; k++) W[k] = g == 0 ? R[k] : (g == 1 ? R[4 + k] : R[8 + k]);
    w0 = o == 0 ? W[0] : (o == 1 ? W[1] : (o == 2 ? W[2] : W[3]));
    w1 = o == 0 ? W[1] : (o == 1 ? W[2] : (o == 2 ? W[3] : W[4]));
    w2 = o == 0 ? W[2] : (o == 1 ? W[3] : (o == 2 ? W[4] : W[5]));
  };
  return line_decode_w(Q[0], win, j, remainder, vs, rvs, found);
}

// threads per probe workgroup: 1,024 for fixed-length keys and hashes (C3 probe 2.74 ->
// 2.59 ms per 256M vs 256: a quarter of the workgroups, each longer), 256 for variable-length
// keys (their per-wave 4 KiB LDS windows; C5 0.325 vs 0.337 ms)
#ifndef RF_PROBE_NT
#define RF_PROBE_NT 1024
#endif
// quad-cooperative probe-line gather (k_probe); 0 = one lane loads its own line
#ifndef RF_PROBE_QUAD
#define RF_PROBE_QUAD 1
#endif
constexpr int PROBE_NT = RF_PROBE_NT;
constexpr int PROBE_NT_VAR = 256;
__host__ __device__ constexpr int probe_nt(int kind) { return kind == IN_VAR ? PROBE_NT_VAR : PROBE_NT; }

// One lane per probe for hashing and decoding. (A cooperative variant that staged 128-byte
// block heads through LDS, 8 lanes per block, measured slower on MI355X -- 3.09 vs 2.34 ms at
// C2; the quad gather below keeps the decode per lane and moves only the line through LDS.)
// Wave table of per-filter probe runs: entry w = (filter of probe 64 w) << 7 | the number of
// the wave's leading probes in that filter's run (64: the whole wave). Built by k_wave_tab
// whenever the run bounds change, so a probe wave finds its filter with ONE scalar load
// instead of a binary search of dependent loads over the run bounds.
__global__ __launch_bounds__(256) void k_wave_tab(const uint64_t* __restrict__ runs, uint32_t nf, uint64_t n,
                                                  uint32_t* __restrict__ tab) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i = w * WAVE;
  if (i >= n) return;
  uint32_t lo = 0, hi = nf;  // largest lo with runs[lo] <= i
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (runs[mid] <= i) lo = mid; else hi = mid;
  }
  const uint64_t left = runs[lo + 1] - i;  // runs[nf] = n
  tab[w] = lo << 7 | (uint32_t)min<uint64_t>(left, WAVE);
}

// filter of probe i (lane `lane` of its wave) from the wave table; lanes past the wave's
// first run boundary step forward over the run bounds
__device__ __forceinline__ uint32_t tab_filter(const uint32_t* __restrict__ tab, const uint64_t* __restrict__ runs,
                                               uint32_t nf, uint64_t i) {
  const uint64_t w = i / WAVE;
  const uint64_t wu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(w >> 32)) << 32) |
                      __builtin_amdgcn_readfirstlane((uint32_t)w);
  const uint32_t t = tab[wu];  // wave-uniform address: a scalar load
  uint32_t lo = t >> 7;
  if ((uint32_t)(i & (WAVE - 1)) >= (t & 127u))
    while (lo + 1 < nf && runs[lo + 1] <= i) lo++;
  return lo;
}

// the probe plan of filter fid; when the whole wave probes one filter (the usual case with
// per-filter runs) it is one scalar load
__device__ __forceinline__ uint4 load_pplan(const uint4* __restrict__ pplans, uint32_t fid, uint32_t nf) {
  const uint32_t fs = __builtin_amdgcn_readfirstlane(fid);
  if (__builtin_amdgcn_ballot_w64(fid != fs) == 0) {
    if (fs >= nf) return make_uint4(0, 0, 0, 1);
#if __HIP_DEVICE_COMPILE__
    // constant address space: a uniform address there is always a scalar (SMEM) load
    typedef __attribute__((address_space(4))) const uint32_t cu32;
    const cu32* c = reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(pplans + fs));
    return make_uint4(c[0], c[1], c[2], c[3]);
#else
    return pplans[fs];
#endif
  }
  return fid < nf ? pplans[fid] : make_uint4(0, 0, 0, 1);
}

// The line half of one probe once its hash and probe plan P are known: bucket, remainder,
// the probe line and its decode. Returns false when the image must be walked instead
// (overflowed line, a bucket too large for the window, or a filter without lines). When the
// whole wave probes one filter, k_probe passes P as wave-uniform values, so everything
// derived from the plan alone (widths, masks, the SWAR field pattern) is computed once per
// wave in scalar registers.
__device__ __forceinline__ bool probe_line(const uint4 P, uint32_t h, const uint4* __restrict__ lines,
                                           uint32_t fp_size, uint64_t& r) {
  const uint32_t vs = P.x & 0xff, rem = (P.x >> 8) & 0xff, rvs = (P.x >> 16) & 0xff, lgl = P.x >> 24;
  r = 0;
  if (P.w) return true;  // unknown filter, or its build failed: nothing found
  if (!lgl) return false;
  const uint32_t fp = h >> (32 - fp_size);
  const uint32_t bucket = rem >= 32 ? 0u : fp >> rem;  // index << lis | bucket in index
  const uint32_t remainder = fp & (rem >= 32 ? 0xffffffffu : ((1u << rem) - 1));
  const v4u* lp = reinterpret_cast<const v4u*>(lines + ((uint64_t)P.y + (bucket >> (lgl - 1))) * 4);
  v4u Q[4];
#pragma unroll
  for (int k = 0; k < 4; k++) Q[k] = lp[k];
  return line_decode(Q, bucket & ((1u << (lgl - 1)) - 1), remainder, vs, rvs, r);
}

// the image walk of one probe (probe_stream from its index slot)
__device__ __forceinline__ uint64_t probe_walk(const uint4 P, uint32_t h, uint32_t fid,
                                               const FilterPlan* __restrict__ plans,
                                               const uint8_t* __restrict__ pages, const uint64_t* __restrict__ slots,
                                               uint32_t fp_size, uint32_t lis, uint32_t page_size) {
  const uint32_t vs = P.x & 0xff, rem = (P.x >> 8) & 0xff, rvs = (P.x >> 16) & 0xff;
  const uint32_t fp = h >> (32 - fp_size);
  const uint32_t bucket = rem >= 32 ? 0u : fp >> rem;
  const uint32_t remainder = fp & (rem >= 32 ? 0xffffffffu : ((1u << rem) - 1));
  const uint64_t hdr = slots[P.z + (bucket >> lis)];
  const uint8_t* pg = pages + (uint64_t)plans[fid].page_base * page_size;
  return probe_stream(bucket & ((1u << lis) - 1), remainder, vs, rvs, pg, hdr, lis);
}

// ---- the probe's fast path ---------------------------------------------------------------
// A full wave of probes that all look into ONE filter (per-filter runs, the usual case) runs with
// every plan field, base address and loop bound in scalar registers, and its lines land in LDS in
// natural order (quad q of the wave reads the line of probe 4q + k in instruction k, lane 4q + t
// loading its quarter t), so each probe reads its encoding with one ds_read_b128 and its remainder
// window with three ds_read_b32 off one address. The SWAR field pattern comes from a table in
// constant memory (one scalar load) instead of being built per wave.
struct FieldOnes {
  uint64_t v[33];
  constexpr FieldOnes() : v() {
    for (uint32_t r = 1; r <= 32; r++) {
      uint64_t L = 0;
      for (uint32_t k = 0; k < 64; k += r) L |= 1ull << k;
      v[r] = L;
    }
  }
};
__constant__ FieldOnes c_field_ones = FieldOnes();

// uniform 32-bit loads through the constant address space: always scalar (SMEM) loads
__device__ __forceinline__ uint32_t sload32(const void* p) {
#if __HIP_DEVICE_COMPILE__
  typedef __attribute__((address_space(4))) const uint32_t cu32;
  return *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(p));
#else
  return *static_cast<const uint32_t*>(p);
#endif
}
__device__ __forceinline__ uint64_t sload64(const void* p) {
  return (uint64_t)sload32(p) | (uint64_t)sload32(static_cast<const uint32_t*>(p) + 1) << 32;
}

// routing_get_bucket_bounds + the remainder scan (src/routing_filter.c:230-279, :1051-1067) on a
// probe line held in LDS (Lw: its 16 dwords, natural order); vs, rvs, L (rvs-bit field ones) are
// wave-uniform. Returns false when the image must be walked (overflowed line, a bucket too big
// for the 96-bit window or for one 64-bit SWAR compare).
__device__ __forceinline__ bool line_decode_u(const uint32_t* Lw, uint32_t j, uint32_t remainder, uint32_t vs,
                                              uint32_t rvs, uint64_t L, uint64_t& found) {
  const v4u E = *reinterpret_cast<const v4u*>(Lw);
  const uint32_t d0 = E.x, d1 = E.y, d2 = E.z, d3 = E.w;
  if ((d0 & d1 & d2 & d3) == 0xffffffffu) return false;  // overflow marker
  uint32_t p1 = 0;  // first bit after terminator j - 1
  if (j) {
    const uint32_t r = j - 1, c0 = __popc(d0), c1 = c0 + __popc(d1), c2 = c1 + __popc(d2);
    const uint32_t x = r >= c2 ? d3 : (r >= c1 ? d2 : (r >= c0 ? d1 : d0));
    const uint32_t base = r >= c2 ? 96u : (r >= c1 ? 64u : (r >= c0 ? 32u : 0u));
    const uint32_t rr = r - (r >= c2 ? c2 : (r >= c1 ? c1 : (r >= c0 ? c0 : 0u)));
    p1 = base + select32(x, rr) + 1;
  }
  const uint64_t e0 = (uint64_t)d1 << 32 | d0, e1 = (uint64_t)d3 << 32 | d2;
  const uint64_t y = p1 >= 128 ? 0ull : (p1 >= 64 ? e1 >> (p1 - 64) : (e0 >> p1) | (p1 ? e1 << (64 - p1) : 0ull));
  if (y == 0) return false;
  const uint32_t c = (uint32_t)__builtin_ctzll(y);  // entries of bucket j
  found = 0;
  if (c == 0) return true;
  const uint32_t b = (p1 - j) * rvs, nb = c * rvs, wi = b >> 5, off = b & 31;
  if (off + nb > 96 || b + nb > 384 || nb > 64) return false;
  const uint64_t M = (L << rvs) - (L << vs);  // remainder part of every field (uniform)
  const uint64_t H = L << (rvs - 1);          // top bit of every remainder part (uniform)
  const uint64_t MH = M & ~H;
  const uint32_t w0 = Lw[4 + wi], w1 = Lw[5 + wi], w2 = Lw[6 + wi];
  // the c fields as one 64-bit word (funnel shifts), compared at once (SWAR, as line_decode_w)
  const uint64_t W = (uint64_t)__builtin_amdgcn_alignbit(w2, w1, off) << 32 | __builtin_amdgcn_alignbit(w1, w0, off);
  const uint64_t Y = W ^ ((uint64_t)(remainder << vs) * L);
  const uint64_t valid = nb == 64 ? ~0ull : (1ull << nb) - 1;
  uint64_t Z = H & valid & ~(((Y & MH) + MH) | Y);  // top bits of the matching fields
  if (vs == 0) {
    found = Z ? 1ull : 0ull;
  } else {
    const uint32_t vmask = (1u << vs) - 1;
    while (Z) {  // one pass per match (usually 0 or 1)
      const uint32_t p = (uint32_t)__builtin_ctzll(Z) + 1 - rvs;  // the field's first bit
      const uint32_t val = (uint32_t)(W >> p) & vmask;
      if (val < 64) found |= 1ull << val;
      Z &= Z - 1;
    }
  }
  return true;
}

// The fast path's LDS buffer per wave: instruction k of the quad gather lands its 1 KiB (16
// lines) at byte k * FAST_KSTRIDE, so the line of probe p = 4g + k sits at k * 1040 + 64 g: the
// 16-byte skew per k puts the 16 lanes of each ds_read_b128 lane group on 16 distinct bank
// quads (without it the four probes of a quad hit the same banks: 4-way conflicts). One extra
// 16-byte slot: a remainder window read at the last line's end (masked bits) stays inside.
#ifndef RF_FAST_KSTRIDE
#define RF_FAST_KSTRIDE 1040
#endif
constexpr uint32_t FAST_KSTRIDE = RF_FAST_KSTRIDE;
constexpr int FAST_WBUF = (3 * FAST_KSTRIDE + 1024) / 16 + 1;

// Sweep 0.. of a full wave of one filter: hash (24-byte keys staged through LDS by LDS-DMA, or
// hashes), gather each probe's 64-B line (quad-cooperative LDS-DMA), decode, one coalesced
// store. False when the wave is not fast-path material (the caller takes the general path).
template <int KIND>
__device__ __forceinline__ bool probe_fast(const uint4* __restrict__ pplans, const FilterPlan* __restrict__ plans,
                                           const uint8_t* __restrict__ pages, const uint64_t* __restrict__ slots,
                                           const uint4* __restrict__ lines, const void* __restrict__ in0,
                                           const uint32_t* __restrict__ wave_tab, uint64_t n,
                                           uint64_t* __restrict__ found, uint32_t fp_size, uint32_t seed, uint32_t lis,
                                           uint32_t page_size, uint32_t nf, uint64_t wf, v4u* sw) {
  if (wf + WAVE > n) return false;
  if (KIND == IN_KEYS24 && ((uintptr_t)in0 & 15)) return false;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  // the wave's keys (or hashes) are requested before its filter is known: their load runs
  // under the two dependent scalar loads of the wave table and the plan instead of after them.
  // A wave that turns out not to be fast-path material leaves the keys where the general path
  // stages them itself (the same LDS slots, the same bytes).
  uint32_t h = 0;
  if constexpr (KIND == IN_KEYS24) {
    // the wave's 64 keys (1,536 contiguous bytes): 16-byte LDS-DMA loads, 12 cache lines
    const uint8_t* kb = static_cast<const uint8_t*>(in0) + wf * 24;
    const uint8_t* kb2 = kb + 1024;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + lane * 16),
                                     (__attribute__((address_space(3))) void*)sw, 16, 0, 2);
    if (lane < 32)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb2 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(sw + WAVE), 16, 0, 2);
  } else {
    h = __builtin_nontemporal_load(static_cast<const uint32_t*>(in0) + wf + lane);
  }
  const uint32_t t = sload32(wave_tab + wf / WAVE);
  if ((t & 127u) != WAVE) return false;  // the wave spans a run boundary
  const uint32_t fs = t >> 7;
  if (fs >= nf) return false;
  const uint4 U = make_uint4(sload32(&pplans[fs].x), sload32(&pplans[fs].y), sload32(&pplans[fs].z),
                             sload32(&pplans[fs].w));
  const uint32_t vs = U.x & 0xff, rem = (U.x >> 8) & 0xff, rvs = (U.x >> 16) & 0xff, lgl = U.x >> 24;
  if (U.w || !lgl || rem == 0 || rem >= 32 || rvs > 32) return false;
  if constexpr (KIND == IN_KEYS24) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync_lds();
    const uint2* k2 = reinterpret_cast<const uint2*>(sw) + 3 * lane;
    const uint2 a = k2[0], b = k2[1], c = k2[2];
    const uint32_t w[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
    h = xxh32_24(w, seed);
  }
  const uint32_t lgG = lgl - 1;
  const uint32_t fp = h >> (32 - fp_size);
  const uint32_t bucket = fp >> rem;
  const uint32_t remainder = fp & ((1u << rem) - 1);
  const uint8_t* fb = reinterpret_cast<const uint8_t*>(lines) + ((uint64_t)U.y << 6);  // the filter's lines
  const uint32_t lo = (bucket >> lgG) << 6, q16 = (lane & 3) << 4;
  uint8_t* sb = reinterpret_cast<uint8_t*>(sw);
#define RF_FAST_LOAD(k)                                                                                       \
  {                                                                                                           \
    const uint32_t lk = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, (k) * 0x55, 0xf, 0xf, false);             \
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(fb + (lk + q16)),        \
                                     (__attribute__((address_space(3))) void*)(sb + (k) * FAST_KSTRIDE), 16, 0, 0); \
  }
  RF_FAST_LOAD(0) RF_FAST_LOAD(1) RF_FAST_LOAD(2) RF_FAST_LOAD(3)
#undef RF_FAST_LOAD
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync_lds();
  const uint32_t* Lw = reinterpret_cast<const uint32_t*>(sb + (lane & 3) * FAST_KSTRIDE + (lane >> 2) * 64);
  const uint64_t L = sload64(&c_field_ones.v[rvs]);
  uint64_t r;
  if (!line_decode_u(Lw, bucket & ((1u << lgG) - 1), remainder, vs, rvs, L, r))
    r = probe_walk(U, h, fs, plans, pages, slots, fp_size, lis, page_size);
#ifdef RF_PROBE_PAD
  {  // diagnostics builds only (tools/ab_build.sh): RF_PROBE_PAD extra VALU per lane
    uint32_t x = h;
#pragma unroll
    for (int k = 0; k < RF_PROBE_PAD; k++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(remainder));
    asm volatile("" ::"v"(x));
  }
#endif
  __builtin_nontemporal_store(r, found + wf + lane);
  return true;
}

template <int KIND>
__global__ __launch_bounds__(probe_nt(KIND)) void k_probe(const uint4* __restrict__ pplans,
                                                    const FilterPlan* __restrict__ plans,
                                                    const uint8_t* __restrict__ pages,
                                                    const uint64_t* __restrict__ slots,
                                                    const uint4* __restrict__ lines,
                                                    const void* __restrict__ in0,
                                                    const uint64_t* __restrict__ offs, uint32_t key_len,
                                                    const uint32_t* __restrict__ filter_id,
                                                    const uint64_t* __restrict__ runs,
                                                    const uint32_t* __restrict__ wave_tab, uint64_t n,
                                                    uint64_t* __restrict__ found, uint32_t fp_size,
                                                    uint32_t seed, uint32_t lis, uint32_t page_size,
                                                    uint32_t num_filters) {
  constexpr int NT = probe_nt(KIND);
  const uint64_t i0 = (uint64_t)xcd_chunk(blockIdx.x, gridDim.x) * NT + threadIdx.x;
  uint32_t h = 0, fid = 0xffffffffu;
  uint4 pp = make_uint4(0, 0, 0, 1);
  constexpr bool WAVE_KEYS = KIND == IN_KEYS24;
  constexpr bool WAVE_VAR = KIND == IN_VAR;
  // per wave: the 24-byte keys' staging (96 x 16 B), then the quad-gathered probe lines
  // (64 x 64 B); variable-length keys stage their window in s_vk and reuse it for the lines
  constexpr bool QUAD = RF_PROBE_QUAD;
  constexpr int WBUF = (QUAD && !WAVE_VAR) ? FAST_WBUF : (WAVE_KEYS ? 96 : 1);
  __shared__ v4u s_wbuf[NT / WAVE][WBUF];
  constexpr uint32_t VCAP = 4096;
  __shared__ __attribute__((aligned(16))) uint32_t s_vk[WAVE_VAR ? NT / WAVE : 1][WAVE_VAR ? VCAP / 4 + 4 : 1];
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t wf = i0 - lane;  // the wave's first probe
  if constexpr ((KIND == IN_KEYS24 || KIND == IN_HASH) && QUAD) {
    if (runs) {
      const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x) / WAVE;
      const uint64_t wfs = (uint64_t)xcd_chunk(blockIdx.x, gridDim.x) * NT + wv * WAVE;  // = wf, in SGPRs
      if (wfs < n && probe_fast<KIND>(pplans, plans, pages, slots, lines, in0, wave_tab, n, found, fp_size, seed,
                                      lis, page_size, num_filters, wfs, s_wbuf[wv]))
        return;
    }
  }
  if constexpr (WAVE_KEYS) {
    // 24-byte keys: the wave's 64 keys (1,536 contiguous bytes) are read with 16-byte
    // coalesced loads -- 12 cache lines per wave, where three strided 8-byte loads per lane
    // touch 36 -- and handed to their lanes through LDS
    if (wf < n) {  // uniform per wave
      if (i0 < n) fid = runs ? tab_filter(wave_tab, runs, num_filters, i0) : __builtin_nontemporal_load(filter_id + i0);
      pp = load_pplan(pplans, fid, num_filters);  // in flight with the key loads
      if (((uintptr_t)in0 & 15) == 0) {
        v4u* sw = s_wbuf[threadIdx.x / WAVE];
        const uint32_t bytes = (uint32_t)min<uint64_t>(WAVE, n - wf) * 24;
        const v4u* src = reinterpret_cast<const v4u*>(static_cast<const uint8_t*>(in0) + wf * 24);
        if (bytes == WAVE * 24) {  // full wave: LDS-DMA, no VGPR round trip
#pragma unroll
          for (uint32_t it = 0; it < 2; it++) {
            const uint32_t j = lane + it * WAVE;
            if (j < 96)
              __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + j),
                                               (__attribute__((address_space(3))) void*)(sw + it * WAVE), 16, 0, 2);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else
#pragma unroll
        for (uint32_t j = lane; j < 96; j += WAVE) {
          if ((j + 1) * 16 <= bytes) {
            sw[j] = __builtin_nontemporal_load(src + j);
          } else if (j * 16 < bytes) {  // an odd key count ends on an 8-byte half
            const uint64_t t = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(src + j));
            sw[j] = v4u{(uint32_t)t, (uint32_t)(t >> 32), 0u, 0u};
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (i0 < n) {
          const uint2* k2 = reinterpret_cast<const uint2*>(sw) + 3 * lane;
          const uint2 a = k2[0], b = k2[1], c = k2[2];
          uint32_t w[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
          h = xxh32_24(w, seed);
        }
      } else if (i0 < n) {
        h = hash_key<KIND, true>(in0, offs, key_len, seed, i0);
      }
    }
  } else if constexpr (WAVE_VAR) {
    // variable-length keys: the wave's 64 keys are one contiguous byte range, read into a
    // 4 KiB LDS window with coalesced 16-byte loads and hashed from there (wave_hash_var)
    uint64_t o0 = 0, o1 = 0;
    if (i0 < n) {
      fid = runs ? tab_filter(wave_tab, runs, num_filters, i0) : __builtin_nontemporal_load(filter_id + i0);
      o0 = offs[i0];
      o1 = offs[i0 + 1];
    }
    pp = load_pplan(pplans, fid, num_filters);
    uint64_t w0 = 0, w1 = 0;
    h = wave_hash_var<VCAP, true>(static_cast<const uint8_t*>(in0), o0, o1, i0 < n, s_vk[threadIdx.x / WAVE], seed,
                                  &w0, &w1);
  } else {
    // the key (or hash) and filter id are independent loads: issued together
    if (i0 < n) {
      if constexpr (KIND == IN_PAIR) {  // routed probes: (local filter id << 32 | hash)
        const uint64_t pr = __builtin_nontemporal_load(static_cast<const uint64_t*>(in0) + i0);
        fid = (uint32_t)(pr >> 32);
        h = (uint32_t)pr;
      } else {
        fid = runs ? tab_filter(wave_tab, runs, num_filters, i0) : __builtin_nontemporal_load(filter_id + i0);
        h = hash_key<KIND, true>(in0, offs, key_len, seed, i0);
      }
    }
    pp = load_pplan(pplans, fid, num_filters);
  }
  const uint32_t fs = __builtin_amdgcn_readfirstlane(fid);
  const bool uniform = __builtin_amdgcn_ballot_w64(fid != fs) == 0;
  if constexpr (QUAD) {
    // Quad-cooperative line gather (full waves probing one filter -- the usual case with
    // per-filter runs; the conditions are wave-uniform, so every lane takes part in the
    // lane exchanges). One 64-B line per probe, but each wave instruction fetches 16 whole
    // lines (quad g = lanes 4g..4g+3 reads one line, 16 B per lane) instead of a 16-B piece
    // of 64 different lines: 64 line requests per wave instead of 256. Instruction k gathers
    // the lines of probes 4g + k (their line index comes from lane 4g + k by a DPP quad
    // broadcast) straight into LDS (LDS-DMA, lane L -> byte 16 L of the k-th KiB); lane q of
    // the quad loads quarter (q + k) & 3, so probe p finds quarter j of its line at
    // KiB p & 3, line slot p >> 2, 16-B slot (j - p) & 3 -- the 16 lanes of each ds_read_b128
    // lane group then hit 16 distinct 4-bank groups (no conflicts). C2 probe 0.842 -> 0.821
    // ms, C3 2.577 -> 2.537 ms per 256M (profiles/r04_quad_ab.json).
    if (wf + WAVE <= n && uniform) {
      const uint4 U = make_uint4(__builtin_amdgcn_readfirstlane(pp.x), __builtin_amdgcn_readfirstlane(pp.y),
                                 __builtin_amdgcn_readfirstlane(pp.z), __builtin_amdgcn_readfirstlane(pp.w));
      const uint32_t vs = U.x & 0xff, rem = (U.x >> 8) & 0xff, rvs = (U.x >> 16) & 0xff, lgl = U.x >> 24;
      if (!U.w && lgl) {
        const uint32_t q = lane & 3;
        const uint32_t fp = h >> (32 - fp_size);
        const uint32_t bucket = rem >= 32 ? 0u : fp >> rem;
        const uint32_t remainder = fp & (rem >= 32 ? 0xffffffffu : ((1u << rem) - 1));
        // the filter's line table (uniform) and this probe's line within it as a 32-bit byte
        // offset: each load is a scalar base plus one VGPR offset (no per-load 64-bit math)
        const uint8_t* fb = reinterpret_cast<const uint8_t*>(lines) + ((uint64_t)U.y << 6);
        const uint32_t lo = (bucket >> (lgl - 1)) << 6;
        v4u* sw;
        if constexpr (WAVE_VAR) sw = reinterpret_cast<v4u*>(s_vk[threadIdx.x / WAVE]);
        else sw = s_wbuf[threadIdx.x / WAVE];
#define RF_QUAD_LOAD(k)                                                                                      \
  {                                                                                                          \
    const uint32_t lk = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, (k) * 0x55, 0xf, 0xf, false);            \
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(fb + lk + (((q + (k)) & 3u) << 4)), \
                                     (__attribute__((address_space(3))) void*)(sw + (k) * WAVE), 16, 0, 0);  \
  }
        RF_QUAD_LOAD(0) RF_QUAD_LOAD(1) RF_QUAD_LOAD(2) RF_QUAD_LOAD(3)
#undef RF_QUAD_LOAD
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // this probe's line in LDS: quarter j at L32 + ((j - lane) & 3) * 4 (dwords). The
        // decode reads the encoding quarter into registers and only the three dwords of its
        // bucket's remainder window from LDS (instead of all four quarters and a 21-way select:
        // the probe is VALU-bound as much as memory-bound)
        const uint32_t* L32 = reinterpret_cast<const uint32_t*>(sw + (lane & 3) * WAVE + (lane >> 2) * 4);
        const v4u E = *reinterpret_cast<const v4u*>(L32 + ((0u - lane) & 3u) * 4);
        auto win = [&](uint32_t wi, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
          // line dword d = 4 + wi + t (d & 15: dwords past the line are never used, the
          // window's bits beyond the bucket are masked)
          auto dw = [&](uint32_t d) -> uint32_t { d &= 15u; return L32[(((d >> 2) - lane) & 3u) * 4 + (d & 3u)]; };
          w0 = dw(4 + wi);
          w1 = dw(5 + wi);
          w2 = dw(6 + wi);
        };
        uint64_t r;
        if (!line_decode_w(E, win, bucket & ((1u << (lgl - 1)) - 1), remainder, vs, rvs, r))
          r = probe_walk(U, h, fs, plans, pages, slots, fp_size, lis, page_size);
        __builtin_nontemporal_store(r, found + i0);
        return;
      }
    }
  }
  // one lane per probe: partial waves, waves across filters, filters without lines
  if (i0 >= n) return;
  uint64_t r;
  bool ok;
  if (uniform) {  // plan fields in scalar registers: the decode's masks are computed once per wave
    const uint4 U = make_uint4(__builtin_amdgcn_readfirstlane(pp.x), __builtin_amdgcn_readfirstlane(pp.y),
                               __builtin_amdgcn_readfirstlane(pp.z), __builtin_amdgcn_readfirstlane(pp.w));
    ok = probe_line(U, h, lines, fp_size, r);
  } else {
    ok = probe_line(pp, h, lines, fp_size, r);
  }
  if (!ok) r = probe_walk(pp, h, fid, plans, pages, slots, fp_size, lis, page_size);
  __builtin_nontemporal_store(r, found + i0);
}

// The probe's memory floor (bench.py roofline.floor_ms; not a lookup): k_probe's fast path with
// its arithmetic taken out -- the same grid and wave order, the same 24-byte key staging by
// LDS-DMA (or hash loads), the same quad gather of one 64-B line per probe from the probe's own
// filter into the same LDS slots, the same coalesced 8-byte store -- but the line comes from a
// multiply-xorshift of the key words instead of XXH32, and the stored word is an XOR of the
// line's quarter instead of its decode. Waves that are not fast-path material store 0.
template <int KIND>
__global__ __launch_bounds__(probe_nt(KIND)) void k_probe_floor(const uint4* __restrict__ pplans,
                                                          const uint4* __restrict__ lines,
                                                          const void* __restrict__ in0,
                                                          const uint32_t* __restrict__ wave_tab, uint64_t n,
                                                          uint64_t* __restrict__ found, uint32_t fp_size,
                                                          uint32_t nf) {
  constexpr int NT = probe_nt(KIND);
  __shared__ v4u s_wbuf[NT / WAVE][FAST_WBUF];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x) / WAVE;
  const uint64_t wf = (uint64_t)xcd_chunk(blockIdx.x, gridDim.x) * NT + wv * WAVE;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  if (wf >= n) return;
  v4u* sw = s_wbuf[wv];
  uint32_t h = 0;
  const bool full = wf + WAVE <= n;
  if constexpr (KIND == IN_KEYS24) {  // requested before the filter is known, as the fast path
    const uint8_t* kb = static_cast<const uint8_t*>(in0) + wf * 24;
    if (full) {
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + lane * 16),
                                       (__attribute__((address_space(3))) void*)sw, 16, 0, 2);
      if (lane < 32)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(sw + WAVE), 16, 0, 2);
    }
  } else {
    if (full) h = __builtin_nontemporal_load(static_cast<const uint32_t*>(in0) + wf + lane);
  }
  const uint32_t t = sload32(wave_tab + wf / WAVE);
  const uint32_t fs = t >> 7;
  uint32_t lgl = 0, rem = 0, base = 0;
  if ((t & 127u) == WAVE && fs < nf && full) {
    const uint32_t x = sload32(&pplans[fs].x);
    lgl = x >> 24;
    rem = (x >> 8) & 0xff;
    base = sload32(&pplans[fs].y);
  }
  if (!lgl || rem == 0 || rem >= 32) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA left in flight at exit
    if (wf + lane < n) found[wf + lane] = 0;
    return;
  }
  if constexpr (KIND == IN_KEYS24) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync_lds();
    const uint2* k2 = reinterpret_cast<const uint2*>(sw) + 3 * lane;
    const uint2 a = k2[0], b = k2[1], c = k2[2];
    h = (a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y) * 0x9e3779b1u;
    h ^= h >> 15;
    h *= 0x85ebca77u;
  }
  const uint32_t bucket = (h >> (32 - fp_size)) >> rem;
  const uint8_t* fb = reinterpret_cast<const uint8_t*>(lines) + ((uint64_t)base << 6);
  const uint32_t lo = (bucket >> (lgl - 1)) << 6, q16 = (lane & 3) << 4;
  uint8_t* sb = reinterpret_cast<uint8_t*>(sw);
#define RF_FLOOR_LOAD(k)                                                                                      \
  {                                                                                                           \
    const uint32_t lk = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, (k) * 0x55, 0xf, 0xf, false);             \
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(fb + (lk + q16)),        \
                                     (__attribute__((address_space(3))) void*)(sb + (k) * FAST_KSTRIDE), 16, 0, 0); \
  }
  RF_FLOOR_LOAD(0) RF_FLOOR_LOAD(1) RF_FLOOR_LOAD(2) RF_FLOOR_LOAD(3)
#undef RF_FLOOR_LOAD
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync_lds();
  const v4u E = *reinterpret_cast<const v4u*>(sb + (lane & 3) * FAST_KSTRIDE + (lane >> 2) * 64);
  __builtin_nontemporal_store((uint64_t)(E[0] ^ E[1] ^ E[2] ^ E[3]), found + wf + lane);
}

// one lookup of hash h in a resident filter given by its group descriptor (its own routing
// config: one launch may answer filters of differently configured kvstores)
__device__ __forceinline__ uint64_t probe_group(const ProbeGroup& G, uint32_t h) {
  const uint32_t fp_size = G.fpl & 0xff, lis = (G.fpl >> 8) & 0xff;
  const uint4 P = make_uint4(G.x, 0u, 0u, G.err);
  uint64_t r = 0;
  if (!probe_line(P, h, G.lines, fp_size, r)) {  // overflowed line / no lines: walk the image
    const uint32_t vs = G.x & 0xff, rem = (G.x >> 8) & 0xff, rvs = (G.x >> 16) & 0xff;
    const uint32_t fp = h >> (32 - fp_size);
    const uint32_t bucket = rem >= 32 ? 0u : fp >> rem;
    const uint32_t remainder = fp & (rem >= 32 ? 0xffffffffu : ((1u << rem) - 1));
    r = probe_stream(bucket & ((1u << lis) - 1), remainder, vs, rvs, G.pages, G.slots[bucket >> lis], lis);
  }
  return r;
}

// ---- lookups against many resident filters in one launch ------------------------------
// Probe i looks up hash in[i] in the filter of group in[n + i] (routing_filter_lookup,
// src/routing_filter.c:985-1073, decoded exactly as k_probe: probe line, image walk when the
// line overflowed). This is the latency path of the drop-in shim: a few to a few thousand
// lookups over up to thousands of filters of different batches. Inputs, group table and
// results may be device memory or pinned host memory read and written over PCIe. When
// done_flag (pinned host memory) is set, every workgroup publishes its results system-wide
// and the last one to finish stores `seq` there: the host waits by polling that word instead
// of synchronising the stream (one HIP call fewer per round trip).
__global__ __launch_bounds__(256) void k_probe_groups(const uint32_t* __restrict__ in,
                                                      const ProbeGroup* __restrict__ groups, uint32_t ng,
                                                      uint64_t n, uint64_t* __restrict__ found,
                                                      uint32_t* __restrict__ counter,
                                                      uint32_t* __restrict__ done_flag, uint32_t seq) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const uint32_t h = in[i], g = in[n + i];
    uint64_t r = 0;
    if (g < ng) r = probe_group(groups[g], h);
    found[i] = r;
  }
  if (done_flag) {
    // every wave's result stores have left before the workgroup signals (guide: producer
    // stores -> vmcnt(0) -> barrier -> one lane's release fence -> vmcnt(0) -> flag)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence_system();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t last = gridDim.x - 1;
      // acq_rel at agent scope: the last workgroup's RMW acquires every earlier workgroup's
      // released results before it publishes the flag
      if (last == 0 || __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == last) {
        if (last) atomicExch(counter, 0u);  // ready for the slot's next launch (stream-ordered)
        __hip_atomic_store(done_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// The smallest calls -- a routing_filter_lookup of one key, a handful of async states -- pass
// their hashes and filter descriptors in the kernel arguments (delivered with the dispatch):
// the kernel reads nothing from host memory before its probe line, one wave answers, and its
// lane 0 publishes the completion word once every result is visible system-wide.
__global__ __launch_bounds__(WAVE) void k_probe_small(SmallProbe a) {
  const uint32_t lane = threadIdx.x;
  if (lane < a.n) {
    const uint32_t h = a.h[lane], g = a.g[lane];
    uint64_t r = 0;
    if (g < a.ng) r = probe_group(a.groups[g], h);
    a.found[lane] = r;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.done_flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- the lookup server ---------------------------------------------------------------------
// One persistent wave answers single lookups (routing_filter_lookup, routing_filter_lookup_async
// states) that the host writes into a ring of SrvReq (rf_plan.h: device memory written through
// the BAR, or pinned host memory): no kernel launch per call (a launch round trip is ~6.5 us on
// MI355X). Each pass reads word 0 of the next 64 slots; the lanes whose word carries their
// ticket's check read the rest of their request, and the prefix whose 16 words all carry it
// (the host's stores arrive in any order) is served: a system-scope acquire drops stale cached
// device data (batches are built by other kernels into pooled memory while this one runs), the
// lanes probe their filter (probe_group, as k_probe_groups does) and store the answer words,
// each carrying the check, so nothing waits for those stores. When nothing is ready, lane 0
// polls the next slot with s_sleep between polls. The wave exits after `idle_ticks` without
// requests, after `life_ticks` in total (s_memrealtime, 100 MHz) or when the host sets the stop
// word after the ring -- every loop iteration checks the clock, so the kernel always ends -- and
// reports the first ticket it did not serve; the host relaunches it from there when more
// requests come.
#ifndef RF_SRV_PROF
#define RF_SRV_PROF 0
#endif
#ifndef RF_SRV_PAIRSTORE
#define RF_SRV_PAIRSTORE 1
#endif
__device__ __forceinline__ uint64_t srv_ld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(WAVE) void k_lookup_server(const SrvReq* __restrict__ ring, SrvRes* __restrict__ res,
                                                        SrvCtl* __restrict__ ctl, uint64_t head, uint64_t gen,
                                                        uint64_t idle_ticks, uint64_t life_ticks) {
  const uint32_t lane = threadIdx.x;
  const uint64_t* stop_word = reinterpret_cast<const uint64_t*>(ring + SRV_RING);  // rf_engine.cpp srv_stop_word
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t_busy = t0, served = 0;
  // a pass looks at the next 64 slots (one word per lane) and, when all of them are ready (a
  // backlog), at the next (SRV_PER - 1) x 64 too; it serves their ready prefix, up to SRV_PER
  // requests per lane
  constexpr uint32_t SRV_PER = 4;
  constexpr uint32_t SRV_USED = 12;  // request words 12-15 are padding
#if RF_SRV_PROF
  uint64_t pf[6] = {0, 0, 0, 0, 0, 0};
  auto stamp = [] {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return __builtin_amdgcn_s_memrealtime();
  };
#endif
  for (;;) {
#if RF_SRV_PROF
    const uint64_t pa = stamp();
#endif
    // every used word of the next 64 slots in one round trip (device memory: ~0.1-0.3 us);
    // a slot is ready when all of its words carry its ticket's check
    uint64_t w[SRV_PER][SRV_USED];
#pragma unroll
    for (uint32_t q = 0; q < SRV_USED; q++) w[0][q] = srv_ld(&ring[(uint32_t)((head + lane) & (SRV_RING - 1))].w[q]);
    // the host's stop word, read beside the requests (no extra round trip), so a busy wave
    // stops too (engine shutdown, a server marked dead)
    const uint64_t stp = lane == 0 ? srv_ld(stop_word) : 0ull;
    if (__shfl(stp, 0)) break;
    uint32_t k;  // the ready prefix
    {
      const uint32_t ck = srv_check(head + lane);
      bool ok = true;
#pragma unroll
      for (uint32_t q = 0; q < SRV_USED; q++) ok = ok && (uint32_t)(w[0][q] >> 32) == ck;
      const uint64_t ready = __builtin_amdgcn_ballot_w64(ok);
      k = ready == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~ready);
    }
    if (k == WAVE) {  // a backlog: the next (SRV_PER - 1) x 64 slots too, all in flight together
#pragma unroll
      for (uint32_t m = 1; m < SRV_PER; m++)
#pragma unroll
        for (uint32_t q = 0; q < SRV_USED; q++)
          w[m][q] = srv_ld(&ring[(uint32_t)((head + lane + WAVE * m) & (SRV_RING - 1))].w[q]);
#pragma unroll
      for (uint32_t m = 1; m < SRV_PER; m++) {
        const uint32_t ck = srv_check(head + lane + WAVE * m);
        bool ok = true;
#pragma unroll
        for (uint32_t q = 0; q < SRV_USED; q++) ok = ok && (uint32_t)(w[m][q] >> 32) == ck;
        const uint64_t ready = __builtin_amdgcn_ballot_w64(ok);
        if (k == WAVE * m) k += ready == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~ready);
      }
    }
    if (k) {
#if RF_SRV_PROF
      const uint64_t pb = stamp();
      const uint64_t pc = pb;
#endif
      {
        // acquire (system scope) once per served pass: no stale cached device data (it
        // invalidates this CU's L1 and the L2)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        uint64_t found[SRV_PER];
#pragma unroll
        for (uint32_t m = 0; m < SRV_PER; m++) {
          const uint32_t i = lane + WAVE * m;
          found[m] = 0;
          if (i < k) {
            ProbeGroup G;
            G.x = (uint32_t)w[m][0];
            G.err = (uint32_t)w[m][1];
            G.fpl = (uint32_t)w[m][2];
            G.pad = 0;
            const uint32_t h = (uint32_t)w[m][3];
            G.lines = reinterpret_cast<const uint4*>((uint64_t)(uint32_t)w[m][4] | ((uint64_t)(uint32_t)w[m][5] << 32));
            G.pages = reinterpret_cast<const uint8_t*>((uint64_t)(uint32_t)w[m][6] | ((uint64_t)(uint32_t)w[m][7] << 32));
            G.slots = reinterpret_cast<const uint64_t*>((uint64_t)(uint32_t)w[m][8] | ((uint64_t)(uint32_t)w[m][9] << 32));
            found[m] = probe_group(G, h);
          }
        }
#if RF_SRV_PAIRSTORE
        // answers: lanes 2j and 2j+1 store the two 16-byte halves of answer j of a group of 32
        // (found, then tag, each word with its check), so one store instruction writes 1 KB of
        // consecutive answers -- whole 64-byte lines over PCIe instead of 8-byte partial writes
        // (each of which the host's copy of the line would see arrive separately)
#pragma unroll
        for (uint32_t r = 0; r < 2 * SRV_PER; r++) {
          if (k > 32 * r) {  // wave-uniform
            const uint32_t m = r >> 1, src = (r & 1) * 32 + (lane >> 1), a = 32 * r + (lane >> 1);
            const uint32_t f0 = __shfl((uint32_t)found[m], src), f1 = __shfl((uint32_t)(found[m] >> 32), src);
            const uint32_t g0 = __shfl((uint32_t)w[m][10], src), g1 = __shfl((uint32_t)w[m][11], src);
            if (a < k) {
              const uint64_t ck = (uint64_t)srv_check(head + a) << 32;
              const uint64_t x = (uint64_t)((lane & 1) ? g0 : f0) | ck, y = (uint64_t)((lane & 1) ? g1 : f1) | ck;
              uint64_t* dst = res[(uint32_t)((head + a) & (SRV_RING - 1))].w + (lane & 1) * 2;
              typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
              const u64x2 v = {x, y};
              // a system-scope store (sc0 sc1, as __hip_atomic_store emits for 8 bytes) of 16 bytes
              asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(dst), "v"(v) : "memory");
            }
          }
        }
#else
        // (A/B: each lane stores its own answer as four 8-byte words)
#pragma unroll
        for (uint32_t m = 0; m < SRV_PER; m++) {
          const uint32_t i = lane + WAVE * m;
          if (i < k) {
            const uint64_t ck = (uint64_t)srv_check(head + i) << 32;
            uint64_t* r = res[(uint32_t)((head + i) & (SRV_RING - 1))].w;
            __hip_atomic_store(r + 0, (found[m] & 0xffffffffull) | ck, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(r + 1, (found[m] >> 32) | ck, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(r + 2, (uint64_t)(uint32_t)w[m][10] | ck, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(r + 3, (uint64_t)(uint32_t)w[m][11] | ck, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
#endif
#if RF_SRV_PROF
        const uint64_t pd = stamp();
        pf[0] += pb - pa;
        pf[1] += pc - pb;
        pf[2] += pd - pc;
        pf[4] += k;
        pf[5] += 1;
#endif
        head += k;
        served += k;
        t_busy = __builtin_amdgcn_s_memrealtime();
        if (t_busy - t0 > life_ticks) break;  // the lifetime bounds a busy wave too (waiters relaunch it)
        continue;
      }
    }
    // idle: poll the next slot's word 0 alone, bounded by the clock
    bool stop = false;
    for (;;) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now - t_busy > idle_ticks || now - t0 > life_ticks) {
        stop = true;
        break;
      }
      uint64_t t1 = 0, st = 0;
      if (lane == 0) {
        t1 = srv_ld(&ring[head & (SRV_RING - 1)].w[0]);
        st = srv_ld(stop_word);
      }
      t1 = __shfl(t1, 0);
      st = __shfl(st, 0);
      if (st) {
        stop = true;
        break;
      }
      if ((uint32_t)(t1 >> 32) == srv_check(head)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (stop) break;
  }
  if (lane == 0) {
#if RF_SRV_PROF
    for (int q = 0; q < 6; q++)  // one server wave at a time: a plain read-add-write
      __hip_atomic_store(&ctl->prof[q], __hip_atomic_load(&ctl->prof[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + pf[q],
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    __hip_atomic_store(&ctl->exit_head, head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&ctl->served, served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&ctl->exit_gen, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- direct placement of an image into host pages (rf_amd_batch_place_image) ----------------
// Blocks [0, count): image page first_page + k -> table[first_page + k] (a device address of
// registered host memory: the stores go over PCIe, 16 bytes per lane). Blocks past them: index
// slots, 256 per block, slot i -> table[num_pages + slot / page_size] + slot % page_size at
// word i % addrs_per_page of the index page table[2 num_pages + i / addrs_per_page]
// (src/routing_filter.c:612-620).
__global__ __launch_bounds__(256) void k_place(const uint8_t* __restrict__ img, const uint64_t* __restrict__ slots,
                                               uint32_t first_page, uint32_t count, uint32_t num_pages,
                                               uint32_t num_indices, uint32_t page_size,
                                               const uint64_t* __restrict__ table, uint32_t addrs_per_page) {
  if (blockIdx.x < count) {
    const uint32_t k = first_page + blockIdx.x;
    const uint4* src = reinterpret_cast<const uint4*>(img + (uint64_t)k * page_size);
    uint4* dst = reinterpret_cast<uint4*>((uintptr_t)table[k]);
    for (uint32_t i = threadIdx.x; i < page_size / 16; i += 256) dst[i] = src[i];
    return;
  }
  const uint32_t i = (blockIdx.x - count) * 256 + threadIdx.x;
  if (i >= num_indices) return;
  const uint64_t s = slots[i];
  const uint64_t v = table[num_pages + s / page_size] + s % page_size;
  uint64_t* ip = reinterpret_cast<uint64_t*>((uintptr_t)table[2ull * num_pages + i / addrs_per_page]);
  ip[i % addrs_per_page] = v;
}

extern "C" int rf_launch_place(void* stream, const uint8_t* img, const uint64_t* slots, uint32_t first_page,
                                uint32_t count, uint32_t num_pages, uint32_t num_indices, uint32_t page_size,
                                const uint64_t* table, uint32_t addrs_per_page) {
  const uint32_t grid = count + (num_indices + 255) / 256;
  if (grid == 0) return 0;
  hipLaunchKernelGGL(k_place, dim3(grid), dim3(256), 0, (hipStream_t)stream, img, slots, first_page, count,
                     num_pages, num_indices, page_size, table, addrs_per_page);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

extern "C" int rf_launch_lookup_server(void* stream, const SrvReq* ring, SrvRes* res, SrvCtl* ctl, uint64_t head,
                                       uint64_t gen, uint64_t idle_ticks, uint64_t life_ticks) {
  hipLaunchKernelGGL(k_lookup_server, dim3(1), dim3(WAVE), 0, (hipStream_t)stream, ring, res, ctl, head, gen,
                     idle_ticks, life_ticks);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

extern "C" int rf_launch_probe_small(void* stream, const SmallProbe* a) {
  hipLaunchKernelGGL(k_probe_small, dim3(1), dim3(WAVE), 0, (hipStream_t)stream, *a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

extern "C" int rf_launch_probe_groups(void* stream, const uint32_t* in, const ProbeGroup* groups, uint32_t ng,
                                      uint64_t n, uint64_t* found, uint32_t* counter, uint32_t* done_flag,
                                      uint32_t seq) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_probe_groups, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, in, groups,
                     ng, n, found, counter, done_flag, seq);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// ======================================================================================
// launch wrappers (called from rf_engine.cpp)
// ======================================================================================
#define CHECK_LAUNCH() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
#define REC(slot) do { if (a.events && (a.ev_mask >> (slot) & 1u)) (void)hipEventRecord((hipEvent_t)a.events[slot], (hipStream_t)a.stream); } while (0)

// dispatch on the input kind (template parameter of the hashing kernels)
#define KIND_SWITCH(kind, L)           \
  switch (kind) {                      \
    case IN_KEYS24: L(IN_KEYS24); break; \
    case IN_KEYS_W: L(IN_KEYS_W); break; \
    case IN_KEYS_B: L(IN_KEYS_B); break; \
    case IN_VAR: L(IN_VAR); break;       \
    default: L(IN_HASH); break;          \
  }

// counts: per coarse bucket counter array (atomically accumulated); gate: see k_hash_count
// gated launches (the fused build's spill fallback, almost never needed) use a small grid
// that strides over the tiles: most of their cost was dispatching one workgroup per tile
constexpr uint32_t GATED_GRID = 256;

template <typename EntT, bool FL = (sizeof(EntT) == 8)>
static int launch_hash_count_t(const LaunchArgs& a, EntT* ent, uint32_t* counts, const uint32_t* gate) {
  dim3 g(gate ? min(a.num_tiles, GATED_GRID) : a.num_tiles), b(TILE_NT);
#define L(K) hipLaunchKernelGGL((k_hash_count<K, EntT, FL>), g, b, 0, (hipStream_t)a.stream, a.plans, a.tile_filter, \
                                a.tile_start, a.in0, a.offs, a.key_len, a.fp_size, a.seed, ent, counts, gate, a.num_tiles)
  KIND_SWITCH(a.kind, L);
#undef L
  CHECK_LAUNCH();
  return 0;
}

template <typename EntT, bool FL = (sizeof(EntT) == 8)>
static int launch_scatter_t(const LaunchArgs& a, EntT* ent, EntT* part, const uint32_t* gate) {
  if (a.num_tiles) {
    hipLaunchKernelGGL((k_scatter<EntT, FL>), dim3(gate ? min(a.num_tiles, GATED_GRID) : a.num_tiles), dim3(SCAT_NT), 0,
                       (hipStream_t)a.stream, a.plans, a.tile_filter, a.tile_start, 0u, a.fp_size, ent, part,
                       a.cb_cursor, gate, a.num_tiles);
    CHECK_LAUNCH();
  }
  if (a.num_old_tiles && !a.flag32) {  // 32-bit incremental builds read the old runs in K4
    hipLaunchKernelGGL((k_scatter<EntT, FL>), dim3(gate ? min(a.num_old_tiles, GATED_GRID) : a.num_old_tiles),
                       dim3(SCAT_NT), 0, (hipStream_t)a.stream, a.plans, a.old_tile_filter, a.old_tile_start, 1u,
                       a.fp_size, ent, part, a.cb_cursor, gate, a.num_old_tiles);
    CHECK_LAUNCH();
  }
  return 0;
}

// K4m for 32-bit incremental builds (RF_AMD_K4M=0: the K4 DUAL sort instead, for A/B;
// round-8 K4 2.22 -> 1.48 ms on one box)
static bool k4m_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RF_AMD_K4M");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

template <typename EntT, bool FL = (sizeof(EntT) == 8), bool DUAL = false>
static int launch_sort_t(const LaunchArgs& a, EntT* ent, EntT* part, const uint32_t* spill) {
  bool merged = false;
  if constexpr (DUAL) {
    if (k4m_enabled()) {
      merged = true;
      hipLaunchKernelGGL(k_cb_merge, dim3(a.num_cb), dim3(SORT_NT), 0, (hipStream_t)a.stream, a.plans, a.cb_filter,
                       a.cb_count, a.cb_start, (const uint32_t*)part, a.old32, a.ob_lo, a.ob_n, a.sorted32, a.idx_cnt,
                       a.idx_start, a.outs, a.overflow, a.lis, a.first_old, a.has_old, spill, a.cb_outs);
      CHECK_LAUNCH();
      // the buckets K4m handed back (bit 31 on their overflow-list entry): up to one workgroup
      // per coarse bucket (early chain rounds hand back nearly all of them); the surplus exits
      hipLaunchKernelGGL((k_cb_sort<EntT, FL, DUAL, true>), dim3(a.num_cb), dim3(SORT_NT), 0, (hipStream_t)a.stream,
                         a.plans, a.cb_filter, a.cb_count, a.cb_start, part, a.old32, a.ob_lo, a.ob_n, a.sorted32,
                         a.idx_cnt, a.idx_start, a.outs, a.overflow, a.lis, a.first_old, a.has_old, spill, a.cb_outs,
                         a.overflow);
    }
  }
  if (!merged) {
    hipLaunchKernelGGL((k_cb_sort<EntT, FL, DUAL>), dim3(a.num_cb), dim3(SORT_NT), 0, (hipStream_t)a.stream, a.plans,
                       a.cb_filter, a.cb_count, a.cb_start, part, a.old32, a.ob_lo, a.ob_n, a.sorted32, a.idx_cnt,
                       a.idx_start, a.outs, a.overflow, a.lis, a.first_old, a.has_old, spill, a.cb_outs, nullptr);
  }
  CHECK_LAUNCH();
  REC(EV_B_SORT);
  hipLaunchKernelGGL((k_cb_sort_big<EntT, FL, DUAL>), dim3(BIG_GRID), dim3(BIG_NT), 0, (hipStream_t)a.stream, a.plans,
                     a.cb_filter, a.cb_count, a.cb_start, part, a.old32, a.ob_lo, a.ob_n, ent, a.sorted32, a.idx_cnt, a.idx_start, a.outs,
                     a.overflow, a.lis, a.first_old, a.has_old, spill, a.cb_outs);
  CHECK_LAUNCH();
  REC(EV_B_SORT_BIG);
  return 0;
}

extern "C" int rf_launch_plines(const LaunchArgs* pa);
static int launch_plines_list(const LaunchArgs& a);

extern "C" int rf_launch_build(const LaunchArgs* pa) {
  const LaunchArgs& a = *pa;
  if (a.wide && a.flag32) {
    // incremental add, 32-bit flagged entries (fp_size + value_size <= 31): the new entries
    // are hashed, counted and scattered; each coarse bucket's run of the (sorted) old
    // entries decoded by rf_launch_old_decode is located by k_old_cb_bounds and read by K4
    // straight from old32 -- the old entries are neither counted nor scattered
    // The new keys take the fused partition (flagged entries into fixed regions of SORT_CAP
    // slots per coarse bucket, spill fallback as for a fresh build); K4 / K4b write each
    // coarse bucket's sorted new + old entries at the scan of the new + old counts
    uint32_t* ent = (uint32_t*)a.ent;
    uint32_t* part = (uint32_t*)a.part;
    if (a.num_tiles) {
#define L(K) hipLaunchKernelGGL((k_hash_scatter<K, true>), dim3(a.num_tiles), dim3(SCAT_NT), 0, (hipStream_t)a.stream, \
                                a.plans, a.tile_filter, a.tile_start, a.in0, a.offs, a.key_len, a.fp_size, a.seed, \
                                part, a.cb_count, a.spill)
      KIND_SWITCH(a.kind, L);
#undef L
      CHECK_LAUNCH();
    }
    // spill fallback (returns at once unless *spill): exact new counts, packed starts, scatter
    if (a.num_tiles) { int rc = launch_hash_count_t<uint32_t, true>(a, ent, a.cb_cursor, a.spill); if (rc) return rc; }
    hipLaunchKernelGGL(k_cb_scan, dim3(a.num_filters), dim3(256), 0, (hipStream_t)a.stream, a.plans, a.cb_cursor,
                       a.cb_count, a.cb_start, a.cb_cursor, a.spill);
    CHECK_LAUNCH();
    if (int rc = launch_scatter_t<uint32_t, true>(a, ent, part, a.spill)) return rc;
    if (a.num_cb) {
      hipLaunchKernelGGL(k_old_cb_bounds, dim3((a.num_cb + 255) / 256), dim3(256), 0, (hipStream_t)a.stream, a.plans,
                         a.cb_filter, a.num_cb, a.old32, a.old_tot, a.fp_size, a.lis, a.ob_lo, a.ob_n, a.cb_count);
      CHECK_LAUNCH();
    }
    REC(EV_B_HASH);
    // the sorted layout: starts of the coarse buckets' new + old counts
    hipLaunchKernelGGL(k_cb_scan, dim3(a.num_filters), dim3(256), 0, (hipStream_t)a.stream, a.plans, a.cb_count,
                       a.cb_count, a.cb_outs, a.cb_outs, nullptr);
    CHECK_LAUNCH();
    REC(EV_B_SCAN);
    REC(EV_B_SCATTER);
    if (int rc = launch_sort_t<uint32_t, true, true>(a, ent, part, a.spill)) return rc;
  } else if (a.wide) {
    // incremental add: 64-bit entries; old entries first (decoded by rf_launch_old_decode)
    uint64_t* ent = (uint64_t*)a.ent;
    uint64_t* part = (uint64_t*)a.part;
    if (a.num_old_tiles) {
      hipLaunchKernelGGL(k_old_count, dim3(a.num_old_tiles), dim3(TILE_NT), 0, (hipStream_t)a.stream, a.plans,
                         a.old_tile_filter, a.old_tile_start, a.fp_size, ent, a.cb_count);
      CHECK_LAUNCH();
    }
    if (a.num_tiles) { int rc = launch_hash_count_t<uint64_t>(a, ent, a.cb_count, nullptr); if (rc) return rc; }
    REC(EV_B_HASH);
    hipLaunchKernelGGL(k_cb_scan, dim3(a.num_filters), dim3(256), 0, (hipStream_t)a.stream, a.plans, a.cb_count,
                       a.cb_count, a.cb_start, a.cb_cursor, nullptr);
    CHECK_LAUNCH();
    REC(EV_B_SCAN);
    if (int rc = launch_scatter_t<uint64_t>(a, ent, part, nullptr)) return rc;
    REC(EV_B_SCATTER);
    if (int rc = launch_sort_t<uint64_t>(a, ent, part, nullptr)) return rc;
  } else {
    // fresh build: fused hash + partition into fixed regions (cb_count = fills)
    uint32_t* ent = (uint32_t*)a.ent;
    uint32_t* part = (uint32_t*)a.part;
    if (a.num_tiles) {
#define L(K) hipLaunchKernelGGL((k_hash_scatter<K>), dim3(a.num_tiles), dim3(SCAT_NT), 0, (hipStream_t)a.stream, \
                                a.plans, a.tile_filter, a.tile_start, a.in0, a.offs, a.key_len, a.fp_size, a.seed, \
                                part, a.cb_count, a.spill)
      KIND_SWITCH(a.kind, L);
#undef L
      CHECK_LAUNCH();
    }
    REC(EV_B_HASH);
    // spill fallback (every kernel returns at once unless *spill): exact counts into
    // cb_cursor, scan -> cb_count / cb_start / cb_cursor, scatter from the entry array
    if (a.num_tiles) { int rc = launch_hash_count_t<uint32_t>(a, ent, a.cb_cursor, a.spill); if (rc) return rc; }
    hipLaunchKernelGGL(k_cb_scan, dim3(a.num_filters), dim3(256), 0, (hipStream_t)a.stream, a.plans, a.cb_cursor,
                       a.cb_count, a.cb_start, a.cb_cursor, a.spill);
    CHECK_LAUNCH();
    REC(EV_B_SCAN);
    if (int rc = launch_scatter_t<uint32_t>(a, ent, part, a.spill)) return rc;
    REC(EV_B_SCATTER);
    if (int rc = launch_sort_t<uint32_t>(a, ent, part, a.spill)) return rc;
  }
  hipLaunchKernelGGL(k_layout, dim3(a.num_filters), dim3(LAYOUT_NT), 0, (hipStream_t)a.stream, a.plans, a.idx_cnt,
                     a.idx_start, a.sorted32, a.first_old, a.has_old, a.pplans_mut, a.slots, a.page_first, a.outs, a.lis, a.page_size);
  CHECK_LAUNCH();
  REC(EV_B_LAYOUT);
  hipLaunchKernelGGL(k_assemble, dim3(a.num_page_slots), dim3(ASM_NT), 0, (hipStream_t)a.stream, a.plans, a.pg_filter,
                     a.idx_cnt, a.idx_start, a.sorted32, a.slots, a.page_first, a.outs, a.pages, a.lines,
                     a.pg_noline, a.lis, a.page_size);
  CHECK_LAUNCH();
  if (a.plines_needed)
    if (int rc = launch_plines_list(a)) return rc;
  REC(EV_B_ASSEMBLE);
  return 0;
}

extern "C" int rf_launch_plines(const LaunchArgs* pa) {
  const LaunchArgs& a = *pa;
  if (!a.line_lmax) return 0;  // no filter of the batch has lines
  const size_t lds = 4ull * (256 / WAVE) * (a.line_lmax + 1);
  hipLaunchKernelGGL(k_plines, dim3((a.num_idx + 3) / 4), dim3(256), lds, (hipStream_t)a.stream, a.plans,
                     a.idx_filter, a.slots, a.pages, a.outs, a.lines, a.num_idx, a.line_lmax, a.lis,
                     a.page_size, a.plines_force);
  CHECK_LAUNCH();
  return 0;
}

// the pages K6 listed in a build (k_plines_list)
static int launch_plines_list(const LaunchArgs& a) {
  if (!a.line_lmax || !a.num_page_slots) return 0;
  const size_t lds = 4ull * (256 / WAVE) * (a.line_lmax + 1);
  const uint32_t grid = a.num_page_slots < 1024 ? a.num_page_slots : 1024;
  hipLaunchKernelGGL(k_plines_list, dim3(grid), dim3(256), lds, (hipStream_t)a.stream, a.plans, a.pg_filter,
                     a.page_first, a.slots, a.pages, a.pg_noline, a.lines, a.line_lmax, a.lis, a.page_size);
  CHECK_LAUNCH();
  return 0;
}

extern "C" int rf_launch_old_decode(const LaunchArgs* pa) {
  const LaunchArgs& a = *pa;
  if (a.num_old_idx == 0) return 0;
  hipLaunchKernelGGL(k_old_counts, dim3((a.num_old_idx + 255) / 256), dim3(256), 0, (hipStream_t)a.stream, a.plans,
                     a.old_idx_filter, a.num_old_idx, a.old_cnt);
  CHECK_LAUNCH();
  hipLaunchKernelGGL(k_old_scan, dim3(a.num_filters), dim3(LAYOUT_NT), 0, (hipStream_t)a.stream, a.plans, a.old_cnt,
                     a.old_pos, a.flag32 ? nullptr : (uint64_t*)a.ent, a.old_tot);
  CHECK_LAUNCH();
  const uint32_t waves_per_block = 256 / WAVE;
  hipLaunchKernelGGL(k_old_decode, dim3((a.num_old_idx + waves_per_block - 1) / waves_per_block), dim3(256), 0,
                     (hipStream_t)a.stream, a.plans, a.old_idx_filter, a.num_old_idx, a.old_pos,
                     a.flag32 ? nullptr : (uint64_t*)a.ent, a.flag32 ? a.old32 : nullptr, a.lis, a.fp_size);
  CHECK_LAUNCH();
  return 0;
}

// Element -> filter map of a batch (tiles, coarse buckets, pages, indices): pre[f] = first
// element of filter f (pre[0] = 0, pre[nf] = n); fof[i] = the f with pre[f] <= i < pre[f + 1]
// (filters with no elements are skipped), start[i] = (i - pre[f]) * mul (a tile's first key).
__global__ __launch_bounds__(256) void k_seg_fill(const uint32_t* __restrict__ pre, uint32_t nf, uint32_t n,
                                                  uint32_t* __restrict__ fof, uint32_t* __restrict__ start,
                                                  uint32_t mul) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t lo = 0, hi = nf;  // pre[lo] <= i < pre[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= i) lo = mid; else hi = mid;
  }
  fof[i] = lo;
  if (start) start[i] = (i - pre[lo]) * mul;
}

extern "C" int rf_launch_seg_fill(void* stream, const uint32_t* pre, uint32_t nf, uint32_t n, uint32_t* fof,
                                  uint32_t* start, uint32_t mul) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_seg_fill, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, pre, nf, n, fof, start, mul);
  CHECK_LAUNCH();
  return 0;
}

extern "C" int rf_launch_wave_tab(void* stream, const uint64_t* runs, uint32_t nf, uint64_t n, uint32_t* tab) {
  const uint64_t nw = (n + WAVE - 1) / WAVE;
  if (nw == 0) return 0;
  hipLaunchKernelGGL(k_wave_tab, dim3((uint32_t)((nw + 255) / 256)), dim3(256), 0, (hipStream_t)stream, runs, nf, n, tab);
  CHECK_LAUNCH();
  return 0;
}

extern "C" int rf_launch_probe_floor(const LaunchArgs* pa, int kind, const void* in0, uint64_t n, uint64_t* found) {
  const LaunchArgs& a = *pa;
  if (n == 0) return 0;
  if (!a.wave_tab || (kind != IN_KEYS24 && kind != IN_HASH)) return (int)hipErrorInvalidValue;
  const int nt = probe_nt(kind);
  dim3 g((uint32_t)((n + nt - 1) / nt)), b(nt);
  if (kind == IN_KEYS24)
    hipLaunchKernelGGL((k_probe_floor<IN_KEYS24>), g, b, 0, (hipStream_t)a.stream, a.pplans, a.lines, in0, a.wave_tab, n,
                       found, a.fp_size, a.num_filters);
  else
    hipLaunchKernelGGL((k_probe_floor<IN_HASH>), g, b, 0, (hipStream_t)a.stream, a.pplans, a.lines, in0, a.wave_tab, n,
                       found, a.fp_size, a.num_filters);
  CHECK_LAUNCH();
  return 0;
}

extern "C" int rf_launch_probe(const LaunchArgs* pa, int kind, const void* in0, const uint64_t* offs,
                               uint32_t key_len, const uint32_t* filter_id, uint64_t n, uint64_t* found) {
  const LaunchArgs& a = *pa;
  if (n == 0) return 0;
  const int nt = probe_nt(kind);
  dim3 g((uint32_t)((n + nt - 1) / nt)), b(nt);
  REC(EV_P_START);
#define PK(K) hipLaunchKernelGGL((k_probe<K>), g, b, 0, (hipStream_t)a.stream, a.pplans, a.plans, a.pages, a.slots, a.lines, in0, offs, key_len, filter_id, a.probe_runs, a.wave_tab, n, found, a.fp_size, a.seed, a.lis, a.page_size, a.num_filters)
  // 8 waves/SIMD: the line probe is bound by outstanding random line fetches (latency x
  // concurrency): 8 waves 1.14 ms, 6 waves 1.20, 5 1.27, 4 1.41 at C2 (round-1 occupancy sweep)
  switch (kind) {
    case IN_KEYS24: PK(IN_KEYS24); break;
    case IN_KEYS_W: PK(IN_KEYS_W); break;
    case IN_KEYS_B: PK(IN_KEYS_B); break;
    case IN_VAR: PK(IN_VAR); break;
    case IN_PAIR: PK(IN_PAIR); break;
    default: PK(IN_HASH); break;
  }
#undef PK
  CHECK_LAUNCH();
  REC(EV_P_END);
  return 0;
}
