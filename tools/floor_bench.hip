// Probe-floor variants (diagnostic tool, not product code).
//
// k_probe_floor (rf_kernels.hip) is the probe's memory floor for ONE access shape: 24-B keys
// staged in LDS by LDS-DMA, one 64-B line per probe gathered quad-cooperatively into LDS, one
// coalesced 8-B store. This tool times variants of that shape on the same grid (1,024-thread
// workgroups, XCD-chunked, probes grouped by filter, each filter's probes over its own table):
//   LW    line bytes gathered per probe: 0 (no line), 16, 32, 64
//   GM    0 = group LDS-DMA (LW/16 lanes per line, lines land in LDS; the shipped form at 64 B)
//         1 = group register gather (lane q of a group of LW/16 loads piece q of each of the
//             group's lines; the pieces are exchanged inside the group by DPP, so every lane
//             ends with its own line in registers: no LDS for lines)
//   ILP   tiles of 64 probes per wave, issued together (keys of all tiles, then all lines)
//   KM    0 = keys staged by LDS-DMA (1,536 B per tile), 1 = keys straight into registers
//         (three 8-B loads per lane), 2 = 4-B hashes in instead of keys
//   HS    0 = multiply-xorshift (as k_probe_floor), 1 = XXH32 of the 24-B key (as k_probe)
// Tables: F filters of T bytes each, n / F probes per filter in contiguous runs (C2: 8 x 8.4 MB,
// 8M probes each; C3: 256 x 2 MB, 2^20 each). Time = HIP events around 10 launches.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/floor_bench.hip -o tools/floor_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int WAVE = 64;
constexpr int NT = 1024;
constexpr uint32_t KSTRIDE = 1040;  // 16-B skew per gather instruction (as FAST_KSTRIDE)

__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t nb) {
  const uint32_t q = nb / 8, r = nb % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return __builtin_rotateleft32(x, r); }
__device__ __forceinline__ uint32_t xxh32_24(const uint32_t w[6], uint32_t seed) {
  constexpr uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U;
  auto rd = [&](uint32_t a, uint32_t in) { return rotl(a + in * P2, 13) * P1; };
  uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
  v1 = rd(v1, w[0]); v2 = rd(v2, w[1]); v3 = rd(v3, w[2]); v4 = rd(v4, w[3]);
  uint32_t h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18) + 24u;
  h = rotl(h + w[4] * P3, 17) * P4;
  h = rotl(h + w[5] * P3, 17) * P4;
  h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
  return h;
}
template <int HS>
__device__ __forceinline__ uint32_t hash6(const uint32_t w[6]) {
  if constexpr (HS == 1) return xxh32_24(w, 42);
  uint32_t h = (w[0] ^ w[1] ^ w[2] ^ w[3] ^ w[4] ^ w[5]) * 0x9e3779b1u;
  h ^= h >> 15;
  return h * 0x85ebca77u;
}

// quad_perm control word: lane q of each quad reads lane p[q]
constexpr int qp(int a, int b, int c, int d) { return a | b << 2 | c << 4 | d << 6; }

// DPP broadcasts with the control word picked by a (compile-time-unrolled) index: each case
// is a literal, as the builtin requires
template <int G>
__device__ __forceinline__ uint32_t bcast(uint32_t x, int k) {  // lanes G g + q <- lane G g + k
  if constexpr (G == 4) {
    switch (k) {
      case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x00, 0xf, 0xf, false);
      case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x55, 0xf, 0xf, false);
      case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xaa, 0xf, 0xf, false);
      default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xff, 0xf, 0xf, false);
    }
  } else if constexpr (G == 2) {
    return k == 0 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)x, qp(0, 0, 2, 2), 0xf, 0xf, false)
                  : (uint32_t)__builtin_amdgcn_mov_dpp((int)x, qp(1, 1, 3, 3), 0xf, 0xf, false);
  } else if constexpr (G == 8) {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane & ~7u) + k) << 2), (int)x);
  }
  return x;
}
template <int G>
__device__ __forceinline__ uint32_t rotq(uint32_t x, int d) {  // lane q <- lane (q + d) % G of its group
  if constexpr (G == 4) {
    switch (d) {
      case 0: return x;
      case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, qp(1, 2, 3, 0), 0xf, 0xf, false);
      case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, qp(2, 3, 0, 1), 0xf, 0xf, false);
      default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, qp(3, 0, 1, 2), 0xf, 0xf, false);
    }
  } else if constexpr (G == 2) {
    return d ? (uint32_t)__builtin_amdgcn_mov_dpp((int)x, qp(1, 0, 3, 2), 0xf, 0xf, false) : x;
  }
  return x;
}

template <int LW, int GM, int ILP, int KM, int HS>
__global__ __launch_bounds__(NT) void k_floor(const uint8_t* __restrict__ keys, const uint8_t* __restrict__ table,
                                              uint64_t tbytes, uint64_t ppf, uint64_t n,
                                              uint64_t* __restrict__ out) {
  constexpr int G = LW / 16 > 0 ? LW / 16 : 1;  // lanes per line
  constexpr int KBUF = (KM == 0 || KM == 3) ? 96 : 0;         // v4u per tile for keys
  constexpr int LBUF = (GM == 0 && LW > 0) ? (int)((KSTRIDE * (G - 1) + 1024) / 16 + 1) : 0;
  // the lines land over the keys' staging (read into registers before the lines are requested), as
  // in k_probe's fast path
  constexpr int PER = (KBUF > LBUF ? KBUF : LBUF) > 0 ? (KBUF > LBUF ? KBUF : LBUF) : 1;
  __shared__ v4u s[NT / WAVE][ILP][PER];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x) / WAVE;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t wf = ((uint64_t)xcd_chunk(blockIdx.x, gridDim.x) * (NT / WAVE) + wv) * (WAVE * ILP);
  if (wf >= n) return;
  const uint64_t fid = wf / ppf;  // wave-uniform
  const uint8_t* fb = table + fid * tbytes;
  const uint32_t nlines = (uint32_t)(tbytes / (LW > 0 ? LW : 1));
  uint32_t h[ILP];
  // 1. keys (or hashes) of every tile
  if constexpr (KM == 3) {
    // diagnostic: the same key traffic (LDS-DMA into the tile's buffer), but the line addresses
    // come from the probe index, so the gathers are issued without waiting for the keys (the
    // buffer's bytes are garbage; only the traffic and the timing matter)
#pragma unroll
    for (int t = 0; t < ILP; t++) {
      const uint8_t* kb = keys + (wf + t * WAVE) * 24;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + lane * 16),
                                       (__attribute__((address_space(3))) void*)&s[wv][t][0], 16, 0, 2);
      if (lane < 32)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)&s[wv][t][WAVE], 16, 0, 2);
      const uint32_t w[6] = {(uint32_t)(wf + t * WAVE + lane), 0x1234567u, 0, 0, 0, 0};
      h[t] = hash6<0>(w);
    }
  } else if constexpr (KM == 0) {
#pragma unroll
    for (int t = 0; t < ILP; t++) {
      const uint8_t* kb = keys + (wf + t * WAVE) * 24;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + lane * 16),
                                       (__attribute__((address_space(3))) void*)&s[wv][t][0], 16, 0, 2);
      if (lane < 32)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)&s[wv][t][WAVE], 16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync_lds();
#pragma unroll
    for (int t = 0; t < ILP; t++) {
      const uint2* k2 = reinterpret_cast<const uint2*>(&s[wv][t][0]) + 3 * lane;
      const uint2 a = k2[0], b = k2[1], c = k2[2];
      const uint32_t w[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
      h[t] = hash6<HS>(w);
    }
  } else if constexpr (KM == 1) {
    uint2 kv[ILP][3];
#pragma unroll
    for (int t = 0; t < ILP; t++) {
      const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + (wf + t * WAVE + lane) * 24);
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const uint64_t v = __builtin_nontemporal_load(kp + j);
        kv[t][j] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
      }
    }
#pragma unroll
    for (int t = 0; t < ILP; t++) {
      const uint32_t w[6] = {kv[t][0].x, kv[t][0].y, kv[t][1].x, kv[t][1].y, kv[t][2].x, kv[t][2].y};
      h[t] = hash6<HS>(w);
    }
  } else {
#pragma unroll
    for (int t = 0; t < ILP; t++)
      h[t] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(keys) + wf + t * WAVE + lane);
  }
  uint32_t acc[ILP];
#pragma unroll
  for (int t = 0; t < ILP; t++) acc[t] = h[t];
  if constexpr (LW > 0) {
    const uint32_t q = lane & (G - 1);
    uint32_t lo[ILP];
#pragma unroll
    for (int t = 0; t < ILP; t++) lo[t] = __umulhi(h[t], nlines) * LW;  // byte offset of the line
    if constexpr (GM == 0) {
      // group LDS-DMA: instruction k lands the lines of probes G g + k (lane G g + q: piece (q + k) % G)
#pragma unroll
      for (int t = 0; t < ILP; t++) {
        uint8_t* sb = reinterpret_cast<uint8_t*>(&s[wv][t][0]);
#pragma unroll
        for (int k = 0; k < G; k++) {
          const uint32_t lk = bcast<G>(lo[t], k);
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(fb + lk + q * 16),
                                           (__attribute__((address_space(3))) void*)(sb + k * KSTRIDE), 16, 0, 0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wave_sync_lds();
#pragma unroll
      for (int t = 0; t < ILP; t++) {
        const uint8_t* sb = reinterpret_cast<const uint8_t*>(&s[wv][t][0]);
        // probe p = lane: its line's pieces are at KiB (p % G), slot p / G
#pragma unroll
        for (int j = 0; j < G; j++) {
          const v4u E = *reinterpret_cast<const v4u*>(sb + (lane % G) * KSTRIDE + (lane / G) * LW + j * 16);
          acc[t] ^= E[0] ^ E[1] ^ E[2] ^ E[3];
        }
      }
    } else {
      // group register gather: instruction k loads, in lane G g + q, piece q of probe G g + k's line
      v4u R[ILP][G];
#pragma unroll
      for (int t = 0; t < ILP; t++) {
#pragma unroll
        for (int k = 0; k < G; k++) {
          const uint32_t lk = bcast<G>(lo[t], k);
          R[t][k] = *reinterpret_cast<const v4u*>(fb + lk + q * 16);  // default policy, as the LDS-DMA gather
        }
      }
#pragma unroll
      for (int t = 0; t < ILP; t++) {
        // exchange: lane q needs piece d' of its own line = R[k = q] of lane d' of its group
        // (sender q' sends R[receiver's q]); for shift d the sender q' sends R[(q' - d) % G]
        v4u mine[G];
#pragma unroll
        for (int d = 0; d < G; d++) {
          v4u x;
#pragma unroll
          for (int c = 0; c < 4; c++) {
            uint32_t v = R[t][0][c];
#pragma unroll
            for (int k = 1; k < G; k++) v = ((q - d) & (G - 1)) == (uint32_t)k ? R[t][k][c] : v;
            x[c] = rotq<G>(v, d);  // receiver q reads sender (q + d) % G
          }
          mine[d] = x;
        }
#pragma unroll
        for (int d = 0; d < G; d++) acc[t] ^= mine[d][0] ^ mine[d][1] ^ mine[d][2] ^ mine[d][3];
      }
    }
  }
#pragma unroll
  for (int t = 0; t < ILP; t++) __builtin_nontemporal_store((uint64_t)acc[t], out + wf + t * WAVE + lane);
}

// Table-part split (round 6, priced in DESIGN §12 first): the probes of each filter gathered in
// NPART passes, pass p gathering only the lines of the p-th part of the table (top bits of the
// hash), so each XCD's L2 holds 1/NPART of its table at a time. Pass 0 stages and hashes the
// keys and writes the 4-B hashes; passes p > 0 read them back. Lanes outside the pass's part
// issue no gather and store nothing (masked 8-B stores).
template <int NPART>
__global__ __launch_bounds__(NT) void k_split(const uint8_t* __restrict__ keys, const uint8_t* __restrict__ table,
                                              uint64_t tbytes, uint64_t ppf, uint64_t n, uint64_t* __restrict__ out,
                                              uint32_t* __restrict__ hbuf, uint32_t pass) {
  __shared__ v4u s[NT / WAVE][(KSTRIDE * 3 + 1024) / 16 + 1];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x) / WAVE;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t wf = ((uint64_t)xcd_chunk(blockIdx.x, gridDim.x) * (NT / WAVE) + wv) * WAVE;
  if (wf >= n) return;
  const uint8_t* fb = table + (wf / ppf) * tbytes;
  const uint32_t nlines = (uint32_t)(tbytes / 64);
  uint32_t h;
  if (pass == 0) {
    const uint8_t* kb = keys + wf * 24;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + lane * 16),
                                     (__attribute__((address_space(3))) void*)&s[wv][0], 16, 0, 2);
    if (lane < 32)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(kb + 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)&s[wv][WAVE], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync_lds();
    const uint2* k2 = reinterpret_cast<const uint2*>(&s[wv][0]) + 3 * lane;
    const uint2 a = k2[0], b = k2[1], c = k2[2];
    const uint32_t w[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
    h = hash6<0>(w);
    if (NPART > 1) __builtin_nontemporal_store(h, hbuf + wf + lane);
    wave_sync_lds();  // every lane's key read before the lines land over them
  } else {
    h = __builtin_nontemporal_load(hbuf + wf + lane);
  }
  const uint32_t lo = __umulhi(h, nlines) * 64, q = lane & 3;
  const uint32_t act = (NPART == 1 || __umulhi(h, NPART) == pass) ? 1u : 0u;
  uint8_t* sb = reinterpret_cast<uint8_t*>(&s[wv][0]);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t lk = bcast<4>(lo, k), ak = bcast<4>(act, k);
    if (ak)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(fb + lk + q * 16),
                                       (__attribute__((address_space(3))) void*)(sb + k * KSTRIDE), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync_lds();
  if (act) {
    const v4u E = *reinterpret_cast<const v4u*>(sb + (lane & 3) * KSTRIDE + (lane >> 2) * 64);
    __builtin_nontemporal_store((uint64_t)(h ^ E[0] ^ E[1] ^ E[2] ^ E[3]), out + wf + lane);
  }
}

__global__ void k_fill(uint32_t* p, uint64_t nw, uint64_t salt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + salt) * 0x9e3779b97f4a7c15ull;
    x ^= x >> 31; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 29;
    p[i] = (uint32_t)x;
  }
}

struct Ctx { const uint8_t* keys; const uint8_t* table; uint64_t T, ppf, n; uint64_t* out; };

template <int LW, int GM, int ILP, int KM, int HS>
float run(const Ctx& c, int reps) {
  const uint64_t per_blk = (uint64_t)NT * ILP;
  dim3 g((unsigned)((c.n + per_blk - 1) / per_blk));
  auto L = [&]() { hipLaunchKernelGGL((k_floor<LW, GM, ILP, KM, HS>), g, dim3(NT), 0, 0, c.keys, c.table, c.T, c.ppf, c.n, c.out); };
  L(); L();
  CK(hipGetLastError());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; r++) L();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return ms / reps;
}

template <int NPART>
float run_split(const Ctx& c, uint32_t* hbuf, int reps) {
  dim3 g((unsigned)((c.n + NT - 1) / NT));
  auto L = [&]() {
    for (uint32_t p = 0; p < NPART; p++)
      hipLaunchKernelGGL((k_split<NPART>), g, dim3(NT), 0, 0, c.keys, c.table, c.T, c.ppf, c.n, c.out, hbuf, p);
  };
  L(); L();
  CK(hipGetLastError());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; r++) L();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  // usage: floor_bench <probes> <filters> <table bytes per filter> [label]
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (64ull << 20);
  const uint64_t F = argc > 2 ? strtoull(argv[2], 0, 0) : 8;
  // each filter's table starts on a 256-B boundary (a misaligned 64-B line spans two cache lines)
  const uint64_t T = (argc > 3 ? strtoull(argv[3], 0, 0) : 8388608) & ~255ull;
  const char* label = argc > 4 ? argv[4] : "";
  const int reps = 10;
  uint8_t *keys, *table; uint64_t* out;
  CK(hipMalloc(&keys, n * 24 + 4096));
  CK(hipMalloc(&out, n * 8));
  CK(hipMalloc(&table, F * T + 4096));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)keys, n * 6, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)table, F * T / 4, 7ull);
  CK(hipDeviceSynchronize());
  Ctx c{keys, table, T, n / F, n, out};
  const double alg = n * 32.0 + F * T / 1.5;  // keys + results + the image (table = 1.5x image)
  printf("# %s: %llu probes, %llu filters x %.2f MB tables (%.0f MB total)\n", label, (unsigned long long)n,
         (unsigned long long)F, T / 1e6, F * T / 1e6);
  auto P = [&](const char* name, float ms) {
    printf("%-44s %8.4f ms  %6.1f ps/probe  alg-frac %.3f\n", name, ms, ms * 1e9 / n, alg / (ms * 1e-3) / 8e12);
    fflush(stdout);
  };
  const int set = getenv("FB_SET") ? atoi(getenv("FB_SET")) : 0;
  if (set == 2) {  // table-part split: NPART passes, each gathering one part of every table
    uint32_t* hbuf;
    CK(hipMalloc(&hbuf, n * 4));
    P("LW64 quad LDS-DMA (k_probe_floor)", run<64, 0, 1, 0, 0>(c, reps));
    P("split 1 part (same kernel, no hash buffer)", run_split<1>(c, hbuf, reps));
    P("split 2 parts", run_split<2>(c, hbuf, reps));
    P("split 3 parts", run_split<3>(c, hbuf, reps));
    P("split 4 parts", run_split<4>(c, hbuf, reps));
    P("LW64 quad LDS-DMA, gathers not waiting on keys", run<64, 0, 1, 3, 0>(c, reps));
    P("LW64 quad LDS-DMA, hashes in", run<64, 0, 1, 2, 0>(c, reps));
    P("LW0  keys LDS-DMA, no line", run<0, 0, 1, 0, 0>(c, reps));
    P("LW0  hashes in, no line", run<0, 0, 1, 2, 0>(c, reps));
    CK(hipFree(hbuf));
    return 0;
  }
  if (set == 1) {  // round-6 second pass: line width, ILP within the LDS budget, 128-B lines
    P("LW0  keys LDS-DMA, no line", run<0, 0, 1, 0, 0>(c, reps));
    P("LW64 quad LDS-DMA (k_probe_floor)", run<64, 0, 1, 0, 0>(c, reps));
    P("LW128 oct LDS-DMA", run<128, 0, 1, 0, 0>(c, reps));
    P("LW32 pair LDS-DMA", run<32, 0, 1, 0, 0>(c, reps));
    P("LW32 pair LDS-DMA ILP2", run<32, 0, 2, 0, 0>(c, reps));
    P("LW16 lane LDS-DMA ILP2", run<16, 0, 2, 0, 0>(c, reps));
    P("LW64 quad reg", run<64, 1, 1, 0, 0>(c, reps));
    P("LW32 pair reg", run<32, 1, 1, 0, 0>(c, reps));
    P("LW32 pair reg ILP2", run<32, 1, 2, 0, 0>(c, reps));
    P("LW16 lane reg ILP2", run<16, 1, 2, 0, 0>(c, reps));
    P("LW16 lane reg ILP4", run<16, 1, 4, 0, 0>(c, reps));
    return 0;
  }
  P("LW0  keys LDS-DMA, no line", run<0, 0, 1, 0, 0>(c, reps));
  P("LW0  keys LDS-DMA, no line, XXH32", run<0, 0, 1, 0, 1>(c, reps));
  P("LW0  keys reg, no line", run<0, 0, 1, 1, 0>(c, reps));
  P("LW0  hashes in, no line", run<0, 0, 1, 2, 0>(c, reps));
  P("LW64 quad LDS-DMA (k_probe_floor)", run<64, 0, 1, 0, 0>(c, reps));
  P("LW64 quad LDS-DMA, XXH32", run<64, 0, 1, 0, 1>(c, reps));
  P("LW64 quad reg", run<64, 1, 1, 0, 0>(c, reps));
  P("LW32 pair LDS-DMA", run<32, 0, 1, 0, 0>(c, reps));
  P("LW32 pair reg", run<32, 1, 1, 0, 0>(c, reps));
  P("LW32 pair reg, XXH32", run<32, 1, 1, 0, 1>(c, reps));
  P("LW16 lane reg", run<16, 1, 1, 0, 0>(c, reps));
  P("LW16 lane LDS-DMA", run<16, 0, 1, 0, 0>(c, reps));
  P("LW64 quad reg ILP2", run<64, 1, 2, 0, 0>(c, reps));
  P("LW32 pair reg ILP2", run<32, 1, 2, 0, 0>(c, reps));
  P("LW32 pair reg ILP2, XXH32", run<32, 1, 2, 0, 1>(c, reps));
  P("LW16 lane reg ILP2", run<16, 1, 2, 0, 0>(c, reps));
  P("LW64 quad reg, keys reg", run<64, 1, 1, 1, 0>(c, reps));
  P("LW32 pair reg, keys reg", run<32, 1, 1, 1, 0>(c, reps));
  P("LW32 pair reg, keys reg ILP2", run<32, 1, 2, 1, 0>(c, reps));
  P("LW32 pair reg, keys reg ILP4", run<32, 1, 4, 1, 0>(c, reps));
  P("LW16 lane reg, keys reg ILP2", run<16, 1, 2, 1, 0>(c, reps));
  P("LW64 quad LDS-DMA, hashes in", run<64, 0, 1, 2, 0>(c, reps));
  P("LW32 pair reg, hashes in", run<32, 1, 1, 2, 0>(c, reps));
  P("LW32 pair reg, hashes in ILP2", run<32, 1, 2, 2, 0>(c, reps));
  return 0;
}
