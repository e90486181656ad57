// rf_device.h -- device-side helpers shared by the routing-filter kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rf {

constexpr int WAVE = 64;

// ---- XXH32 (published xxHash algorithm; the reference's platform_hash32,
//      src/platform_linux/platform_hash.h:23) ----------------------------------------
constexpr uint32_t XP1 = 2654435761U, XP2 = 2246822519U, XP3 = 3266489917U,
                   XP4 = 668265263U, XP5 = 374761393U;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) {
  return __builtin_rotateleft32(x, r);
}
__device__ __forceinline__ uint32_t xround(uint32_t acc, uint32_t in) {
  return rotl32(acc + in * XP2, 13) * XP1;
}
__device__ __forceinline__ uint32_t xavalanche(uint32_t h) {
  h ^= h >> 15; h *= XP2; h ^= h >> 13; h *= XP3; h ^= h >> 16;
  return h;
}

// 24-byte key held as 6 little-endian words (the filter_test / BASELINE key format)
__device__ __forceinline__ uint32_t xxh32_24(const uint32_t w[6], uint32_t seed) {
  uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
  v1 = xround(v1, w[0]); v2 = xround(v2, w[1]); v3 = xround(v3, w[2]); v4 = xround(v4, w[3]);
  uint32_t h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  h += 24u;
  h = rotl32(h + w[4] * XP3, 17) * XP4;
  h = rotl32(h + w[5] * XP3, 17) * XP4;
  return xavalanche(h);
}

// Generic length, 4-byte aligned base: word loads.
__device__ __forceinline__ uint32_t xxh32_words(const uint32_t* p, uint32_t len, uint32_t seed) {
  uint32_t h, i = 0;
  if (len >= 16) {
    uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    uint32_t nstripe = len / 16;
    for (uint32_t s = 0; s < nstripe; s++) {
      v1 = xround(v1, p[4 * s]); v2 = xround(v2, p[4 * s + 1]);
      v3 = xround(v3, p[4 * s + 2]); v4 = xround(v4, p[4 * s + 3]);
    }
    i = nstripe * 16;
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + XP5;
  }
  h += len;
  for (; i + 4 <= len; i += 4) h = rotl32(h + p[i / 4] * XP3, 17) * XP4;
  if (i < len) {
    uint32_t w = p[i / 4];
    for (; i < len; i++) {
      h = rotl32(h + (w & 0xffu) * XP5, 11) * XP1;
      w >>= 8;
    }
  }
  return xavalanche(h);
}

// Arbitrary alignment: gfx950 global loads accept unaligned addresses, so each 16-byte
// stripe is ONE dwordx4 load (memcpy lets the compiler emit it) and every load stays inside
// the key's own bytes.
__device__ __forceinline__ uint32_t pick4u(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return q == 0 ? a : q == 1 ? b : q == 2 ? c : d;
}

__device__ __forceinline__ uint32_t xxh32_unaligned(const uint8_t* p, uint32_t len, uint32_t seed);

// One key per lane with nothing else in flight (probes, k_hash): for keys of 16..128 bytes
// every load of the key is issued before any is used; other lengths take xxh32_unaligned.
// (The partition keeps the stripe loop: it hashes 8 keys per lane at once, and the extra
// registers cost it more than the loop's waits.)
__device__ __forceinline__ uint32_t xxh32_unaligned_prefetch(const uint8_t* p, uint32_t len, uint32_t seed) {
  constexpr uint32_t MS = 8;
  if (len >= 16 && len <= 16 * MS) {
    // Every load of the key is issued before any is used (a stripe loop would wait for
    // each stripe in turn): the full 16-byte stripes, and the key's last 16 bytes, which
    // hold the tail (len % 16 bytes) at their end. All loads stay inside the key.
    const uint32_t ns = len / 16;
    uint4 st[MS];
#pragma unroll
    for (uint32_t s = 0; s < MS; s++)
      if (s < ns) __builtin_memcpy(&st[s], p + 16 * s, 16);
    uint4 tl;
    __builtin_memcpy(&tl, p + len - 16, 16);
    uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
#pragma unroll
    for (uint32_t s = 0; s < MS; s++)
      if (s < ns) {
        v1 = xround(v1, st[s].x); v2 = xround(v2, st[s].y); v3 = xround(v3, st[s].z); v4 = xround(v4, st[s].w);
      }
    uint32_t h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18) + len;
    const uint32_t r = len - 16 * ns;  // tail bytes, at offsets [16 - r, 16) of tl
    // 4 bytes of tl from byte offset o (o <= 12)
    auto word_at = [&](uint32_t o) -> uint32_t {
      const uint32_t q = o >> 2, sh = (o & 3) * 8;
      const uint32_t lo = pick4u(q, tl.x, tl.y, tl.z, tl.w), hi = pick4u(q, tl.y, tl.z, tl.w, 0u);
      return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
    };
    uint32_t o = 16 - r;
#pragma unroll
    for (uint32_t k = 0; k < 3; k++)
      if (o + 4 <= 16) {
        h = rotl32(h + word_at(o) * XP3, 17) * XP4;
        o += 4;
      }
#pragma unroll
    for (uint32_t k = 0; k < 3; k++)
      if (o < 16) {
        const uint32_t q = o >> 2, sh = (o & 3) * 8;
        h = rotl32(h + ((pick4u(q, tl.x, tl.y, tl.z, tl.w) >> sh) & 0xffu) * XP5, 11) * XP1;
        o++;
      }
    return xavalanche(h);
  }
  return xxh32_unaligned(p, len, seed);
}

__device__ __forceinline__ uint32_t xxh32_unaligned(const uint8_t* p, uint32_t len, uint32_t seed) {
  uint32_t h, i = 0;
  if (len >= 16) {
    uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    for (; i + 16 <= len; i += 16) {
      uint4 w;
      __builtin_memcpy(&w, p + i, 16);
      v1 = xround(v1, w.x); v2 = xround(v2, w.y); v3 = xround(v3, w.z); v4 = xround(v4, w.w);
    }
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + XP5;
  }
  h += len;
  for (; i + 4 <= len; i += 4) {
    uint32_t w;
    __builtin_memcpy(&w, p + i, 4);
    h = rotl32(h + w * XP3, 17) * XP4;
  }
  for (; i < len; i++) h = rotl32(h + (uint32_t)p[i] * XP5, 11) * XP1;
  return xavalanche(h);
}

// XXH32 of `len` bytes at byte offset `boff` of an LDS word array (any alignment): each
// little-endian word is funnel-shifted out of two aligned LDS words (v_alignbyte_b32).
// Reads up to two words past the key's last byte: the caller pads the array.
__device__ __forceinline__ uint32_t xxh32_lds(const uint32_t* sw, uint32_t boff, uint32_t len, uint32_t seed) {
  const uint32_t* p = sw + (boff >> 2);
  const uint32_t sh = boff & 3;
  auto word = [&](uint32_t i) -> uint32_t { return __builtin_amdgcn_alignbyte(p[i + 1], p[i], sh); };
  uint32_t h, i = 0;
  if (len >= 16) {
    uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint32_t ns = len >> 4;
    for (uint32_t s = 0; s < ns; s++) {
      v1 = xround(v1, word(4 * s)); v2 = xround(v2, word(4 * s + 1));
      v3 = xround(v3, word(4 * s + 2)); v4 = xround(v4, word(4 * s + 3));
    }
    i = 4 * ns;
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + XP5;
  }
  h += len;
  const uint32_t nw = len >> 2;
  for (; i < nw; i++) h = rotl32(h + word(i) * XP3, 17) * XP4;
  if (len & 3) {
    uint32_t w = word(nw);
    for (uint32_t b = 0; b < (len & 3); b++) {
      h = rotl32(h + (w & 0xffu) * XP5, 11) * XP1;
      w >>= 8;
    }
  }
  return xavalanche(h);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t lane) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), lane) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, lane);
}
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Variable-length keys, one per lane, hashed from a wave-private LDS window of CAP bytes
// (CAP a multiple of 16; `sw` holds CAP/4 + 2 words, 16-byte aligned). A wave's keys are
// contiguous in the key buffer (offsets increase with the key number), so the window is
// filled by coalesced 16-byte loads of the whole byte range -- where one unaligned load
// per lane per stripe touches up to 64 cache lines per instruction -- and each lane then
// reads its key from LDS. The window is 16-byte aligned in the address space, so its
// loads never leave the 4 KiB pages that hold the keys. [*win0, *win1) is the staged
// address range, kept across calls for keys that continue the same byte stream; a key
// longer than CAP - 15 bytes is hashed straight from global memory.
template <uint32_t CAP, bool NT>
__device__ __forceinline__ uint32_t wave_hash_var(const uint8_t* keys, uint64_t o0, uint64_t o1, bool valid,
                                                  uint32_t* sw, uint32_t seed, uint64_t* win0,
                                                  uint64_t* win1) {
  static_assert(CAP % 16 == 0, "window is whole 16-byte chunks");
  constexpr uint32_t IT = (CAP / 16 + WAVE - 1) / WAVE;
  typedef unsigned int v4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t kb = (uint64_t)(uintptr_t)keys;
  const uint64_t vm = __ballot(valid);
  if (!vm) return 0;
  const uint64_t aend = (kb + readlane64(o1, 63 - __builtin_clzll(vm)) + 15) & ~15ull;
  uint32_t h = 0;
  bool pending = valid;
  for (;;) {
    if (pending && kb + o0 >= *win0 && kb + o1 <= *win1) {
      h = xxh32_lds(sw, (uint32_t)(kb + o0 - *win0), (uint32_t)(o1 - o0), seed);
      pending = false;
    }
    const uint64_t m = __ballot(pending);
    if (!m) break;
    const uint32_t first = __builtin_ctzll(m);
    const uint64_t a0 = (kb + readlane64(o0, first)) & ~15ull;
    const uint64_t a1 = min(aend, a0 + CAP);
    if (lane == first && kb + o1 > a1) {  // longer than the window: straight from HBM
      h = xxh32_unaligned(keys + o0, (uint32_t)(o1 - o0), seed);
      pending = false;
    }
    wave_sync_lds();  // every lane's reads of the old window are done
    const uint32_t n16 = (uint32_t)(a1 - a0) / 16;
    const v4* src = reinterpret_cast<const v4*>((uintptr_t)a0);
    // LDS-DMA (global_load_lds_dwordx4): every chunk of the window in flight at once with
    // no VGPR destination; instruction `it` fills bytes [1 KiB * it, +1 KiB) lane-linearly
#pragma unroll
    for (uint32_t it = 0; it < IT; it++) {
      const uint32_t j = lane + it * WAVE;
      if (j < n16)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + j),
                                         (__attribute__((address_space(3))) void*)(sw + it * WAVE * 4), 16, 0,
                                         NT ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync_lds();
    *win0 = a0;
    *win1 = a1;
  }
  return h;
}

// ---- scans ------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    uint32_t y = __shfl_up(x, d, WAVE);
    if (lane >= d) x += y;
  }
  return x;
}

// Block-wide exclusive scan. s_tmp needs NT/64 + 1 words. Returns the exclusive prefix,
// writes the block total to *total. Contains barriers: call from every thread.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_tmp, uint32_t* total) {
  constexpr int NW = NT / WAVE;
  const int w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  uint32_t inc = wave_incl_scan(x);
  if (lane == WAVE - 1) s_tmp[w] = inc;
  __syncthreads();
  if (threadIdx.x < WAVE) {
    uint32_t v = (int)threadIdx.x < NW ? s_tmp[threadIdx.x] : 0u;
    uint32_t vi = wave_incl_scan(v);
    if ((int)threadIdx.x < NW) s_tmp[threadIdx.x] = vi - v;
    if ((int)threadIdx.x == NW - 1) s_tmp[NW] = vi;
  }
  __syncthreads();
  uint32_t r = s_tmp[w] + inc - x;
  *total = s_tmp[NW];
  __syncthreads();
  return r;
}

// In-place exclusive scan of x[k] over the elements j = k * NT + threadIdx.x (k-major
// order), so the loads and stores around it are lane-consecutive (coalesced, no LDS bank
// conflicts). s_w: PER * NT/64 + 1 words. Contains barriers: call from every thread.
template <int NT, int PER>
__device__ __forceinline__ void block_excl_scan_kmajor(uint32_t (&x)[PER], uint32_t* s_w, uint32_t* total) {
  constexpr int NW = NT / WAVE, M = PER * NW, Q = (M + WAVE - 1) / WAVE;
  const int w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t inc = wave_incl_scan(x[k]);
    if (lane == WAVE - 1) s_w[k * NW + w] = inc;
    x[k] = inc - x[k];
  }
  __syncthreads();
  if (threadIdx.x < WAVE) {  // one wave scans the M wave totals in (k, wave) order
    uint32_t v[Q], sum = 0;
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int i = threadIdx.x * Q + q;
      v[q] = i < M ? s_w[i] : 0u;
      sum += v[q];
    }
    uint32_t e = wave_incl_scan(sum) - sum;
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int i = threadIdx.x * Q + q;
      if (i < M) s_w[i] = e;
      e += v[q];
    }
    if (threadIdx.x == WAVE - 1) s_w[M] = e;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; k++) x[k] += s_w[k * NW + w];
  *total = s_w[M];
  __syncthreads();
}

// ---- unaligned little-endian reads from filter page bytes (4-byte aligned buffer) -------
__device__ __forceinline__ uint64_t ld_u64_unaligned(const uint8_t* base, uint64_t byte_off) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base) + (byte_off >> 2);
  uint32_t sh = (uint32_t)(byte_off & 3) * 8;
  uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  if (sh == 0) return lo;
  uint64_t hi = w[2];
  return (lo >> sh) | (hi << (64 - sh));
}
__device__ __forceinline__ uint32_t ld_bits(const uint8_t* base, uint64_t bitpos, uint32_t nbits) {
  if (nbits == 0) return 0;
  uint64_t v = ld_u64_unaligned(base, bitpos >> 3) >> (bitpos & 7);
  return (uint32_t)(v & ((nbits >= 32) ? 0xffffffffull : ((1ull << nbits) - 1)));
}

// position of the k-th (0-based) set bit of x (requires popcount(x) > k)
__device__ __forceinline__ uint32_t select64(uint64_t x, uint32_t k) {
  for (uint32_t i = 0; i < k; i++) x &= x - 1;
  return (uint32_t)__builtin_ctzll(x);
}

}  // namespace rf
