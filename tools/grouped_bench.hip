// Microbenchmark (diagnostic tool, not product code): SURVEY §7's grouped probe against the
// direct probe, at C2's shape (64M probes of 24-B keys over 8 filters whose 64-B line tables
// are 8.4 MB each, probes grouped by filter as bench.py issues them) and C3's (256M probes over
// 256 filters of 1M keys, 2.1 MB of lines each, run as 4 launches of 64M).
//   direct : per probe, read its key, derive its line, gather the 64-B line (quad-cooperative,
//            as k_probe's fast path), write one 8-B result in probe order (coalesced).
//   grouped: pass A partitions the probes by line range (RANGE_LINES lines = 64 KiB, LDS-sized)
//            with a fused count + reserve + scatter of 8-B (probe index, line, hash bits)
//            records into fixed-capacity regions; pass B gives each range one workgroup that
//            stages its 64 KiB of lines in LDS once and answers the range's probes from LDS,
//            writing each result to its probe's slot (a scattered 8-B store: results must come
//            back in probe order). "B, results in range order" writes them coalesced instead
//            (what B would cost if the caller could take results permuted: a lower bound).
// The arithmetic on the line is a stand-in (XOR of 16 B) in both: this measures the memory
// system, like k_probe_floor. Times from HIP events, median of 5 after 2 warm-ups.
// build: hipcc --offload-arch=gfx950 -O3 tools/grouped_bench.hip -o tools/grouped_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr uint32_t RANGE_LINES = 1024;   // 64 KiB of lines per range (LDS)
constexpr uint32_t TILE = 16384;         // probes per partition workgroup
constexpr uint32_t PNT = 512;            // partition threads
constexpr uint32_t MAX_RANGES = 2048;

__device__ __forceinline__ uint32_t mix3(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t x = a ^ (b * 0x9e3779b97f4a7c15ull) ^ (c >> 7) ^ (c << 29);
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33;
  return (uint32_t)x;
}

// the probe's line: filter f's table holds lpf lines (a power of two)
__device__ __forceinline__ uint32_t line_of(const uint64_t* keys, uint64_t i, uint32_t f, uint32_t lg_lpf, uint32_t* hbits) {
  const uint64_t* k = keys + 3 * i;
  const uint32_t h = mix3(__builtin_nontemporal_load(k), __builtin_nontemporal_load(k + 1), __builtin_nontemporal_load(k + 2));
  *hbits = h;
  return (f << lg_lpf) | (h >> (32 - lg_lpf));
}

// direct: one lane per probe, quad-cooperative 64-B line gather through LDS (k_probe's fast path)
__global__ __launch_bounds__(1024) void k_direct(const uint64_t* __restrict__ keys, const uint4* __restrict__ lines,
                                                 uint64_t n, uint64_t per_f, uint32_t lg_lpf,
                                                 uint64_t* __restrict__ out) {
  __shared__ uint4 s_l[1024 / 64][4 * 64 + 4];
  const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x / 64;
  uint32_t hb = 0, ln = 0;
  if (i < n) ln = line_of(keys, i, (uint32_t)(i / per_f), lg_lpf, &hb);
  // quad q of the wave fetches line of probe 4g + k in instruction k: lane L loads quarter L & 3
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t lk = __shfl(ln, (lane & ~3u) + k, 64);
    s_l[w][k * 64 + lane] = lines[(uint64_t)lk * 4 + (lane & 3)];
  }
  __syncthreads();
  const uint4 v = s_l[w][(lane & 3) * 64 + (lane & ~3u) + ((lane + 1) & 3)];
  if (i < n) __builtin_nontemporal_store((uint64_t)(v.x ^ v.y ^ v.z ^ v.w ^ hb), out + i);
}

// pass A: per tile, LDS histogram of ranges, one atomic per (tile, range) to reserve space in
// the range's fixed region, scatter of 8-B records (probe index << 32 | line-in-range << 22 | hash bits)
__global__ __launch_bounds__(PNT) void k_partition(const uint64_t* __restrict__ keys, uint64_t n, uint64_t per_f,
                                                   uint32_t lg_lpf, uint32_t nranges, uint32_t region,
                                                   uint32_t* __restrict__ fill, uint64_t* __restrict__ recs) {
  __shared__ uint32_t s_cnt[MAX_RANGES];
  __shared__ uint32_t s_base[MAX_RANGES];
  constexpr int PER = TILE / PNT;
  for (uint32_t r = threadIdx.x; r < nranges; r += PNT) s_cnt[r] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
  uint32_t ln[PER], hb[PER], rk[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint64_t i = t0 + k * PNT + threadIdx.x;
    if (i < n) {
      ln[k] = line_of(keys, i, (uint32_t)(i / per_f), lg_lpf, &hb[k]);
      rk[k] = atomicAdd(&s_cnt[ln[k] / RANGE_LINES], 1u);
    }
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < nranges; r += PNT)
    s_base[r] = s_cnt[r] ? atomicAdd(&fill[r], s_cnt[r]) : 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint64_t i = t0 + k * PNT + threadIdx.x;
    if (i < n) {
      const uint32_t r = ln[k] / RANGE_LINES, slot = s_base[r] + rk[k];
      if (slot < region)
        recs[(uint64_t)r * region + slot] = (i << 32) | ((uint64_t)(ln[k] % RANGE_LINES) << 22) | (hb[k] & 0x3fffff);
    }
  }
}

// pass B: one workgroup per range: its lines into LDS once, then its probes answered from LDS
template <bool SCATTER>
__global__ __launch_bounds__(1024) void k_answer(const uint4* __restrict__ lines, const uint32_t* __restrict__ fill,
                                                 const uint64_t* __restrict__ recs, uint32_t region,
                                                 uint64_t* __restrict__ out) {
  __shared__ uint4 s_lines[RANGE_LINES * 4];
  const uint32_t r = blockIdx.x;
  const uint4* src = lines + (uint64_t)r * RANGE_LINES * 4;
  for (uint32_t j = threadIdx.x; j < RANGE_LINES * 4; j += 1024) s_lines[j] = src[j];
  __syncthreads();
  const uint32_t cnt = min(fill[r], region);
  const uint64_t* rr = recs + (uint64_t)r * region;
  for (uint32_t j = threadIdx.x; j < cnt; j += 1024) {
    const uint64_t rec = __builtin_nontemporal_load(rr + j);
    const uint32_t l = (uint32_t)(rec >> 22) & (RANGE_LINES - 1), hb = (uint32_t)rec & 0x3fffff;
    const uint4 v = s_lines[l * 4 + (hb & 3)];
    const uint64_t res = v.x ^ v.y ^ v.z ^ v.w ^ hb;
    if (SCATTER) out[rec >> 32] = res;
    else __builtin_nontemporal_store(res, out + (uint64_t)r * region + j);
  }
}

__global__ void k_init(uint64_t* p, uint64_t n, uint64_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + seed) * 0x9e3779b97f4a7c15ull;
    x ^= x >> 31; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 29;
    p[i] = x;
  }
}

template <typename F>
static float timed(F&& f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  std::vector<float> t;
  for (int r = 0; r < 5; r++) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[2];
}

static void shape(const char* name, uint32_t nf, uint32_t lg_lpf, uint32_t launches) {
  const uint64_t n = 64ull << 20;                   // probes per launch
  const uint32_t fpl = nf / launches;               // filters per launch
  const uint64_t per_f = n / fpl;
  const uint64_t nlines = (uint64_t)fpl << lg_lpf;  // one launch's filters
  const uint32_t nranges = (uint32_t)(nlines / RANGE_LINES);
  const uint32_t region = (uint32_t)(n / nranges + 8 * std::sqrt((double)n / nranges) + 64);
  uint64_t *keys, *out, *recs;
  uint4* lines;
  uint32_t* fill;
  CK(hipMalloc(&keys, n * 24));
  CK(hipMalloc(&out, std::max<uint64_t>(n, (uint64_t)nranges * region) * 8));
  CK(hipMalloc(&lines, nlines * 64));
  CK(hipMalloc(&recs, (uint64_t)nranges * region * 8));
  CK(hipMalloc(&fill, nranges * 4));
  k_init<<<1024, 256>>>(keys, n * 3, 1);
  k_init<<<1024, 256>>>(reinterpret_cast<uint64_t*>(lines), nlines * 8, 2);
  CK(hipDeviceSynchronize());
  const dim3 gd((uint32_t)((n + 1023) / 1024)), ga((uint32_t)((n + TILE - 1) / TILE));
  const float t_direct = timed([&] { k_direct<<<gd, 1024>>>(keys, lines, n, per_f, lg_lpf, out); }) * launches;
  const float t_a = timed([&] {
    CK(hipMemsetAsync(fill, 0, nranges * 4));
    k_partition<<<ga, PNT>>>(keys, n, per_f, lg_lpf, nranges, region, fill, recs);
  }) * launches;
  const float t_b = timed([&] { k_answer<true><<<nranges, 1024>>>(lines, fill, recs, region, out); }) * launches;
  const float t_b0 = timed([&] { k_answer<false><<<nranges, 1024>>>(lines, fill, recs, region, out); }) * launches;
  std::vector<uint32_t> hf(nranges);
  CK(hipMemcpy(hf.data(), fill, nranges * 4, hipMemcpyDeviceToHost));
  const uint32_t mx = *std::max_element(hf.begin(), hf.end());
  printf("%s: %u filters x 2^%u lines (%.1f MB of lines each), %u launch(es) of 64M probes; ranges of %u lines: %u per launch, region %u (fullest %u%s)\n",
         name, nf, lg_lpf, (double)(64ull << lg_lpf) / 1e6, launches, RANGE_LINES, nranges, region, mx,
         mx > region ? ", OVERFLOWED" : "");
  printf("  direct (quad gather, results in probe order)   %.3f ms\n", t_direct);
  printf("  grouped: A partition %.3f + B answer, scattered results %.3f = %.3f ms\n", t_a, t_b, t_a + t_b);
  printf("  grouped: A partition %.3f + B answer, results in range order %.3f = %.3f ms (lower bound: permuted output)\n",
         t_a, t_b0, t_a + t_b0);
  CK(hipFree(keys)); CK(hipFree(out)); CK(hipFree(lines)); CK(hipFree(recs)); CK(hipFree(fill));
}

int main() {
  shape("C2", 8, 17, 1);      // 8 x 8.4 MB line tables (8M keys per filter)
  shape("C3", 256, 15, 4);    // 256 x 2.1 MB (2^20 keys per filter), 64 filters per launch
  return 0;
}
