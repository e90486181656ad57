// Microbenchmark (diagnostic tool, not product code): what does one random W-byte line fetch
// per probe cost on MI355X, beside the probe's 24 B key read + 8 B result write?
//   mode 0: stream only (read 24 B key, write 8 B) per item
//   mode 1: gather only (one random W-byte line per item)
//   mode 2: stream + gather (the probe's access pattern)
// layout L: 0 = one lane loads the whole line (W/16 dwordx4 loads); 1 = W/16 consecutive
// lanes load 16 B each of one line (a line per lane group; all lanes of a group still
// stream their own key)
// build: hipcc --offload-arch=gfx950 -O3 tools/gather_bench.hip -o /tmp/gather_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}

template <int W, int MODE, int LAYOUT>
__global__ __launch_bounds__(256) void k(const uint4* __restrict__ keys, const uint4* __restrict__ table,
                                         uint32_t nlines, uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t h = 0;
  if (MODE != 1) {
    const uint32_t* kp = reinterpret_cast<const uint32_t*>(keys) + i * 6;
    const uint64_t* k8 = reinterpret_cast<const uint64_t*>(kp);
    const uint64_t a = __builtin_nontemporal_load(k8), b = __builtin_nontemporal_load(k8 + 1),
                   c = __builtin_nontemporal_load(k8 + 2);
    h = mix(a ^ (b << 17) ^ (c >> 9) ^ c ^ i);  // keys are constant: i keeps lines random
  } else {
    h = mix(i);
  }
  uint32_t acc = h;
  if (MODE != 0) {
    constexpr int Q = W / 16;
    if (LAYOUT == 0) {
      const uint4* lp = table + (uint64_t)(h % nlines) * Q;
      uint4 v[Q];
#pragma unroll
      for (int q = 0; q < Q; q++) v[q] = lp[q];
#pragma unroll
      for (int q = 0; q < Q; q++) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    } else {
      // lane group of Q lanes: lane t of the group loads part t of each of the group's Q lines
      const uint32_t t = threadIdx.x % Q;
      uint4 v[Q];
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const uint32_t hq = __shfl(h, (threadIdx.x & ~(Q - 1)) + q, 64);
        v[q] = table[(uint64_t)(hq % nlines) * Q + t];
      }
#pragma unroll
      for (int q = 0; q < Q; q++) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    }
  }
  if (MODE == 1) {
    if (acc == 0x12345678u) out[i] = acc;  // keep the loads alive
  } else {
    __builtin_nontemporal_store((uint64_t)acc, out + i);
  }
}

template <int W, int MODE, int LAYOUT>
float run(const uint4* keys, const uint4* table, uint32_t nlines, uint64_t n, uint64_t* out) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  dim3 g((unsigned)((n + 255) / 256));
  for (int w = 0; w < 2; w++) hipLaunchKernelGGL((k<W, MODE, LAYOUT>), g, dim3(256), 0, 0, keys, table, nlines, n, out);
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k<W, MODE, LAYOUT>), g, dim3(256), 0, 0, keys, table, nlines, n, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

template <int W>
void sweep(const uint4* keys, const uint4* table, size_t table_bytes, uint64_t n, uint64_t* out) {
  const uint32_t nl = (uint32_t)(table_bytes / W);
  const float g0 = run<W, 1, 0>(keys, table, nl, n, out);
  const float g1 = W > 16 ? run<W, 1, 1>(keys, table, nl, n, out) : g0;
  const float s0 = run<W, 2, 0>(keys, table, nl, n, out);
  const float s1 = W > 16 ? run<W, 2, 1>(keys, table, nl, n, out) : s0;
  printf("table %6.1f MB  W %3d B | gather lane %.3f ms (%.0f GB/s line bytes)  group %.3f ms | stream+gather lane %.3f ms  group %.3f ms\n",
         table_bytes / 1e6, W, g0, n * (double)W / g0 / 1e6, g1, s0, s1);
}

int main(int argc, char** argv) {
  const uint64_t n = 64ull << 20;
  uint4 *keys, *table; uint64_t* out;
  CK(hipMalloc(&keys, n * 24));
  CK(hipMalloc(&out, n * 8));
  const size_t tmax = 256ull << 20;
  CK(hipMalloc(&table, tmax));
  CK(hipMemset(keys, 0x5a, n * 24));
  CK(hipMemset(table, 0x33, tmax));
  printf("stream only (24 B read + 8 B write per item, %llu items): %.3f ms\n", (unsigned long long)n,
         run<16, 0, 0>(keys, table, 1, n, out));
  const size_t sizes[] = {2ull << 20, 8ull << 20, 64ull << 20, 200ull << 20};
  for (size_t tb : sizes) {
    sweep<16>(keys, table, tb, n, out);
    sweep<32>(keys, table, tb, n, out);
    sweep<64>(keys, table, tb, n, out);
    sweep<128>(keys, table, tb, n, out);
  }
  return 0;
}
