// Microbenchmark (diagnostic tool, not product code): is "24 B key stream + one random 64-B
// line per probe" latency-bound or request-bound on MI355X? Compares
//   A: one probe per lane (key load -> hash -> dependent line load -> store), full grid;
//   B: grid-stride loop, next probe's key loaded while this probe's line is in flight;
//   C: grid-stride loop, P probes per lane per iteration (P keys, P lines in flight).
// build: hipcc --offload-arch=gfx950 -O3 tools/gather_pipe.hip -o tools/gather_pipe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}
struct K3 { uint64_t a, b, c; };
__device__ __forceinline__ K3 ldk(const uint64_t* keys, uint64_t i) {
  const uint64_t* p = keys + i * 3;
  return K3{__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1), __builtin_nontemporal_load(p + 2)};
}
__device__ __forceinline__ uint32_t hk(K3 k, uint64_t i) { return mix(k.a ^ (k.b << 17) ^ (k.c >> 9) ^ k.c ^ i); }
__device__ __forceinline__ uint32_t use(const uint4 (&v)[4], uint32_t h) {
  uint32_t acc = h;
#pragma unroll
  for (int q = 0; q < 4; q++) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
  return acc;
}

__global__ __launch_bounds__(256) void kA(const uint64_t* __restrict__ keys, const uint4* __restrict__ table,
                                          uint32_t nl, uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t h = hk(ldk(keys, i), i);
  const uint4* lp = table + (uint64_t)(h % nl) * 4;
  uint4 v[4];
#pragma unroll
  for (int q = 0; q < 4; q++) v[q] = lp[q];
  __builtin_nontemporal_store((uint64_t)use(v, h), out + i);
}

__global__ __launch_bounds__(256) void kB(const uint64_t* __restrict__ keys, const uint4* __restrict__ table,
                                          uint32_t nl, uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  K3 k = ldk(keys, i);
  for (; i < n; i += stride) {
    const uint32_t h = hk(k, i);
    const uint4* lp = table + (uint64_t)(h % nl) * 4;
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = lp[q];
    if (i + stride < n) k = ldk(keys, i + stride);
    __builtin_nontemporal_store((uint64_t)use(v, h), out + i);
  }
}

template <int P>
__global__ __launch_bounds__(256) void kC(const uint64_t* __restrict__ keys, const uint4* __restrict__ table,
                                          uint32_t nl, uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * P;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * P + threadIdx.x; i0 < n; i0 += stride) {
    K3 k[P];
#pragma unroll
    for (int p = 0; p < P; p++) k[p] = i0 + p * 256 < n ? ldk(keys, i0 + p * 256) : K3{0, 0, 0};
    uint32_t h[P];
    uint4 v[P][4];
#pragma unroll
    for (int p = 0; p < P; p++) {
      h[p] = hk(k[p], i0 + p * 256);
      const uint4* lp = table + (uint64_t)(h[p] % nl) * 4;
#pragma unroll
      for (int q = 0; q < 4; q++) v[p][q] = lp[q];
    }
#pragma unroll
    for (int p = 0; p < P; p++)
      if (i0 + p * 256 < n) __builtin_nontemporal_store((uint64_t)use(v[p], h[p]), out + i0 + p * 256);
  }
}

template <typename F>
float timeit(F launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch(); launch();
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int r = 0; r < reps; r++) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  const uint64_t n = 64ull << 20;
  uint64_t *keys, *out; uint4* table;
  CK(hipMalloc(&keys, n * 24)); CK(hipMalloc(&out, n * 8)); CK(hipMalloc(&table, 256ull << 20));
  CK(hipMemset(keys, 0x5a, n * 24)); CK(hipMemset(table, 0x33, 256ull << 20));
  int cus = 256;
  const size_t sizes[] = {2ull << 20, 4ull << 20, 8ull << 20, 67ull << 20};
  for (size_t tb : sizes) {
    const uint32_t nl = (uint32_t)(tb / 64);
    const unsigned gA = (unsigned)(n / 256);
    float a = timeit([&] { hipLaunchKernelGGL(kA, dim3(gA), dim3(256), 0, 0, keys, table, nl, n, out); });
    printf("table %5.1f MB  A %.3f ms |", tb / 1e6, a);
    for (int wpc : {8, 16, 32}) {
      const unsigned g = cus * wpc / 4;
      float b = timeit([&] { hipLaunchKernelGGL(kB, dim3(g), dim3(256), 0, 0, keys, table, nl, n, out); });
      float c2 = timeit([&] { hipLaunchKernelGGL(kC<2>, dim3(g), dim3(256), 0, 0, keys, table, nl, n, out); });
      float c4 = timeit([&] { hipLaunchKernelGGL(kC<4>, dim3(g), dim3(256), 0, 0, keys, table, nl, n, out); });
      printf(" %2d w/CU: B %.3f C2 %.3f C4 %.3f |", wpc, b, c2, c4);
    }
    printf("\n");
  }
  return 0;
}
