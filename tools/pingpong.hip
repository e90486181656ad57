// Microbenchmark (diagnostic tool, not product code): host <-> GPU round trip through pinned
// coherent host memory, without a kernel launch per request, against a launch per request.
//   persistent: one wave polls a request word in host memory (system-scope loads, s_sleep
//               between polls), answers by storing a result word; the host spins on it.
//               The kernel's loop is bounded by s_memrealtime (max lifetime) and a stop flag.
//   launch:     one 64-thread kernel per request that stores the result word (what a
//               launch-based lookup round trip costs at minimum).
// build: hipcc --offload-arch=gfx950 -O3 tools/pingpong.hip -o /tmp/pingpong
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_server(uint64_t* req, uint64_t* res, uint64_t* ctl, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = 0, served = 0;
  for (;;) {
    const uint64_t r = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (r != last) {
      last = r;
      served++;
      __hip_atomic_store(res, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      continue;
    }
    if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __hip_atomic_store(ctl + 1, served, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_once(uint64_t* res, uint64_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(res, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  uint64_t *req, *res, *ctl;
  CK(hipHostMalloc(&req, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&res, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&ctl, 64, hipHostMallocCoherent | hipHostMallocMapped));
  *req = 0; *res = 0; ctl[0] = ctl[1] = 0;
  hipStream_t st, sm;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // a CU-masked stream gets an HSA queue of its own: the persistent kernel never blocks work
  // queued on other streams
  uint32_t mask[8] = {1u, 0, 0, 0, 0, 0, 0, 0};
  const hipError_t me = hipExtStreamCreateWithCUMask(&sm, 8, mask);
  printf("cu-masked stream: %s\n", me == hipSuccess ? "ok" : hipGetErrorString(me));
  if (me != hipSuccess) sm = st;
  // launch per request
  for (int w = 0; w < 100; w++) { hipLaunchKernelGGL(k_once, dim3(1), dim3(64), 0, st, res, (uint64_t)w + 1); CK(hipStreamSynchronize(st)); }
  const int N = 20000;
  double t = now_us();
  for (int i = 1; i <= N; i++) {
    const uint64_t v = 1000 + i;
    hipLaunchKernelGGL(k_once, dim3(1), dim3(64), 0, st, res, v);
    while (__atomic_load_n(res, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
  }
  const double launch_us = (now_us() - t) / N;
  CK(hipStreamSynchronize(st));
  // persistent server (at most 3 s)
  *res = 0;
  hipLaunchKernelGGL(k_server, dim3(1), dim3(64), 0, sm, req, res, ctl, (uint64_t)300000000);
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  for (int i = 1; i <= 100; i++) {
    __atomic_store_n(req, (uint64_t)i, __ATOMIC_RELEASE);
    while (__atomic_load_n(res, __ATOMIC_ACQUIRE) != (uint64_t)i) __builtin_ia32_pause();
  }
  t = now_us();
  for (int i = 101; i <= 100 + N; i++) {
    __atomic_store_n(req, (uint64_t)i, __ATOMIC_RELEASE);
    while (__atomic_load_n(res, __ATOMIC_ACQUIRE) != (uint64_t)i) __builtin_ia32_pause();
  }
  const double persist_us = (now_us() - t) / N;
  // meanwhile other work on another stream must not be blocked by the server: 200 launch +
  // stream-sync round trips on a plain stream while the server runs, then the same after it
  // stopped (first sample and median of each: a cold first launch vs a steady cost)
  auto other = [&](double* first, double* med) {
    double v[200];
    for (int i = 0; i < 200; i++) {
      const double t1 = now_us();
      hipLaunchKernelGGL(k_once, dim3(1), dim3(64), 0, st, res + 1, (uint64_t)i);
      CK(hipStreamSynchronize(st));
      v[i] = now_us() - t1;
    }
    *first = v[0];
    std::sort(v, v + 200);
    *med = v[100];
  };
  double run_first, run_med, idle_first, idle_med;
  std::this_thread::sleep_for(std::chrono::milliseconds(20));  // st idle for a while, as in round 4
  other(&run_first, &run_med);
  __atomic_store_n(ctl, (uint64_t)1, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(sm));
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  other(&idle_first, &idle_med);
  const double other_us = run_first;
  printf("{\"launch_roundtrip_us\": %.2f, \"persistent_roundtrip_us\": %.2f, \"other_stream_kernel_us_while_server_runs\": {\"first\": %.1f, \"median\": %.1f}, \"other_stream_kernel_us_server_stopped\": {\"first\": %.1f, \"median\": %.1f}, \"served\": %llu}\n",
         launch_us, persist_us, other_us, run_med, idle_first, idle_med, (unsigned long long)ctl[1]);
  return 0;
}
