// Microbenchmark (diagnostic tool, not product code): where should the lookup server's request
// ring live? The server wave polls tickets and reads payloads; today both sit in pinned
// coherent host memory, so every poll is a PCIe read (RF_SRV_PROF: 4.3 us per 64-ticket poll,
// 1.3 us per payload read). Alternative: the ring in fine-grained device memory that the host
// writes through the BAR (posted writes), the wave polling its own HBM.
//   1. which allocations the host can reach (hsa_amd_pointer_info: accessible agents);
//   2. per mode: the wave's latency of a 64-lane, 8-B-per-lane poll (system-scope loads) and of
//      a dependent 64-lane 64-B payload read;
//   3. per mode: ping-pong round trip (host stores request t, wave polls it, answers in pinned
//      host memory, host spins on the answer);
//   4. the host's cost of writing a 64-B request into each mode (stores + sfence).
// Every kernel loop is bounded by s_memrealtime. build:
//   hipcc --offload-arch=gfx950 -O3 tools/vram_ring.hip -o tools/vram_ring -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <atomic>
#include <csetjmp>
#include <csignal>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// wave-side latency: `iters` rounds of (64-lane poll of 8 B each, then 64-lane read of a 64-B
// line each, dependent on the poll), timed with s_memrealtime (100 MHz)
__global__ void k_lat(const uint64_t* tick, const uint4* pay, uint64_t* out, int iters, int mode_payload) {
  const uint32_t lane = threadIdx.x;
  uint64_t acc = 0, tp = 0, tq = 0;
  for (int i = 0; i < iters; i++) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t a = __builtin_amdgcn_s_memrealtime();
    const uint64_t t = __hip_atomic_load(&tick[(lane + acc) & 63], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    acc += t & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t b = __builtin_amdgcn_s_memrealtime();
    tp += b - a;
    if (mode_payload) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      const uint4* p = pay + ((lane + acc) & 63) * 4;
      uint4 x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
      acc += (x0.x ^ x1.y ^ x2.z ^ x3.w) & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tq += __builtin_amdgcn_s_memrealtime() - b;
    }
  }
  if (lane == 0) {
    out[0] = tp;
    out[1] = tq;
    out[2] = acc;
  }
}

// ping-pong: the wave (lane 0) polls req[0] (system scope) until it changes, answers in res[0]
__global__ void k_server(const uint64_t* req, uint64_t* res, uint64_t* ctl, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = 0, served = 0;
  for (;;) {
    const uint64_t r = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (r != last) {
      last = r;
      served++;
      __hip_atomic_store(res, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      continue;
    }
    if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __hip_atomic_store(ctl + 1, served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// server emulation: the wave polls 64 published-ticket words from head (slot t holds t + 1 once
// request t is published), serves the ready prefix (head += k) and reports head in host memory;
// the host producer keeps at most 64 requests ahead of it. Poll time summed over served polls.
__global__ void k_srvemu(const uint64_t* pub, uint64_t* hd, uint64_t* out, uint64_t n_total, uint64_t max_ticks) {
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t head = 0, tpoll = 0, npoll = 0, nidle = 0;
  for (;;) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t a = __builtin_amdgcn_s_memrealtime();
    const uint64_t tk = __hip_atomic_load(&pub[(head + lane) & 255], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t ready = __builtin_amdgcn_ballot_w64(tk == head + lane + 1);
    const uint32_t k = ready == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~ready);
    const uint64_t b = __builtin_amdgcn_s_memrealtime();
    if (k) {
      tpoll += b - a;
      npoll++;
      head += k;
      if (lane == 0) __hip_atomic_store(hd, head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      nidle++;
      __builtin_amdgcn_s_sleep(2);
    }
    if (head >= n_total || b - t0 > max_ticks) break;
  }
  if (lane == 0) {
    out[0] = tpoll;
    out[1] = npoll;
    out[2] = head;
    out[3] = nidle;
    out[4] = __builtin_amdgcn_s_memrealtime() - t0;
  }
}

struct Pools {
  hsa_agent_t cpu{}, gpu{};
  hsa_amd_memory_pool_t gpu_fine{}, gpu_coarse{};
  bool have_fine = false, have_coarse = false;
};

static hsa_status_t agent_cb(hsa_agent_t a, void* d) {
  Pools* P = (Pools*)d;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !P->cpu.handle) P->cpu = a;
  if (t == HSA_DEVICE_TYPE_GPU && !P->gpu.handle) P->gpu = a;
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* d) {
  Pools* P = (Pools*)d;
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !P->have_fine) { P->gpu_fine = p; P->have_fine = true; }
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !P->have_coarse) { P->gpu_coarse = p; P->have_coarse = true; }
  return HSA_STATUS_SUCCESS;
}

static sigjmp_buf g_jb;
static void segv_handler(int) { siglongjmp(g_jb, 1); }
// a host store + load on ptr under a SIGSEGV guard (a fault here is the host's, not the GPU's)
static bool host_touch(void* ptr, const char* name) {
  struct sigaction sa, old_segv, old_bus;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = segv_handler;
  sigaction(SIGSEGV, &sa, &old_segv);
  sigaction(SIGBUS, &sa, &old_bus);
  bool ok = false;
  if (sigsetjmp(g_jb, 1) == 0) {
    volatile uint64_t* q = (volatile uint64_t*)ptr;
    q[0] = 0x1234567ull;
    _mm_sfence();
    ok = q[0] == 0x1234567ull;
  }
  sigaction(SIGSEGV, &old_segv, nullptr);
  sigaction(SIGBUS, &old_bus, nullptr);
  printf("# %s: host store/load %s\n", name, ok ? "ok" : "FAULTED or mismatched");
  return ok;
}

static bool cpu_accessible(const Pools& P, void* ptr, const char* name) {
  hsa_amd_pointer_info_t info;
  memset(&info, 0, sizeof(info));
  info.size = sizeof(info);
  uint32_t n = 0;
  hsa_agent_t* ags = nullptr;
  const hsa_status_t s = hsa_amd_pointer_info(ptr, &info, malloc, &n, &ags);
  bool cpu = false;
  for (uint32_t i = 0; i < n; i++) cpu |= ags[i].handle == P.cpu.handle;
  printf("# %s: pointer_info %d type %d host %p agents %u cpu_access %d\n", name, (int)s, (int)info.type,
         info.hostBaseAddress, n, (int)cpu);
  free(ags);
  return s == HSA_STATUS_SUCCESS && cpu;
}

int main() {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  if (hsa_init() != HSA_STATUS_SUCCESS) { printf("hsa_init failed\n"); return 1; }
  Pools P;
  hsa_iterate_agents(agent_cb, &P);
  hsa_amd_agent_iterate_memory_pools(P.gpu, pool_cb, &P);
  printf("# gpu fine pool %d coarse pool %d\n", (int)P.have_fine, (int)P.have_coarse);

  const size_t SZ = 1 << 16;
  struct Mode { const char* name; uint8_t* p; };
  std::vector<Mode> modes;
  uint8_t* h = nullptr;
  CK(hipHostMalloc((void**)&h, SZ, hipHostMallocCoherent | hipHostMallocMapped));
  memset(h, 0, SZ);
  modes.push_back({"host_coherent", h});
  // device fine-grained memory through HSA, opened to the CPU
  if (P.have_fine) {
    void* v = nullptr;
    hsa_status_t s = hsa_amd_memory_pool_allocate(P.gpu_fine, SZ, 0, &v);
    if (s == HSA_STATUS_SUCCESS) {
      s = hsa_amd_agents_allow_access(1, &P.cpu, nullptr, v);
      printf("# vram_fine_hsa: allocate ok, allow_access(cpu) %d\n", (int)s);
      cpu_accessible(P, v, "vram_fine_hsa");
      if (s == HSA_STATUS_SUCCESS && host_touch(v, "vram_fine_hsa")) {
        memset(v, 0, SZ);
        modes.push_back({"vram_fine_hsa", (uint8_t*)v});
      }
    } else {
      printf("# vram_fine_hsa: allocate failed %d\n", (int)s);
    }
  }
  // hipExtMallocWithFlags fine-grained / uncached: reported only (host access if the runtime opened it)
  {
    void* v = nullptr;
    if (hipExtMallocWithFlags(&v, SZ, hipDeviceMallocFinegrained) == hipSuccess) {
      cpu_accessible(P, v, "hip_finegrained");
      if (host_touch(v, "hip_finegrained")) { memset(v, 0, SZ); modes.push_back({"hip_finegrained", (uint8_t*)v}); }
    }
    void* u = nullptr;
    if (hipExtMallocWithFlags(&u, SZ, hipDeviceMallocUncached) == hipSuccess) {
      cpu_accessible(P, u, "hip_uncached");
      if (host_touch(u, "hip_uncached")) { memset(u, 0, SZ); modes.push_back({"hip_uncached", (uint8_t*)u}); }
    }
  }
  uint64_t *res, *ctl, *out;
  CK(hipHostMalloc((void**)&res, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&ctl, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&out, 64, hipHostMallocCoherent | hipHostMallocMapped));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (const Mode& m : modes) {
    // 2. wave-side latencies
    const int IT = 2000;
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, st, (const uint64_t*)m.p, (const uint4*)(m.p + 4096), out, 10, 1);
    CK(hipStreamSynchronize(st));
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, st, (const uint64_t*)m.p, (const uint4*)(m.p + 4096), out, IT, 1);
    CK(hipStreamSynchronize(st));
    const double poll_us = out[0] * 0.01 / IT, pay_us = out[1] * 0.01 / IT;
    // 3. ping-pong: request word in this mode, answer in host memory
    uint64_t* req = (uint64_t*)(m.p + 8192);
    __atomic_store_n(req, 0ull, __ATOMIC_RELEASE);
    _mm_sfence();
    *res = 0;
    ctl[0] = ctl[1] = 0;
    hipLaunchKernelGGL(k_server, dim3(1), dim3(64), 0, st, req, res, ctl, (uint64_t)200000000);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    const int N = 20000;
    double t0 = 0;
    bool ok = true;
    for (int i = 1; i <= N + 200 && ok; i++) {
      if (i == 201) t0 = now_us();
      __atomic_store_n(req, (uint64_t)i, __ATOMIC_RELEASE);
      _mm_sfence();
      const double ts = now_us();
      while (__atomic_load_n(res, __ATOMIC_ACQUIRE) != (uint64_t)i) {
        __builtin_ia32_pause();
        if (now_us() - ts > 100000) { ok = false; break; }
      }
    }
    const double rt_us = ok ? (now_us() - t0) / N : -1;
    __atomic_store_n(ctl, 1ull, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(st));
    // 4. host cost of a 64-B request write (8 stores + sfence), 200k times over 64 slots
    uint64_t* w = (uint64_t*)(m.p + 16384);
    const int W = 200000;
    const double tw = now_us();
    for (int i = 0; i < W; i++) {
      uint64_t* q = w + (i & 63) * 8;
      for (int k = 0; k < 7; k++) q[k] = (uint64_t)i + k;
      _mm_sfence();
      __atomic_store_n(q + 7, (uint64_t)i, __ATOMIC_RELEASE);
      _mm_sfence();
    }
    const double write_ns = (now_us() - tw) * 1000.0 / W;
    // host read cost of one word (the reaper would read answers; here for reference)
    volatile uint64_t sink = 0;
    const double tr = now_us();
    for (int i = 0; i < 20000; i++) sink += w[(i & 63) * 8];
    const double read_ns = (now_us() - tr) * 1000.0 / 20000;
    // 5. server emulation: producer thread (this one) publishes N requests, each a 64-B payload
    //    line then its ticket word, with plain stores or non-temporal stores (+ sfence)
    double emu[2][4];
    for (int nt = 0; nt < 2; nt++) {
      uint64_t* pub = (uint64_t*)(m.p + 32768);
      uint64_t* pay = (uint64_t*)(m.p + 36864);  // 256 x 64 B
      for (int i = 0; i < 256; i++) pub[i] = 0;
      _mm_sfence();
      volatile uint64_t* hd = res + 2;
      *hd = 0;
      const uint64_t NREQ = 200000;
      hipLaunchKernelGGL(k_srvemu, dim3(1), dim3(64), 0, st, (const uint64_t*)pub, (uint64_t*)(res + 2), out, NREQ,
                         (uint64_t)300000000);
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      const double te = now_us();
      for (uint64_t t = 0; t < NREQ; t++) {
        const double tw0 = now_us();
        while (t >= *hd + 64) {
          __builtin_ia32_pause();
          if (now_us() - tw0 > 100000) break;
        }
        uint64_t* q = pay + (t & 255) * 8;
        if (nt) {
          for (int k = 0; k < 8; k++) _mm_stream_si64((long long*)&q[k], (long long)(t + k));
          _mm_sfence();
          _mm_stream_si64((long long*)&pub[t & 255], (long long)(t + 1));
          _mm_sfence();
        } else {
          for (int k = 0; k < 8; k++) q[k] = t + k;
          __atomic_store_n(&pub[t & 255], t + 1, __ATOMIC_RELEASE);
        }
      }
      CK(hipStreamSynchronize(st));
      emu[nt][0] = (now_us() - te) / NREQ * 1000.0;                 // ns per request end to end
      emu[nt][1] = out[1] ? out[0] * 10.0 / out[1] : -1;            // ns per served poll
      emu[nt][2] = out[1] ? (double)out[2] / out[1] : -1;           // requests per served poll
      emu[nt][3] = (double)out[2];
    }
    printf("{\"mode\": \"%s\", \"emu_plain\": {\"ns_per_req\": %.1f, \"poll_ns\": %.0f, \"per_poll\": %.1f, \"served\": %.0f}, "
           "\"emu_nt\": {\"ns_per_req\": %.1f, \"poll_ns\": %.0f, \"per_poll\": %.1f, \"served\": %.0f}}\n",
           m.name, emu[0][0], emu[0][1], emu[0][2], emu[0][3], emu[1][0], emu[1][1], emu[1][2], emu[1][3]);
    printf("{\"mode\": \"%s\", \"wave_poll64_us\": %.3f, \"wave_payload64B_us\": %.3f, \"pingpong_us\": %.3f, "
           "\"served\": %llu, \"host_write64B_ns\": %.1f, \"host_read8B_ns\": %.1f}\n",
           m.name, poll_us, pay_us, rt_us, (unsigned long long)ctl[1], write_ns, read_ns);
    fflush(stdout);
  }
  return 0;
}
