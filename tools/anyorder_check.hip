// Measurement tool (not product code): does an any-order packet (hipExtAnyOrderLaunch) behind a
// persistent, LDS-filling kernel start before that kernel ends?  A: one 1024-thread workgroup per
// CU with 160 KB of LDS taking work items from a counter for ~0.5 ms (as k_bpe_short); B: a small
// kernel with a large by-value argument (as k_c3_list with Work) whose last workgroup writes a
// host word; the host polls the word and reports how long after the launches it arrived.
//   hipcc --offload-arch=gfx950 -O3 tools/anyorder_check.hip -o tools/anyorder_check
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

struct Big {  // a by-value argument of the size of the encode path's Work
  uint32_t* ctr;
  uint32_t* host;
  uint32_t seq;
  uint64_t pad[60];
};

__device__ unsigned long long g_st[4];  // A end (max), B first start (min), B report time

__global__ __launch_bounds__(1024) void k_persist(uint32_t* ctr, uint4* buf, uint32_t items) {
  extern __shared__ uint4 s[];
  __shared__ uint32_t s_k;
  for (;;) {
    if (threadIdx.x == 0) s_k = atomicAdd(ctr, 1u);
    __syncthreads();
    const uint32_t k = s_k;
    __syncthreads();
    if (k >= items) {
      if (threadIdx.x == 0) atomicMax(&g_st[0], (unsigned long long)wall_clock64());
      break;
    }
    uint4 v = buf[(size_t)k * 1024 + threadIdx.x];
    for (int r = 0; r < 64; r++) {
      s[(threadIdx.x + r * 7) & 8191] = v;
      __syncthreads();
      v.x += s[(threadIdx.x * 3 + r) & 8191].y;
    }
    buf[(size_t)k * 1024 + threadIdx.x] = v;
  }
}

__global__ __launch_bounds__(256) void k_report_small(uint32_t* ctr, uint32_t* host, uint32_t seq) {
  if (threadIdx.x == 0) atomicMin(&g_st[1], (unsigned long long)wall_clock64());
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x >= 64) return;
  uint32_t last = 0;
  if ((threadIdx.x & 63) == 0) last = atomicAdd(ctr + 1, 1u) == gridDim.x - 1 ? 1u : 0u;
  if (!__builtin_amdgcn_readfirstlane(last)) return;
  if (threadIdx.x == 0) g_st[2] = wall_clock64();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (threadIdx.x == 0) __hip_atomic_store(host, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

__global__ __launch_bounds__(256) void k_report(Big b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x >= 64) return;
  uint32_t last = 0;
  if ((threadIdx.x & 63) == 0) last = atomicAdd(b.ctr + 1, 1u) == gridDim.x - 1 ? 1u : 0u;
  if (!__builtin_amdgcn_readfirstlane(last)) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (threadIdx.x == 0) __hip_atomic_store(b.host, b.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

int main() {
  const uint32_t items = 6000;
  uint4* buf;
  uint32_t *ctr, *host;
  CK(hipMalloc(&buf, (size_t)items * 1024 * 16));
  CK(hipMemset(buf, 0, (size_t)items * 1024 * 16));
  CK(hipMalloc(&ctr, 64));
  CK(hipHostMalloc(&host, 64, hipHostMallocCoherent));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipFuncSetAttribute((const void*)k_persist, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int mode = 0; mode < 11; mode++) {
    const int grid_a = mode == 8 ? cus - 8 : mode == 9 ? cus / 2 : mode == 10 ? cus - 1 : cus;
    for (int rep = 0; rep < 4; rep++) {
      CK(hipMemset(ctr, 0, 64));
      unsigned long long init[4] = {0, ~0ull, 0, 0};
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_st), init, sizeof(init)));
      CK(hipDeviceSynchronize());
      Big b{};
      b.ctr = ctr;
      b.host = host;
      b.seq = (uint32_t)(mode * 100 + rep + 1);
      const auto t0 = std::chrono::steady_clock::now();
      if (mode == 3) {
        void* args[] = {&ctr, &buf, (void*)&items};
        CK(hipExtLaunchKernel((const void*)k_persist, dim3(cus), dim3(1024), args, 156 * 1024, s, nullptr, nullptr, 0));
      } else {
        k_persist<<<grid_a, 1024, 156 * 1024, s>>>(ctr, buf, items);
      }
      const uint32_t ao = (uint32_t)hipExtAnyOrderLaunch;
      if (mode == 0) k_report<<<158, 256, 0, s>>>(b);
      else if (mode <= 3) hipExtLaunchKernelGGL(k_report, dim3(158), dim3(256), 0, s, nullptr, nullptr, mode == 2 ? 0u : ao, b);
      else if (mode == 4) hipExtLaunchKernelGGL(k_report_small, dim3(158), dim3(256), 0, s, nullptr, nullptr, ao, ctr, host, b.seq);
      else if (mode == 5) hipExtLaunchKernelGGL(k_report_small, dim3(158), dim3(64), 0, s, nullptr, nullptr, ao, ctr, host, b.seq);
      else if (mode == 6) hipExtLaunchKernelGGL(k_report_small, dim3(1024), dim3(64), 0, s, nullptr, nullptr, ao, ctr, host, b.seq);
      else if (mode == 7) hipExtLaunchKernelGGL(k_report_small, dim3(8), dim3(64), 0, s, nullptr, nullptr, ao, ctr, host, b.seq);
      else hipExtLaunchKernelGGL(k_report_small, dim3(158), dim3(256), 0, s, nullptr, nullptr, ao, ctr, host, b.seq);
      CK(hipGetLastError());
      while (__atomic_load_n(host, __ATOMIC_ACQUIRE) != b.seq) {
      }
      const auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(s));
      const auto t2 = std::chrono::steady_clock::now();
      unsigned long long gs[4];
      CK(hipMemcpyFromSymbol(gs, HIP_SYMBOL(g_st), sizeof(gs)));
      if (rep > 0)
        printf("mode %d (%s): report after %.1f us, both kernels done after %.1f us; device: B first start %.1f us, "
               "B last %.1f us from A's end\n", mode,
               mode == 0 ? "plain B" : mode == 1 ? "B any-order" : mode == 2 ? "B ext, in order" : mode == 3 ? "A ext, B any-order"
               : mode == 4 ? "small-arg B any-order 158x256" : mode == 5 ? "small-arg B 158x64" : mode == 6 ? "small-arg B 1024x64"
               : mode == 7 ? "small-arg B 8x64" : mode == 8 ? "A on cus-8, B 158x256 any-order"
               : mode == 9 ? "A on cus/2, B any-order" : "A on cus-1, B any-order",
               std::chrono::duration<double, std::micro>(t1 - t0).count(),
               std::chrono::duration<double, std::micro>(t2 - t0).count(),
               mode >= 4 ? ((double)(long long)(gs[1] - gs[0])) / 100.0 : 0.0,
               mode >= 4 ? ((double)(long long)(gs[2] - gs[0])) / 100.0 : 0.0);
    }
  }
  return 0;
}
