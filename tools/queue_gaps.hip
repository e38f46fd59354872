// Measurement tool (not product code): the device-side gap between two kernels for the ways the
// encode call orders its streams -- same stream, an event record in between, a second stream
// waiting on that event, a second stream waiting on a value the first kernel writes -- after a
// first kernel that leaves `dirty` MB of written data behind.  Times come from the kernels
// themselves (wall_clock64, 100 MHz): the first kernel's last workgroup stamps its end, the
// second kernel's first workgroup its start.
//   hipcc --offload-arch=gfx950 -O3 tools/queue_gaps.hip -o tools/queue_gaps && tools/queue_gaps
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

// stamps[0] = end of A (last workgroup), stamps[1] = start of B (first workgroup, atomic min)
__global__ void k_writer(uint4* buf, size_t n16, uint32_t* ticket, uint64_t* stamps, uint32_t* flag, uint32_t seq) {
  if (threadIdx.x == 0) atomicMin((unsigned long long*)&stamps[2], (unsigned long long)wall_clock64());
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    buf[i] = make_uint4((uint32_t)i, seq, 1, 2);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t t = atomicAdd(ticket, 1u);
    if (t == gridDim.x - 1) {
      *ticket = 0;
      stamps[0] = wall_clock64();
      if (flag) {
        __threadfence_system();
        __atomic_store_n(flag, seq, __ATOMIC_RELEASE);
      }
    }
  }
}

// A as a persistent-style grid: one 1024-thread workgroup per CU holding 142 KB of LDS (as k_bpe_short)
__global__ __launch_bounds__(1024) void k_writer_lds(uint4* buf, size_t n16, uint32_t* ticket, uint64_t* stamps,
                                                     uint32_t* flag, uint32_t seq) {
  extern __shared__ uint4 s_lds[];
  if (threadIdx.x == 0) atomicMin((unsigned long long*)&stamps[2], (unsigned long long)wall_clock64());
  s_lds[threadIdx.x] = make_uint4(seq, 0, 0, 0);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    buf[i] = make_uint4((uint32_t)i, s_lds[threadIdx.x].x, 1, 2);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t t = atomicAdd(ticket, 1u);
    if (t == gridDim.x - 1) {
      *ticket = 0;
      stamps[0] = wall_clock64();
    }
  }
}

__global__ __launch_bounds__(1024) void k_reader_lds(const uint4* buf, uint64_t* stamps, uint32_t* out) {
  extern __shared__ uint4 s_img[];
  if (threadIdx.x == 0) atomicMin((unsigned long long*)&stamps[1], (unsigned long long)wall_clock64());
  for (uint32_t i = threadIdx.x; i < 96 * 1024 / 16; i += blockDim.x) s_img[i] = buf[i];
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s_img[blockIdx.x & 63].x;
}

__global__ void k_reader(const uint4* buf, uint64_t* stamps, uint32_t* out) {
  if (threadIdx.x == 0) atomicMin((unsigned long long*)&stamps[1], (unsigned long long)wall_clock64());
  // a little work: read one line per workgroup
  if (threadIdx.x == 0) out[blockIdx.x] = buf[(size_t)blockIdx.x * 64].x;
}

int main(int argc, char** argv) {
  const size_t dirty_mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
  const int reps = 20;
  const size_t n16 = dirty_mb * (1u << 20) / 16;
  uint4* buf;
  uint32_t *ticket, *out, *flag_dev, *flag_host;
  uint64_t* stamps;
  CK(hipMalloc(&buf, std::max<size_t>(n16, 4096 * 64) * 16));
  CK(hipMalloc(&ticket, 4));
  CK(hipMemset(ticket, 0, 4));
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMalloc(&flag_dev, 4));
  CK(hipMemset(flag_dev, 0, 4));
  CK(hipHostMalloc(&flag_host, 4, hipHostMallocCoherent));
  *flag_host = 0;
  CK(hipHostMalloc(&stamps, 32, hipHostMallocCoherent));
  int wv = 0;
  CK(hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, 0));
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev_t, ev_n;
  CK(hipEventCreate(&ev_t));
  CK(hipEventCreateWithFlags(&ev_n, hipEventDisableTiming));
  printf("dirty %zu MB, stream wait value supported %d, wall clock %d kHz\n", dirty_mb, wv, khz);
  const char* names[] = {"same stream", "same stream + timing event", "same stream + no-timing event",
                         "2nd stream waits no-timing event", "2nd stream waits value (device flag)",
                         "2nd stream waits value (host flag)", "same stream + 2nd stream waits event on it",
                         "encode fork: event, copy + kernel on 2 streams, 142 KB B",
                         "same stream, 142 KB B", "same stream + event, 142 KB B",
                         "same stream, B any-order launch", "A with start/stop events (no markers)",
                         "A with events, B any-order", "B any-order with events", "A 1-per-CU 142 KB, B any-order",
                         "B any-order with a stop event only", "B any-order with a start event only",
                         "A 1-per-CU 160 KB, B any-order", "A 1-per-CU 156 KB, B any-order", "A 1-per-CU 152 KB, B any-order"};
  uint32_t seq = 0;
  hipStream_t s3;
  CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  uint32_t* hbuf;
  CK(hipHostMalloc(&hbuf, 4096, hipHostMallocCoherent));
  CK(hipFuncSetAttribute((const void*)k_reader_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 142 * 1024));
  CK(hipFuncSetAttribute((const void*)k_writer_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 20; mode++) {
    double ev_ms = 0, a_ms = 0;
    if ((mode == 4 || mode == 5) && !wv) continue;
    std::vector<double> gaps;
    for (int r = 0; r < reps; r++) {
      seq++;
      stamps[0] = 0;
      stamps[1] = ~0ull;
      stamps[2] = ~0ull;
      uint32_t* flag = mode == 4 ? flag_dev : mode == 5 ? flag_host : nullptr;
      CK(hipDeviceSynchronize());
      if (mode == 11 || mode == 12) {
        void* args[] = {&buf, (void*)&n16, &ticket, &stamps, &flag, &seq};
        CK(hipExtLaunchKernel((const void*)k_writer, dim3(2048), dim3(256), args, 0, s1, e0, e1, 0));
      } else if (mode == 14 || mode >= 17) {
        void* args[] = {&buf, (void*)&n16, &ticket, &stamps, &flag, &seq};
        const size_t lds = mode == 14 ? 142 * 1024 : mode == 17 ? 160 * 1024 : mode == 18 ? 156 * 1024 : 152 * 1024;
        CK(hipExtLaunchKernel((const void*)k_writer_lds, dim3(256), dim3(1024), args, lds, s1, nullptr, nullptr, 0));
      } else {
        k_writer<<<2048, 256, 0, s1>>>(buf, n16, ticket, stamps, flag, seq);
      }
      hipStream_t sb = s1;
      if (mode == 1) CK(hipEventRecord(ev_t, s1));
      if (mode == 2 || mode == 3 || mode == 6) CK(hipEventRecord(ev_n, s1));
      if (mode == 3) {
        CK(hipStreamWaitEvent(s2, ev_n, 0));
        sb = s2;
      }
      if (mode == 4 || mode == 5) {
        CK(hipStreamWaitValue32(s2, flag, seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
        sb = s2;
      }
      if (mode == 6) CK(hipStreamWaitEvent(s2, ev_n, 0));  // (the other stream's wait only)
      if (mode == 7 || mode == 9) CK(hipEventRecord(ev_n, s1));
      if (mode == 7) {
        CK(hipStreamWaitEvent(s2, ev_n, 0));
        CK(hipMemcpyAsync(hbuf, out, 128, hipMemcpyDeviceToHost, s2));
        CK(hipStreamWaitEvent(s3, ev_n, 0));
        k_reader<<<64, 64, 0, s3>>>(buf, stamps + 2, out + 2048);
        CK(hipMemcpyAsync(hbuf + 64, out, 4, hipMemcpyDeviceToHost, s3));
      }
      if (mode == 10 || mode >= 12) {
        void* args[] = {&buf, &stamps, &out};
        CK(hipExtLaunchKernel((const void*)k_reader, dim3(1024), dim3(64), args, 0, s1,
                              mode == 13 || mode == 16 ? e0 : nullptr, mode == 13 || mode == 15 ? e1 : nullptr,
                              hipExtAnyOrderLaunch));
      } else if (mode >= 7 && mode <= 9) k_reader_lds<<<256, 1024, 142 * 1024, s1>>>(buf, stamps, out);
      else k_reader<<<1024, 64, 0, sb>>>(buf, stamps, out);
      CK(hipDeviceSynchronize());
      if (r >= 3) gaps.push_back((double)(int64_t)(stamps[1] - stamps[0]) * 1e3 / khz);
      if (mode == 11) {
        float v = 0;
        CK(hipEventElapsedTime(&v, e0, e1));
        ev_ms = v;
        a_ms = (double)(int64_t)(stamps[0] - stamps[2]) * 1.0 / khz;
      }
    }
    std::sort(gaps.begin(), gaps.end());
    printf("%-46s gap A end -> B start: median %7.2f us  min %7.2f  max %7.2f\n", names[mode], gaps[gaps.size() / 2],
           gaps.front(), gaps.back());
    if (mode == 11) printf("   A: events %.4f ms, device stamps (first start -> last end) %.4f ms\n", ev_ms, a_ms);
  }
  return 0;
}
