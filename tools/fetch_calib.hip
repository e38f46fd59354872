// FETCH_SIZE calibration on known byte counts, in the access shapes of the merge passes (VERDICT r05
// #3; MI355X_MICROARCH.md "HBM": FETCH_SIZE is calibrated only for 16-B-per-lane streaming reads).
// Profiling helper, not product code.  Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip
// -o tools/fetch_calib.  Run under rocprofv3 --pmc (one launch per kernel below; tools/pmc_calib.sh
// makes the passes and prints bytes per access).
//
//   k_stream16     16 B per lane, coalesced, over 2 GiB (past the 256 MiB Infinity Cache): the
//                  streaming shape (the guide's reference: FETCH = half the bytes)
//   k_gather_line  one 4-B load per 128-B line, lines in a random order (a permutation: every line
//                  of a 2 GiB table exactly once, no reuse): tallied bytes per missing line
//   k_gather_half  two 4-B loads per line at +0 and +64 by the same lane: 1 request per line means
//                  the L2 fetches whole 128-B lines, 2 means 64-B halves
//   k_gather_tab8  8-B loads at random slots of a 32 MiB table (the narrow merge table of a 50k
//                  vocabulary), 64M of them: the merge passes' global-table probes, L2 misses served
//                  by the Infinity Cache
//   k_text_words   the merge passes' text loads: each lane reads 5 consecutive dwords at its own
//                  piece start, pieces 12 B apart on average (a class list's stride), over 1 GiB
//   k_store16, k_store_line4, k_store_dense4   WRITE_SIZE: 16-B coalesced stores over 1 GiB, one
//                  4-B store per 128-B line (each line of 2 GiB once, random order: scattered record
//                  stores), 4-B stores of consecutive dwords over 1 GiB
//
// Each kernel writes one sum per lane (so the loads are not dead) into a small output.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));    \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void k_stream16(const uint4* __restrict__ a, uint64_t n16, uint32_t* __restrict__ out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// line i of the table in a random order without an index array: (i * odd + c) mod 2^k is a
// permutation of [0, 2^k)
__device__ __forceinline__ uint64_t line_of(uint64_t i, uint64_t mask) { return (i * 0x9E3779B1ull + 12345ull) & mask; }

__global__ void k_gather_line(const uint32_t* __restrict__ tab, uint64_t n_lines, uint32_t* __restrict__ out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_lines; i += (uint64_t)gridDim.x * blockDim.x)
    s += tab[line_of(i, n_lines - 1) * 32 + (i & 15)];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_gather_half(const uint32_t* __restrict__ tab, uint64_t n_lines, uint32_t* __restrict__ out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_lines; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = line_of(i, n_lines - 1) * 32;
    s += tab[b] + tab[b + 16];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_gather_tab8(const uint64_t* __restrict__ tab, uint32_t mask, uint64_t n, uint32_t* __restrict__ out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    const uint64_t e = tab[h & mask];
    s += (uint32_t)e ^ (uint32_t)(e >> 32);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// piece i starts at 12 i + (0..3): lanes' pieces ~12 B apart, as consecutive entries of a class
// list; each lane reads its piece's 5 dwords
__global__ void k_text_words(const uint8_t* __restrict__ text, uint64_t n, uint32_t* __restrict__ out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = (12 * i + ((i * 0x9E3779B1ull) >> 40) % 4) & ~3ull;
#pragma unroll
    for (int k = 0; k < 5; k++) s += *reinterpret_cast<const uint32_t*>(text + a + 4 * k);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// stores: 16 B per lane coalesced; one 4-B store per 128-B line (lines in a random order, each
// once: a scattered record store); 4-B stores of consecutive dwords by consecutive lanes
__global__ void k_store16(uint4* __restrict__ a, uint64_t n16) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ void k_store_line4(uint32_t* __restrict__ tab, uint64_t n_lines) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_lines; i += (uint64_t)gridDim.x * blockDim.x)
    tab[line_of(i, n_lines - 1) * 32 + (i & 31)] = (uint32_t)i;
}

__global__ void k_store_dense4(uint32_t* __restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

int main() {
  const uint64_t kBig = 2ull << 30;                 // 2 GiB: past the Infinity Cache
  const uint64_t n_lines = kBig / 128;              // 2^24 lines
  const uint64_t kTab8 = 32ull << 20;               // 32 MiB table of u64
  const uint64_t n_tab8 = 64ull << 20;              // 64M probes
  const uint64_t n_text = (1ull << 30) / 12;        // pieces over ~1 GiB of text
  const int grid = 256 * 8, block = 256;
  uint8_t* big;
  uint32_t* out;
  uint64_t* tab8;
  CK(hipMalloc(&big, kBig + 64));
  CK(hipMalloc(&out, (size_t)grid * block * 4));
  CK(hipMalloc(&tab8, kTab8));
  CK(hipMemset(big, 1, kBig + 64));
  CK(hipMemset(tab8, 2, kTab8));
  CK(hipDeviceSynchronize());
  // (tools/pmc_calib.sh reads the counters per kernel name; each kernel once, the 2 GiB table
  // streamed through between the gathers so that no line they read is still cached)
  k_stream16<<<grid, block>>>((const uint4*)big, kBig / 16, out);
  k_gather_line<<<grid, block>>>((const uint32_t*)big, n_lines, out);
  k_stream16<<<grid, block>>>((const uint4*)big, kBig / 16, out);
  k_gather_half<<<grid, block>>>((const uint32_t*)big, n_lines, out);
  k_gather_tab8<<<grid, block>>>(tab8, (uint32_t)(kTab8 / 8 - 1), n_tab8, out);
  k_stream16<<<grid, block>>>((const uint4*)big, kBig / 16, out);
  k_text_words<<<grid, block>>>(big, n_text, out);
  k_store16<<<grid, block>>>((uint4*)big, (kBig / 2) / 16);
  k_stream16<<<grid, block>>>((const uint4*)big, kBig / 16, out);
  k_store_line4<<<grid, block>>>((uint32_t*)big, n_lines);
  k_stream16<<<grid, block>>>((const uint4*)big, kBig / 16, out);
  k_store_dense4<<<grid, block>>>((uint32_t*)big, (kBig / 2) / 4);
  CK(hipDeviceSynchronize());
  printf("{\"stream16_bytes\": %llu, \"gather_lines\": %llu, \"gather_half_loads\": %llu, \"tab8_probes\": %llu, "
         "\"tab8_table_bytes\": %llu, \"text_pieces\": %llu, \"text_span_bytes\": %llu, \"store16_bytes\": %llu, "
         "\"store_lines\": %llu, \"store_dense4_bytes\": %llu}\n",
         (unsigned long long)kBig, (unsigned long long)n_lines, (unsigned long long)(2 * n_lines),
         (unsigned long long)n_tab8, (unsigned long long)kTab8, (unsigned long long)n_text,
         (unsigned long long)(12 * n_text + 20), (unsigned long long)(kBig / 2), (unsigned long long)n_lines,
         (unsigned long long)(kBig / 2));
  return 0;
}
