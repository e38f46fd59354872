// HIP kernels (gfx950) of the INL-BPE trainer's pair counting.
//
// Reference (Complexity-ML/complexity-tokenizer v0.3.3, src/trainer.rs):
//   compute_initial_pairs    :341-367  rayon fold/reduce of a (a, b) -> sum of word freqs histogram
//   apply_merge_incremental  :522-590  every word scanned for the merged pair, the pair replaced
//                                      left to right, +-freq deltas for the neighbouring pairs
//
// Words live in HBM as a CSR token array (word w: tok[wstart[w] .. wstart[w] + wlen[w]), shrinking
// in place as merges apply) with a u32 frequency each.  Pair counts (initial histogram and per-merge
// deltas) accumulate in an open-addressing table of u64 keys a << 32 | b and i64 values, by device
// atomics (they execute at the memory side, so workgroups on different XCDs add into one table
// exactly; integer sums are order-independent, hence bit-exact).  A slot's first insert appends
// the slot to a used list; the drain pass moves the used slots' (key, count) pairs out and resets
// them, so a merge costs O(its deltas), not O(table), to read back.  No MFMA: integer/hash work.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "trainer_internal.h"

namespace ctok_train {

__device__ __forceinline__ uint32_t slot_of(uint64_t key, uint32_t mask) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32) & mask;
}

// count += v for key (inserting it on first use)
__device__ __forceinline__ void table_add(const PairTable& T, uint64_t key, int64_t v) {
  uint32_t h = slot_of(key, T.mask);
  for (;;) {
    uint64_t k = T.keys[h];
    if (k == kEmptyKey) {
      k = atomicCAS((unsigned long long*)&T.keys[h], (unsigned long long)kEmptyKey, (unsigned long long)key);
      if (k == kEmptyKey) {  // this thread took the slot
        T.used[atomicAdd(T.n_used, 1u)] = h;
        k = key;
      }
    }
    if (k == key) {
      atomicAdd((unsigned long long*)&T.vals[h], (unsigned long long)v);
      return;
    }
    h = (h + 1) & T.mask;
  }
}

// compute_initial_pairs: thread per word (grid-stride)
__global__ __launch_bounds__(256) void k_count_pairs(Words W, PairTable T) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < W.n_words; w += gridDim.x * blockDim.x) {
    const uint32_t* t = W.tok + W.wstart[w];
    const uint32_t n = W.wlen[w];
    const int64_t f = (int64_t)W.wfreq[w];
    for (uint32_t i = 0; i + 1 < n; i++) table_add(T, ((uint64_t)t[i] << 32) | t[i + 1], f);
  }
}

// apply_merge_incremental for pair (a, b) -> nid: thread per word, the reference's left-to-right
// loop verbatim (after a merge at i the scan stays at i), deltas into T, merged occurrences'
// frequencies summed into *tok_freq.
__global__ __launch_bounds__(256) void k_apply_merge(Words W, PairTable T, uint32_t a, uint32_t b, uint32_t nid,
                                                     unsigned long long* tok_freq) {
  unsigned long long mine = 0;
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < W.n_words; w += gridDim.x * blockDim.x) {
    uint32_t* t = W.tok + W.wstart[w];
    uint32_t n = W.wlen[w];
    if (n < 2) continue;
    const int64_t f = (int64_t)W.wfreq[w];
    uint32_t i = 0;
    bool changed = false;
    while (i + 1 < n) {
      if (t[i] == a && t[i + 1] == b) {
        if (i > 0) table_add(T, ((uint64_t)t[i - 1] << 32) | a, -f);
        if (i + 2 < n) table_add(T, ((uint64_t)b << 32) | t[i + 2], -f);
        t[i] = nid;
        for (uint32_t j = i + 1; j + 1 < n; j++) t[j] = t[j + 1];  // Vec::remove(i + 1)
        n--;
        if (i > 0) table_add(T, ((uint64_t)t[i - 1] << 32) | nid, f);
        if (i + 1 < n) table_add(T, ((uint64_t)nid << 32) | t[i + 1], f);
        mine += (unsigned long long)f;
        changed = true;
      } else {
        i++;
      }
    }
    if (changed) W.wlen[w] = n;
  }
  // one atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
  if ((threadIdx.x & 63) == 0 && mine) atomicAdd(tok_freq, mine);
}

// Move the used slots out (keys, counts; *n_out = count) and reset them.
__global__ __launch_bounds__(256) void k_drain(PairTable T, uint64_t* out_keys, int64_t* out_vals) {
  const uint32_t n = *T.n_used;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t h = T.used[i];
    out_keys[i] = T.keys[h];
    out_vals[i] = T.vals[h];
    T.keys[h] = kEmptyKey;
    T.vals[h] = 0;
  }
}

static uint32_t grid_for(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (uint32_t)(g < 1 ? 1 : g > 8192 ? 8192 : g);
}

hipError_t launch_count_pairs(const Words& W, const PairTable& T, hipStream_t s) {
  if (W.n_words) k_count_pairs<<<grid_for(W.n_words), 256, 0, s>>>(W, T);
  return hipGetLastError();
}

hipError_t launch_apply_merge(const Words& W, const PairTable& T, uint32_t a, uint32_t b, uint32_t nid,
                              unsigned long long* tok_freq, hipStream_t s) {
  if (W.n_words) k_apply_merge<<<grid_for(W.n_words), 256, 0, s>>>(W, T, a, b, nid, tok_freq);
  return hipGetLastError();
}

hipError_t launch_drain(const PairTable& T, uint64_t max_used, uint64_t* out_keys, int64_t* out_vals, hipStream_t s) {
  k_drain<<<grid_for(max_used), 256, 0, s>>>(T, out_keys, out_vals);
  return hipGetLastError();
}

}  // namespace ctok_train
