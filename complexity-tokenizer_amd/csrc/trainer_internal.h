// Internal interfaces between the trainer host (trainer_host.cpp) and its kernels (trainer.hip).
// Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ctok_train {

constexpr uint64_t kEmptyKey = ~0ull;  // no pair (a, b) has a = b = 0xFFFFFFFF

struct Words {        // device CSR of the training words
  uint32_t* tok;      // tokens; word w at tok[wstart[w] .. + wlen[w]) (shrinks in place)
  const uint32_t* wstart;
  uint32_t* wlen;
  const uint32_t* wfreq;
  uint32_t n_words;
};

struct PairTable {    // open addressing, key a << 32 | b, i64 count; capacity mask + 1
  uint64_t* keys;
  int64_t* vals;
  uint32_t mask;
  uint32_t* used;     // slots taken since the last drain
  uint32_t* n_used;
};

hipError_t launch_count_pairs(const Words& W, const PairTable& T, hipStream_t s);
hipError_t launch_apply_merge(const Words& W, const PairTable& T, uint32_t a, uint32_t b, uint32_t nid,
                              unsigned long long* tok_freq, hipStream_t s);
hipError_t launch_drain(const PairTable& T, uint64_t max_used, uint64_t* out_keys, int64_t* out_vals, hipStream_t s);

}  // namespace ctok_train
