// HIP kernels (gfx950 / CDNA4) for the padded batch encode: encoded ids -> Encoding rows as
// [rows, width] arrays of ids, attention mask, type ids and special-tokens mask.
//
// Reference path (Complexity-ML/complexity-tokenizer v0.3.3):
//   Tokenizer.__call__ / encode_batch_with_padding / encode_batch_to_encoding
//                                          src/bindings/tokenizer.rs:46-201, :326-371
//   encode_to_encoding_impl                src/huggingface/mod.rs:358-392 (merge pair, process(ids,
//                                          None), masks extended by the added count, mark_special)
//   encode_batch_with_padding              src/huggingface/mod.rs:483-509
//   Encoding::from_ids / merge / truncate / pad   src/encoding.rs:45-131, :240-253
//
// Per row: n = ids of the row (pair: na + nb), P = the processed length (n times each $A item +
// one per special item), L = min(P, max_len) when truncating, then pad to the target.  Cell i of
// the content: the processed id, attention 1, type id (i < n ? i >= na : 0 -- the pair's ids are
// type 1, the post-processor's additions type 0), special mask (i >= n, or the id is a special
// token when marking).  Padding cells: pad id, attention 0, type 0, special 1.  A pure gather +
// streaming write: HBM-bound, one thread per output cell, consecutive lanes -> consecutive cells.
#include <hip/hip_runtime.h>

#include "ctok_internal.h"

namespace ctok_dev {

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

struct PadRow {
  uint64_t base;  // first id of the row in w.ids
  uint32_t n, na;
  uint64_t P, L;
};

__device__ __forceinline__ PadRow pad_row(const PadWork& w, uint32_t r, uint32_t nA, uint32_t nS) {
  PadRow x;
  const uint32_t a = w.pairs ? 2 * r : r;
  x.base = w.tok_off[a];
  const uint64_t ea = w.tok_off[a + 1];
  const uint64_t e = w.pairs ? w.tok_off[a + 2] : ea;
  x.na = (uint32_t)(ea - x.base);
  x.n = (uint32_t)(e - x.base);
  x.P = w.use_tpl ? (uint64_t)nA * x.n + nS : x.n;
  x.L = (w.truncate && x.P > w.max_len) ? w.max_len : x.P;
  return x;
}

__device__ __forceinline__ void count_items(const PadWork& w, uint32_t& nA, uint32_t& nS) {
  nA = 0;
  nS = 0;
  for (uint32_t k = 0; k < w.n_items; k++) {
    if (w.items[k] == kPadItemA) nA++;
    else nS++;
  }
}

// row lengths, the longest content, and the reference's panic when a template drops ids
// (`processed_ids.len() - encoding.ids.len()` underflows, src/huggingface/mod.rs:378)
__global__ void k_pad_len(PadWork w) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t nA, nS;
  count_items(w, nA, nS);
  uint64_t L = 0;
  if (r < w.n_rows) {
    const PadRow x = pad_row(w, r, nA, nS);
    if (x.P < x.n) atomicOr(&w.counters[2], 1u);
    L = x.L;
    w.row_len[r] = L > w.target ? L : w.target;
  }
  // wave maximum, one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t u = __shfl_xor(L, o, 64);
    L = u > L ? u : L;
  }
  if ((threadIdx.x & 63) == 0 && L) atomicMax((unsigned long long*)w.counters, (unsigned long long)L);
}

__device__ __forceinline__ bool is_special(const PadWork& w, uint32_t id) {
  uint32_t lo = 0, hi = w.n_special;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t v = w.special_ids[mid];
    if (v == id) return true;
    if (v < id) lo = mid + 1;
    else hi = mid;
  }
  return false;
}

__device__ __forceinline__ void pad_cell(const PadWork& w, uint32_t r, uint64_t c, uint32_t nA, uint32_t nS) {
  const PadRow x = pad_row(w, r, nA, nS);
  const uint64_t rowlen = x.L > w.target ? x.L : w.target;
  const uint64_t pad = rowlen - x.L;
  bool is_pad;
  uint64_t i = 0;
  if (c >= rowlen) {
    is_pad = true;  // past a ragged row's end: filled like padding
  } else if (w.pad_left) {
    is_pad = c < pad;
    i = c - pad;
  } else {
    is_pad = c >= x.L;
    i = c;
  }
  uint32_t id = w.pad_id, attn = 0, type = 0, spec = 1;
  if (!is_pad) {
    if (w.use_tpl) {
      uint64_t off = 0;
      for (uint32_t k = 0; k < w.n_items; k++) {
        const uint32_t it = w.items[k];
        const uint64_t len = it == kPadItemA ? x.n : 1;
        if (i < off + len) {
          id = it == kPadItemA ? w.ids[x.base + (i - off)] : it;
          break;
        }
        off += len;
      }
    } else {
      id = w.ids[x.base + i];
    }
    attn = 1;
    type = (i < x.n && i >= x.na) ? 1u : 0u;
    spec = (i >= x.n || (w.mark && is_special(w, id))) ? 1u : 0u;
  }
  const uint64_t o = (uint64_t)r * w.width + c;
  w.out_ids[o] = id;
  if (w.out_attn) w.out_attn[o] = attn;
  if (w.out_type) w.out_type[o] = type;
  if (w.out_special) w.out_special[o] = spec;
}

// one thread per output cell (grid-stride over rows * width, row-major: consecutive lanes write
// consecutive cells of a row)
__global__ __launch_bounds__(256) void k_pad_rows(PadWork w) {
  uint32_t nA, nS;
  count_items(w, nA, nS);
  const uint64_t total = (uint64_t)w.n_rows * w.width;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t cell = (uint64_t)blockIdx.x * 256 + threadIdx.x; cell < total; cell += stride) {
    const uint32_t r = (uint32_t)(cell / w.width);
    pad_cell(w, r, cell - (uint64_t)r * w.width, nA, nS);
  }
}

hipError_t launch_pad_len(const PadWork& w, hipStream_t s) {
  if (w.n_rows) k_pad_len<<<(w.n_rows + 255) / 256, 256, 0, s>>>(w);
  return hipGetLastError();
}

hipError_t launch_pad_rows(const PadWork& w, hipStream_t s) {
  const uint64_t total = (uint64_t)w.n_rows * w.width;
  if (!total) return hipSuccess;
  const uint64_t blocks = (total + 255) / 256;
  k_pad_rows<<<(uint32_t)(blocks < 65536 ? blocks : 65536), 256, 0, s>>>(w);
  return hipGetLastError();
}

}  // namespace ctok_dev
