// HIP kernels (gfx950 / CDNA4) for batch decode: token ids -> UTF-8 text.
//
// Reference path (Complexity-ML/complexity-tokenizer v0.3.3):
//   HuggingFaceTokenizer::decode_batch(_with_options)   src/huggingface/mod.rs:771-785
//   -> decode_impl                                       src/huggingface/mod.rs:710-747
//      skip special tokens (model.vocab string is a special added token)   :716-726
//      Vocab::get_token per id (model.vocab only)                          :729-732
//      ByteLevel decoder: chars -> bytes, from_utf8_lossy                  src/decoders.rs:94-119
//      (or BpeTokenizer::decode: raw token strings, src/bpe.rs:170-176, for an unknown decoder)
//      clean_up_tokenization_spaces: 15 replaces + split_whitespace/join   src/huggingface/mod.rs:749-767
//
// Every id maps to a fixed byte string (its token's chars mapped back to bytes), so the batch
// is first gathered into `raw` (the concatenation) -- an HBM-bound id -> bytes gather.  Lossy
// UTF-8 and the clean-up then act per document on `raw`, and both are local:
//   * a maximal invalid subpart (lossy) is decided from at most 3 bytes on either side;
//   * every clean-up pattern consists of ' ' and the 14 bytes . , ! ? : ; " ' ( ) [ ] - ("set
//     bytes"), and each replace only deletes spaces, so the 15 passes act independently on each
//     maximal run of set bytes (a lane replays them on the run);
//   * split_whitespace + join(" ") keeps one ' ' for the first surviving unit of each white-space
//     run between two non-white-space units, and drops leading/trailing white space (marked per
//     doc by k_dec_trim).
// So every input byte emits 0, 1 or 3 (U+FFFD) output bytes; a tile-level count, a scan and a
// rewrite produce the packed output.
#include <hip/hip_runtime.h>

#include "ctok_internal.h"

namespace ctok_dev {

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

constexpr int kDecPer = 16;               // ids (gather) or bytes (clean-up) per thread
constexpr int kDecStage = 32768;          // LDS staging bytes for a chunk's output
constexpr int kHalo = 64;                 // doc-start bitmap margin around a clean-up tile
constexpr int kWinBits = kDecTile + 2 * kHalo;
constexpr int kWinWords = kWinBits / 32;

// ------------------------------------------------------------------------------------------
// helpers

// exclusive scan over a 256-thread block; sh needs 4 u32
__device__ __forceinline__ uint32_t dec_block_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) sh[wid] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = sh[k];
    base += k < wid ? x : 0u;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

__device__ __forceinline__ uint32_t dec_len_of(uint32_t y, uint32_t opts) {
  if ((opts & kDecOptSkipSpecial) && (y & kDecSpecial)) return 0;
  return y & kDecLenMask;
}

// first d in [0, n] with off[d] >= x (off sorted, n + 1 entries)
__device__ __forceinline__ uint32_t lower_bound_u64(const uint64_t* off, uint32_t n, uint64_t x) {
  uint32_t lo = 0, hi = n + 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (off[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Copy a chunk's staged bytes s_stage[a, a + n) to dst[g0 + a, g0 + a + n), g0 16-byte aligned:
// whole 16-byte blocks with one store, the partial first / last blocks byte by byte (the
// neighbouring workgroups write the other bytes of those blocks).
__device__ __forceinline__ void store_staged(const uint8_t* s_stage, uint32_t a, uint32_t n, uint8_t* dst) {
  const uint32_t nblk = (a + n + 15) / 16;
  for (uint32_t b = threadIdx.x; b < nblk; b += blockDim.x) {
    const uint32_t lo = b * 16, hi = lo + 16;
    if (lo >= a && hi <= a + n) {
      *reinterpret_cast<uint4*>(dst + lo) = *reinterpret_cast<const uint4*>(s_stage + lo);
    } else {
      const uint32_t j0 = lo > a ? lo : a, j1 = hi < a + n ? hi : a + n;
      for (uint32_t j = j0; j < j1; j++) dst[j] = s_stage[j];
    }
  }
}

// ------------------------------------------------------------------------------------------
// K0: offsets check (tok_off[0] == 0, non-decreasing, tok_off[n_docs] == n_ids)

__global__ void k_dec_check(DecWork w) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d > w.n_docs) return;
  const uint64_t o = w.tok_off[d];
  bool bad = (d == 0 && o != 0) || (d == w.n_docs && o != w.n_ids) || o > w.n_ids;
  if (d < w.n_docs && w.tok_off[d + 1] < o) bad = true;
  if (bad) atomicOr(&w.counters[0], 1u);
}

// ------------------------------------------------------------------------------------------
// K1: decoded bytes per chunk of kDecChunk ids (lane-strided loads), non-ASCII flag

__global__ __launch_bounds__(256) void k_dec_len(DecWork w, DecTables t) {
  __shared__ uint32_t sh[4];
  const uint32_t base = blockIdx.x * kDecChunk;
  uint32_t sum = 0, flags = 0;
#pragma unroll
  for (int k = 0; k < kDecPer; k++) {
    const uint32_t i = base + k * 256 + threadIdx.x;
    if (i < w.n_ids) {
      const uint32_t id = w.ids[i];
      const uint32_t y = id < t.n_ent ? t.ent[id].y : 0u;
      const uint32_t l = dec_len_of(y, w.opts);
      sum += l;
      flags |= l ? y : 0u;
    }
  }
  uint32_t tot;
  (void)dec_block_scan(sum, sh, &tot);
  if (threadIdx.x == 0) {
    w.chunk_off[blockIdx.x] = tot;
    atomicAdd(reinterpret_cast<unsigned long long*>(w.counters + 2), (unsigned long long)tot);
  }
  if (__any(flags & kDecNonAscii) && (threadIdx.x & 63) == 0) atomicOr(&w.counters[1], 1u);
}

hipError_t launch_dec_len(const DecWork& w, const DecTables& t, uint32_t* tmp, uint64_t tmp_cap, hipStream_t s) {
  k_dec_check<<<(w.n_docs + 1 + 255) / 256, 256, 0, s>>>(w);
  HIPCHK(hipGetLastError());
  if (w.n_chunks) {
    k_dec_len<<<w.n_chunks, 256, 0, s>>>(w, t);
    HIPCHK(hipGetLastError());
  }
  return scan_u32(w.chunk_off, w.chunk_off, w.n_chunks, nullptr, tmp, tmp_cap, s);
}

// ------------------------------------------------------------------------------------------
// K2: gather.  Workgroup per chunk: the ids' decoded lengths are scanned in the block, their
// bytes staged in LDS at the chunk's global alignment and stored as 16-byte blocks; the docs
// whose first id lies in the chunk get their byte offset from the per-id prefix in LDS.

__global__ __launch_bounds__(256) void k_dec_gather(DecWork w, DecTables t, uint8_t* __restrict__ dst,
                                                    uint64_t* __restrict__ dst_off) {
  __shared__ uint32_t s_pre[kDecChunk + 1];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[kDecStage + 16];
  __shared__ uint32_t sh[4];
  __shared__ uint32_t s_d0;
  const uint32_t c = blockIdx.x, base = c * kDecChunk;
  const uint32_t i0 = base + threadIdx.x * kDecPer;
  if (threadIdx.x == 0) s_d0 = lower_bound_u64(w.tok_off, w.n_docs, base);
  uint32_t e_off[kDecPer], e_len[kDecPer];
  uint32_t sum = 0;
  if (i0 + kDecPer <= w.n_ids && ((uintptr_t)w.ids & 15) == 0) {
    uint32_t idv[kDecPer];
#pragma unroll
    for (int q = 0; q < kDecPer / 4; q++) {
      const uint4 v = *reinterpret_cast<const uint4*>(w.ids + i0 + 4 * q);
      idv[4 * q] = v.x; idv[4 * q + 1] = v.y; idv[4 * q + 2] = v.z; idv[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < kDecPer; k++) {
      const uint2 e = idv[k] < t.n_ent ? t.ent[idv[k]] : make_uint2(0, 0);
      e_off[k] = e.x;
      e_len[k] = dec_len_of(e.y, w.opts);
      sum += e_len[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < kDecPer; k++) {
      const uint32_t i = i0 + k;
      const uint32_t id = i < w.n_ids ? w.ids[i] : 0xFFFFFFFFu;
      const uint2 e = id < t.n_ent ? t.ent[id] : make_uint2(0, 0);
      e_off[k] = e.x;
      e_len[k] = dec_len_of(e.y, w.opts);
      sum += e_len[k];
    }
  }
  uint32_t tot;
  const uint32_t ex = dec_block_scan(sum, sh, &tot);
  {
    uint32_t r = ex;
#pragma unroll
    for (int k = 0; k < kDecPer; k++) {
      s_pre[threadIdx.x * kDecPer + k] = r;
      r += e_len[k];
    }
    if (threadIdx.x == 0) s_pre[kDecChunk] = tot;
  }
  const uint32_t gbase = w.chunk_off[c];
  if (tot <= kDecStage) {
    const uint32_t a = gbase & 15;
    uint32_t r = a + ex;
#pragma unroll
    for (int k = 0; k < kDecPer; k++) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(t.bytes + e_off[k]);
      for (uint32_t j = 0; j < e_len[k]; j += 4) {
        const uint32_t v = src[j >> 2];
        const uint32_t m = e_len[k] - j < 4 ? e_len[k] - j : 4;
        for (uint32_t q = 0; q < m; q++) s_stage[r + j + q] = (uint8_t)(v >> (8 * q));
      }
      r += e_len[k];
    }
    __syncthreads();
    store_staged(s_stage, a, tot, dst + (gbase - a));
  } else {
    uint32_t r = gbase + ex;
#pragma unroll
    for (int k = 0; k < kDecPer; k++) {
      for (uint32_t j = 0; j < e_len[k]; j++) dst[r + j] = t.bytes[e_off[k] + j];
      r += e_len[k];
    }
    __syncthreads();
  }
  // docs whose first id is in this chunk (tok_off == n_ids belongs to the last chunk)
  const uint64_t end = c + 1 == w.n_chunks ? (uint64_t)w.n_ids + 1 : (uint64_t)base + kDecChunk;
  for (uint32_t d = s_d0 + threadIdx.x; d <= w.n_docs; d += 256) {
    const uint64_t to = w.tok_off[d];
    if (to >= end) break;
    dst_off[d] = (uint64_t)gbase + s_pre[to - base];
  }
}

hipError_t launch_dec_gather(const DecWork& w, const DecTables& t, uint8_t* dst, uint64_t* dst_off, hipStream_t s) {
  if (w.n_chunks) k_dec_gather<<<w.n_chunks, 256, 0, s>>>(w, t, dst, dst_off);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// UTF-8 units (from_utf8_lossy, core::str::lossy::Utf8Chunks) and white space

__device__ __forceinline__ bool is_cont(uint32_t b) { return (b & 0xC0u) == 0x80u; }

// Doc boundaries near a clean-up tile: an LDS bitmap of the doc starts (and the end, n_raw) in
// the window [ws, ws + kWinBits); outside it, a binary search of raw_off.
struct Bounds {
  const uint64_t* off;
  uint32_t n_docs;
  uint32_t ws;
  const uint32_t* bits;
  __device__ __forceinline__ bool at(uint32_t q) const {
    const uint32_t r = q - ws;
    if (q >= ws && r < (uint32_t)kWinBits) return (bits[r >> 5] >> (r & 31)) & 1u;
    const uint32_t d = lower_bound_u64(off, n_docs, q);
    return d <= n_docs && off[d] == q;
  }
};

__device__ void build_bounds(const uint64_t* off, uint32_t n_docs, uint32_t ws, uint32_t* s_bits, uint32_t* s_d) {
  for (int i = threadIdx.x; i < kWinWords; i += blockDim.x) s_bits[i] = 0;
  if (threadIdx.x == 0) *s_d = lower_bound_u64(off, n_docs, ws);
  __syncthreads();
  for (uint32_t d = *s_d + threadIdx.x; d <= n_docs; d += blockDim.x) {
    const uint64_t o = off[d];
    if (o >= (uint64_t)ws + kWinBits) break;
    const uint32_t r = (uint32_t)(o - ws);
    atomicOr(&s_bits[r >> 5], 1u << (r & 31));
  }
  __syncthreads();
}

// The unit (maximal valid sequence, or maximal invalid subpart) starting at byte q, which is a
// unit start: its length | 0x100 when valid.  Bytes past the doc's end read as 0 (safe_get).
__device__ __forceinline__ uint32_t unit_at(const uint8_t* raw, const Bounds& bd, uint32_t q) {
  const uint32_t c = raw[q];
  if (c < 0x80) return 1 | 0x100;
  auto nx = [&](uint32_t m) -> uint32_t { return bd.at(q + m) ? 0u : (uint32_t)raw[q + m]; };
  if (c >= 0xC2 && c <= 0xDF) return is_cont(nx(1)) ? (2 | 0x100) : 1;
  if (c >= 0xE0 && c <= 0xEF) {
    const uint32_t c1 = nx(1);
    const bool ok = c == 0xE0 ? (c1 >= 0xA0 && c1 <= 0xBF) : c == 0xED ? (c1 >= 0x80 && c1 <= 0x9F) : is_cont(c1);
    if (!ok) return 1;
    return is_cont(nx(2)) ? (3 | 0x100) : 2;
  }
  if (c >= 0xF0 && c <= 0xF4) {
    const uint32_t c1 = nx(1);
    const bool ok = c == 0xF0 ? (c1 >= 0x90 && c1 <= 0xBF) : c == 0xF4 ? (c1 >= 0x80 && c1 <= 0x8F) : is_cont(c1);
    if (!ok) return 1;
    if (!is_cont(nx(2))) return 2;
    return is_cont(nx(3)) ? (4 | 0x100) : 3;
  }
  return 1;
}

// Start of the unit holding byte p: the nearest preceding non-continuation byte (within 3 bytes
// and the same doc) when its unit reaches p, else p itself.
__device__ __forceinline__ uint32_t unit_start(const uint8_t* raw, const Bounds& bd, uint32_t p) {
  if (!is_cont(raw[p])) return p;
#pragma unroll
  for (uint32_t k = 1; k <= 3; k++) {
    if (bd.at(p - k + 1)) return p;  // p - k + 1 starts a doc: p - k belongs to the previous one
    const uint32_t c = raw[p - k];
    if (is_cont(c)) continue;
    if (c >= 0xC0 && (unit_at(raw, bd, p - k) & 0xFF) > k) return p - k;
    return p;
  }
  return p;
}

// White_Space (Rust char::is_whitespace, 25 code points) for a valid unit of length l at q.
__device__ __forceinline__ bool unit_is_ws(const uint8_t* raw, uint32_t q, uint32_t l) {
  const uint32_t c = raw[q];
  if (l == 1) return (c >= 0x09 && c <= 0x0D) || c == 0x20;
  if (l == 2) return c == 0xC2 && (raw[q + 1] == 0x85 || raw[q + 1] == 0xA0);
  if (l != 3) return false;
  const uint32_t c1 = raw[q + 1], c2 = raw[q + 2];
  if (c == 0xE1) return c1 == 0x9A && c2 == 0x80;
  if (c == 0xE3) return c1 == 0x80 && c2 == 0x80;
  if (c != 0xE2) return false;
  if (c1 == 0x80) return c2 <= 0x8A || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF;
  return c1 == 0x81 && c2 == 0x9F;
}

__device__ __forceinline__ bool del_at(const uint32_t* delbits, uint32_t q) { return (delbits[q >> 5] >> (q & 31)) & 1u; }

// ------------------------------------------------------------------------------------------
// K3: trimmed white space.  Thread per doc: the white-space units before the first and after
// the last non-white-space unit are marked deleted (split_whitespace drops them).

__global__ void k_dec_trim(DecWork w) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= w.n_docs) return;
  const uint32_t ds = (uint32_t)w.raw_off[d], de = (uint32_t)w.raw_off[d + 1];
  if (ds == de) return;
  const Bounds bd{w.raw_off, w.n_docs, 0xFFFFFFFFu - kWinBits, nullptr};  // global search only
  uint32_t p = ds;
  while (p < de) {
    const uint32_t u = unit_at(w.raw, bd, p);
    if (!(u & 0x100) || !unit_is_ws(w.raw, p, u & 0xFF)) break;
    atomicOr(&w.delbits[p >> 5], 1u << (p & 31));
    p += u & 0xFF;
  }
  if (p >= de) return;
  uint32_t q = de;  // units ending at q, walked backwards down to the first non-white-space unit
  while (q > p) {
    const uint32_t u0 = unit_start(w.raw, bd, q - 1);
    const uint32_t u = unit_at(w.raw, bd, u0);
    if (!(u & 0x100) || !unit_is_ws(w.raw, u0, u & 0xFF)) break;
    atomicOr(&w.delbits[u0 >> 5], 1u << (u0 & 31));
    q = u0;
  }
}

// ------------------------------------------------------------------------------------------
// K4: the 15 replaces of clean_up_tokenization_spaces on each run of set bytes.  Thread per
// run start (runs of >= 2 bytes; no pattern matches one byte), replaying the passes in order on
// the run's alive positions; runs of <= 64 bytes keep the alive set in a register.

__device__ __forceinline__ bool is_set_byte(uint32_t b) {
  switch (b) {
    case ' ': case '.': case ',': case '!': case '?': case ':': case ';': case '"': case '\'':
    case '(': case ')': case '[': case ']': case '-': return true;
    default: return false;
  }
}

// pass k: pattern (p0, p1) and whether the space is the first (1) or the second (2) char
__constant__ uint8_t c_pat[14][3] = {{' ', '.', 1}, {' ', ',', 1}, {' ', '!', 1}, {' ', '?', 1}, {' ', ':', 1},
                                     {' ', ';', 1}, {'"', ' ', 2}, {' ', '"', 1}, {'\'', ' ', 2}, {' ', '\'', 1},
                                     {'(', ' ', 2}, {' ', ')', 1}, {'[', ' ', 2}, {' ', ']', 1}};

struct RegAlive {  // alive positions of a run of n <= 64 bytes
  uint64_t m;
  uint32_t n;
  __device__ uint32_t next(uint32_t k) const {  // first alive > k (n if none); k = ~0u: first
    const uint64_t r = k == 0xFFFFFFFFu ? m : (k >= 63 ? 0ull : (m & (~0ull << (k + 1))));
    return r ? (uint32_t)__ffsll((unsigned long long)r) - 1 : n;
  }
  __device__ void kill(uint32_t k) { m &= ~(1ull << k); }
};

struct MemAlive {  // longer runs: the alive set is the complement of delbits (this thread owns the run)
  uint32_t* del;
  uint32_t rs, n;
  __device__ bool dead(uint32_t k) const {
    const uint32_t q = rs + k;
    return (__hip_atomic_load(&del[q >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (q & 31)) & 1u;
  }
  __device__ uint32_t next(uint32_t k) const {
    uint32_t j = k == 0xFFFFFFFFu ? 0 : k + 1;
    while (j < n && dead(j)) j++;
    return j;
  }
  __device__ void kill(uint32_t k) { const uint32_t q = rs + k; atomicOr(&del[q >> 5], 1u << (q & 31)); }
};

template <typename A>
__device__ void replay_run(const uint8_t* run, A& al) {
  const uint32_t n = al.n;
  for (int k = 0; k < 14; k++) {
    const uint32_t p0 = c_pat[k][0], p1 = c_pat[k][1], sp = c_pat[k][2];
    uint32_t i = al.next(0xFFFFFFFFu);
    while (i < n) {
      const uint32_t j = al.next(i);
      if (j >= n) break;
      if (run[i] == p0 && run[j] == p1) {
        al.kill(sp == 1 ? i : j);
        i = al.next(j);
      } else {
        i = j;
      }
    }
  }
  // " - " -> "-"
  uint32_t i = al.next(0xFFFFFFFFu);
  while (i < n) {
    const uint32_t j = al.next(i);
    if (j >= n) break;
    const uint32_t l = al.next(j);
    if (l >= n) break;
    if (run[i] == ' ' && run[j] == '-' && run[l] == ' ') {
      al.kill(i);
      al.kill(l);
      i = al.next(l);
    } else {
      i = j;
    }
  }
}

__global__ __launch_bounds__(256) void k_dec_runs(DecWork w) {
  __shared__ uint32_t s_bits[kWinWords];
  __shared__ uint32_t s_d;
  const uint32_t ts = blockIdx.x * kDecTile;
  const uint32_t ws = ts >= (uint32_t)kHalo ? ts - kHalo : 0u;
  build_bounds(w.raw_off, w.n_docs, ws, s_bits, &s_d);
  const Bounds bd{w.raw_off, w.n_docs, ws, s_bits};
  const uint32_t p0 = ts + threadIdx.x * kDecPer;
  for (uint32_t k = 0; k < (uint32_t)kDecPer; k++) {
    const uint32_t p = p0 + k;
    if (p >= w.n_raw) break;
    if (!is_set_byte(w.raw[p])) continue;
    if (!bd.at(p) && is_set_byte(w.raw[p - 1])) continue;  // not a run start
    uint32_t e = p + 1;
    while (e < w.n_raw && !bd.at(e) && is_set_byte(w.raw[e])) e++;
    const uint32_t n = e - p;
    if (n < 2) continue;
    if (n <= 64) {
      RegAlive al{n == 64 ? ~0ull : ((1ull << n) - 1), n};
      replay_run(w.raw + p, al);
      const uint64_t dead = ~al.m & (n == 64 ? ~0ull : ((1ull << n) - 1));
      for (uint32_t q = 0; q < n; q++)
        if ((dead >> q) & 1ull) atomicOr(&w.delbits[(p + q) >> 5], 1u << ((p + q) & 31));
    } else {
      MemAlive al{w.delbits, p, n};
      replay_run(w.raw + p, al);
    }
  }
}

hipError_t launch_dec_prepare(const DecWork& w, hipStream_t s) {
  if (!(w.opts & kDecOptCleanup) || !w.n_raw) return hipSuccess;
  // runs first: a run longer than 64 bytes keeps its replay state in delbits, which must hold
  // only that run's own deletions while it is replayed
  k_dec_runs<<<w.n_tiles, 256, 0, s>>>(w);
  HIPCHK(hipGetLastError());
  k_dec_trim<<<(w.n_docs + 255) / 256, 256, 0, s>>>(w);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// K5 / K6: output bytes per input byte, counted per tile, then written.
// emit(p) = count | first byte << 8 (count 3 = U+FFFD).

__device__ __forceinline__ uint32_t dec_emit(const DecWork& w, const Bounds& bd, uint32_t p, bool cl) {
  const uint8_t* raw = w.raw;
  const uint32_t b = raw[p];
  if (b < 0x80) {
    if (!cl) return 1 | (b << 8);
    const bool ws = (b >= 0x09 && b <= 0x0D) || b == 0x20;
    if (!ws) return 1 | (b << 8);
  }
  const uint32_t u0 = unit_start(raw, bd, p);
  const uint32_t u = unit_at(raw, bd, u0);
  const bool valid = u & 0x100;
  if (u0 != p) {  // inside a unit
    if (!valid) return 0;
    if (cl && unit_is_ws(raw, u0, u & 0xFF)) return 0;
    return 1 | (b << 8);
  }
  if (!valid) return 3 | (0xEFu << 8);
  if (!cl || !unit_is_ws(raw, p, u & 0xFF)) return 1 | (b << 8);
  // a white-space unit: one ' ' if it is the first surviving unit of its run
  if (del_at(w.delbits, p)) return 0;
  uint32_t q = p;
  for (;;) {
    if (bd.at(q)) return 0;
    const uint32_t v0 = unit_start(raw, bd, q - 1);
    if (del_at(w.delbits, v0)) { q = v0; continue; }
    const uint32_t v = unit_at(raw, bd, v0);
    return ((v & 0x100) && unit_is_ws(raw, v0, v & 0xFF)) ? 0u : (1u | (0x20u << 8));
  }
}

template <bool kWrite>
__global__ __launch_bounds__(256) void k_dec_emit(DecWork w, uint8_t* __restrict__ out, uint64_t* __restrict__ out_off) {
  __shared__ uint32_t s_bits[kWinWords];
  __shared__ uint32_t s_d;
  __shared__ uint32_t sh[4];
  __shared__ uint16_t s_pre[kWrite ? kDecTile + 1 : 1];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[kWrite ? 3 * kDecTile + 32 : 16];
  const uint32_t ts = blockIdx.x * kDecTile;
  const uint32_t ws = ts >= (uint32_t)kHalo ? ts - kHalo : 0u;
  build_bounds(w.raw_off, w.n_docs, ws, s_bits, &s_d);
  const Bounds bd{w.raw_off, w.n_docs, ws, s_bits};
  const bool cl = w.opts & kDecOptCleanup;
  const uint32_t p0 = ts + threadIdx.x * kDecPer;
  uint32_t em[kDecPer];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < kDecPer; k++) {
    const uint32_t p = p0 + k;
    em[k] = p < w.n_raw ? dec_emit(w, bd, p, cl) : 0u;
    sum += em[k] & 0xFF;
  }
  uint32_t tot;
  const uint32_t ex = dec_block_scan(sum, sh, &tot);
  if (!kWrite) {
    if (threadIdx.x == 0) w.tile_cnt[blockIdx.x] = tot;
    return;
  }
  const uint32_t gbase = w.tile_cnt[blockIdx.x];
  const uint32_t a = gbase & 15;
  uint32_t r = ex;
#pragma unroll
  for (int k = 0; k < kDecPer; k++) {
    s_pre[threadIdx.x * kDecPer + k] = (uint16_t)r;
    const uint32_t c = em[k] & 0xFF;
    if (c == 1) s_stage[a + r] = (uint8_t)(em[k] >> 8);
    else if (c == 3) { s_stage[a + r] = 0xEF; s_stage[a + r + 1] = 0xBF; s_stage[a + r + 2] = 0xBD; }
    r += c;
  }
  if (threadIdx.x == 0) s_pre[kDecTile] = (uint16_t)tot;
  __syncthreads();
  store_staged(s_stage, a, tot, out + (gbase - a));
  // docs starting in this tile (raw_off == n_raw belongs to the last tile)
  const uint64_t end = blockIdx.x + 1 == w.n_tiles ? (uint64_t)w.n_raw + 1 : (uint64_t)ts + kDecTile;
  if (threadIdx.x == 0) s_d = lower_bound_u64(w.raw_off, w.n_docs, ts);
  __syncthreads();
  for (uint32_t d = s_d + threadIdx.x; d <= w.n_docs; d += 256) {
    const uint64_t o = w.raw_off[d];
    if (o >= end) break;
    out_off[d] = (uint64_t)gbase + s_pre[o - ts];
  }
}

hipError_t launch_dec_count(const DecWork& w, uint32_t* tmp, uint64_t tmp_cap, hipStream_t s) {
  if (w.n_tiles) {
    k_dec_emit<false><<<w.n_tiles, 256, 0, s>>>(w, nullptr, nullptr);
    HIPCHK(hipGetLastError());
  }
  return scan_u32(w.tile_cnt, w.tile_cnt, w.n_tiles, nullptr, tmp, tmp_cap, s);
}

hipError_t launch_dec_write(const DecWork& w, uint8_t* out, uint64_t* out_off, hipStream_t s) {
  if (w.n_tiles) k_dec_emit<true><<<w.n_tiles, 256, 0, s>>>(w, out, out_off);
  return hipGetLastError();
}

}  // namespace ctok_dev
