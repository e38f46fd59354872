// HIP kernels (gfx950 / CDNA4) for the batch ByteLevel-BPE encode path.
//
// Reference path (Complexity-ML/complexity-tokenizer v0.3.3):
//   HuggingFaceTokenizer::encode_batch   src/huggingface/mod.rs:694-696
//   -> encode                            src/huggingface/mod.rs:551-613
//      NFC                               src/normalizers.rs:47
//      byte_level_pretokenize            src/pretokenizers.rs:158-185 (GPT2_PATTERN :11-15)
//      added-token split                 src/huggingface/mod.rs:566-675
//      BpeTokenizer::encode              src/bpe.rs:88-153
//
// Data layout in HBM (all offsets u32: one call covers < 4 GiB of text):
//   text[B] u8, doc_off[D+1] u64 (input) ->
//   tfirst (each tile's first document) ->
//   pbits: 1 bit per byte (piece start), 4 KiB tiles of 64 64-byte words ->
//   per tile: wpref (pieces before each word), class lists of pieces still to merge, prec[j]
//   (record of piece j: a whole-piece hit's id, u16 on narrow vocabularies), pdoc, tile_np,
//   tile_tok ->
//   per tile: scratch (the merged pieces' ids, by length-class region), mrec[k] (count and place
//   of the tile's k-th merged piece), tile_tok scanned to each tile's first id ->
//   ids[T] u32 + tok_off[D+1] u64 (output).
// No array is indexed by a global piece number, so no pass has to wait for a global piece count.
//
// The regex of GPT2_PATTERN is evaluated as a "piece starts here" predicate over code-point
// classes {White_Space, L, N, other} (derivation in DESIGN.md), bit-parallel on 64-bit masks.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <type_traits>

#include "ctok_internal.h"
#include "seg_lane.h"

namespace ctok_dev {

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

// A kernel launch with Lx's start / stop events (recorded by its own dispatch) through
// hipExtLaunchKernel, or a plain launch when it has none.
template <typename F, typename... A>
static void launch_lx(const Lx& x, F k, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, A... a) {
  if (x.start || x.stop)
    hipExtLaunchKernelGGL(k, grid, block, lds, s, x.start, x.stop, 0u, a...);
  else
    hipLaunchKernelGGL(k, grid, block, lds, s, a...);
}

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kDead = 0xFFFFFFFFu;
constexpr uint32_t kSel = kNoRank - 1;  // marks a merge site during a parallel round

// ------------------------------------------------------------------------------------------
// small device helpers

// The call's report (Work::report; one wave, after k_segment has completed): the counters, with
// the class-3 shards summed into counters[kCtrC3Count], into the pinned host words, a
// system-scope release, then the call's sequence number (see k_report).
__device__ __forceinline__ void write_report(const Work& w) {
  const uint32_t lane = threadIdx.x & 63;
  // the class-3 shards (kC3Shards == 64: one per lane): their exclusive prefix into c3pre for
  // k_bpe_sparse, their sum into the report (all ones when a shard overflowed its capacity)
  uint32_t c3 = 0;
  if (w.c3_max) {
    const uint32_t c = w.counters[kNumCounters + lane];
    uint32_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = (uint32_t)__shfl_up((int)inc, o, 64);
      if (lane >= (uint32_t)o) inc += v;
    }
    w.c3pre[lane] = inc - c;
    if (lane == 63) w.c3pre[64] = inc;
    c3 = __shfl((int)inc, 63, 64);
    if (__ballot(c > w.c3_max / kC3Shards)) c3 = ~0u;
  }
  if (lane < (uint32_t)kNumCounters) w.report[lane] = lane == (uint32_t)kCtrC3Count ? c3 : w.counters[lane];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(&w.report[kNumCounters], w.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (and the sequence number itself on its way)
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Wave minimum in uniform control flow (all 64 lanes active): DPP within each row of 16 (quad
// swaps, half-row and row mirrors, fused into v_min), then the four row minima through
// readlane.  About 10 instructions and no LDS round trip, against six ds_bpermute waits for the
// shuffle form above; the long-piece rounds are latency-bound, with two reductions per round.
__device__ __forceinline__ uint32_t wave_min_full_u32(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));   // lane ^ 1
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));   // lane ^ 2
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return min(min(a, b), min(c, d));
}

// Wave sum in uniform control flow, the same DPP row reduction as wave_min_full_u32.
__device__ __forceinline__ uint32_t wave_sum_full_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);   // lane ^ 1
  v += (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);   // lane ^ 2
  v += (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// u32 inclusive wave scan in uniform control flow (all 64 lanes active): DPP row shifts within
// each row of 16, then row broadcasts 15 / 31 -- six fused v_add, against six ds_bpermute round
// trips for the shuffle form (k_segment's and k_emit's per-round scans are on their critical
// paths).  Preferred over the template for u32 arguments.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ uint32_t lane63(uint32_t v) { return __builtin_amdgcn_readlane(v, 63); }

// block-wide exclusive scan; nthreads = blockDim.x (multiple of 64, <= 1024)
template <typename T>
__device__ T block_excl_scan(T v, T* smem /*[17]*/, T* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) smem[wid] = inc;
  __syncthreads();
  if (wid == 0) {
    T s = lane < nw ? smem[lane] : T(0);
    T si = wave_incl_scan(s);
    if (lane < nw) smem[lane] = si - s;
    if (lane == nw - 1) smem[16] = si;
  }
  __syncthreads();
  T r = inc - v + smem[wid];
  if (total) *total = smem[16];
  __syncthreads();
  return r;
}

// Wave-uniform values are moved to SGPRs with readfirstlane: the loop exits and the chain walk
// then branch on scalars, so the wave can never split around the cross-lane reductions (a split
// wave reduces over inactive lanes and never terminates).
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Range checks of decoded piece records (opt-in build: -DCTOK_CHECK, tools/build_variant.sh):
// a record out of range prints where it was found and traps, instead of steering a gather
// through garbage offsets (round 5's r05_v12 fault: unwritten merged records).  The host then
// also fills mrec with all ones before each call, so a record no pass wrote is out of range too.
#ifdef CTOK_CHECK
#define CTOK_CHECK_REC(cond, ...)                                                            \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      printf(__VA_ARGS__);                                                                 \
      __builtin_trap();                                                                    \
    }                                                                                      \
  } while (0)
#else
#define CTOK_CHECK_REC(cond, ...) do { } while (0)
#endif

// Diagnostic (CTOK_WGREC=1, Work::wgrec non-null): workgroup `blockIdx.x` of kernel slot k records
// its start and end (wall clock, 100 MHz), its CU (xcc | se | cu) and a count.  The host prints,
// per kernel, the CUs used and the spread of the workgroups' starts and ends (ctok_host.cpp).
constexpr uint32_t kWgRecMax = 1024;  // (4 kernel slots: short, mid<2>, mid<3>, sparse)
// (stateless: the record's place is recomputed at the end from the kernel argument, so that no
// register stays live across the kernel -- the 64-slot pass is at its register limit)
struct WgRec {
  static __device__ __forceinline__ void begin(uint64_t* base, uint32_t k) {
    if (base && threadIdx.x == 0 && blockIdx.x < kWgRecMax) {
      uint64_t* p = base + ((size_t)k * kWgRecMax + blockIdx.x) * 4;
      p[0] = (uint64_t)wall_clock64();
      p[2] = __smid();
    }
  }
  static __device__ __forceinline__ void end(uint64_t* base, uint32_t k, uint32_t count) {
    if (base && threadIdx.x == 0 && blockIdx.x < kWgRecMax) {
      uint64_t* p = base + ((size_t)k * kWgRecMax + blockIdx.x) * 4;
      p[1] = (uint64_t)wall_clock64();
      p[3] = count;
    }
  }
};

// NFC speculation failed in k_segment (a code point NFC might change): the rest of this pass is
// discarded (the host checks, normalises and runs the pipeline again), so the kernels after
// k_segment return at once instead of merging text that will be re-encoded.
__device__ __forceinline__ bool spec_failed(const Work& w) { return w.nfc_watch == 1 && uni(w.counters[12]) != 0; }

// pieces in the long list (k_segment counts them all; past long_cap they were not stored and the
// host reruns the call with the safe capacities)
__device__ __forceinline__ uint32_t long_count(const Work& w) { return min(w.counters[0], w.long_cap); }

// wave-aggregated append to an LDS counter: returns this lane's slot (lanes with take == false
// get garbage).  One ds_add per wave instead of one per lane.
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool take) {
  const uint64_t m = __ballot(take);
  uint32_t base = 0;
  if (m) {
    const uint32_t leader = __ffsll((unsigned long long)m) - 1;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t b = 0;
    if (lane == leader) b = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __builtin_amdgcn_readlane(b, leader);
  }
  return base + (uint32_t)__popcll(m & lanemask_lt());
}

__device__ __forceinline__ int u8len(uint8_t b) {
  return b < 0x80 ? 1 : (b >> 5) == 6 ? 2 : (b >> 4) == 14 ? 3 : 4;
}

__device__ __forceinline__ int cls_ascii(uint32_t c) {
  // 0 White_Space, 1 letter, 2 number, 3 other
  if (c == 32 || (c >= 9 && c <= 13)) return 0;
  if ((c | 32) >= 'a' && (c | 32) <= 'z') return 1;
  if (c >= '0' && c <= '9') return 2;
  return 3;
}

__device__ __forceinline__ int cls_of(uint32_t cp, const Tables& t) {
  if (cp < 0x80) return cls_ascii(cp);
  if (cp >= 0x110000) return 3;
  const uint32_t blk = t.cls_s1[cp >> 8];
  const uint32_t w = t.cls_s2[blk * 64 + ((cp & 255) >> 2)];
  return (w >> ((cp & 3) * 2)) & 3;
}


// A long-piece round of merge value r applies every occurrence of r at once, except when the table
// is not rank-monotone and r's merge is eager (Tables::eager): then the leftmost one alone, as the
// sequential loop would before a lower-ranked merge the first one enables.  (Wave-uniform r: a
// scalar load.)
__device__ __forceinline__ bool serial_round(const Tables& t, uint32_t r) {
  return !t.proper && ((t.eager[r >> 5] >> (r & 31)) & 1u) != 0;
}
// first_cascade (the rounds of an eager merge): the sequential loop takes the sites of rank r left
// to right, and after each one the pairs it made -- (the left neighbour, or nid when the site two
// tokens before was merged just before; nid) and (nid, the next token as it is) -- compete with the
// remaining sites.  While none of them ranks below r it goes on with the next site; the first site
// that makes a lower-ranked pair is the last one it applies before that pair's merge.  So a round
// applies the sites up to and including the first such one (all of them when there is none), which
// is the sequential result for any merge table; the lookups of this check never set the panic flag
// (they go to a sink counter): a pair they see is formed, and looked up again, only if its site is
// applied.  (x, x) runs of an eager merge take the leftmost site alone.

// Merge-table value of an entry: the merge priority.  Compact tables (new ids strictly increasing
// in rank, the usual layout) store the merged token id itself, so the minimum value is both the
// winning pair and its new id; otherwise the rank is stored and the new id is looked up.
__device__ __forceinline__ bool value_panics(const Tables& t, uint32_t v) {
  return t.compact ? v == kPanicVal : v >= t.n_ranks;
}
__device__ __forceinline__ uint32_t new_id_of(const Tables& t, uint32_t v) {
  return t.compact ? v : t.rank_newid[v];
}

// value of pair (a, b) or kNoRank.  Sets the panic bit when the reference would index
// BpeTokenizer.merges out of range (src/bpe.rs:141).
__device__ __forceinline__ uint32_t rank_of(const Tables& t, uint32_t a, uint32_t b, uint32_t* err) {
  const uint64_t key = ((uint64_t)a << kIdBits) | b;
  uint32_t h = mhash(a, b) & t.merge_mask;
  for (;;) {
    const uint64_t e = t.merge_tab[h];
    if ((e & kKeyMask) == key) {
      const uint32_t r = (uint32_t)(e >> 42);
      if (value_panics(t, r)) { atomicOr(err, kErrPanic); return kNoRank; }
      return r;
    }
    if (e == kEmpty) return kNoRank;
    h = (h + 1) & t.merge_mask;
  }
}

// ------------------------------------------------------------------------------------------
// doc-start bitmap

// Each tile's first document (k_segment finds the doc starts of its 64 words from it): tfirst[t] =
// the first doc d with doc_off[d] >= the tile's context word (t * kTile - 64), written by thread d
// for the tiles whose context word lies in (doc_off[d - 1], doc_off[d]] -- at most 64 of them
// (a document over ~250 KB leaves the rest at ~0 from k_clear, and k_segment searches for those);
// and the empty documents, counted into counters[kCtrEmptyDocs] (one atomic per wave).  It
// replaces a doc-start bitmap of n_bytes / 8 bytes, zeroed, written and read back every call.
__global__ __launch_bounds__(256) void k_tilefirst(const uint64_t* __restrict__ off, uint32_t n_docs, uint32_t n_tiles,
                                                   uint32_t* __restrict__ tfirst, uint32_t* __restrict__ counters) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  bool empty = false;
  if (d <= n_docs && n_tiles) {
    const uint64_t y = off[d];
    empty = d < n_docs && y == off[d + 1];
    // tiles t with off[d - 1] < t * kTile - 64 <= y (d = 0: every t with t * kTile - 64 <= y)
    const uint64_t t_lo = d ? (off[d - 1] + 64) / kTile + 1 : 0ull;
    const uint64_t t_hi = min((y + 64) / kTile, (uint64_t)n_tiles - 1);
    for (uint64_t t = t_lo; t <= t_hi && t < t_lo + 64; t++) tfirst[t] = d;
  } else if (d < n_docs) {
    empty = off[d] == off[d + 1];
  }
  const uint64_t me = __ballot(empty);
  if (me && (threadIdx.x & 63) == (uint32_t)__ffsll((unsigned long long)me) - 1)
    atomicAdd(&counters[kCtrEmptyDocs], (uint32_t)__popcll(me));
}

// The same for one tile, by bisection (k_segment: a tile whose context word lies inside a document
// longer than k_tilefirst's 64 tiles).  Wave-uniform.
__device__ uint32_t tile_first_search(const uint64_t* off, uint32_t n_docs, uint32_t tile) {
  const uint64_t key = tile ? (uint64_t)tile * kTile - 64 : 0ull;
  uint32_t lo = 0, hi = n_docs;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (__builtin_amdgcn_readfirstlane((uint32_t)(off[mid] < key))) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Zeroes the call's counters (when asked) and the NFC watch bitmap (nfc_watch 2) in one launch.
__device__ __forceinline__ void clear_words(uint32_t* __restrict__ p, uint64_t n) {
  const uint64_t n4 = n / 4;
  uint4* p4 = reinterpret_cast<uint4*>(p);  // (hipMalloc'd: 256-byte aligned)
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256)
    p4[i] = make_uint4(0u, 0u, 0u, 0u);
  if (blockIdx.x == 0 && threadIdx.x < n - 4 * n4) p[4 * n4 + threadIdx.x] = 0u;
}

__global__ __launch_bounds__(256) void k_clear(uint32_t* __restrict__ bits, uint64_t n, uint32_t* __restrict__ counters,
                                               uint32_t* __restrict__ tfirst, uint32_t n_tiles) {
  if (bits) clear_words(bits, n);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n_tiles; i += gridDim.x * 256) tfirst[i] = ~0u;
  if (blockIdx.x == 0 && counters && threadIdx.x < (uint32_t)kCounterWords) counters[threadIdx.x] = 0u;
}

uint64_t nfc_bits_words(uint64_t n_bytes) { return (n_bytes + 2047) / 2048 + 8; }

hipError_t launch_docstart(const Work& w, hipStream_t s, bool zero_counters, Lx x, Lx x2) {
  const bool nfc = w.nfc_watch == 2;
  const uint64_t n = nfc ? nfc_bits_words(w.n_bytes) : 0;
  const uint64_t work = std::max<uint64_t>(n / 4, w.n_tiles);
  launch_lx(x, k_clear, (unsigned)std::min<uint64_t>((work + 255) / 256 + 1, 8ull * w.n_cus), 256, 0, s,
            nfc ? w.nfc_bits : nullptr, n, zero_counters ? w.counters : nullptr, w.tfirst, w.n_tiles);
  if (w.n_tiles) launch_lx(x2, k_tilefirst, (w.n_docs + 1 + 255) / 256, 256, 0, s, w.doc_off, w.n_docs, w.n_tiles, w.tfirst, w.counters);
  else if (w.n_docs)  // (no text: only the empty-document count)
    k_tilefirst<<<(w.n_docs + 255) / 256, 256, 0, s>>>(w.doc_off, w.n_docs, 0, w.tfirst, w.counters);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// pre-tokenizer: piece-start bitmap, bit-parallel, one 64-byte word per lane (k_segment below;
// the per-word logic is csrc/seg_lane.h).  Positions >= n_bytes read as doc starts (D), which
// closes every run at the end of the text.

__device__ __forceinline__ uint16_t nfc16(const Tables& t, uint32_t cp) {
  if (cp >= 0x110000) return 0;
  return t.nfc_s2[t.nfc_s1[cp >> 8] * 256 + (cp & 255)];
}

// Neighbour lanes' words (k_segment: lane l needs lanes l - 1 and l + 1), by DPP wave shifts
// (wave_shr:1 / wave_shl:1, GFX9) instead of ds_bpermute: lane 0 (shr) and lane 63 (shl) keep
// their own value, as __shfl_up / __shfl_down leave it.  Uniform control flow only.
__device__ __forceinline__ uint32_t dpp_prev(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x130, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v) {
  return (uint64_t)dpp_prev((uint32_t)v) | ((uint64_t)dpp_prev((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ uint64_t shfl_down64(uint64_t v) {
  return (uint64_t)dpp_next((uint32_t)v) | ((uint64_t)dpp_next((uint32_t)(v >> 32)) << 32);
}

// Bytes s .. s + 4*NW - 1 of the text as NW little-endian words, read with NW + 1 aligned dword
// loads whose addresses are clamped into the buffer: every load is unconditional (a predicated
// per-byte load makes hipcc branch and wait vmcnt(0) around each one); bytes past the piece or the
// text are garbage and must be masked by the caller.
template <int NW>
__device__ __forceinline__ void load_words(const uint8_t* text, uint32_t s, uint32_t n_bytes, uint32_t (&wv)[NW]) {
  const uint32_t a0 = s & ~3u;
  const uint32_t last = (n_bytes - 1) & ~3u;
  uint32_t d[NW + 1];
#pragma unroll
  for (int j = 0; j <= NW; j++) d[j] = *reinterpret_cast<const uint32_t*>(text + min(a0 + 4 * j, last));
  const uint32_t sh = s & 3u;
#pragma unroll
  for (int j = 0; j < NW; j++) wv[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
}

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int k) { return (w >> (8 * (k & 3))) & 255u; }




// Whole-piece table lookup given the first probed slot e (at h): the vocab id, or kNone.
__device__ __forceinline__ uint32_t piece_probe(const Tables& t, uint4 e, uint32_t h, uint32_t lo, uint32_t hi,
                                                uint32_t n) {
  while (e.z != 0) {  // linear probing past the first slot (rare)
    if (e.x == lo && e.y == hi && e.z == n) return e.w;
    h = (h + 1) & t.piece_mask;
    e = t.piece_tab[h];
  }
  return kNone;
}

// position of the k-th (0-based) set bit of x (k < popcount(x))
__device__ __forceinline__ uint32_t select_bit(uint64_t x, uint32_t k) {
  uint32_t pos = 0;
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t c = __popc(lo);
  uint32_t v = lo;
  if (k >= c) { k -= c; v = hi; pos = 32; }
#pragma unroll
  for (int wdt = 16; wdt >= 1; wdt >>= 1) {
    const uint32_t m = (1u << wdt) - 1u;
    c = __popc(v & m);
    if (k >= c) { k -= c; v >>= wdt; pos += wdt; }
  }
  return pos;
}




// One wavefront per tile, kSegWaves tiles per workgroup, no workgroup barrier.  Lane l owns the
// 64-byte word g0 - 1 + l: lane 0 is the previous tile's last word (context only), lanes 1..62
// are the tile's words, lane 63 is the next tile's first word (look-ahead: where the tile's last
// piece ends; its bits 62-63 depend on a word no lane holds and are not used).
//  A. per lane: the word's class / byte masks by SWAR tests (csrc/seg_lane.h); non-ASCII code
//     points classified per code point; doc starts from the doc bitmap;
//  B. per lane: the piece-start predicate, the neighbouring words' masks by cross-lane shuffles;
//  C. thread per piece (piece j = the j-th start of the tile): length from the next start, then
//     routing: a piece of <= 8 bytes that is one self-encoding vocab token is finished here with
//     one whole-piece probe; every other piece is appended to its tile's class list (<= 8 B,
//     9..16 B, 17..32 B) or to the long list, so that the merge passes run dense, length-uniform
//     waves.
// (amdgpu_waves_per_eu(7): at most 72 VGPRs, 7 waves per SIMD; without it the compiler takes 72-73
// and this kernel runs at 6-7; C4 k_segment 2.78 -> 2.67 ms, 8 waves spill: 2.96 ms,
// profiles/r03/v30_ab_seg_waves_per_eu.txt)
// Diagnostic build only (-DCTOK_SEG_STAMPS): shader-clock stamps at k_segment's phase boundaries,
// one row of 8 u64 per tile in Work::stamps (read by the host with CTOK_STAMPS=1); the production
// build executes none.  Read the phases' shares, not the build's run time.
#ifdef CTOK_SEG_STAMPS
#define SEG_STAMP(k)                                                                              \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long t_;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                     \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (w.stamps && lane == 0) w.stamps[(size_t)tile * 8 + (k)] = t_;                            \
  } while (0)
#else
#define SEG_STAMP(k) do { } while (0)
#endif
// R16: u16 piece records (Work::rec16); a template parameter, not a branch on the flag: both store
// paths in one kernel cost 18 more spilled SGPRs
template <bool R16>
__global__ __launch_bounds__(64 * kSegWaves) __attribute__((amdgpu_waves_per_eu(7))) void k_segment(Work w, Tables t) {
  __shared__ uint16_t s_pos_all[kSegWaves][64 * kSegUnroll + 8];  // one round's piece starts
  // per wave: 3 spare words, the 4 bytes before the context word, the context word, the tile, the
  // look-ahead word, the 4 bytes after it, 3 spare words (rows of 1032 words: every lane's 64-byte
  // word starts 16-byte aligned for its four 16-byte stores)
  __shared__ __attribute__((aligned(16))) uint32_t s_text_all[kSegWaves][(kTileWords + 2) * 16 + 8];
  __shared__ uint64_t s_D_all[kSegWaves][64];
  constexpr uint32_t kSegLongCap = 32;  // long pieces staged per tile (the list entries)
  __shared__ uint64_t s_long_all[kSegWaves][kSegLongCap];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = uni(threadIdx.x >> 6);
  const uint32_t tile = uni(blockIdx.x * kSegWaves + wid);
  if (tile >= w.n_tiles) return;
  uint16_t* s_pos = s_pos_all[wid];
  SEG_STAMP(0);
  const uint32_t B = w.n_bytes;
  const uint32_t t0 = tile * kTile;
  const int64_t g = (int64_t)tile * kTileWords - 1 + lane;  // this lane's word
  const bool first = lane == 0, last = lane == 63;

  // ---- A
  uint32_t x[16];
  uint64_t D, valid;
  {
    const int64_t x0 = g * 64;
    if (x0 >= 0 && x0 + 64 <= (int64_t)B) {
      const uint4* p = reinterpret_cast<const uint4*>(w.text + x0);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint4 v = p[k];
        x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
      }
      valid = ~0ull;
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) x[k] = 0;
      valid = 0;
      if (x0 >= 0 && x0 < (int64_t)B) {  // the text's last, partial word
        const uint32_t n = B - (uint32_t)x0;
        valid = (1ull << n) - 1;
        for (uint32_t i = 0; i < n; i++) x[i >> 2] |= (uint32_t)w.text[x0 + i] << (8 * (i & 3));
      }
    }
  }
  // the first 64 documents from the tile's first (k_tilefirst), loaded right behind the text
  // (their starts give the doc-start bits below; the mask work on the text runs meanwhile)
  uint32_t dfirst = uni(w.tfirst[tile]);
  if (dfirst == ~0u) dfirst = tile_first_search(w.doc_off, w.n_docs, tile);  // (inside a document > 250 KB)
  uint64_t xs0 = ~0ull, ys0 = ~0ull;
  if (dfirst + lane < w.n_docs) {
    xs0 = w.doc_off[dfirst + lane];
    ys0 = w.doc_off[dfirst + lane + 1];
  }
  seg::Masks m = seg::ascii_masks(x);
  {  // doc-start bits of the 64 words [base, base + 4096): the non-empty documents starting there,
     // from the tile's first document on (k_tilefirst), 64 at a time (C4: one round)
    uint64_t* s_D = s_D_all[wid];
    s_D[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint64_t base = (uint64_t)t0 - 64;  // (tile 0: -64, wrapping; the sums below wrap back)
    const uint64_t lim = (uint64_t)t0 + 4032;  // the window's end
    auto mark = [&](uint64_t xs, uint64_t ys) {  // (xs = ~0: no document)
      const bool in = xs < lim;
      if (in && xs != ys) {
        const uint64_t r = xs - base;
        atomicOr((unsigned long long*)&s_D[r >> 6], 1ull << (r & 63));
      }
      return in;
    };
    if (__ballot(mark(xs0, ys0)) == ~0ull) {  // every lane's doc started inside: look further (rare)
      for (uint32_t d = dfirst + 64;; d += 64) {
        const uint32_t i = d + lane;
        uint64_t xs = ~0ull, ys = ~0ull;
        if (i < w.n_docs) {
          xs = w.doc_off[i];
          ys = w.doc_off[i + 1];
        }
        if (__ballot(mark(xs, ys)) != ~0ull) break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t x0 = g * 64;
    if (x0 < 0) D = 0;
    else if (x0 >= (int64_t)B) D = ~0ull;
    else D = s_D[lane] | ~valid;
  }
  s_D_all[wid][lane] = D;
  // every lane's word in LDS: the tile's bytes (and the look-ahead word) for the whole-piece
  // probes (s_text: the tile's first byte), the context word too for the code point decoding below
  uint32_t* s_all = s_text_all[wid] + 4;  // (s_all[-1]: the 4 bytes before the context word)
  uint32_t* s_text = s_all + 16;
  // the context word's first code point can start in the word before it (its first byte is a
  // continuation byte): the 4 bytes before it
  if (first && (x[0] & 0xC0u) == 0x80u && g * 64 >= 4)
    s_all[-1] = *reinterpret_cast<const uint32_t*>(w.text + g * 64 - 4);
#pragma unroll
  for (int k = 0; k < 4; k++)
    *reinterpret_cast<uint4*>(s_all + lane * 16 + 4 * k) = make_uint4(x[4 * k], x[4 * k + 1], x[4 * k + 2], x[4 * k + 3]);
  if (last) {  // the 4 bytes after the look-ahead word: a code point starting in its last bytes
               // runs into them (zero past the text)
    const int64_t xe = g * 64 + 64;
    uint32_t v = 0;
    if (xe + 4 <= (int64_t)B) {
      v = *reinterpret_cast<const uint32_t*>(w.text + xe);
    } else {
      for (int64_t i = xe; i < (int64_t)B && i < xe + 4; i++) v |= (uint32_t)w.text[i] << (8 * (uint32_t)(i - xe));
    }
    s_all[64 * 16] = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  SEG_STAMP(1);
  if (m.NA) {  // non-ASCII code points: classes and NFC flags from the two-level tables
    constexpr int kSegCp = 4;
    bool nfc_bad = false;
    auto set_class = [&](int cl, uint64_t bits) {
      if (cl == 0) m.W |= bits & m.NA;
      else if (cl == 1) m.L |= bits & m.NA;
      else if (cl == 2) m.N |= bits & m.NA;
    };
    // continuation bytes (10xxxxxx), SWAR over the word's dwords
    uint64_t cont = 0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
      const uint32_t c0 = x[k] & ~(x[k] << 1) & seg::kHi, c1 = x[k + 1] & ~(x[k + 1] << 1) & seg::kHi;
      cont |= (uint64_t)seg::pack8(c0, c1) << (4 * k);
    }
    cont &= m.NA;
    const uint64_t lead_cont = cont & ~(cont + 1);  // continuation bytes at the start of the word
    if (lead_cont) {  // a code point whose lead is in the previous word: classified on its own
      // the bytes before this word are staged just before it (the previous lane's word, or for
      // the context word s_all[-1]): the lead is 1..3 bytes back (at most 3 steps back, as a
      // walk over the text would take)
      const uint32_t pw = s_all[lane * 16 - 1];  // bytes x0 - 4 .. x0 - 1
      const int32_t back = ((pw >> 24) & 0xC0u) != 0x80u ? 1 : ((pw >> 16) & 0xC0u) != 0x80u ? 2 : 3;
      const int32_t a = (int32_t)lane * 64 - back;  // byte address in s_all (-3 .. -1 for the context word)
      const uint32_t v = __builtin_amdgcn_alignbyte(s_all[(a >> 2) + 1], s_all[a >> 2], (uint32_t)a & 3u);
      const uint32_t b0 = v & 255u, b1 = (v >> 8) & 0x3Fu, b2 = (v >> 16) & 0x3Fu, b3 = (v >> 24) & 0x3Fu;
      const int l = u8len((uint8_t)b0);
      const uint32_t c = l == 2 ? ((b0 & 0x1Fu) << 6) | b1
                       : l == 3 ? ((b0 & 0x0Fu) << 12) | (b1 << 6) | b2
                       : l == 4 ? ((b0 & 0x07u) << 18) | (b1 << 12) | (b2 << 6) | b3 : b0;
      const int rc = t.cp_fast ? cp_range_class(c) : -1;
      const int cw = rc >= 0 ? rc : (cls_of(c, t) | (nfc16(t, c) != 0 ? 4 : 0));
      nfc_bad |= (cw & 4) != 0;
      set_class(cw & 3, lead_cont);
    }
    // every other code point starts at a lead byte in this word: decoded and looked up 8 at a
    // time, so the byte loads, then both first-level table loads, then both second-level table
    // loads of the 8 are in flight together (instead of a chain of dependent loads per code point)
    uint64_t leads = m.NA & ~cont;
    while (leads) {
      uint32_t pos[kSegCp], cp[kSegCp], len[kSegCp];
#pragma unroll
      for (int k = 0; k < kSegCp; k++) {
        pos[k] = leads ? (uint32_t)__builtin_ctzll(leads) : 64u;
        leads &= leads ? leads - 1 : 0ull;
      }
#pragma unroll
      for (int k = 0; k < kSegCp; k++) {
        // the code point's bytes from LDS (this lane's word and the next: s_all is contiguous;
        // valid UTF-8 never runs past the text, whose bytes past B read as zero)
        const uint32_t a = lane * 64 + min(pos[k], 63u);
        const uint32_t v = __builtin_amdgcn_alignbyte(s_all[(a >> 2) + 1], s_all[a >> 2], a & 3);
        const uint32_t b0 = v & 255u, b1 = (v >> 8) & 0x3Fu, b2 = (v >> 16) & 0x3Fu, b3 = (v >> 24) & 0x3Fu;
        const int l = u8len((uint8_t)b0);
        len[k] = (uint32_t)l;
        cp[k] = l == 2 ? ((b0 & 0x1Fu) << 6) | b1
              : l == 3 ? ((b0 & 0x0Fu) << 12) | (b1 << 6) | b2
              : l == 4 ? ((b0 & 0x07u) << 18) | (b1 << 12) | (b2 << 6) | b3 : b0;
      }
      int rc[kSegCp];  // range-test class, -1: look it up
      uint32_t s1[kSegCp];
#pragma unroll
      for (int k = 0; k < kSegCp; k++) {
        rc[k] = t.cp_fast ? cp_range_class(cp[k]) : -1;
        const bool in = pos[k] < 64 && cp[k] < 0x110000 && rc[k] < 0;
        // BMP code points: class and NFC flag in one load from the direct table (cls_bmp); the
        // rare supplementary ones outside the fast ranges: two-level lookups in the branch below
        s1[k] = in && cp[k] < 0x10000 ? (uint32_t)t.cls_bmp[cp[k] >> 1] : 0u;
      }
#pragma unroll
      for (int k = 0; k < kSegCp; k++) {
        if (pos[k] >= 64) continue;
        const uint32_t c = cp[k];
        int cl = 3;
        bool nf = false;
        if (rc[k] >= 0) {
          cl = rc[k];
        } else if (c < 0x80) {
          cl = cls_ascii(c);
        } else if (c < 0x10000) {
          const uint32_t v = s1[k] >> ((c & 1u) * 4);
          cl = (int)(v & 3u);
          nf = (v & 4u) != 0;
        } else if (c < 0x110000) {
          cl = cls_of(c, t);
          nf = nfc16(t, c) != 0;
        }
        nfc_bad |= nf;
        const uint32_t p = pos[k];
        const uint64_t bits = (len[k] >= 64 - p ? ~0ull : ((1ull << len[k]) - 1)) << p;
        set_class(cl, bits);
      }
    }
    if (nfc_bad && w.nfc_watch) {
      atomicOr(&w.counters[12], 1u);
      if (w.nfc_watch == 2 && g >= 0) atomicOr(&w.nfc_bits[g >> 5], 1u << (g & 31));  // (splice mode only)
    }
  }
  SEG_STAMP(2);
  // contraction letters only where an apostrophe could use them (this word's or the previous
  // word's last two bytes)
  // (every lane takes part in each shuffle: a lane that is inactive at a ds_bpermute hands its
  // neighbour zeros)
  uint64_t pQ = shfl_up64(m.Q);
  if (first) pQ = 0;
  seg::Letters lt{0, 0, 0, 0, 0};
  if (m.Q | (pQ >> 62)) lt = seg::letter_masks(x, m.NA);

  // ---- B
  uint64_t st;
  {
    uint64_t pW = shfl_up64(m.W), pL = shfl_up64(m.L), pN = shfl_up64(m.N);
    if (first) pW = pL = pN = 0;
    uint64_t nW = shfl_down64(m.W), nL = shfl_down64(m.L), nD = shfl_down64(D);
    seg::Letters nl{shfl_down64(lt.T1), shfl_down64(lt.R), shfl_down64(lt.Le), shfl_down64(lt.V), shfl_down64(lt.LL)};
    if (last) {
      nW = nL = nD = 0;
      nl = seg::Letters{0, 0, 0, 0, 0};
    }
    const uint64_t A = seg::attached(m, D, pW, nW, nD);
    uint64_t pA = shfl_up64(A);
    if (first) pA = 0;
    uint64_t C1, C2;
    seg::contractions(m, lt, D, A, pA, ~(pW | pL | pN), nL, nD, nl, C1, C2);
    uint64_t pC1 = shfl_up64(C1), pC2 = shfl_up64(C2);
    if (first) pC1 = pC2 = 0;
    st = seg::starts(m, D, pW, pL, pN, A, pA, C1, C2, pC1, pC2) & valid;
    if (last) st &= (1ull << 62) - 1;
    if (!first && !last) {  // piece-start bitmap
      const uint64_t gw = (uint64_t)g * 2;
      if (gw < w.n_words) w.pbits[gw] = (uint32_t)st;
      if (gw + 1 < w.n_words) w.pbits[gw + 1] = (uint32_t)(st >> 32);
    }
  }
  // documents starting in the tile: its words' doc-start bits within the text (summed at the end)
  uint32_t nd = (!first && !last) ? (uint32_t)__popcll(D & valid) : 0u;
  const uint32_t c = (!first && !last) ? (uint32_t)__popcll(st) : 0u;
  const uint32_t inc = wave_incl_scan(c);
  if (!first && !last) w.wpref[(size_t)tile * 64 + lane - 1] = (uint16_t)(inc - c);
  const uint32_t np = lane63(inc);
  // where the tile's last piece ends (look-ahead lane): 0xFFFF = unknown (longer than the
  // look-ahead can tell: a long piece)
  const uint32_t tile_end =
      uni((uint32_t)__shfl((int)(st ? (uint32_t)(kTileWords * 64 + __builtin_ctzll(st))
                                    : ((uint64_t)B <= (uint64_t)t0 + kTile + 62 ? (uint32_t)(B - t0) : 0xFFFFu)),
                           63, 64));
  // expansion state: the starts of this lane's word and the pieces of the tile before it
  const uint64_t stw = (!first && !last) ? st : 0ull;
  const uint32_t prew = inc - c;
  uint32_t wcur = 1;  // the first word lane that can hold the next window's first piece (wave-uniform)

  SEG_STAMP(3);
  // ---- C: thread per piece, kSegUnroll pieces per lane per round with their LDS lookups and
  // table probes issued together (each round is one dependent global round trip)
  const bool generic = t.n_at != 0;  // added tokens can match inside pieces: no whole-piece shortcut
  using RecT = typename std::conditional<R16, uint16_t, uint32_t>::type;
  RecT* prec = (RecT*)w.prec + (size_t)tile * kTileSlots;
  uint32_t* pdoc = w.pdoc + (size_t)tile * (kTileSlots / 32);
  uint32_t hits = 0;
  uint32_t nm = 0;  // merged pieces so far (wave-uniform): the next ordinal
  uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0;  // class-list lengths (wave-uniform)
  uint32_t nlong = 0;  // long pieces staged in s_long_all (wave-uniform)
  uint32_t by0 = 0, by1 = 0, by2 = 0;        // this lane's bytes in class lists 0..2 (id regions)
  constexpr int U = kSegUnroll;
  constexpr uint32_t W = 64 * U;  // pieces per round
  for (uint32_t j0 = 0; j0 < np; j0 += W) {
    // expansion of this round's window [j0, j0 + W]: s_pos[j - j0] = start of piece j (the
    // entry past the window is the next round's first piece, peeked, not consumed).
    // Half-words over the lanes: lane l takes half (l & 1) of word wb + (l >> 1), 32 words per
    // pass (a window of 256 pieces spans ~18 words of English text: one pass), and walks its
    // half's set bits -- a trip count of the busiest half (~10), against ten VALU per word of
    // the round-3 word-serial walk (C4 k_segment 2.72 -> 2.66 ms, profiles/r05/v16_*).
    for (uint32_t wb = wcur;; wb += 32) {  // (wave-uniform)
      const uint32_t wl = wb + (lane >> 1), src = min(wl, 63u);
      const uint32_t lo32 = (uint32_t)__shfl((int)(uint32_t)stw, (int)src, 64);
      const uint32_t hi32 = (uint32_t)__shfl((int)(uint32_t)(stw >> 32), (int)src, 64);
      const uint32_t pw = (uint32_t)__shfl((int)prew, (int)src, 64);
      const bool hi = (lane & 1) != 0;
      uint32_t bits = wl <= (uint32_t)kTileWords ? (hi ? hi32 : lo32) : 0u;
      uint32_t k = pw + (hi ? (uint32_t)__popc(lo32) : 0u);  // piece index of the half's first start
      if (k > j0 + W || k + (uint32_t)__popc(bits) <= j0) bits = 0;  // no piece of the window
      const uint32_t pos0 = (wl - 1) * 64 + (hi ? 32u : 0u);
      while (bits) {
        const uint32_t b = (uint32_t)__builtin_ctz(bits);
        if (k >= j0 && k <= j0 + W) s_pos[k - j0] = (uint16_t)(pos0 + b);
        bits &= bits - 1u;
        k++;
      }
      const uint32_t wn = wb + 32;  // the next pass's first word: needed when it starts a piece of the window
      if (wn > (uint32_t)kTileWords || uni(__builtin_amdgcn_readlane(prew, wn)) > j0 + W) break;
    }
    {  // the last word whose first piece index is within the window (the next window starts there)
      const uint64_t inw = __ballot(lane >= wcur && lane <= (uint32_t)kTileWords && prew <= j0 + W);
      if (inw) wcur = 63u - (uint32_t)__builtin_clzll(inw);
    }

    if (lane == 0 && np <= j0 + W) s_pos[np - j0] = (uint16_t)tile_end;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t sl[U], n[U], cls[U], plo[U], phi[U], h[U], doc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t j = j0 + 64 * u + lane;
      sl[u] = 0;
      n[u] = 0;
      doc[u] = 0;
      cls[u] = 4;  // 0..2 class lists, 3 long, 4 done (or inactive), 5 probe, 6 class list 3
      if (j < np) {
        sl[u] = s_pos[64 * u + lane];
        doc[u] = (uint32_t)(s_D_all[wid][(sl[u] >> 6) + 1] >> (sl[u] & 63)) & 1u;
        const uint32_t el = s_pos[64 * u + lane + 1];
        if (el == 0xFFFFu || el - sl[u] > (generic ? (uint32_t)kShortMax : (uint32_t)kMedMax)) {
          cls[u] = 3;
        } else {
          n[u] = el - sl[u];
          cls[u] = generic ? 0 : n[u] > 32 ? 6 : n[u] > 16 ? 2 : n[u] > 8 ? 1 : 5;
        }
      }
      // whole-piece probe key: the piece's raw bytes (from LDS), zero-padded to 8
      const uint32_t a = sl[u] >> 2, sh = sl[u] & 3;
      const uint32_t d0 = s_text[a], d1 = s_text[a + 1], d2 = s_text[a + 2];
      const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
      const uint32_t nn = n[u];
      plo[u] = nn >= 4 ? w0 : w0 & ((1u << (8 * nn)) - 1u);
      phi[u] = nn >= 8 ? w1 : nn <= 4 ? 0u : w1 & ((1u << (8 * (nn - 4))) - 1u);
      // lanes without a probe read the spare empty slot past the table (one shared line)
      h[u] = cls[u] == 5 ? piece_hash(plo[u], phi[u], nn) & t.piece_mask : t.piece_mask + 1;
    }
    // all first probes in flight together (unrolled by hand: a loop over u around the probing
    // loop would not unroll, and the arrays would go to scratch)
    uint32_t hitv[U];
#define CTOK_PROBE_LOAD(u) const uint4 e##u = t.piece_tab[h[u]];
#define CTOK_PROBE_USE(u) hitv[u] = piece_probe(t, e##u, h[u], plo[u], phi[u], n[u]);
    static_assert(U == 4 || U == 8, "kSegUnroll: 4 or 8");
    CTOK_PROBE_LOAD(0) CTOK_PROBE_LOAD(1) CTOK_PROBE_LOAD(2) CTOK_PROBE_LOAD(3)
    if constexpr (U == 8) {
      CTOK_PROBE_LOAD(4) CTOK_PROBE_LOAD(5) CTOK_PROBE_LOAD(6) CTOK_PROBE_LOAD(7)
      CTOK_PROBE_USE(4) CTOK_PROBE_USE(5) CTOK_PROBE_USE(6) CTOK_PROBE_USE(7)
    }
    CTOK_PROBE_USE(0) CTOK_PROBE_USE(1) CTOK_PROBE_USE(2) CTOK_PROBE_USE(3)
#undef CTOK_PROBE_LOAD
#undef CTOK_PROBE_USE
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t j = j0 + 64 * u + lane;
      uint32_t rec = kRecMerged32;  // a later pass produces the piece's ids (its mrec slot)
      // (written as flag arithmetic: an if / else-if chain assigning cls[u] in each arm was
      // miscompiled by this hipcc in the unrolled loop)
      if (cls[u] == 5) {
        const bool hit = hitv[u] != kNone;
        rec = hit ? hitv[u] : kRecMerged32;
        hits += hit ? 1u : 0u;
        cls[u] = hit ? 4u : 0u;
      }
      // every piece's record: whole coalesced lines (u16 on narrow vocabularies)
      if (j < np) {
        prec[j] = (RecT)rec;
      }
      const uint64_t dm = __ballot(j < np && doc[u]);  // doc-start bits of the 64 pieces
      if (lane == 0 && j0 + 64 * u < np)
        *reinterpret_cast<uint2*>(pdoc + ((j0 + 64 * u) >> 5)) = make_uint2((uint32_t)dm, (uint32_t)(dm >> 32));
    }
    {  // the tile's class-0 list is full: the rest of its class-0 pieces go to the long list (one
       // uniform test per round; the per-piece fix-up only in the rare round that crosses w.k0)
      uint32_t tot0 = n0;
#pragma unroll
      for (int u = 0; u < U; u++) tot0 += (uint32_t)__popcll(__ballot(cls[u] == 0));
      if (tot0 > w.k0) {
        uint32_t c = n0;
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t m = __ballot(cls[u] == 0);
          if (cls[u] == 0 && c + __popcll(m & lanemask_lt()) >= w.k0) cls[u] = 3;
          c += (uint32_t)__popcll(m);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t below = lanemask_lt();
      // the piece's ordinal among the tile's merged pieces (inactive lanes have class 4)
      const uint64_t mm = __ballot(cls[u] != 4);
      const uint32_t ord = nm + (uint32_t)__popcll(mm & below);
      nm += (uint32_t)__popcll(mm);
      const uint32_t e = list_entry(sl[u], ord, n[u]);
      {  // the wave owns its tile's lists: running counts in scalar registers, no atomics
        const uint64_t m0 = __ballot(cls[u] == 0);
        const uint64_t m1 = __ballot(cls[u] == 1), m2 = __ballot(cls[u] == 2);
        const uint64_t m3 = __ballot(cls[u] == 6);
        if (cls[u] == 0) w.list0[(size_t)tile * w.k0 + n0 + __popcll(m0 & below)] = e;
        if (cls[u] == 1) w.list1[(size_t)tile * kCap1 + n1 + __popcll(m1 & below)] = e;
        if (cls[u] == 2) w.list2[(size_t)tile * kCap2 + n2 + __popcll(m2 & below)] = e;
        if (cls[u] == 6) w.list3[(size_t)tile * kCap3 + n3 + __popcll(m3 & below)] = e;
        by0 += cls[u] == 0 ? n[u] : 0u;
        by1 += cls[u] == 1 ? n[u] : 0u;
        by2 += cls[u] == 2 ? n[u] : 0u;
        n0 += __popcll(m0);
        n1 += __popcll(m1);
        n2 += __popcll(m2);
        n3 += __popcll(m3);
      }
      const uint64_t lm = __ballot(cls[u] == 3);
      // long pieces staged in LDS; one global atomic for the tile's whole batch at the end (a
      // returned atomic per round on the shared counter stalled the wave for its round trip)
      if (lm && nlong + (uint32_t)__popcll(lm) <= kSegLongCap) {
        if (cls[u] == 3) {
          const uint32_t el = s_pos[64 * u + lane + 1];
          const uint32_t ln = el == 0xFFFFu ? 0u : min(el - sl[u], 0x7FFFFu);
          s_long_all[wid][nlong + __popcll(lm & lanemask_lt())] =
              (uint64_t)(t0 + sl[u]) | ((uint64_t)ord << 32) | ((uint64_t)ln << 44);
        }
        nlong += (uint32_t)__popcll(lm);
      } else if (lm) {  // (past kSegLongCap long pieces in the tile: one global atomic per wave)
        const uint32_t leader = __ffsll((unsigned long long)lm) - 1;
        uint32_t b = 0;
        if (lane == leader) b = atomicAdd(&w.counters[0], (uint32_t)__popcll(lm));
        b = __builtin_amdgcn_readlane(b, leader);
        const uint32_t li = b + __popcll(lm & lanemask_lt());
        if (cls[u] == 3 && li < w.long_cap)
        {
          // the length when the piece ends within the look-ahead (0: k_long_len finds its end)
          const uint32_t el = s_pos[64 * u + lane + 1];
          const uint32_t ln = el == 0xFFFFu ? 0u : min(el - sl[u], 0x7FFFFu);
          w.long_list[li] = (uint64_t)(t0 + sl[u]) | ((uint64_t)ord << 32) | ((uint64_t)ln << 44);
        }
        if (lane == leader && b + __popcll(lm) > w.long_cap) atomicOr(&w.counters[kCtrOverflow], 1u);
      }
    }
    // every lane has read this round's s_pos before the next round's expansion overwrites it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (nlong) {  // the tile's staged long pieces: one reservation, coalesced entry stores
    uint32_t b = 0;
    if (lane == 0) b = atomicAdd(&w.counters[0], nlong);
    b = __builtin_amdgcn_readfirstlane(b);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < nlong && b + lane < w.long_cap) w.long_list[b + lane] = s_long_all[wid][lane];
    if (lane == 0 && b + nlong > w.long_cap) atomicOr(&w.counters[kCtrOverflow], 1u);
  }
  SEG_STAMP(4);
  hits = wave_sum_full_u32(hits);
  by0 = wave_sum_full_u32(by0);
  by1 = wave_sum_full_u32(by1);
  by2 = wave_sum_full_u32(by2);
  nd = wave_sum_full_u32(nd);
  if (lane == 0) {
    w.tile_tok[tile] = hits;  // initial token count (the merge passes add theirs atomically)
    w.tile_doc[tile] = nd;
    w.tile_np[tile] = np;
    // id regions of the register passes (ids <= bytes per piece; all four fit in kTileSlots:
    // the lists hold pieces that start in the tile and end within its 62-byte look-ahead)
    w.tregion[tile] = make_uint2(by0 | ((by0 + by1) << 16), by0 + by1 + by2);
  }
  if (lane < kNumClasses)  // (the merge passes move them to the end of what they consumed)
    w.rend[(size_t)lane * w.n_tiles + tile] = lane == 0 ? 0u : lane == 1 ? by0 : lane == 2 ? by0 + by1 : by0 + by1 + by2;
  if (lane < kNumClasses)
    w.tcls[(size_t)lane * w.n_tiles + tile] = lane == 0 ? n0 : lane == 1 ? n1 : lane == 2 ? n2 : n3;
  if (lane == 0 && n2) w.counters[kCtrAnyMid] = 1;  // plain stores: every writer stores 1
  if (lane == 0 && n3) w.counters[kCtrAnyC3] = 1;
  // the sparse class-3 queue (k_bpe_sparse): the tile's class-3 entries into one of kC3Shards
  // shards, its count into the shard's counter (one counter for every tile: C5 k_segment
  // 1.7 -> 5.9 ms, its atomics serialised on one address); a shard that overflows its capacity
  // keeps counting, and the report then steers the call to the register pass
  if (n3 && w.c3_max) {
    const uint32_t sh = tile & (kC3Shards - 1), cap = w.c3_max / kC3Shards;
    uint32_t b = 0;
    if (lane == 0) b = atomicAdd(&w.counters[kNumCounters + sh], n3);
    b = __builtin_amdgcn_readfirstlane(b);
    for (uint32_t j = lane; j < n3; j += 64)
      if (b + j < cap) w.c3q[(size_t)sh * cap + b + j] = (tile << 7) | j;
  }
  SEG_STAMP(5);
#ifdef CTOK_SEG_STAMPS
  if (w.stamps && lane == 0) w.stamps[(size_t)tile * 8 + 6] = np;
#endif
}

hipError_t launch_segment(const Work& w, const Tables& t, hipStream_t s, Lx x) {
  const uint32_t grid = (w.n_tiles + kSegWaves - 1) / kSegWaves;
  if (w.n_tiles && w.rec16) launch_lx(x, k_segment<true>, grid, 64 * kSegWaves, 0, s, w, t);
  else if (w.n_tiles) launch_lx(x, k_segment<false>, grid, 64 * kSegWaves, 0, s, w, t);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// BPE, short pieces: one thread per piece, the working tokens and pair ranks in LDS
// (thread-interleaved columns: entry j of thread t at [j*256 + t], conflict-free).

struct AddedMatch {  // first occurrence of added token k in bytes[0, n) honouring its flags
  __device__ static int64_t find(const Tables& t, uint32_t k, const uint8_t* s, uint32_t n) {
    const uint8_t* pat = t.at_bytes + t.at_off[k];
    const uint32_t m = t.at_off[k + 1] - t.at_off[k];
    if (m > n) return -1;
    for (uint32_t pos = 0; pos + m <= n; pos++) {
      uint32_t j = 0;
      while (j < m && s[pos + j] == pat[j]) j++;
      if (j < m) continue;
      // first occurrence found: the flags are checked only here (src/huggingface/mod.rs:637-675)
      const uint8_t f = t.at_flags[k];
      if (f & 1) {  // single_word: Rust is_alphanumeric of the neighbouring byte-mapped chars
        if (pos > 0 && t.bytemap_alnum[s[pos - 1]]) return -1;
        if (pos + m < n && t.bytemap_alnum[s[pos + m]]) return -1;
      }
      // byte-mapped chars are never White_Space: lstrip/rstrip pass only at the edges
      if ((f & 2) && pos > 0) return -1;
      if ((f & 4) && pos + m < n) return -1;
      return pos;
    }
    return -1;
  }
};

#define TOK(i) s_tok[(i) * NT + tid]
#define RK(i) s_rk[(i) * NT + tid]

// BPE over bytes[0, n) (n <= the slots per thread), appending ids to out; returns the id count.
// s_tok / s_rk hold NT threads' slots interleaved.
template <uint32_t NT>
__device__ __forceinline__ uint32_t bpe_short(const Tables& t, const uint8_t* bytes, uint32_t n,
                                              const int32_t* s_b2id, uint32_t* s_tok, uint32_t* s_rk,
                                              uint32_t tid, uint32_t* out, uint32_t* err) {
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; i++) {
    const int32_t id = s_b2id[bytes[i]];
    if (id >= 0) TOK(m++) = (uint32_t)id;
  }
  if (m >= 2) {
    for (uint32_t i = 0; i + 1 < m; i++) RK(i) = rank_of(t, TOK(i), TOK(i + 1), err);
    while (m >= 2) {
      uint32_t best = kNoRank, bi = 0;
      for (uint32_t i = 0; i + 1 < m; i++) {
        const uint32_t r = RK(i);
        if (r < best) { best = r; bi = i; }
      }
      if (best == kNoRank) break;
      TOK(bi) = new_id_of(t, best);
      for (uint32_t i = bi + 1; i + 1 < m; i++) TOK(i) = TOK(i + 1);
      for (uint32_t i = bi + 1; i + 2 < m; i++) RK(i) = RK(i + 1);
      m--;
      if (bi > 0) RK(bi - 1) = rank_of(t, TOK(bi - 1), TOK(bi), err);
      if (bi + 1 < m) RK(bi) = rank_of(t, TOK(bi), TOK(bi + 1), err);
    }
  }
  for (uint32_t i = 0; i < m; i++) out[i] = TOK(i);
  return m;
}

// ------------------------------------------------------------------------------------------
// Merge passes over the per-tile class lists.  Workgroup b takes K consecutive tiles and treats
// their lists as one concatenated list (prefix of the K counts in LDS); entry q -> its tile by a
// binary search over those K offsets.  Token counts are summed per tile in LDS and added to
// tile_tok with one atomic per (workgroup, tile); no two workgroups share a (class, tile).

// s_tsum[l] starts at tile t0 + l's region base for class cls (tregion, cls >= 0) or at 0: the
// merge passes allocate their ids from it (and add the difference to tile_tok at the flush).
// (K <= 256 tiles: the first K/64 waves scan 64 counts each, then add the earlier waves' totals;
// the workgroup has at least K threads)
template <int K>
__device__ __forceinline__ uint32_t tile_share_init(const uint32_t* counts, uint32_t n_tiles, uint32_t t0,
                                                    uint32_t* s_pre, uint32_t* s_tsum, const uint2* tregion = nullptr,
                                                    int cls = -1, uint32_t* s_tbase = nullptr) {
  static_assert(K >= 1 && K <= 256 && (K & (K - 1)) == 0, "K: power of two <= 256");
  constexpr uint32_t kW = (K + 63) / 64;
  __shared__ uint32_t s_wsum[4];
  const uint32_t l = threadIdx.x, wv = l >> 6;
  const bool in = l < K && t0 + l < n_tiles;
  uint32_t c = 0, inc = 0;
  if (wv < kW) {
    c = in ? counts[t0 + l] : 0u;
    inc = wave_incl_scan(c);
    if (kW > 1 && (l & 63) == 63) s_wsum[wv] = inc;
  }
  if constexpr (kW > 1) __syncthreads();
  if (wv < kW) {
#pragma unroll
    for (uint32_t v = 0; v + 1 < kW; v++) inc += v < wv ? s_wsum[v] : 0u;
    if (l < K) {
      s_pre[l] = inc - c;
      uint32_t b0 = 0;
      if (cls > 0 && in) b0 = region_base(tregion[t0 + l], cls);
      s_tsum[l] = b0;
      if (s_tbase) s_tbase[l] = b0;
    }
    if (l == (K < 64 ? 63u : (uint32_t)K - 1)) s_pre[K] = inc;
  }
  __syncthreads();
  return s_pre[K];
}

template <int K>
__device__ __forceinline__ uint32_t tile_of(const uint32_t* s_pre, uint32_t q) {
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = K / 2; step >= 1; step >>= 1)
    if (s_pre[lo + step] <= q) lo += step;
  return lo;
}

template <int K>
__device__ __forceinline__ void tile_share_flush(const Work& w, uint32_t t0, uint32_t t1, const uint32_t* s_tsum,
                                                 const uint32_t* s_tbase = nullptr, int cls = -1) {
  __syncthreads();
  if (threadIdx.x < K && t0 + threadIdx.x < t1) {
    const uint32_t v = s_tsum[threadIdx.x] - (s_tbase ? s_tbase[threadIdx.x] : 0u);
    if (v) atomicAdd(&w.tile_tok[t0 + threadIdx.x], v);
    if (cls >= 0 && v) w.rend[(size_t)cls * w.n_tiles + t0 + threadIdx.x] = s_tsum[threadIdx.x];
  }
}

constexpr int kTilesGeneric = 2;  // tiles per workgroup, generic pass over list0

// Generic thread-per-piece kernel (LDS working arrays; handles dropped bytes and added tokens).
// MID = false: every piece of list0 (launched instead of the register passes when the tokenizer
// has added tokens that can match inside a piece); MID = true: the pieces the register passes
// found to contain a byte whose char is not in the vocab (mid_list).
// MID pieces can be up to kMedMax bytes (class 3 finds them too): 64 slots, 128 threads.
template <bool MID>
__global__ __launch_bounds__(MID ? 128 : 256) void k_bpe_generic(Work w, Tables t) {
  if (spec_failed(w)) return;
  constexpr uint32_t NT = MID ? 128 : 256;
  constexpr uint32_t SLOTS = MID ? kMedMax : kShortMax;
  __shared__ uint32_t s_tok[SLOTS * NT];
  __shared__ uint32_t s_rk[SLOTS * NT];
  __shared__ int32_t s_b2id[256];
  __shared__ uint32_t s_pre[kTilesGeneric + 1], s_tsum[kTilesGeneric];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 256; i += NT) s_b2id[i] = t.byte2id[i];
  uint32_t* err = &w.counters[2];
  uint32_t E, t0 = 0;
  if (MID) {
    __syncthreads();
    E = min(w.counters[4], w.mid_cap);
  } else {
    t0 = blockIdx.x * kTilesGeneric;
    E = tile_share_init<kTilesGeneric>(w.tcls, w.n_tiles, t0, s_pre, s_tsum);
  }
  const uint32_t stride = MID ? gridDim.x * NT : NT;
  for (uint32_t q = (MID ? blockIdx.x * NT : 0) + tid; q < E; q += stride) {
    uint32_t s, o, n, tile, kt = 0;  // o: the piece's ordinal (its mrec slot)
    if (MID) {
      const uint64_t e = w.mid_list[q];
      s = (uint32_t)e;
      o = (uint32_t)(e >> 32) & 0xFFFu;
      n = (uint32_t)(e >> 48);
      tile = s / kTile;
    } else {
      kt = tile_of<kTilesGeneric>(s_pre, q);
      tile = t0 + kt;
      const uint32_t e = w.list0[(size_t)tile * w.k0 + (q - s_pre[kt])];
      s = tile * kTile + (e & 0xFFFu);
      o = ent_ord(e);
      n = ent_len(e);
    }
    const uint8_t* bytes = w.text + s;
    // ids go to the tile's region of the piece's length class, after what the merge passes used
    // there (the region holds the bytes of every piece of the class: ids <= bytes)
    const uint32_t cl = n <= 8 ? 0u : n <= 16 ? 1u : n <= 32 ? 2u : 3u;
    const uint32_t pos = atomicAdd(&w.rend[(size_t)(MID ? cl : 0u) * w.n_tiles + tile], n);
    uint32_t* out = w.scratch + (size_t)tile * kTileSlots + pos;
    uint32_t cnt = 0;
    if (t.n_at == 0) {
      cnt = bpe_short<NT>(t, bytes, n, s_b2id, s_tok, s_rk, tid, out, err);
    } else {
      // added-token split of the word (src/huggingface/mod.rs:566-610), on raw bytes
      uint32_t pos = 0;
      while (pos < n) {
        int32_t best = -1;
        uint32_t blen = 0;
        for (uint32_t k = 0; k < t.n_at; k++) {
          const uint32_t m = t.at_off[k + 1] - t.at_off[k];
          if (AddedMatch::find(t, k, bytes + pos, n - pos) == 0 && (best < 0 || m > blen)) { best = (int32_t)k; blen = m; }
        }
        if (best >= 0) { out[cnt++] = t.at_id[best]; pos += blen; continue; }
        uint32_t nxt = n - pos;
        for (uint32_t k = 0; k < t.n_at; k++) {
          const int64_t f = AddedMatch::find(t, k, bytes + pos, n - pos);
          if (f > 0 && (uint32_t)f < nxt) nxt = (uint32_t)f;
        }
        cnt += bpe_short<NT>(t, bytes + pos, nxt, s_b2id, s_tok, s_rk, tid, out + cnt, err);
        pos += nxt;
      }
    }
    w.mrec[(size_t)tile * kTileSlots + o] = rec_short(cnt, pos);
    if (MID) atomicAdd(&w.tile_tok[tile], cnt);
    else atomicAdd(&s_tsum[kt], cnt);
  }
  if (!MID) tile_share_flush<kTilesGeneric>(w, t0, w.n_tiles, s_tsum);
}

// ------------------------------------------------------------------------------------------
// BPE fast path: pieces of <= N bytes merged by one thread with the tokens and pair ranks in
// registers (fully unrolled, compile-time slot indices; no LDS for the working set, so occupancy
// is set by VGPRs alone).  All first-probe loads of the initial pairs issue back to back.

__device__ __forceinline__ uint32_t resolve_rank(const Tables& t, uint64_t key, uint32_t h, uint64_t e, uint32_t* err) {
  for (;;) {
    if ((e & kKeyMask) == key) {
      const uint32_t r = (uint32_t)(e >> 42);
      if (value_panics(t, r)) { atomicOr(err, kErrPanic); return kNoRank; }
      return r;
    }
    if (e == kEmpty) return kNoRank;
    h = (h + 1) & t.merge_mask;
    e = t.merge_tab[h];
  }
}

__device__ __forceinline__ uint64_t pair_key(uint32_t a, uint32_t b) { return ((uint64_t)a << kIdBits) | b; }

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;

// The LDS image of the merge passes: hot table + Bloom filter (ctok_internal.h).
struct PairLds {
  const lds_u64* hot;  // bucket c = hot[2c], hot[2c + 1]
  const lds_u32* bloom;
  bool no_bloom = false;  // (HOT = false) no filter in LDS: every lookup goes to the global table
};

// Rank lookup, LDS stage: the pair's value from the hot table, else kNoRank; `global` is set
// when the hot table missed and the Bloom filter cannot rule the pair out.  HOT = false: the
// Bloom filter only (workgroups that keep 32 KiB of LDS instead of 96).
template <bool HOT>
__device__ __forceinline__ uint32_t rank_lds(const PairLds& P, uint32_t a, uint32_t b, uint32_t h1, uint32_t h2,
                                             bool& global) {
  if constexpr (!HOT) {
    if (P.no_bloom) {
      global = true;
      return kNoRank;
    }
  }
  const uint32_t b1 = (h1 >> 12) & (kBloomBits - 1), b2 = (h2 >> 12) & (kBloomBits - 1);
  const uint32_t f = (P.bloom[b1 >> 5] >> (b1 & 31)) & (P.bloom[b2 >> 5] >> (b2 & 31)) & 1u;
  if constexpr (!HOT) {
    global = f != 0;
    return kNoRank;
  }
  const uint32_t c1 = 2 * (h1 & (kHotBuckets - 1)), c2 = 2 * (h2 & (kHotBuckets - 1));
  const uint64_t x0 = P.hot[c1], x1 = P.hot[c1 + 1], y0 = P.hot[c2], y1 = P.hot[c2 + 1];
  // entry = value << 42 | a << 21 | b: compare the 42-bit key as (lo 32, hi 10)
  const uint32_t klo = (a << kIdBits) | b, khi = a >> (32 - kIdBits);
  uint32_t v = kNoRank;
  bool hit = false;
  auto chk = [&](uint64_t e) {
    const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
    const bool m = lo == klo && (hi & 0x3FFu) == khi;
    v = m ? (hi >> 10) : v;
    hit |= m;
  };
  chk(x0);
  chk(x1);
  chk(y0);
  chk(y1);
  global = !hit && f;
  return v;
}

// One pair lookup of a merge pass, split in two so that the global-table load (issued by
// start, only when the LDS stage cannot decide) overlaps the caller's other work before finish.
// NARROW = false: the 42-bit-key tables (mhash / mhash2); true: the 32-bit-key tables (key16,
// ctok_internal.h), whose hashes and bucket compares take about half the VALU.
template <bool NARROW, bool HOT> struct Probe;

template <bool HOT>
struct Probe<false, HOT> {
  uint32_t a, b, h, r;
  uint64_t e;
  bool g;
  __device__ __forceinline__ void start(const Tables& t, const PairLds& P, uint32_t a_, uint32_t b_, bool live) {
    a = a_;
    b = b_;
    h = mhash(a, b);
    r = rank_lds<HOT>(P, a, b, h, mhash2(h), g);
    g = g && live;
    e = 0;
    if (g) e = t.merge_tab[h & t.merge_mask];
  }
  __device__ __forceinline__ uint32_t finish(const Tables& t, uint32_t* err) {
    if (g) r = resolve_rank(t, pair_key(a, b), h & t.merge_mask, e, err);
    return r;
  }
};

template <bool HOT>
struct Probe<true, HOT> {
  uint32_t k, h, r;
  uint64_t e;
  bool g;
  __device__ __forceinline__ void start(const Tables& t, const PairLds& P, uint32_t a, uint32_t b, bool live) {
    a &= 0xFFFFu;  // (ids < 2^16; known to the compiler, the hashes use 24-bit multiplies)
    b &= 0xFFFFu;
    k = key16(a, b);
    h = hash16_h(a, b);
    const uint32_t h2 = hash16_g(a, b);
    const uint32_t b1 = h & (kBloomBits - 1), b2 = h2 >> 14;
    const uint32_t f = (P.bloom[b1 >> 5] >> (b1 & 31)) & (P.bloom[b2 >> 5] >> (b2 & 31)) & 1u;
    const uint32_t c1 = 2 * (h >> 20), c2 = 2 * (h2 >> 20);
    const uint64_t x0 = P.hot[c1], x1 = P.hot[c1 + 1], y0 = P.hot[c2], y1 = P.hot[c2 + 1];
    uint32_t v = kNoRank;
    bool hit = false;
    auto chk = [&](uint64_t x) {
      const bool m = (uint32_t)x == k;
      v = m ? (uint32_t)(x >> 32) : v;
      hit |= m;
    };
    chk(x0);
    chk(x1);
    chk(y0);
    chk(y1);
    r = v;
    g = !hit && f && live;
    e = 0;
    if (g) e = t.merge16[h & t.merge16_mask];
  }
  __device__ __forceinline__ uint32_t finish(const Tables& t, uint32_t* err) {
    if (g) {
      uint32_t s = h & t.merge16_mask;
      for (;;) {
        if ((uint32_t)e == k) {
          r = (uint32_t)(e >> 32);
          if (value_panics(t, r)) { atomicOr(err, kErrPanic); r = kNoRank; }
          break;
        }
        if (e == kEmpty) { r = kNoRank; break; }
        s = (s + 1) & t.merge16_mask;
        e = t.merge16[s];
      }
    }
    return r;
  }
};

template <int N> struct LdsClass;
template <> struct LdsClass<8> { static constexpr int cls = 0; static constexpr uint32_t cap = kCap0; };
template <> struct LdsClass<16> { static constexpr int cls = 1; static constexpr uint32_t cap = kCap1; };
template <> struct LdsClass<32> { static constexpr int cls = 2; static constexpr uint32_t cap = kCap2; };
template <> struct LdsClass<64> { static constexpr int cls = 3; static constexpr uint32_t cap = kCap3; };

template <int N>
__device__ __forceinline__ const uint32_t* class_list(const Work& w) {
  return N == 8 ? w.list0 : N == 16 ? w.list1 : N == 32 ? w.list2 : w.list3;
}
template <int N>
__device__ __forceinline__ uint32_t class_cap(const Work& w) {
  return N == 8 ? w.k0 : LdsClass<N>::cap;
}

// The merge loop on the first N register slots of tk / rk (compile-time indices only, so the
// arrays stay in registers): branch-free over the slots, the lowest (rank, position) pair is
// merged, the slots right of it shift left by one, the two new pairs' ranks are looked up.
// Returns true when it stopped because the piece shrank to <= stop tokens (the caller continues
// on fewer slots), false when no pair can merge.  Slots >= m hold kDead / kNoRank.
template <int N, bool COMPACT, bool HOT, bool NARROW>
__device__ __forceinline__ bool merge_slots(const Tables& t, const PairLds& P, uint32_t* tk, uint32_t* rk,
                                            uint32_t& m, uint32_t stop, uint32_t* err) {
  for (;;) {
    if (m <= stop) return true;
    uint32_t key = ~0u;  // rank << 6 | position: one v_min per slot (ranks < 2^22, N <= 64)
#pragma unroll
    for (int k = 0; k < N - 1; k++) key = min(key, (rk[k] << 6) | (uint32_t)k);
    const uint32_t best = key >> 6, bi = key & 63u;
    if (best == kNoRank) return false;
    const uint32_t nid = COMPACT ? best : t.rank_newid[best];
    uint32_t L = 0, R = 0;
#pragma unroll
    for (int k = 0; k < N; k++) {
      L = ((uint32_t)k + 1 == bi) ? tk[k] : L;
      R = ((uint32_t)k == bi + 2) ? tk[k] : R;
    }
    const bool has_l = bi > 0, has_r = bi + 2 < m;
    Probe<NARROW, HOT> pl, pr;
    pl.start(t, P, L, nid, has_l);
    pr.start(t, P, nid, R, has_r);
#pragma unroll
    for (int k = 0; k < N; k++) {  // ascending: tk[k+1] is read before it is overwritten
      const uint32_t nxt_t = k + 1 < N ? tk[k + 1] : kDead;
      const uint32_t nxt_r = k + 1 < N ? rk[k + 1] : kNoRank;
      const bool gt = (uint32_t)k > bi;
      tk[k] = gt ? nxt_t : ((uint32_t)k == bi ? nid : tk[k]);
      rk[k] = gt ? nxt_r : rk[k];
    }
    m--;
    const uint32_t rl = has_l ? pl.finish(t, err) : kNoRank;
    const uint32_t rr = has_r ? pr.finish(t, err) : kNoRank;
#pragma unroll
    for (int k = 0; k < N - 1; k++)
      rk[k] = ((uint32_t)k + 1 == bi) ? rl : (((uint32_t)k == bi) ? rr : rk[k]);
  }
}

// The last tier (<= 8 tokens) with the working state in LDS instead of registers: positions stay
// fixed, a live mask says which slots still hold a token, and slot s keeps the key
// rank << 3 | s of the pair its token starts (~0 when the slot is dead or last).  A merge then
// reads the keys (four ds_read2st64, a v_min tree), writes three keys and one token, and reads its
// two neighbours by index; the register tiers' N-wide select / shift chains (~100 VALU per merge
// at N = 8) are gone.  Tokens are u16 (narrow vocabularies: every id < 2^16), so 1024 threads'
// state (48 B each) fits beside the 96 KiB image.  Pair lookups use the 32-bit-key tables.
//   keys:   s_key[s * NT + tid] (u32; read two at a time with ds_read2st64)
//   tokens: s_tok[s * NT + tid] (u16)
// Semantics are merge_slots': the lowest (rank, position) pair merges (src/bpe.rs:118-149).
typedef __attribute__((address_space(3))) uint16_t lds_u16;

// out_of(m) returns where the piece's m ids go (called once, after the last merge).
template <bool COMPACT, bool HOT, uint32_t NT, typename OutOf>
__device__ __forceinline__ uint32_t merge_lds8(const Tables& t, const PairLds& P, const uint32_t* tk, const uint32_t* rk,
                                               uint32_t m, lds_u32* s_key, lds_u16* s_tok, uint32_t* err,
                                               OutOf&& out_of) {
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    s_key[k * NT + tid] = (uint32_t)k + 1 < m ? (rk[k] << 3) | (uint32_t)k : ~0u;
    s_tok[k * NT + tid] = (uint16_t)tk[k];
  }
  // live slots, with a sentinel at bit 8 (so every "next live" search finds a bit)
  uint32_t lv = ((1u << m) - 1u) | 0x100u;
  for (;;) {
    uint32_t kk[8];
#pragma unroll
    for (int k = 0; k < 8; k++) kk[k] = s_key[k * NT + tid];
    const uint32_t best = min(min(min(kk[0], kk[1]), min(kk[2], kk[3])), min(min(kk[4], kk[5]), min(kk[6], kk[7])));
    if (best >= (kNoRank << 3)) break;
    const uint32_t bi = best & 7u, r = best >> 3;
    // (ids < 2^16: the mask lets the hashes use 24-bit multiplies)
    const uint32_t nid = (COMPACT ? r : t.rank_newid[r]) & 0xFFFFu;
    const uint32_t p = bi + 1 + (uint32_t)__builtin_ctz(lv >> (bi + 1));  // the right token's slot
    const uint32_t q = p + 1 + (uint32_t)__builtin_ctz(lv >> (p + 1));    // the token after it (8: none)
    const bool has_r = q < 8;
    const uint32_t lo = lv & ((1u << bi) - 1u);
    const bool has_l = lo != 0;
    const uint32_t pv = 31u - (uint32_t)__builtin_clz(lo | 1u);           // the token before
    const uint32_t L = s_tok[pv * NT + tid], R = s_tok[min(q, 7u) * NT + tid];
    s_tok[bi * NT + tid] = (uint16_t)nid;
    s_key[p * NT + tid] = ~0u;
    lv &= ~(1u << p);
    m--;
    Probe<true, HOT> pl, pr;
    pl.start(t, P, L, nid, has_l);
    pr.start(t, P, nid, R, has_r);
    const uint32_t rl = pl.finish(t, err), rr = pr.finish(t, err);
    if (has_l) s_key[pv * NT + tid] = (rl << 3) | pv;
    s_key[bi * NT + tid] = has_r ? (rr << 3) | bi : ~0u;
  }
  // live tokens in slot order to out[0 .. m)
  uint32_t* out = out_of(m);
#pragma unroll
  for (int k = 0; k < 8; k++)
    if ((lv >> k) & 1u) out[__popc(lv & ((1u << k) - 1u))] = s_tok[k * NT + tid];
  return m;
}

// Workgroup-shared scratch of a merge pass.
template <uint32_t SORTCAP, int KT = 64>
struct PassLds {
  uint32_t pre[KT + 1], tsum[KT], tbase[KT], stat[2], bcnt[4], bfill[4], chunk, take, next;
  uint16_t perm[SORTCAP];  // the chunk's entries ordered by length bucket
};

// Merge pass over one length class (N = 8, 16, 32 slots), run by a persistent grid:
// workgroups take chunks of w.unit-tile units from a counter (up to KT / w.unit units at once when the
// previous chunk left most of the workgroup idle: sparse classes) (counters[ctr_chunk(class)]) and walk the chunk's
// class lists as one concatenated list (see tile_share_init).  Thread per piece, tokens and pair
// ranks in registers (fully unrolled, compile-time slots).
// `load` fills the workgroup's LDS tables (image, byte -> id); it runs at the first chunk with
// work, so a workgroup that finds only empty lists never reads the 32..96 KiB image (`loaded`
// is shared by the passes of one kernel).
// L8: the <= 8-token tier runs in LDS (merge_lds8, narrow vocabularies; s_key / s_tok its state).
template <int N, bool COMPACT, bool HOT, uint32_t NT, uint32_t SORTCAP, bool L8 = false, int KT = 64, typename Load>
__device__ __forceinline__ void class_pass(const Work& w, const Tables& t, const PairLds& P, const int32_t* s_b2id,
                                           PassLds<SORTCAP, KT>& S, bool& loaded, Load&& load,
                                           lds_u32* s_key = nullptr, lds_u16* s_tok = nullptr) {
  using LC = LdsClass<N>;
  constexpr int K = KT;
  static_assert(KT <= (int)NT, "a thread per chunk tile");
  const uint32_t tid = threadIdx.x;
  uint32_t* err = &w.counters[2];
  const uint32_t* list = class_list<N>(w);
  const uint32_t cap = class_cap<N>(w);
  const uint32_t* counts = w.tcls + (size_t)LC::cls * w.n_tiles;
  uint32_t st_bytes = 0, st_ids = 0;
  if (tid < 2) S.stat[tid] = 0;
  // length buckets (4 per class): a wavefront's pieces then have similar lengths, hence
  // similar merge counts, and fewer of its lanes idle while the longest piece finishes
  constexpr uint32_t blo = N == 8 ? 1 : N / 2 + 1, bw = N == 64 ? 8 : N == 32 ? 4 : 2;
  auto bucket = [&](uint32_t n) { return min(3u, (n - blo) / bw); };
  // chunks of K tiles dealt dynamically (one atomic per chunk, taken by thread 0 and broadcast
  // through LDS): workgroups that start late, or whose CU is shared, take fewer chunks
  __syncthreads();
  uint32_t take = 1;  // units of the next chunk (workgroup-uniform)
  const uint32_t U = w.unit;
  for (;;) {
    if (tid == 0) {
      S.chunk = atomicAdd(&w.counters[ctr_chunk(LC::cls)], take);
      S.take = take;
      S.next = 0;
    }
    __syncthreads();
    const uint32_t c0 = S.chunk * U;
    if (c0 >= w.n_tiles) break;
    const uint32_t tb1 = min(w.n_tiles, c0 + U * S.take);
    const uint32_t E = tile_share_init<K>(counts, tb1, c0, S.pre, S.tsum, w.tregion, LC::cls, S.tbase);
    if (E && !loaded) {  // E is workgroup-uniform (read from LDS after a barrier)
      load();
      loaded = true;
      __syncthreads();
    }
    const bool sorted = N > 8 && E <= SORTCAP;  // <= 8 B pieces: few merges, sorting does not pay
    if (sorted) {
      if (tid < 4) { S.bcnt[tid] = 0; S.bfill[tid] = 0; }
      __syncthreads();
      for (uint32_t q = tid; q < E; q += NT) {  // bucket sizes (one LDS add per wave and bucket)
        const uint32_t kt = tile_of<K>(S.pre, q);
        const uint32_t b = bucket(ent_len(list[(size_t)(c0 + kt) * cap + (q - S.pre[kt])]));
#pragma unroll
        for (uint32_t bb = 0; bb < 4; bb++) {
          const uint64_t m = __ballot(b == bb);
          if (m && (threadIdx.x & 63) == __ffsll((unsigned long long)m) - 1) atomicAdd(&S.bcnt[bb], (uint32_t)__popcll(m));
        }
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t acc = 0;
        for (int bb = 0; bb < 4; bb++) {
          const uint32_t c = S.bcnt[bb];
          S.bfill[bb] = acc;
          acc += c;
        }
      }
      __syncthreads();
      for (uint32_t q = tid; q < E; q += NT) {  // scatter entry numbers into bucket order
        const uint32_t kt = tile_of<K>(S.pre, q);
        const uint32_t b = bucket(ent_len(list[(size_t)(c0 + kt) * cap + (q - S.pre[kt])]));
#pragma unroll
        for (uint32_t bb = 0; bb < 4; bb++) {
          const uint32_t slot = wave_append(&S.bfill[bb], b == bb);
          if (b == bb) S.perm[slot] = (uint16_t)q;
        }
      }
      __syncthreads();
    }
    auto entry = [&](uint32_t i, uint32_t& kt) {
      const uint32_t q = sorted ? (uint32_t)S.perm[i] : i;
      kt = tile_of<K>(S.pre, q);
      return list[(size_t)(c0 + kt) * cap + (q - S.pre[kt])];
    };
    auto start_of = [&](uint32_t e, uint32_t kt) { return (c0 + kt) * kTile + (e & 0xFFFu); };
    // one piece: list entry e of chunk tile kt, its first N bytes in wv
    // `hook` runs before the piece's first store (the pipeline below waits there for its
    // look-ahead loads, not behind the stores at its next step)
    auto body = [&](uint32_t e, uint32_t kt, const uint32_t* wv, auto&& hook) {
        const uint32_t tile = c0 + kt;
        const uint32_t s = tile * kTile + (e & 0xFFFu);
        const uint32_t o = ent_ord(e);
        const uint32_t n = ent_len(e);
        uint32_t tk[N], rk[N];
        bool missing = false;
        {
#pragma unroll
          for (int k = 0; k < N; k++) {
            const int32_t id = s_b2id[byte_of(wv[k >> 2], k)];
            missing |= ((uint32_t)k < n) & (id < 0);
            tk[k] = (uint32_t)id;
          }
        }
        if (missing) {  // a byte char absent from the vocab is dropped: generic path
          hook();
          const uint32_t mi = atomicAdd(&w.counters[4], 1u);
          if (mi < w.mid_cap)
            w.mid_list[mi] = (uint64_t)s | ((uint64_t)o << 32) | ((uint64_t)n << 48);
          else
            atomicOr(&w.counters[kCtrOverflow], 1u);
          return;
        }
        // initial pair ranks: every initial pair is a byte pair, one load each from the 256 x 256
        // byte-pair table (L2-resident), all in flight together
        {
          uint32_t bytes[N];
#pragma unroll
          for (int k = 0; k < N; k++) bytes[k] = byte_of(wv[k >> 2], k);
#pragma unroll
          for (int k = 0; k < N - 1; k++) rk[k] = t.pair0[(bytes[k] << 8) | bytes[k + 1]];
#pragma unroll
          for (int k = 0; k < N - 1; k++) {
            const bool live = (uint32_t)k + 1 < n;
            if (live && rk[k] != kNoRank && value_panics(t, rk[k])) atomicOr(err, kErrPanic);
            rk[k] = (live && !(rk[k] != kNoRank && value_panics(t, rk[k]))) ? rk[k] : kNoRank;
          }
        }
        rk[N - 1] = kNoRank;
        uint32_t m = n;
        // tiers: N slots while the piece has more than N/2 tokens, then N/2, ... down to 8 slots
        bool more = true;
        if constexpr (N >= 64) more = merge_slots<64, COMPACT, HOT, L8>(t, P, tk, rk, m, 32, err);
        if constexpr (N >= 32) {
          if (more) more = merge_slots<32, COMPACT, HOT, L8>(t, P, tk, rk, m, 16, err);
        }
        if constexpr (N >= 16) {
          if (more) more = merge_slots<16, COMPACT, HOT, L8>(t, P, tk, rk, m, 8, err);
        }
        // ids go to the next free slots of the tile's region for this class (dense: a wave's
        // stores fill whole lines), the record points at them
        hook();
        uint32_t pos = 0;
        auto out_of = [&](uint32_t mm) {
          pos = atomicAdd(&S.tsum[kt], mm);
          return w.scratch + (size_t)tile * kTileSlots + pos;
        };
        if (L8 && more) {
          m = merge_lds8<COMPACT, HOT, NT>(t, P, tk, rk, m, s_key, s_tok, err, out_of);
        } else {
          if (!L8 && more) merge_slots<8, COMPACT, HOT, L8>(t, P, tk, rk, m, 0, err);
          uint32_t* out = out_of(m);
#pragma unroll
          for (int k = 0; k < N; k++)
            if ((uint32_t)k < m) out[k] = tk[k];
        }
        CTOK_CHECK_REC(m >= 1 && m <= n && pos + m <= (uint32_t)kTileSlots && o < (uint32_t)kTileSlots,
                       "[ctok check] class pass N=%d tile %u: record m=%u n=%u pos=%u ordinal=%u\n", N, tile, m, n, pos, o);
        w.mrec[(size_t)tile * kTileSlots + o] = rec_short(m, pos);
        st_bytes += n;
        st_ids += m;
    };
    if constexpr (N > 32) {
      // 64 slots: no registers to spare for a pipeline; a static stride over the chunk
      for (uint32_t i = tid; i < E; i += NT) {
        uint32_t kt;
        const uint32_t e = entry(i, kt);
        uint32_t wv[N / 4];
        load_words<N / 4>(w.text, start_of(e, kt), w.n_bytes, wv);
        body(e, kt, wv, [] {});
      }
    } else {
      // Each wavefront takes blocks of 64 entries from S.next (one LDS atomic per block): a wave
      // whose pieces merge quickly takes more blocks, so the chunk's waves finish together
      // instead of each owning a fixed stride of the chunk (which cost 8% (<= 8 B) .. 15%
      // (9..16 B) of the pass at the chunk barrier).  Software pipeline over a wave's blocks b0,
      // b1, b2: the list entry is loaded two blocks ahead and the piece's text dwords one block
      // ahead, so the merges of one piece hide the two dependent global loads of the next.  The
      // look-ahead registers are only loaded here (aligned at their use) and are waited for
      // inside the piece's body before its stores (`hook`): vmcnt counts loads and stores
      // together in issue order, so a wait for them at the top of the next step would also wait
      // for the stores.
      const uint32_t lane = tid & 63;
      auto take = [&]() -> uint32_t {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(&S.next, 64u);
        return uni((uint32_t)__shfl((int)b, 0, 64));
      };
      constexpr int kPw = N / 4;
      uint32_t e0 = 0, kt0 = 0, e1 = 0, kt1 = 0;
      uint32_t d0[kPw + 1], sh0 = 0;  // the next piece's text dwords (unaligned) and its byte shift
#pragma unroll
      for (int k = 0; k <= kPw; k++) d0[k] = 0;
      const uint32_t last = (w.n_bytes - 1) & ~3u;
      auto issue_words = [&](uint32_t s) {
        const uint32_t a0 = s & ~3u;
#pragma unroll
        for (int k = 0; k <= kPw; k++) d0[k] = *reinterpret_cast<const uint32_t*>(w.text + min(a0 + 4 * k, last));
        sh0 = s & 3u;
      };
      auto hook = [&]() {
        static_assert(kPw <= 8, "hook operands");
        if constexpr (kPw == 2) asm volatile("" ::"v"(d0[0]), "v"(d0[1]), "v"(d0[2]), "v"(e1));
        else if constexpr (kPw == 4)
          asm volatile("" ::"v"(d0[0]), "v"(d0[1]), "v"(d0[2]), "v"(d0[3]), "v"(d0[4]), "v"(e1));
        else
          asm volatile("" ::"v"(d0[0]), "v"(d0[1]), "v"(d0[2]), "v"(d0[3]), "v"(d0[4]), "v"(d0[5]), "v"(d0[6]),
                       "v"(d0[7]), "v"(d0[8]), "v"(e1));
      };
      uint32_t b0 = take();
      uint32_t b1 = b0 < E ? take() : E;
      if (b0 + lane < E) {
        e0 = entry(b0 + lane, kt0);
        issue_words(start_of(e0, kt0));
      }
      if (b1 + lane < E) e1 = entry(b1 + lane, kt1);
      hook();
      while (b0 < E) {  // wave-uniform
        const uint32_t i = b0 + lane;
        const uint32_t b2 = b1 < E ? take() : E;
        const uint32_t e = e0, kt = kt0;
        uint32_t wv[kPw];
#pragma unroll
        for (int k = 0; k < kPw; k++) wv[k] = __builtin_amdgcn_alignbyte(d0[k + 1], d0[k], sh0);
        e0 = e1;
        kt0 = kt1;
        if (b1 + lane < E) issue_words(start_of(e0, kt0));
        if (b2 + lane < E) e1 = entry(b2 + lane, kt1);
        b0 = b1;
        b1 = b2;
        if (i < E) body(e, kt, wv, hook);
        else hook();
      }
    }
    tile_share_flush<K>(w, c0, tb1, S.tsum, S.tbase, LC::cls);
    // size the next chunk for about two entries per thread (up to K tiles): sparse classes take
    // several units at once, dense ones one; never more than a fair share of the units left, so
    // the last chunks stay small (C2: 504 units for 256 workgroups)
    const uint32_t units = (w.n_tiles + U - 1) / U, next = S.chunk + S.take;
    const uint32_t share = next < units ? (units - next) / gridDim.x : 0u;
    take = min(min((uint32_t)K / U, max(1u, share)), N <= 16 ? 64u : max(1u, (2 * NT * S.take + E) / (E + 1)));
    __syncthreads();
  }
  // statistics: bytes merged and ids produced by this pass (algorithmic bytes for the roofline)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    st_bytes += (uint32_t)__shfl_xor((int)st_bytes, o, 64);
    st_ids += (uint32_t)__shfl_xor((int)st_ids, o, 64);
  }
  if ((tid & 63) == 0) {
    atomicAdd(&S.stat[0], st_bytes);
    atomicAdd(&S.stat[1], st_ids);
  }
  __syncthreads();
  if (tid == 0) {
    atomicAdd(&w.counters[ctr_stat(LC::cls)], S.stat[0]);
    atomicAdd(&w.counters[ctr_stat(LC::cls) + 1], S.stat[1]);
  }
  __syncthreads();
}

// (Round 5 also built a lane-group variant of this pass -- 8 / 16 lanes per piece, -DCTOK_SHORT_LG:
// 4.3x slower, VALU-issue bound; DESIGN.md 4.2.  It is kept out of this file as
// profiles/r05/patches/short_lane_group.diff.)

// Pieces of <= 16 bytes (classes 0 and 1): one workgroup per CU holding the whole LDS image
// (hot table + Bloom filter); a workgroup moves on to class 1 as soon as class 0 has no chunk
// left, with no kernel boundary in between.  NARROW (every id < 2^16): 1024 threads, the last
// tier's state in LDS (merge_lds8); else 1024 threads, all tiers in registers.
// Narrow: the workgroup size and the sort buffer share the LDS left beside the image with
// merge_lds8's 48 B per thread; 1024 threads with a 7168-entry sort buffer (LDS 163,648 B) take
// k_bpe_short 3.57 -> 3.51 ms on C4 against 960 with 8192 (profiles/r04/v12_ab_short_nt1024_c4.txt).
// (Compile-time knobs for A/B builds.)
#ifndef CTOK_SHORT_NT
#define CTOK_SHORT_NT 1024
#endif
#ifndef CTOK_SHORT_SORTCAP
#define CTOK_SHORT_SORTCAP 7168
#endif
template <bool NARROW> struct ShortCfg {
  static constexpr uint32_t NT = NARROW ? CTOK_SHORT_NT : 1024;
  static constexpr uint32_t SORTCAP = NARROW ? CTOK_SHORT_SORTCAP : kSortCap;
};
// tiles per chunk of the <= 16 B passes (dense classes: ~100 + ~60 pieces per tile on C4; 128
// tiles per chunk measured 3% slower, profiles/r02/v30_ab_short_kt128.txt)
constexpr int kShortKT = 64;

template <bool COMPACT, bool NARROW>
__global__ __launch_bounds__(1024) void k_bpe_short(Work w, Tables t, uint32_t passes) {
  if (w.report && blockIdx.x == 0 && threadIdx.x < 64) write_report(w);  // (k_report's work: see there)
  if (spec_failed(w)) return;
  constexpr uint32_t NT = ShortCfg<NARROW>::NT;
  extern __shared__ __attribute__((aligned(16))) uint4 s_img[];
  __shared__ int32_t s_b2id[256];
  __shared__ PassLds<ShortCfg<NARROW>::SORTCAP, kShortKT> S;
  __shared__ uint32_t s_key[NARROW ? 8 * NT : 1];
  __shared__ uint16_t s_tok[NARROW ? 8 * NT : 1];
  const uint32_t tid = threadIdx.x;
  const uint4* img = NARROW ? t.lds16_image : t.lds_image;
  auto load = [&] {
    for (uint32_t i = tid; i < kLdsImageBytes / 16; i += NT) s_img[i] = img[i];
    for (uint32_t i = tid; i < 256; i += NT) s_b2id[i] = t.byte2id[i];
  };
  bool loaded = false;
  const PairLds P{(const lds_u64*)s_img, (const lds_u32*)(s_img + kHotBuckets)};
  lds_u32* sk = (lds_u32*)s_key;
  lds_u16* st = (lds_u16*)s_tok;
  WgRec::begin(w.wgrec, 0);
  // passes: bit 0 the <= 8 B class, bit 1 the 9..16 B class (both, except in the timing A/B
  // CTOK_DBG_MODE=30, which launches them as two kernels to time them apart)
  if (passes & 1u)
    class_pass<8, COMPACT, true, NT, ShortCfg<NARROW>::SORTCAP, NARROW, kShortKT>(w, t, P, s_b2id, S, loaded, load, sk, st);
  if (passes & 2u)
    class_pass<16, COMPACT, true, NT, ShortCfg<NARROW>::SORTCAP, NARROW, kShortKT>(w, t, P, s_b2id, S, loaded, load, sk, st);
  WgRec::end(w.wgrec, 0, loaded ? 1u : 0u);
}

// ------------------------------------------------------------------------------------------
// Sparse 33..64 B class (round 6).  On English-like text class 3 is a few pieces per thousand
// tiles (C4: ~600 pieces in 322k tiles; C2 or a 1/8 C4 shard: ~70), and the register pass
// (k_bpe_mid<3>: a thread per piece over 64 slots, ~1,300 VALU per merge) then costs one thread's
// whole merge chain: 90 us on C2, 190 us on C4 for a few kilobytes.  k_segment queues each tile's
// class-3 pieces in one of 64 shards (Work::c3q; a shard per tile % 64, so its atomics spread
// over 64 counters); when the report counts at most Work::c3_max of them, the host launches
// k_bpe_sparse instead of the register pass: its waves take the queue's pieces one at a time from
// a counter and merge each on the whole wavefront (merge_wave64), its ids into the tile's class-3
// region (reserved from rend, as the dropped-byte pass does) and its merged record in mrec --
// what the register pass would write.  (Round 6's first build gathered the list in a kernel of
// its own, on a stream forked after k_segment; k_segment appending to one list -- one atomic per
// tile on one counter -- took C5's k_segment from 1.7 to 5.9 ms; folding the pass into the 17..32
// B pass's workgroups put its merge chains at that pass's end, +20..40 us on a 1/8 C4 shard; waves
// scanning 64-tile chunks of the class counts themselves left a dense chunk's pieces to one wave:
// C5-NFC's sub-batch 2.4 -> 17 ms.)

// The merge loop of one <= 64-token piece on a whole wavefront: lane k holds token k (positions
// stay put) and the value of the pair its token starts (kNoRank when it starts none); the live
// mask lv (wave-uniform, in SGPRs) marks the lanes that still hold a token.  A merge is a 64-lane
// minimum of value << 6 | lane (the lowest value, leftmost on ties: src/bpe.rs:118-149, as
// merge_slots), its neighbours found with scalar bit scans of lv, the two new pairs looked up at
// once by lanes 0 and 1, and three selects -- a chain of ~40 instructions and one LDS probe per
// merge where the register pass spends ~1,300 on one lane.  Returns the token count.
template <bool COMPACT, bool NARROW>
__device__ __forceinline__ uint32_t merge_wave64(const Tables& t, const PairLds& P, uint32_t& tok, uint32_t rk,
                                                 uint64_t& lv, uint32_t* err) {
  const uint32_t lane = threadIdx.x & 63;
  for (;;) {
    const uint32_t best = wave_min_full_u32((rk << 6) | lane);
    const uint32_t r = best >> 6, bi = best & 63u;
    if (r == kNoRank) break;
    const uint32_t nid = COMPACT ? r : uni(t.rank_newid[r]);
    const uint64_t right = lv & ~((2ull << bi) - 1ull);  // live lanes past bi (bi < 63: it starts a pair)
    const uint32_t p = (uint32_t)__builtin_ctzll(right);  // the right token
    const uint64_t after = right & (right - 1ull);
    const bool has_r = after != 0;
    const uint32_t q = has_r ? (uint32_t)__builtin_ctzll(after) : 0u;  // the token after it
    const uint64_t left = lv & ((1ull << bi) - 1ull);
    const bool has_l = left != 0;
    const uint32_t pv = has_l ? 63u - (uint32_t)__builtin_clzll(left) : 0u;  // the token before
    const uint32_t L = __builtin_amdgcn_readlane(tok, pv), R = __builtin_amdgcn_readlane(tok, q);
    uint32_t v = kNoRank;
    if (lane < 2) {  // lane 0: (L, nid), lane 1: (nid, R)
      Probe<NARROW, true> pr;
      pr.start(t, P, lane == 0 ? L : nid, lane == 0 ? nid : R, lane == 0 ? has_l : has_r);
      v = pr.finish(t, err);
    }
    const uint32_t rl = __builtin_amdgcn_readlane(v, 0), rr = __builtin_amdgcn_readlane(v, 1);
    tok = lane == bi ? nid : tok;
    rk = (has_l && lane == pv) ? rl : rk;
    rk = lane == bi ? (has_r ? rr : kNoRank) : rk;
    rk = lane == p ? kNoRank : rk;
    lv &= ~(1ull << p);
  }
  return (uint32_t)__popcll(lv);
}

// One wave's share of the sparse class-3 pass (see above): n pieces in the sharded queue c3q
// (shard i: pieces c3pre[i] .. c3pre[i + 1] - 1 of the pass, at c3q + i * cap); P / s_b2id: the
// workgroup's LDS image.
template <bool COMPACT, bool NARROW>
__device__ __forceinline__ void sparse_c3(const Work& w, const Tables& t, const PairLds& P, const int32_t* s_b2id,
                                          uint32_t n) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t cap = w.c3_max / kC3Shards;
  const uint32_t pre = w.c3pre[lane];  // (kC3Shards == 64: shard `lane`'s first piece)
  uint32_t* err = &w.counters[2];
  uint32_t st_bytes = 0, st_ids = 0;
  for (;;) {
    // (every lane takes part, lane 0 adding 1: no divergent branch around the atomic)
    const uint32_t k = uni(atomicAdd(&w.counters[kCtrC3Take], lane == 0 ? 1u : 0u));
    if (k >= n) break;
    // its shard: the last one starting at or before k (empty shards share their successor's start)
    const uint32_t sh = 63u - (uint32_t)__builtin_clzll(__ballot(pre <= k));
    const uint32_t qe = uni(w.c3q[(size_t)sh * cap + (k - __builtin_amdgcn_readlane(pre, sh))]);
    const uint32_t tile = qe >> 7;
    const uint32_t e = uni(w.list3[(size_t)tile * kCap3 + (qe & 127u)]);
    const uint32_t s = tile * kTile + (e & 0xFFFu), o = ent_ord(e), len = ent_len(e);
    // lane k: byte k, its token, the value of the byte pair it starts (the 256 x 256 table)
    const uint32_t b0 = lane < len ? w.text[s + lane] : 0u;
    const uint32_t b1 = lane + 1 < len ? w.text[s + lane + 1] : 0u;
    const int32_t id = s_b2id[b0];
    if (__ballot(lane < len && id < 0)) {  // a byte char absent from the vocab: the generic pass drops it
      if (lane == 0) {
        const uint32_t mi = atomicAdd(&w.counters[4], 1u);
        if (mi < w.mid_cap) w.mid_list[mi] = (uint64_t)s | ((uint64_t)o << 32) | ((uint64_t)len << 48);
        else atomicOr(&w.counters[kCtrOverflow], 1u);
      }
      continue;
    }
    uint32_t rk = lane + 1 < len ? t.pair0[(b0 << 8) | b1] : kNoRank;
    if (rk != kNoRank && value_panics(t, rk)) {
      atomicOr(err, kErrPanic);
      rk = kNoRank;
    }
    uint32_t tok = (uint32_t)id;
    uint64_t lv = len >= 64 ? ~0ull : (1ull << len) - 1ull;
    const uint32_t m = merge_wave64<COMPACT, NARROW>(t, P, tok, rk, lv, err);
    uint32_t pos = 0;
    if (lane == 0) pos = atomicAdd(&w.rend[3ull * w.n_tiles + tile], m);
    pos = uni(pos);
    if ((lv >> lane) & 1u) w.scratch[(size_t)tile * kTileSlots + pos + __popcll(lv & lanemask_lt())] = tok;
    CTOK_CHECK_REC(m >= 1 && m <= len && pos + m <= (uint32_t)kTileSlots,
                   "[ctok check] sparse class 3 tile %u: record m=%u n=%u pos=%u\n", tile, m, len, pos);
    if (lane == 0) {
      w.mrec[(size_t)tile * kTileSlots + o] = rec_short(m, pos);
      atomicAdd(&w.tile_tok[tile], m);
    }
    st_bytes += len;
    st_ids += m;
  }
  if (lane == 0 && st_bytes) {  // statistics: bytes merged / ids produced by class 3
    atomicAdd(&w.counters[ctr_stat(3)], st_bytes);
    atomicAdd(&w.counters[ctr_stat(3) + 1], st_ids);
  }
}

constexpr int kSparseWaves = 16;  // waves per k_bpe_sparse workgroup (beside the 96 KiB image: one per CU)

template <bool COMPACT, bool NARROW>
__global__ __launch_bounds__(64 * kSparseWaves) void k_bpe_sparse(Work w, Tables t, uint32_t n) {
  if (spec_failed(w)) return;
  WgRec::begin(w.wgrec, 3);
  extern __shared__ __attribute__((aligned(16))) uint4 s_dyn[];
  __shared__ int32_t s_b2id[256];
  const uint32_t tid = threadIdx.x;
  const uint4* img = NARROW ? t.lds16_image : t.lds_image;
  for (uint32_t i = tid; i < kLdsImageBytes / 16; i += 64 * kSparseWaves) s_dyn[i] = img[i];
  for (uint32_t i = tid; i < 256; i += 64 * kSparseWaves) s_b2id[i] = t.byte2id[i];
  __syncthreads();
  const PairLds P{(const lds_u64*)s_dyn, (const lds_u32*)(s_dyn + kHotBuckets)};
  sparse_c3<COMPACT, NARROW>(w, t, P, s_b2id, n);
  __syncthreads();
  WgRec::end(w.wgrec, 3, 1);
}


// Pieces of 17..32 bytes (CLS = 2, on the main stream after k_bpe_short) or 33..64 bytes (CLS = 3,
// e.g. runs of CJK letters, 3 bytes each): 512-thread workgroups (two waves per SIMD at <= 256
// VGPRs: 32 or 64 register slots per thread) with the whole LDS image.  One class per kernel:
// the fully unrolled 64- and 32-slot loops together overflow the instruction cache.
// Class 3 is launched twice, once on the side stream after the long-piece tiers and once on the
// main stream after class 2; both instances take chunks from the same counter, so a handful of
// class-3 pieces (long merge chains) is done by the side instance in the shadow of the main
// stream's passes, and a large class 3 (multilingual text) is shared by both as CUs free up.
// Most tiles per chunk of the 17..32 B / 33..64 B passes: these classes can be sparse (C4: ~5
// class-2 pieces per tile), where 64 tiles left most of a 512-thread workgroup idle per chunk.
// NT: threads per workgroup.  The 17..32 B pass runs at 768 (three waves per SIMD at 168 VGPRs,
// 152 KiB of LDS) when the call has no long pieces -- on C4 0.60 -> 0.55 ms --, else at 512: with
// long pieces the side stream's tiers share the CUs, and 768 made C5 slower (+0.12 ms,
// profiles/r05/v17_ab_mid768_c4_c5.txt).
template <int CLS> struct MidCfg { static constexpr int KT = 256; };

template <bool COMPACT, int CLS, bool NARROW, uint32_t NT = 512>
__global__ __launch_bounds__(NT) void k_bpe_mid(Work w, Tables t) {
  if (spec_failed(w)) return;
  constexpr int KT = MidCfg<CLS>::KT;
  extern __shared__ __attribute__((aligned(16))) uint4 s_img[];
  __shared__ int32_t s_b2id[256];
  __shared__ PassLds<kSortCap, KT> S;
  __shared__ uint32_t s_key[NARROW ? 8 * NT : 1];
  __shared__ uint16_t s_tok[NARROW ? 8 * NT : 1];
  // (the image is loaded up front: a lazy load pushes the 64-slot pass into scratch; the kernel
  // returns at once when k_segment found no piece of its class)
  if constexpr (CLS == 2) WgRec::begin(w.wgrec, 1);  // (not in the 64-slot pass: it is at its register limit)
  if (w.counters[CLS == 2 ? kCtrAnyMid : kCtrAnyC3] == 0) {
    if constexpr (CLS == 2) WgRec::end(w.wgrec, 1, 0);
    return;
  }
  // every chunk already taken (the other instance of class 3 got there first): one read for the
  // whole workgroup, so its waves leave together (a wave that stayed would find thread 0 gone)
  __shared__ uint32_t s_left;
  if (threadIdx.x == 0)
    s_left = (uint64_t)__atomic_load_n(&w.counters[ctr_chunk(CLS)], __ATOMIC_RELAXED) * w.unit < w.n_tiles;
  __syncthreads();
  if (!s_left) {
    if constexpr (CLS == 2) WgRec::end(w.wgrec, 1, 0);
    return;
  }
  const uint32_t tid = threadIdx.x;
  const uint4* img = NARROW ? t.lds16_image : t.lds_image;
  for (uint32_t i = tid; i < kLdsImageBytes / 16; i += NT) s_img[i] = img[i];
  for (uint32_t i = tid; i < 256; i += NT) s_b2id[i] = t.byte2id[i];
  bool loaded = true;
  const PairLds P{(const lds_u64*)s_img, (const lds_u32*)(s_img + kHotBuckets)};
  class_pass<CLS == 2 ? 32 : 64, COMPACT, true, NT, kSortCap, NARROW, KT>(w, t, P, s_b2id, S, loaded, [] {},
                                                                         (lds_u32*)s_key, (lds_u16*)s_tok);
  if constexpr (CLS == 2) WgRec::end(w.wgrec, 1, 1);
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): the attribute is set
// on the current device's instance of the kernel, and ctok_exec.devices launches from one host
// thread per device at once, so the flag is a per-device bit under a lock (one per kernel).
struct LdsAttr {
  std::mutex mu;
  uint64_t done = 0;  // bit d: set on device d (ordinals >= 64 set it on every call)
};
static hipError_t lds_attr_once(LdsAttr& a, const void* fn, size_t bytes) {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  const uint64_t bit = dev < 64 ? 1ull << dev : 0ull;
  std::lock_guard<std::mutex> lk(a.mu);
  if (a.done & bit) return hipSuccess;
  HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  a.done |= bit;
  return hipSuccess;
}

template <bool C, int CLS, bool NW>
static hipError_t launch_mid_t(const Work& w, const Tables& t, hipStream_t s, const Lx& x) {
  static LdsAttr attr;
  HIPCHK(lds_attr_once(attr, (const void*)k_bpe_mid<C, CLS, NW>, kLdsImageBytes));
  if (!w.n_tiles) return hipSuccess;
  const uint32_t grid = min((w.n_tiles + w.unit - 1) / w.unit, w.n_cus);
  if constexpr (CLS == 2) {
    if (w.mid_wide) {
      static LdsAttr attr768;
      HIPCHK(lds_attr_once(attr768, (const void*)k_bpe_mid<C, CLS, NW, 768>, kLdsImageBytes));
      launch_lx(x, k_bpe_mid<C, CLS, NW, 768>, grid, 768, kLdsImageBytes, s, w, t);
      return hipGetLastError();
    }
  }
  launch_lx(x, k_bpe_mid<C, CLS, NW>, grid, 512, kLdsImageBytes, s, w, t);
  return hipGetLastError();
}
template <bool C, int CLS>
static hipError_t launch_mid(const Work& w, const Tables& t, hipStream_t s, const Lx& x = {}) {
  return t.narrow ? launch_mid_t<C, CLS, true>(w, t, s, x) : launch_mid_t<C, CLS, false>(w, t, s, x);
}

template <bool C, bool NW>
static hipError_t launch_short_t(const Work& w, const Tables& t, hipStream_t s, const Lx& x) {
  static LdsAttr attr;
  HIPCHK(lds_attr_once(attr, (const void*)k_bpe_short<C, NW>, kLdsImageBytes));
  if (!w.n_tiles) return hipSuccess;
  // (Work::short_wgs: fewer workgroups than CUs leave CUs to the side stream's passes from the start)
  const uint32_t grid = min((w.n_tiles + w.unit - 1) / w.unit, w.short_wgs ? min(w.short_wgs, w.n_cus) : w.n_cus);
  if (t.dbg == 30) {
    k_bpe_short<C, NW><<<grid, ShortCfg<NW>::NT, kLdsImageBytes, s>>>(w, t, 1u);
    k_bpe_short<C, NW><<<grid, ShortCfg<NW>::NT, kLdsImageBytes, s>>>(w, t, 2u);
  } else {
    launch_lx(x, k_bpe_short<C, NW>, grid, ShortCfg<NW>::NT, kLdsImageBytes, s, w, t, 3u);
  }
  return hipGetLastError();
}
template <bool C>
static hipError_t launch_short(const Work& w, const Tables& t, hipStream_t s, const Lx& x) {
  return t.narrow ? launch_short_t<C, true>(w, t, s, x) : launch_short_t<C, false>(w, t, s, x);
}

template <bool C, bool NW>
static hipError_t launch_sparse_t(const Work& w, const Tables& t, uint32_t n_pieces, hipStream_t s, const Lx& x) {
  static LdsAttr attr;
  HIPCHK(lds_attr_once(attr, (const void*)k_bpe_sparse<C, NW>, kLdsImageBytes));
  const uint32_t grid = std::max(1u, std::min((n_pieces + kSparseWaves - 1) / kSparseWaves, w.n_cus));  // (a wave per piece at most)
  launch_lx(x, k_bpe_sparse<C, NW>, grid, 64 * kSparseWaves, kLdsImageBytes, s, w, t, n_pieces);
  return hipGetLastError();
}

hipError_t launch_c3_sparse(const Work& w, const Tables& t, uint32_t n_pieces, hipStream_t s, Lx x) {
  if (!n_pieces || n_pieces > w.c3_max || !w.n_tiles) return hipSuccess;
  if (t.compact)
    return t.narrow ? launch_sparse_t<true, true>(w, t, n_pieces, s, x) : launch_sparse_t<true, false>(w, t, n_pieces, s, x);
  return t.narrow ? launch_sparse_t<false, true>(w, t, n_pieces, s, x) : launch_sparse_t<false, false>(w, t, n_pieces, s, x);
}

hipError_t launch_bpe_class(const Work& w, const Tables& t, int cls, hipStream_t s, Lx x) {
  if (t.n_at != 0) {  // every <= 32 B piece is in list0
    if (cls == 0 && w.n_tiles)
      launch_lx(x, k_bpe_generic<false>, (w.n_tiles + kTilesGeneric - 1) / kTilesGeneric, 256, 0, s, w, t);
    return hipGetLastError();
  }
  switch (cls) {
    case 0: return t.compact ? launch_short<true>(w, t, s, x) : launch_short<false>(w, t, s, x);  // classes 0 and 1
    case 2: return t.compact ? launch_mid<true, 2>(w, t, s, x) : launch_mid<false, 2>(w, t, s, x);
    case 4: return t.compact ? launch_mid<true, 3>(w, t, s, x) : launch_mid<false, 3>(w, t, s, x);  // main-stream instance
    case 3:  // pieces with dropped bytes, found by the merge passes (none when every byte's char is in the vocab)
      if (t.all_bytes) return hipSuccess;
      launch_lx(x, k_bpe_generic<true>, 64, 128, 0, s, w, t);
      return hipGetLastError();
    default:
      return hipSuccess;
  }
}

// ------------------------------------------------------------------------------------------
// BPE, long pieces: one wavefront per piece over a doubly linked token list in global memory.
// Each round finds the global minimum rank r (wave reduction).  If the merge table is
// rank-monotone ("proper": every merge consuming token z ranks after every merge producing
// z), the sequential algorithm applies all non-overlapping occurrences of r left to right
// before any other merge, so they are applied in one parallel round; (x,x) chains and
// non-monotone tables fall back to the exact sequential order.

// Working state of one long piece.  GMEM = arrays in global memory (any length): every access
// is an agent-scope relaxed atomic (`global_load/store ... sc1`, served by L2), so lanes of the
// wave see each other's stores between rounds (the vector L1 does not).  LDS = arrays in the
// wave's slice of LDS (pieces up to kLdsPos), accessed through address-space-3 pointers so the
// compiler emits in-order ds_read/ds_write (never flat).
template <bool GMEM>
struct LongState;

template <>
struct LongState<true> {
  uint32_t* tok;
  uint32_t* nxt;
  uint32_t* prv;
  uint32_t* rk;
  static __device__ __forceinline__ uint32_t ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  static __device__ __forceinline__ void st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ uint32_t Tok(uint32_t i) const { return ld(tok + i); }
  __device__ __forceinline__ uint32_t Nxt(uint32_t i) const { return ld(nxt + i); }
  __device__ __forceinline__ uint32_t Prv(uint32_t i) const { return ld(prv + i); }
  __device__ __forceinline__ uint32_t Rk(uint32_t i) const { return ld(rk + i); }
  __device__ __forceinline__ void sTok(uint32_t i, uint32_t v) const { st(tok + i, v); }
  __device__ __forceinline__ void sNxt(uint32_t i, uint32_t v) const { st(nxt + i, v); }
  __device__ __forceinline__ void sPrv(uint32_t i, uint32_t v) const { st(prv + i, v); }
  __device__ __forceinline__ void sRk(uint32_t i, uint32_t v) const { st(rk + i, v); }
  static __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
  }
};

template <>
struct LongState<false> {
  lds_u32* tok;
  lds_u32* nxt;
  lds_u32* prv;
  lds_u32* rk;
  __device__ __forceinline__ uint32_t Tok(uint32_t i) const { return tok[i]; }
  __device__ __forceinline__ uint32_t Nxt(uint32_t i) const { return nxt[i]; }
  __device__ __forceinline__ uint32_t Prv(uint32_t i) const { return prv[i]; }
  __device__ __forceinline__ uint32_t Rk(uint32_t i) const { return rk[i]; }
  __device__ __forceinline__ void sTok(uint32_t i, uint32_t v) const { tok[i] = v; }
  __device__ __forceinline__ void sNxt(uint32_t i, uint32_t v) const { nxt[i] = v; }
  __device__ __forceinline__ void sPrv(uint32_t i, uint32_t v) const { prv[i] = v; }
  __device__ __forceinline__ void sRk(uint32_t i, uint32_t v) const { rk[i] = v; }
  static __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
};

template <bool G>
__device__ __forceinline__ void merge_one(const Tables& t, const LongState<G>& L, uint32_t i, uint32_t nid,
                                          uint32_t* err) {
  const uint32_t j = L.Nxt(i);
  const uint32_t nj = L.Nxt(j);
  L.sTok(i, nid);
  L.sTok(j, kDead);
  L.sRk(j, kNoRank);
  L.sNxt(i, nj);
  if (nj != kNone) L.sPrv(nj, i);
  L.sRk(i, nj != kNone ? rank_of(t, nid, L.Tok(nj), err) : kNoRank);
  const uint32_t p = L.Prv(i);
  if (p != kNone) L.sRk(p, rank_of(t, L.Tok(p), nid, err));
}


template <bool G>
__device__ uint32_t bpe_wave(const Tables& t, const uint8_t* bytes, uint32_t n, const LongState<G>& L, uint32_t* out,
                             uint32_t* err, uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63;
  // initial ids, dropping bytes whose char is not in the vocab (order-preserving compaction)
  uint32_t m = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += 64) {
    const uint32_t i = i0 + lane;
    const int32_t id = i < n ? t.byte2id[bytes[i]] : -1;
    const uint64_t bal = __ballot(id >= 0);
    if (id >= 0) L.sTok(m + __popcll(bal & lanemask_lt()), (uint32_t)id);
    m = uni(m + __popcll(bal));
  }
  L.sync();
  if (m == 0) return 0;
  for (uint32_t i = lane; i < m; i += 64) {
    L.sNxt(i, i + 1 < m ? i + 1 : kNone);
    L.sPrv(i, i > 0 ? i - 1 : kNone);
    L.sRk(i, i + 1 < m ? rank_of(t, L.Tok(i), L.Tok(i + 1), err) : kNoRank);
  }
  L.sync();
  for (;;) {
    uint32_t lmin = kNoRank;
    for (uint32_t i = lane; i < m; i += 64) lmin = min(lmin, L.Rk(i));
    const uint32_t r = uni(wave_min_u32(lmin));
    if (r == kNoRank) break;
    const uint32_t nid = uni(new_id_of(t, r));
    uint32_t lpos = kNone;
    for (uint32_t i = lane; i < m; i += 64) {
      if (L.Rk(i) == r) { lpos = i; break; }
    }
    const uint32_t lm = uni(wave_min_u32(lpos));
    const uint32_t chain = uni(L.Tok(lm) == L.Tok(L.Nxt(lm)) ? 1u : 0u);
    // sites past `cut` wait for a later round (eager merges, see first_cascade)
    uint32_t cut = kNone;
    if (serial_round(t, r) && !chain) {
      uint32_t c = kNone;
      for (uint32_t i = lane; i < m; i += 64) {
        if (L.Rk(i) != r) continue;
        const uint32_t pp = L.Prv(i), j = L.Nxt(i), nj = L.Nxt(j);
        const bool left_site = pp != kNone && L.Prv(pp) != kNone && L.Rk(L.Prv(pp)) == r;
        const uint32_t rl = pp == kNone ? kNoRank : rank_of(t, left_site ? nid : L.Tok(pp), nid, sink);
        const uint32_t rr = nj == kNone ? kNoRank : rank_of(t, nid, L.Tok(nj), sink);
        if (rl < r || rr < r) c = min(c, i);
      }
      cut = uni(wave_min_u32(c));
    }
    if (serial_round(t, r) && chain) {
      merge_one(t, L, lm, nid, err);  // every lane performs the same update
    } else if (chain) {
      // (x,x) runs: the sequential left-to-right order, walked by the whole wave in lockstep
      for (uint32_t i = lm; i != kNone; i = uni(L.Nxt(i))) {
        if (uni(L.Rk(i)) == r) merge_one(t, L, i, nid, err);
      }
    } else {
      // phase A: splice out the right token of every occurrence (up to cut)
      for (uint32_t i = lane; i < m; i += 64) {
        if (L.Rk(i) != r || (cut != kNone && i > cut)) continue;
        const uint32_t j = L.Nxt(i);
        const uint32_t nj = L.Nxt(j);
        L.sTok(i, nid);
        L.sTok(j, kDead);
        L.sRk(j, kNoRank);
        L.sRk(i, kSel);
        L.sNxt(i, nj);
        if (nj != kNone) L.sPrv(nj, i);
      }
      L.sync();
      // phase B: ranks of the new pairs (left pair only when its left end is not a site)
      for (uint32_t i = lane; i < m; i += 64) {
        if (L.Rk(i) != kSel) continue;
        const uint32_t nj = L.Nxt(i);
        L.sRk(i, nj != kNone ? rank_of(t, nid, L.Tok(nj), err) : kNoRank);
        const uint32_t p = L.Prv(i);
        if (p != kNone && L.Rk(p) != kSel) L.sRk(p, rank_of(t, L.Tok(p), nid, err));
      }
    }
    L.sync();
    // (no per-round read of the panic flag: a panicking pair ranks as kNoRank, so the loop still
    // ends, and the host discards the batch -- a global load per round would double its latency)
  }
  // emit surviving tokens in order
  uint32_t c = 0;
  for (uint32_t i0 = 0; i0 < m; i0 += 64) {
    const uint32_t i = i0 + lane;
    const uint32_t v = i < m ? L.Tok(i) : kDead;
    const uint64_t bal = __ballot(v != kDead);
    if (v != kDead) out[c + __popcll(bal & lanemask_lt())] = v;
    c = uni(c + __popcll(bal));
  }
  return c;
}

constexpr uint32_t kLdsPos = 2048;  // positions per wave in LDS (4 u32 arrays: 32 KiB per wave)
constexpr uint32_t kWaveMax = 64 * 64;  // longest piece of the dense wave tiers (k_bpe_wave)

template <bool G>
__device__ uint32_t long_piece(const Tables& t, const uint8_t* bytes, uint32_t n, const LongState<G>& L,
                               uint32_t* out, uint32_t* err) {
  const uint32_t lane = threadIdx.x & 63;
  if (t.n_at == 0) return bpe_wave<G>(t, bytes, n, L, out, err, err - 2 + kCtrSink);
  uint32_t cnt = 0, pos = 0;
  while (pos < n) {  // every lane computes the same added-token split; kept in SGPRs
    int32_t best = -1;
    uint32_t blen = 0;
    for (uint32_t k = 0; k < t.n_at; k++) {
      const uint32_t m = t.at_off[k + 1] - t.at_off[k];
      if (AddedMatch::find(t, k, bytes + pos, n - pos) == 0 && (best < 0 || m > blen)) { best = (int32_t)k; blen = m; }
    }
    best = (int32_t)uni((uint32_t)best);
    blen = uni(blen);
    if (best >= 0) {
      if (lane == 0) out[cnt] = t.at_id[best];
      cnt++;
      pos += blen;
      continue;
    }
    uint32_t nxt = n - pos;
    for (uint32_t k = 0; k < t.n_at; k++) {
      const int64_t f = AddedMatch::find(t, k, bytes + pos, n - pos);
      if (f > 0 && (uint32_t)f < nxt) nxt = (uint32_t)f;
    }
    nxt = uni(nxt);
    cnt = uni(cnt + bpe_wave<G>(t, bytes + pos, nxt, L, out + cnt, err, err - 2 + kCtrSink));
    pos += nxt;
  }
  return cnt;
}

// End of the piece starting at s: the next set bit of the piece-start bitmap, else n_bytes.
// Wave-uniform (64 bitmap words per step).
__device__ __forceinline__ uint32_t piece_end(const Work& w, uint32_t s) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t first = (s + 1) >> 5, sh = (s + 1) & 31;
  for (uint32_t base = first; base < w.n_words; base += 64) {
    const uint32_t idx = base + lane;
    uint32_t v = idx < w.n_words ? w.pbits[idx] : 0u;
    if (idx == first) v &= ~0u << sh;
    const uint64_t m = __ballot(v != 0);
    if (m) {
      const uint32_t l = uni(__ffsll((unsigned long long)m) - 1);
      const uint32_t vv = uni((uint32_t)__shfl((int)v, (int)l, 64));
      return min(w.n_bytes, ((base + l) << 5) + (uint32_t)__builtin_ctz(vv));
    }
  }
  return w.n_bytes;
}

// One wavefront per long piece, pieces dealt to waves by a static stride (no work-queue
// atomics: every loop bound and index is a scalar, so the wave never splits).  GMEM selects the
// tier: LDS for pieces up to kLdsPos positions, global memory beyond.
template <bool GMEM>
__global__ __launch_bounds__(256) void k_bpe_long(Work w, Tables t) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_long[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = uni(threadIdx.x >> 6);
  const uint32_t n_long = uni(long_count(w));
  const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
  uint32_t* err = &w.counters[2];
  for (uint32_t li = uni(blockIdx.x * (blockDim.x >> 6) + wid); li < n_long; li += n_waves) {
    const uint64_t e = w.long_list[li];
    const uint32_t s = uni((uint32_t)e);
    const uint32_t o = uni(long_ord(e));
    const uint32_t n = uni(piece_end(w, s) - s);
    // tiers: LDS up to kLdsPos positions, global memory beyond (only beyond the dense wave tiers
    // when those run, i.e. without added tokens)
    const uint32_t gmin = (t.n_at != 0 || t.dbg == 7) ? kLdsPos : kWaveMax;
    if (GMEM != (n > gmin)) continue;
    const uint8_t* bytes = w.text + s;
    uint32_t* out = w.lids + w.long_pos[li];
    uint32_t cnt;
    if constexpr (GMEM) {
      uint32_t* lw = w.lw + 4 * (size_t)w.lw_pos[li];
      LongState<true> L{lw, lw + n, lw + 2 * (size_t)n, lw + 3 * (size_t)n};
      cnt = long_piece<true>(t, bytes, n, L, out, err);
    } else {
      lds_u32* lds = (lds_u32*)s_long + wid * 4 * kLdsPos;
      LongState<false> L{lds, lds + kLdsPos, lds + 2 * kLdsPos, lds + 3 * kLdsPos};
      cnt = long_piece<false>(t, bytes, n, L, out, err);
    }
    if (lane == 0) {
      const uint32_t tile = s / kTile;
      w.long_cnt[li] = cnt;
      w.mrec[(size_t)tile * kTileSlots + o] = kRecLong | li;
      atomicAdd(&w.tile_tok[tile], cnt);
    }
  }
}

// ------------------------------------------------------------------------------------------
// BPE, pieces of kMedMax+1 .. 64K bytes without added tokens: one wavefront per piece, the
// piece's tokens and pair ranks dense in the wave's LDS slice (position p in lane p % 64 of
// step p / 64).  A round: r = wave minimum of the pair ranks; the merge sites are every
// position whose pair has rank r (proper tables: occurrences never overlap unless the pair is
// (x, x), where runs take every other site from the left, as the sequential loop does;
// non-monotone tables: the leftmost site only); the sites' right tokens are dropped while the
// survivors are compacted into the other buffer (ballot prefix counts), and only pairs that
// touch a new token are looked up again (Bloom filter in LDS, global table on a Bloom hit).
// The live token count shrinks every round, and so does the work per round.

template <int K>
struct WaveSlice {  // per-wave LDS slice: 64K positions (compacted in place every round)
  static constexpr uint32_t C = 64 * K;
  static constexpr uint32_t kBytes = 8 * C + 2 * (C + 64) + 2 * C;
  lds_u32* base;  // tok | rk | chg | sel | pos (u16: the token's first initial position, window rounds)
  __device__ __forceinline__ lds_u32* tok() const { return base; }
  __device__ __forceinline__ lds_u32* rk() const { return base + C; }
  __device__ __forceinline__ __attribute__((address_space(3))) uint8_t* chg() const {
    return (__attribute__((address_space(3))) uint8_t*)(base + 2 * C);
  }
  __device__ __forceinline__ __attribute__((address_space(3))) uint8_t* sel() const {
    return (__attribute__((address_space(3))) uint8_t*)(base + 2 * C) + C + 64;
  }
  __device__ __forceinline__ __attribute__((address_space(3))) uint16_t* pos() const {
    return (__attribute__((address_space(3))) uint16_t*)(sel() + C + 64);
  }
};

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// value of pair (a, b) (never a byte pair): LDS hot table (HOT) and Bloom filter, the global
// table when neither settles it
template <bool HOT>
__device__ __forceinline__ uint32_t rank_pair(const Tables& t, const PairLds& P, uint32_t a, uint32_t b,
                                              uint32_t* err) {
  const uint32_t h1 = mhash(a, b);
  bool g;
  const uint32_t v = rank_lds<HOT>(P, a, b, h1, mhash2(h1), g);
  if (!g) return v;
  const uint32_t h = h1 & t.merge_mask;
  return resolve_rank(t, pair_key(a, b), h, t.merge_tab[h], err);
}

template <int K, bool HOT>
__device__ uint32_t bpe_wave_dense(const Tables& t, const PairLds& P, const int32_t* s_b2id, const uint8_t* bytes,
                                   uint32_t n, const WaveSlice<K>& S, uint32_t* out, uint32_t* err, uint32_t* sink,
                                 uint32_t* rounds = nullptr /* += this piece's rounds (per-wave register) */) {
  const uint32_t lane = threadIdx.x & 63;
  lds_u32* tok = S.tok();
  lds_u32* rk = S.rk();
  auto chg = S.chg();
  auto sel = S.sel();
  auto pos = S.pos();
  // initial ids (bytes whose char is not in the vocab are dropped: order-preserving compaction);
  // the raw bytes go to chg for the initial pair ranks
  uint32_t m = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += 64) {
    const uint32_t i = i0 + lane;
    const int32_t id = i < n ? s_b2id[bytes[i]] : -1;
    const uint64_t bal = __ballot(id >= 0);
    if (id >= 0) {
      const uint32_t q = m + __popcll(bal & lanemask_lt());
      tok[q] = (uint32_t)id;
      chg[q] = bytes[i];
    }
    m = uni(m + __popcll(bal));
  }
  wave_sync_lds();
  if (m == 0) return 0;
  // initial pairs are byte pairs: the 256 x 256 byte-pair table (byte pairs are left out of the
  // LDS image; every later pair holds a merged token)
#pragma unroll 4
  for (uint32_t p = lane; p < m; p += 64) {
    uint32_t r = kNoRank;
    if (p + 1 < m) {
      r = t.pair0[((uint32_t)chg[p] << 8) | chg[p + 1]];
      if (r != kNoRank && value_panics(t, r)) {
        atomicOr(err, kErrPanic);
        r = kNoRank;
      }
    }
    rk[p] = r;
    pos[p] = (uint16_t)p;
  }
  const uint32_t m0 = m;  // initial positions (window rounds: token spans are in these units)
  wave_sync_lds();
  uint32_t nr = 0;  // rounds (statistics: ctok_stats.long_rounds)
  for (;;) {
    nr++;
    uint32_t lmin = kNoRank;
#pragma unroll 8
    for (uint32_t p = lane; p < m; p += 64) lmin = min(lmin, (uint32_t)rk[p]);
    const uint32_t r = uni(wave_min_full_u32(lmin));
    if (r == kNoRank) break;
    const uint32_t nid = uni(new_id_of(t, r));
    // sites: positions whose pair has rank r; lm = the leftmost
    uint32_t lpos = kNone;
#pragma unroll 4
    for (uint32_t p = lane; p < m; p += 64) {
      const bool site = rk[p] == r;
      sel[p] = site ? 1 : 0;
      lpos = min(lpos, site ? p : kNone);
    }
    const uint32_t lm = uni(wave_min_full_u32(lpos));
    const bool chain = uni(tok[lm] == tok[lm + 1] ? 1u : 0u) != 0;
    wave_sync_lds();
    if (serial_round(t, r) && chain) {
      for (uint32_t p = lane; p < m; p += 64) sel[p] = p == lm ? 1 : 0;
      wave_sync_lds();
    } else if (serial_round(t, r)) {
      // eager merge (first_cascade): the sites up to the first whose sequential new pairs
      // include a lower rank
      uint32_t c = kNone;
      for (uint32_t p = lane; p < m; p += 64) {
        if (!sel[p]) continue;
        const bool left_site = p >= 2 && sel[p - 2];
        const uint32_t rl = p == 0 ? kNoRank : rank_pair<HOT>(t, P, left_site ? nid : (uint32_t)tok[p - 1], nid, sink);
        const uint32_t rr = p + 2 >= m ? kNoRank : rank_pair<HOT>(t, P, nid, tok[p + 2], sink);
        if (rl < r || rr < r) c = min(c, p);
      }
      const uint32_t cm = uni(wave_min_full_u32(c));
      if (cm != kNone) {
        for (uint32_t p = lane; p < m; p += 64)
          if (p > cm) sel[p] = 0;
        wave_sync_lds();
      }
    } else if (chain) {
      // (x, x): in a run of consecutive sites the sequential loop merges the 1st, 3rd, ... one
      // (the choice goes through chg, rewritten by the compaction below)
      for (uint32_t p = lane; p < m; p += 64) {
        uint32_t d = 0;
        if (sel[p]) {
          while (d < p && sel[p - 1 - d]) d++;
        }
        chg[p] = (sel[p] && (d & 1) == 0) ? 1 : 0;
      }
      wave_sync_lds();
      for (uint32_t p = lane; p < m; p += 64) sel[p] = chg[p];
      wave_sync_lds();
    }
    // window rounds (t.window, see bpe_wave_seg): a pair p of rank rc > r merges too when every
    // other pair starting in its window [pos(x) - left(x), end(y) + right(y)) ranks above rc
    // (pos: each token's first initial position, carried through the compaction; end(y) = the
    // next token's pos).  Only local minima are checked (both neighbour pairs lie in every
    // window); the scans walk out from p and stop at the window's ends or the first lower pair.
    if (t.window) {
      for (uint32_t p = lane; p + 1 < m; p += 64) {
        const uint32_t rc = rk[p];
        if (rc == kNoRank || rc == r || (p > 0 && (uint32_t)rk[p - 1] <= rc) || (uint32_t)rk[p + 1] <= rc) continue;
        const uint32_t wl = t.wmeta[tok[p]] & 0xFFFFu, wr = t.wmeta[tok[p + 1]] >> 16;
        const uint32_t p0 = pos[p];
        uint32_t lo = p0 > wl ? p0 - wl : 0u;
        uint32_t hi = (p + 2 < m ? (uint32_t)pos[p + 2] : m0) + wr;
        if (serial_round(t, rc)) {
          // eager candidate (not rank-monotone; see bpe_wave_seg): its new pairs with today's
          // neighbours rank above it, and the window covers the neighbours' own windows
          const uint32_t nn = new_id_of(t, rc);
          const uint32_t rl = p > 0 ? rank_pair<HOT>(t, P, tok[p - 1], nn, sink) : kNoRank;
          const uint32_t rr = p + 2 < m ? rank_pair<HOT>(t, P, nn, tok[p + 2], sink) : kNoRank;
          if (rl <= rc || rr <= rc) continue;
          if (p > 0) {
            const uint32_t wlu = t.wmeta[tok[p - 1]] & 0xFFFFu, pu = pos[p - 1];
            lo = min(lo, pu > wlu ? pu - wlu : 0u);
          }
          if (p + 2 < m) hi = max(hi, (p + 3 < m ? (uint32_t)pos[p + 3] : m0) + (t.wmeta[tok[p + 2]] >> 16));
        }
        bool fire = true;
        for (uint32_t j = p; fire && j > 0;) {
          --j;
          if ((uint32_t)pos[j] < lo) break;
          fire = (uint32_t)rk[j] > rc;
        }
        for (uint32_t j = p + 1; fire && j + 1 < m; j++) {
          if ((uint32_t)pos[j] >= hi) break;
          fire = (uint32_t)rk[j] > rc;
        }
        if (fire) sel[p] = 1;
      }
      wave_sync_lds();
    }
    // in-place compaction: a site's right neighbour is dropped, the site takes its new id (nid,
    // or in window rounds its own rank's).  Position p moves to q <= p; a step reads its 64
    // positions before it writes, and later steps read only positions past every q written so far.
    uint32_t base = 0;
    for (uint32_t p0 = 0; p0 < m; p0 += 64) {
      const uint32_t p = p0 + lane;
      const bool in = p < m;
      const bool site = in && sel[p];
      const bool dead = in && p > 0 && sel[p - 1];
      const bool alive = in && !dead;
      const uint32_t tv = in ? (uint32_t)tok[p] : 0u, rv = in ? (uint32_t)rk[p] : 0u;
      const uint32_t pv = in ? (uint32_t)pos[p] : 0u;
      const uint64_t bal = __ballot(alive);
      if (alive) {
        const uint32_t q = base + __popcll(bal & lanemask_lt());
        tok[q] = site ? (t.window ? new_id_of(t, rv) : nid) : tv;
        rk[q] = rv;
        pos[q] = (uint16_t)pv;
        chg[q] = site ? 1 : 0;
      }
      base = uni(base + __popcll(bal));
    }
    m = base;
    if (lane == 0) chg[m] = 0;
    wave_sync_lds();
    // pairs touching a new token get their rank again
    for (uint32_t p = lane; p < m; p += 64) {
      if (chg[p] | chg[p + 1]) rk[p] = p + 1 < m ? rank_pair<HOT>(t, P, tok[p], tok[p + 1], err) : kNoRank;
    }
    wave_sync_lds();
    // (no per-round read of the panic flag: a panicking pair ranks as kNoRank, so the loop still
    // ends, and the host discards the batch -- a global load per round would double its latency)
  }
#pragma unroll 4
  for (uint32_t p = lane; p < m; p += 64) out[p] = tok[p];
  if (rounds) *rounds += nr;
  return m;
}

// Long pieces (hundreds to thousands of tokens): positions stay put and are linked into a list
// (nxt / prv, u16); lane l owns the contiguous segment [l*S, (l+1)*S), in four groups of S/4
// positions whose ranks it keeps in registers with each group's minimum.  A round costs a
// 64-lane minimum, then only the lanes that hold a site look at the group(s) holding it, and
// only groups whose ranks changed are reloaded -- instead of every round sweeping and compacting
// the whole piece.
template <int K>
struct SegSlice {  // per-wave LDS slice for up to 64K positions
  static constexpr uint32_t C = 64 * K;
  static constexpr uint32_t kBytes = 12 * C + 256 + 1024;
  lds_u32* base;  // tok[C] | rk[C] | nxt[C] u16 | prv[C] u16 (the raw bytes until the list is built) |
                  // dirty[256] u8 (per group) | gmin[256] u32 (per group: its minimum rank, window rounds)
  __device__ __forceinline__ lds_u32* tok() const { return base; }
  __device__ __forceinline__ lds_u32* rk() const { return base + C; }
  __device__ __forceinline__ __attribute__((address_space(3))) uint16_t* nxt() const {
    return (__attribute__((address_space(3))) uint16_t*)(base + 2 * C);
  }
  __device__ __forceinline__ __attribute__((address_space(3))) uint16_t* prv() const { return nxt() + C; }
  __device__ __forceinline__ __attribute__((address_space(3))) uint8_t* dirty() const {
    return (__attribute__((address_space(3))) uint8_t*)(prv() + C);
  }
  __device__ __forceinline__ lds_u32* gmin() const { return (lds_u32*)(dirty() + 256); }
};

constexpr uint32_t kNoPos = 0xFFFFu;

template <int K, bool HOT>
__device__ uint32_t bpe_wave_seg(const Tables& t, const PairLds& P, const int32_t* s_b2id, const uint8_t* bytes,
                                 uint32_t n, const SegSlice<K>& S, uint32_t* out, uint32_t* err, uint32_t* sink,
                                 uint32_t* rounds = nullptr /* += this piece's rounds (per-wave register) */) {
  static_assert(K % 16 == 0 && K <= 64, "segment width: a multiple of 16, at most 64");
  constexpr uint32_t R = K / 4;  // registers per group
  const uint32_t lane = threadIdx.x & 63;
  lds_u32* tok = S.tok();
  lds_u32* rk = S.rk();
  auto nxt = S.nxt();
  auto prv = S.prv();
  auto raw = S.prv();  // (the raw bytes, for the byte-pair ranks, until prv is built)
  auto dirty = S.dirty();
  // initial ids (dropped bytes compacted away); raw bytes parked in prv for the byte-pair ranks.
  // The byte loads of 16 rows of 64 (coalesced) are issued together, then the rows are
  // compacted: one global latency per 1 KiB instead of one per 64 bytes.
  uint32_t m = 0;
  for (uint32_t j0 = 0; j0 * 64 < n; j0 += 16) {
    uint32_t bb[16];
    int32_t id[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t i = (j0 + j) * 64 + lane;
      bb[j] = i < n ? (uint32_t)bytes[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) id[j] = ((j0 + j) * 64 + lane < n) ? s_b2id[bb[j]] : -1;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint64_t bal = __ballot(id[j] >= 0);
      if (id[j] >= 0) {
        const uint32_t q = m + __popcll(bal & lanemask_lt());
        tok[q] = (uint32_t)id[j];
        raw[q] = (uint16_t)bb[j];
      }
      m = uni(m + __popcll(bal));
    }
  }
  wave_sync_lds();
  if (m == 0) return 0;
  // lane l owns positions [l*SW, l*SW + SW) in four groups of G = SW/4 positions: SW is a
  // multiple of 16, so a group's ranks are read with G/4 independent 16-byte LDS loads into
  // v[g*R ..] (one LDS latency per group instead of one per position); positions >= m hold
  // kNoRank.  Group of position p (its dirty flag): p / G, by a multiply-high (p < 2^16).
  const uint32_t SW = min((uint32_t)K, (((m + 63) / 64) + 15) & ~15u);
  const uint32_t G = SW >> 2;
  const uint32_t gmag = (uint32_t)(((1ull << 32) + G - 1) / G);
  auto unit = [&](uint32_t p) { return __umulhi(p, gmag); };
  const uint32_t a0 = lane * SW;
  auto pos = [&](uint32_t b) { return a0 + (b / R) * G + (b % R); };  // site bit -> position
  // initial pair ranks, 16 positions at a time (their byte-pair table loads in flight together)
  for (uint32_t k0 = 0; k0 < SW; k0 += 16) {
    uint32_t sb[17], r[16];
#pragma unroll
    for (int k = 0; k < 17; k++) sb[k] = a0 + k0 + k < m ? (uint32_t)raw[a0 + k0 + k] : 0u;
#pragma unroll
    for (int k = 0; k < 16; k++) r[k] = a0 + k0 + k + 1 < m ? t.pair0[(sb[k] << 8) | sb[k + 1]] : kNoRank;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t p = a0 + k0 + k;
      if (r[k] != kNoRank && value_panics(t, r[k])) {
        atomicOr(err, kErrPanic);
        r[k] = kNoRank;
      }
      rk[p] = r[k];
      if (p < m) nxt[p] = p + 1 < m ? (uint16_t)(p + 1) : (uint16_t)kNoPos;
    }
  }
  wave_sync_lds();  // (every raw byte read before prv overwrites them)
  for (uint32_t k = 0; k < SW; k++) {
    const uint32_t p = a0 + k;
    if (p < m) prv[p] = p > 0 ? (uint16_t)(p - 1) : (uint16_t)kNoPos;
  }
  wave_sync_lds();
  lds_u32* dirty32 = (lds_u32*)dirty;
  dirty32[lane] = 0x01010101u;  // first round: every lane loads its groups
  uint32_t v[K];
  uint32_t gm[4] = {kNoRank, kNoRank, kNoRank, kNoRank};
  wave_sync_lds();
  uint32_t nr = 0;  // rounds (statistics: ctok_stats.long_rounds)
  for (;;) {
    nr++;
    const uint32_t dw = dirty32[lane];
    if (dw) {  // (re)load the changed groups' ranks and their minima
#pragma unroll
      for (int g = 0; g < 4; g++) {
        if (dw & (0xFFu << (8 * g))) {
          const uint4* src = (const uint4*)(rk + a0 + g * G);
          uint32_t mn = kNoRank;
#pragma unroll
          for (int q = 0; q < (int)R / 4; q++) {
            const uint4 x = (uint32_t)(4 * q) < G ? src[q] : make_uint4(kNoRank, kNoRank, kNoRank, kNoRank);
            v[g * R + 4 * q] = x.x;
            v[g * R + 4 * q + 1] = x.y;
            v[g * R + 4 * q + 2] = x.z;
            v[g * R + 4 * q + 3] = x.w;
            mn = min(min(mn, min(x.x, x.y)), min(x.z, x.w));
          }
          gm[g] = mn;
        }
      }
      dirty32[lane] = 0;
    }
    const uint32_t smin = min(min(gm[0], gm[1]), min(gm[2], gm[3]));
    const uint32_t r = uni(wave_min_full_u32(smin));
    if (r == kNoRank) break;
    const uint32_t nid = uni(new_id_of(t, r));
    // this segment's sites as a bit mask (bit g*R + k: position a0 + g*G + k), from the groups
    // whose minimum is r; the leftmost site decides the mode
    uint64_t sites = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {
      if (gm[g] == r) {
#pragma unroll
        for (int k = 0; k < (int)R; k++) sites |= (uint64_t)(v[g * R + k] == r) << (g * R + k);
      }
    }
    const uint32_t first = sites ? pos((uint32_t)__builtin_ctzll(sites)) : kNone;
    // every site holds the same pair (rank r's), so a lane tells (x, x) from its own first site
    // (no second wave reduction on the round's critical path)
    bool chain = false;
    if (sites) chain = tok[first] == tok[nxt[first]];
    const bool eager = serial_round(t, r);
    const bool chain_any = __ballot(chain) != 0;
    if (eager && chain_any) {
      const uint32_t lm = uni(wave_min_full_u32(first));
      sites = first == lm ? (sites & (~sites + 1)) : 0ull;  // the leftmost site only
    } else if (eager) {
      // eager merge (first_cascade): the sites up to the first whose sequential new pairs
      // include a lower rank; the left pair of a site whose left neighbour's left neighbour is
      // a site is (nid, nid), its right pair (nid, the next token as it is now)
      uint32_t c = kNone;
      for (uint64_t rest = sites; rest;) {
        const uint32_t p = pos((uint32_t)__builtin_ctzll(rest));
        rest &= rest - 1;
        const uint32_t pp = prv[p], q = nxt[p];
        const uint32_t nq = nxt[q];
        const uint32_t ppp = pp != kNoPos ? (uint32_t)prv[pp] : kNoPos;
        const bool left_site = ppp != kNoPos && rk[ppp] == r;
        Probe<false, HOT> pl, pr;
        pl.start(t, P, left_site ? nid : (pp != kNoPos ? (uint32_t)tok[pp] : 0u), nid, pp != kNoPos);
        pr.start(t, P, nid, nq != kNoPos ? (uint32_t)tok[nq] : 0u, nq != kNoPos);
        const uint32_t rl = pp != kNoPos ? pl.finish(t, sink) : kNoRank;
        const uint32_t rr = nq != kNoPos ? pr.finish(t, sink) : kNoRank;
        if (rl < r || rr < r) c = min(c, p);
      }
      const uint32_t cm = uni(wave_min_full_u32(c));
      if (cm != kNone) {
        uint64_t keep = 0;
        for (uint64_t rest = sites; rest;) {
          const uint32_t k = (uint32_t)__builtin_ctzll(rest);
          rest &= rest - 1;
          if (pos(k) <= cm) keep |= 1ull << k;
        }
        sites = keep;
      }
    } else if (chain && sites) {
      // (x, x) runs: the 1st, 3rd, ... site of a run (d = sites before p in its run)
      uint64_t keep = 0, rest = sites;
      uint32_t d = 0, last = kNone;
      while (rest) {
        const uint32_t k = (uint32_t)__builtin_ctzll(rest);
        rest &= rest - 1;
        const uint32_t p = pos(k);
        if (last != kNone && prv[p] == last) {
          d++;
        } else {  // run start, or a run entering from the previous segment: walk back
          d = 0;
          for (uint32_t q = prv[p]; q != kNoPos && rk[q] == r; q = prv[q]) d++;
        }
        last = p;
        if ((d & 1) == 0) keep |= 1ull << k;
      }
      sites = keep;
    }
    // Window rounds (t.window: token instances span exactly their strings' lengths; the argument
    // below is for a rank-monotone table -- every pair a merge makes ranks after it -- and holds for
    // any candidate whose merge is not eager; eager ones get the extra check further down).  Besides the sites of the
    // round's rank r, a pair c = (x, y) of rank rc > r merges now when no other pair starting in
    // its window [c - left(x), end(y) + right(y)) ranks <= rc, left(x) / right(y) being the
    // longest left / right side of any merge with x on the right / y on the left (Tables::wmeta).
    // Exact: the sequential loop (src/bpe.rs:88-153) takes merges in non-decreasing rank order,
    // so before c it can only touch x or y by merging some u into (u, x) or (y, v) at a rank <
    // rc; u (v) spans at most left(x) (right(y)) positions next to c, and the first merge
    // building it was a pair of today's tokens inside that span ranked below rc -- which the
    // window excludes.  So c is the first merge that touches x or y, and applying it now leaves
    // the rest of the sequence unchanged (every pair it makes ranks above rc).  Checked at group
    // granularity: c must be its group's only minimum, and every other group the window
    // overlaps must have a larger minimum (gmin, published here each round); a window over more
    // than kWinGroups groups is not checked.  Random-letter 4 KiB runs (C3): ~820 rounds -> ~30.
    uint64_t bsites = 0;
    if (t.window) {
      constexpr uint32_t kWinGroups = 16;
      lds_u32* gmin = S.gmin();
#pragma unroll
      for (int g = 0; g < 4; g++) gmin[4 * lane + g] = gm[g];
      uint32_t cp[4], cb[4];
#pragma unroll
      for (int g = 0; g < 4; g++) {
        cp[g] = kNone;
        cb[g] = 0;
        if (gm[g] != kNoRank && gm[g] != r) {
          uint32_t eq = 0;
#pragma unroll
          for (int k = 0; k < (int)R; k++) eq |= (uint32_t)(v[g * R + k] == gm[g]) << k;
          if (__popc(eq) == 1) {
            const uint32_t k = (uint32_t)__builtin_ctz(eq);
            cb[g] = g * R + k;
            cp[g] = a0 + g * G + k;
          }
        }
      }
      wave_sync_lds();
      uint32_t q[4], tc[4], tq[4], nq[4];
#pragma unroll
      for (int g = 0; g < 4; g++) {
        q[g] = cp[g] != kNone ? (uint32_t)nxt[cp[g]] : kNoPos;
        tc[g] = cp[g] != kNone ? (uint32_t)tok[cp[g]] : 0u;
      }
#pragma unroll
      for (int g = 0; g < 4; g++) {
        tq[g] = q[g] != kNoPos ? (uint32_t)tok[q[g]] : 0u;
        nq[g] = q[g] != kNoPos ? (uint32_t)nxt[q[g]] : kNoPos;
      }
      uint32_t wl[4], wr[4];
#pragma unroll
      for (int g = 0; g < 4; g++) {
        wl[g] = q[g] != kNoPos ? (t.wmeta[tc[g]] & 0xFFFFu) : 0u;
        wr[g] = q[g] != kNoPos ? (t.wmeta[tq[g]] >> 16) : 0u;
      }
      uint32_t lo_x[4], end_x[4];  // window bounds widened for eager candidates (below)
#pragma unroll
      for (int g = 0; g < 4; g++) {
        lo_x[g] = kNone;
        end_x[g] = 0;
      }
      if (!t.proper) {
        // Not rank-monotone (tiktoken-style lists): a candidate whose merge is eager -- some merge
        // consuming its token n ranks below it -- also needs its new pairs with today's
        // neighbours, (u, n) and (n, v), to rank above it, and its window widened to u's and v's
        // own windows ([u - left(u), end(v) + right(v))), so that neither neighbour can change
        // before the sequential loop reaches it; then nothing it makes is taken earlier than the
        // sequential loop would take it.  A non-eager candidate needs neither: every pair its
        // token n makes, with any neighbour, ranks above it (the monotone argument).  Model and
        // random non-monotone tables: tests/window_model.py, tests/test_window_rule.py.
        bool eg[4];
        uint32_t pu[4], tu[4], tv[4], nv[4], nn[4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
          eg[g] = q[g] != kNoPos && serial_round(t, gm[g]);
          pu[g] = eg[g] ? (uint32_t)prv[cp[g]] : kNoPos;
          nn[g] = eg[g] ? new_id_of(t, gm[g]) : 0u;
        }
#pragma unroll
        for (int g = 0; g < 4; g++) {
          tu[g] = pu[g] != kNoPos ? (uint32_t)tok[pu[g]] : 0u;
          tv[g] = eg[g] && nq[g] != kNoPos ? (uint32_t)tok[nq[g]] : 0u;
          nv[g] = eg[g] && nq[g] != kNoPos ? (uint32_t)nxt[nq[g]] : kNoPos;
        }
        Probe<false, HOT> PL[4], PR[4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
          PL[g].start(t, P, tu[g], nn[g], pu[g] != kNoPos);
          PR[g].start(t, P, nn[g], tv[g], eg[g] && nq[g] != kNoPos);
        }
#pragma unroll
        for (int g = 0; g < 4; g++) {
          if (!eg[g]) continue;
          const uint32_t rl = pu[g] != kNoPos ? PL[g].finish(t, sink) : kNoRank;
          const uint32_t rr = nq[g] != kNoPos ? PR[g].finish(t, sink) : kNoRank;
          if (rl <= gm[g] || rr <= gm[g]) {
            q[g] = kNoPos;  // (not a candidate this round)
            continue;
          }
          if (pu[g] != kNoPos) {
            const uint32_t wlu = t.wmeta[tu[g]] & 0xFFFFu;
            lo_x[g] = pu[g] >= wlu ? pu[g] - wlu : 0u;
          }
          if (nq[g] != kNoPos) end_x[g] = (nv[g] == kNoPos ? m : nv[g]) + (t.wmeta[tv[g]] >> 16);
        }
      }
#pragma unroll
      for (int g = 0; g < 4; g++) {
        if (q[g] == kNoPos) continue;
        const uint32_t c = cp[g];
        const uint32_t lo = min(c >= wl[g] ? c - wl[g] : 0u, lo_x[g]);
        const uint32_t end = min(max((nq[g] == kNoPos ? m : nq[g]) + wr[g], end_x[g]), m);
        const uint32_t h0 = unit(lo), h1 = unit(end - 1), own = unit(c);
        if (h1 - h0 >= kWinGroups) continue;
        bool ok = true;
        for (uint32_t h = h0; h <= h1; h++)
          if (h != own && (uint32_t)gmin[h] <= gm[g]) {
            ok = false;
            break;
          }
        if (ok) bsites |= 1ull << cb[g];
      }
      sites |= bsites;
    }
    // A lane's sites go four at a time, the LDS reads (and in phase B the pair lookups, global
    // loads included) of the four in flight together: no read of a phase depends on a write of
    // the same phase (a site's right neighbour q is never a site; the left neighbour pp of a site
    // may be a site, whose phase-A writes the barrier orders first).
    constexpr int kB = 4;
    auto take = [&](uint64_t& rest, uint32_t (&p)[kB]) {
#pragma unroll
      for (int i = 0; i < kB; i++) {
        p[i] = rest ? pos((uint32_t)__builtin_ctzll(rest)) : kNone;
        rest &= rest - 1;
      }
    };
    // One pass (the common round: every site holds a pair (a, b) with a != b, all of them merge,
    // and no lane holds more than kB): the new pairs' tokens are read from the state before the
    // merges -- a site's right pair is (nid, the token after its right neighbour, nid when that
    // is a site itself), its left pair (the token before it, or nid with the site before that
    // when that one merges into it) -- so their lookups, global loads included, are in flight
    // while the merges are written, instead of after a second walk of the list.
    if (!eager && !chain_any && __ballot(__popcll(sites) > (uint32_t)kB || bsites != 0) == 0) {
      uint32_t p[kB], q[kB], pp[kB], nq[kB], ppp[kB], tpp[kB], rnq[kB], tnq[kB], rppp[kB];
      uint64_t rest = sites;
      take(rest, p);
#pragma unroll
      for (int i = 0; i < kB; i++) {
        q[i] = p[i] != kNone ? (uint32_t)nxt[p[i]] : kNoPos;
        pp[i] = p[i] != kNone ? (uint32_t)prv[p[i]] : kNoPos;
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        nq[i] = q[i] != kNoPos ? (uint32_t)nxt[q[i]] : kNoPos;
        ppp[i] = pp[i] != kNoPos ? (uint32_t)prv[pp[i]] : kNoPos;
        tpp[i] = pp[i] != kNoPos ? (uint32_t)tok[pp[i]] : 0u;
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        rnq[i] = nq[i] != kNoPos ? (uint32_t)rk[nq[i]] : kNoRank;
        tnq[i] = nq[i] != kNoPos ? (uint32_t)tok[nq[i]] : 0u;
        rppp[i] = ppp[i] != kNoPos ? (uint32_t)rk[ppp[i]] : kNoRank;
      }
      Probe<false, HOT> R[kB], L[kB];
      uint32_t lpos[kB];
#pragma unroll
      for (int i = 0; i < kB; i++) {
        const bool left_site = rppp[i] == r;  // (rank r: a site, which takes pp in)
        lpos[i] = left_site ? ppp[i] : pp[i];
        R[i].start(t, P, nid, rnq[i] == r ? nid : tnq[i], p[i] != kNone && nq[i] != kNoPos);
        L[i].start(t, P, left_site ? nid : tpp[i], nid, p[i] != kNone && pp[i] != kNoPos);
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        if (p[i] == kNone) continue;
        tok[p[i]] = nid;
        tok[q[i]] = kDead;
        rk[q[i]] = kNoRank;
        nxt[p[i]] = (uint16_t)nq[i];
        if (nq[i] != kNoPos) prv[nq[i]] = (uint16_t)p[i];
        dirty[unit(q[i])] = 1;
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        if (p[i] == kNone) continue;
        const uint32_t rr = R[i].finish(t, err), rl = L[i].finish(t, err);
        rk[p[i]] = nq[i] != kNoPos ? rr : kNoRank;
        dirty[unit(p[i])] = 1;
        if (pp[i] != kNoPos) {
          rk[lpos[i]] = rl;
          dirty[unit(lpos[i])] = 1;
        }
      }
      wave_sync_lds();
      continue;
    }
    // phase A: every selected site merges with its right neighbour (window rounds: each site
    // with its own rank's new id; no site is another site's right neighbour, whose rank this
    // phase overwrites)
    for (uint64_t rest = sites; rest;) {
      uint32_t p[kB], q[kB], nq[kB], np[kB];
      take(rest, p);
#pragma unroll
      for (int i = 0; i < kB; i++) {
        q[i] = p[i] != kNone ? (uint32_t)nxt[p[i]] : kNoPos;
        np[i] = nid;
        if (t.window && p[i] != kNone) np[i] = (uint32_t)rk[p[i]];
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        nq[i] = p[i] != kNone ? (uint32_t)nxt[q[i]] : kNoPos;
        if (t.window && p[i] != kNone) np[i] = new_id_of(t, np[i]);
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        if (p[i] == kNone) continue;
        tok[p[i]] = np[i];
        tok[q[i]] = kDead;
        rk[q[i]] = kNoRank;
        nxt[p[i]] = (uint16_t)nq[i];
        if (nq[i] != kNoPos) prv[nq[i]] = (uint16_t)p[i];
        dirty[unit(q[i])] = 1;
      }
    }
    wave_sync_lds();
    // phase B: the new pairs' ranks.  When the left neighbour pp is itself a site, its right-pair
    // lookup and this site's left-pair lookup are the same pair (nid, nid) and write the same rank.
    for (uint64_t rest = sites; rest;) {
      uint32_t p[kB], q[kB], pp[kB], tq[kB], tp[kB], ts[kB];
      take(rest, p);
#pragma unroll
      for (int i = 0; i < kB; i++) {
        q[i] = p[i] != kNone ? (uint32_t)nxt[p[i]] : kNoPos;
        pp[i] = p[i] != kNone ? (uint32_t)prv[p[i]] : kNoPos;
        ts[i] = nid;
        if (t.window && p[i] != kNone) ts[i] = (uint32_t)tok[p[i]];
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        tq[i] = q[i] != kNoPos ? (uint32_t)tok[q[i]] : 0u;
        tp[i] = pp[i] != kNoPos ? (uint32_t)tok[pp[i]] : 0u;
      }
      Probe<false, HOT> R[kB], L[kB];
#pragma unroll
      for (int i = 0; i < kB; i++) {
        R[i].start(t, P, ts[i], tq[i], q[i] != kNoPos);
        L[i].start(t, P, tp[i], ts[i], pp[i] != kNoPos);
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        if (p[i] == kNone) continue;
        const uint32_t rr = R[i].finish(t, err), rl = L[i].finish(t, err);
        rk[p[i]] = q[i] != kNoPos ? rr : kNoRank;
        dirty[unit(p[i])] = 1;
        if (pp[i] != kNoPos) {
          rk[pp[i]] = rl;
          dirty[unit(pp[i])] = 1;
        }
      }
    }
    wave_sync_lds();
    // (no per-round read of the panic flag: a panicking pair ranks as kNoRank, so the loop still
    // ends, and the host discards the batch -- a global load per round would double its latency)
  }
  // surviving tokens in position order (rows of 64 positions, 16 rows' LDS reads at a time)
  uint32_t c = 0;
  for (uint32_t i0 = 0; i0 < m; i0 += 16 * 64) {
    uint32_t tv[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t i = i0 + (uint32_t)j * 64 + lane;
      tv[j] = i < m ? (uint32_t)tok[i] : kDead;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint64_t bal = __ballot(tv[j] != kDead);
      if (tv[j] != kDead) out[c + __popcll(bal & lanemask_lt())] = tv[j];
      c = uni(c + __popcll(bal));
    }
  }
  if (rounds) *rounds += nr;
  return c;
}

// Long-piece order.  k_long_len: a wavefront per long piece finds its length (parked in
// long_cnt until a tier overwrites it with the piece's id count) and counts the bucket of each
// piece > kDenseMax B (workgroup histogram in LDS, one global add per non-empty bucket);
// k_long_order: the buckets' exclusive scan (every workgroup computes it, workgroup 0 stores it)
// and the scatter of those pieces' list indices, longest bucket first (LDS ranks within a
// 256-piece step, one global reservation per bucket and step).  The segmented tiers take their
// pieces from their own range of long_ord through a counter: the longest pieces start first and
// a wave that finishes early takes the next one, so a tier's makespan is about its total rounds
// over its waves (with a static stride one wave could draw several of the longest pieces).
// Pieces <= kDenseMax B (many, short: a counter per piece would be a contended atomic each) are
// dealt to the dense tier by a static stride over the long list.
constexpr uint32_t kDenseMax = 256;

// (lwn[li]: the piece's length when the global-memory tier takes it (> gmin bytes), else 0; its
// scan places the pieces' state in lw, the scan of long_cnt places their ids in lids)
__global__ __launch_bounds__(256) void k_long_len(Work w, uint32_t* lwn, uint32_t gmin) {
  __shared__ uint32_t s_hist[kLhBuckets];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n_long = uni(long_count(w));
  const uint32_t n_waves = gridDim.x * 4;
  if (threadIdx.x < (uint32_t)kLhBuckets) s_hist[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t li = uni(blockIdx.x * 4 + (threadIdx.x >> 6)); li < n_long; li += n_waves) {
    const uint64_t e = w.long_list[li];
    const uint32_t s = uni((uint32_t)e);
    const uint32_t kn = uni(long_len(e));  // (k_segment's, when the piece ended within its look-ahead)
    const uint32_t n = kn ? kn : uni(piece_end(w, s) - s);
    if (lane == 0) {
      w.long_cnt[li] = n;
      lwn[li] = n > gmin ? n : 0u;
      if (n > kDenseMax) atomicAdd(&s_hist[long_bucket(n)], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < (uint32_t)kLhBuckets && s_hist[threadIdx.x])
    atomicAdd(&w.long_hist[kLhHist + threadIdx.x], s_hist[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_long_order(Work w) {
  __shared__ uint32_t s_scan[kLhBuckets + 1], s_cnt[kLhBuckets], s_base[kLhBuckets];
  const uint32_t tid = threadIdx.x;
  const uint32_t n_long = long_count(w);
  if (tid == 0) {
    uint32_t a = 0;
    for (int d = 0; d < kLhBuckets; d++) {
      s_scan[d] = a;
      a += w.long_hist[kLhHist + d];
    }
    s_scan[kLhBuckets] = a;
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid <= (uint32_t)kLhBuckets) w.long_hist[kLhScan + tid] = s_scan[tid];
  if (s_scan[kLhBuckets] == 0) return;  // no piece > kDenseMax B
  for (uint32_t b0 = blockIdx.x * 256; b0 < n_long; b0 += gridDim.x * 256) {
    if (tid < (uint32_t)kLhBuckets) s_cnt[tid] = 0;
    __syncthreads();
    const uint32_t li = b0 + tid;
    const uint32_t n = li < n_long ? w.long_cnt[li] : 0u;
    const uint32_t d = long_bucket(n);
    uint32_t r = 0;
    if (n > kDenseMax) r = atomicAdd(&s_cnt[d], 1u);
    __syncthreads();
    if (tid < (uint32_t)kLhBuckets && s_cnt[tid]) s_base[tid] = atomicAdd(&w.long_hist[kLhFill + tid], s_cnt[tid]);
    __syncthreads();
    if (n > kDenseMax) w.long_ord[s_scan[d] + s_base[d] + r] = li;
    __syncthreads();
  }
}

// One wavefront per piece of (LO, 64K] bytes; NW waves per workgroup, each taking the tier's
// pieces (a range of long_ord, longest first) from a counter.  LDS: the merge-table image (HOT:
// hot table + Bloom filter, 96 KiB; else the Bloom filter, 32 KiB) and one slice per wave.
template <int K, uint32_t LO, int NW, bool HOT, bool SEG, bool NOB = false>
__global__ __launch_bounds__(64 * NW) void k_bpe_wave(Work w, Tables t) {
  constexpr uint32_t kSlice = SEG ? SegSlice<K>::kBytes : WaveSlice<K>::kBytes;
  constexpr uint32_t HI = 64u * K;
  static_assert(HI <= 4096 && LO % 64 == 0 && LO < HI, "tier bounds: multiples of the 64 B buckets");
  extern __shared__ __attribute__((aligned(16))) uint4 s_dyn[];
  __shared__ int32_t s_b2id[256];
  constexpr uint32_t kImg = NOB ? 0u : HOT ? kLdsImageBytes / 16 : kBloomWords / 4;  // uint4 units
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wid = uni(tid >> 6);
  static_assert(SEG ? LO >= kDenseMax : HI <= kDenseMax, "ordered tiers: > kDenseMax B; dense tier: <= kDenseMax B");
  const uint32_t n_long = uni(long_count(w));
  const uint32_t lo = SEG ? uni(w.long_hist[kLhScan + kLhBuckets - HI / 64]) : 0u;
  const uint32_t hi = SEG ? uni(w.long_hist[kLhScan + kLhBuckets - LO / 64]) : n_long;
  // (a workgroup past the tier's piece count has nothing to take: return before the image load;
  // the dense tier's workgroups check that they meet a piece of the tier)
  if (lo >= hi || blockIdx.x * NW >= hi - lo) return;
  if constexpr (!SEG) {
    __shared__ uint32_t s_any;
    if (tid == 0) s_any = 0;
    __syncthreads();
    for (uint32_t li = blockIdx.x * NW + wid; li < n_long; li += gridDim.x * NW) {
      if (w.long_cnt[li] <= HI) {
        if (lane == 0) s_any = 1;
        break;
      }
    }
    __syncthreads();
    if (s_any == 0) return;
  }
  // (HOT: hot table + the filter of the other pairs; else the filter of all pairs, stored after
  // the image)
  const uint4* img = HOT ? t.lds_image : t.lds_image + kLdsImageBytes / 16;
  for (uint32_t i = tid; i < kImg; i += 64 * NW) s_dyn[i] = img[i];
  for (uint32_t i = tid; i < 256; i += 64 * NW) s_b2id[i] = t.byte2id[i];
  __syncthreads();
  const PairLds P = HOT ? PairLds{(const lds_u64*)s_dyn, (const lds_u32*)(s_dyn + kHotBuckets)}
                        : PairLds{nullptr, (const lds_u32*)s_dyn, NOB};
  lds_u32* slice = (lds_u32*)((__attribute__((address_space(3))) uint8_t*)(s_dyn + kImg) + (size_t)wid * kSlice);
  uint32_t* err = &w.counters[2];
  uint32_t rounds = 0;  // this wave's rounds over its pieces (statistics; one atomic at the end)
  for (uint32_t step = uni(blockIdx.x * NW + wid);; step += gridDim.x * NW) {
    uint32_t li;
    if constexpr (SEG) {
      // every lane takes part (lane 0 adds 1, the others 0): no divergent branch around the
      // atomic, whose structurised form (a divergent loop exit) once re-ran a piece forever
      const uint32_t k = uni(atomicAdd(&w.long_hist[kLhTake + HI / 64], lane == 0 ? 1u : 0u));
      if (k >= hi - lo) break;
      li = uni(w.long_ord[lo + k]);
    } else {
      if (step >= n_long) break;
      li = step;
    }
    const uint32_t n = uni(w.long_cnt[li]);
    if (!SEG && n > HI) continue;
    const uint64_t e = w.long_list[li];
    const uint32_t s = uni((uint32_t)e);
    const uint32_t o = uni(long_ord(e));
    uint32_t cnt;
    uint32_t* sink = &w.counters[kCtrSink];
    uint32_t* out = w.lids + w.long_pos[li];
    if constexpr (SEG) cnt = bpe_wave_seg<K, HOT>(t, P, s_b2id, w.text + s, n, SegSlice<K>{slice}, out, err, sink, &rounds);
    else cnt = bpe_wave_dense<K, HOT>(t, P, s_b2id, w.text + s, n, WaveSlice<K>{slice}, out, err, sink, &rounds);
    if (lane == 0) {
      const uint32_t tile = s / kTile;
      w.long_cnt[li] = cnt;
      w.mrec[(size_t)tile * kTileSlots + o] = kRecLong | li;
      atomicAdd(&w.tile_tok[tile], cnt);
    }
  }
  if (lane == 0 && rounds) atomicAdd(&w.counters[kCtrRounds], rounds);
}

template <int K, uint32_t LO, int NW, bool HOT, bool SEG, bool NOB = false>
static hipError_t launch_wave(const Work& w, const Tables& t, uint32_t grid, hipStream_t s) {
  static LdsAttr attr;
  const size_t slice = SEG ? SegSlice<K>::kBytes : WaveSlice<K>::kBytes;
  const size_t lds = (NOB ? 0 : HOT ? kLdsImageBytes : kBloomWords * 4) + (size_t)NW * slice;
  HIPCHK(lds_attr_once(attr, (const void*)k_bpe_wave<K, LO, NW, HOT, SEG, NOB>, lds));
  k_bpe_wave<K, LO, NW, HOT, SEG, NOB><<<grid, 64 * NW, lds, s>>>(w, t);
  return hipGetLastError();
}

// Long-piece preparation (side stream): lengths and the tiers' order (k_long_len, k_long_order),
// then the places of every piece's ids in lids (scan of the lengths: ids <= bytes) and of the
// global-memory tier's state in lw (scan of lwn).  long_pos[n_long] / lw_pos[n_long] hold the
// totals, which the host reads back to size lids and lw before it launches the tiers.
hipError_t launch_long_prep(const Work& w, const Tables& t, hipStream_t s, uint32_t n_long, uint32_t* lwn,
                            uint32_t* tmp, uint64_t tmp_cap) {
  if (n_long == 0) return hipSuccess;
  auto cap = [](uint32_t want, uint32_t most) { return std::max(1u, std::min(want, most)); };
  const bool added = t.n_at != 0 || t.dbg == 7;
  HIPCHK(hipMemsetAsync(w.long_hist, 0, kLhWords * sizeof(uint32_t), s));
  k_long_len<<<cap((n_long + 3) / 4, 4 * w.n_cus), 256, 0, s>>>(w, lwn, added ? kLdsPos : kWaveMax);
  if (!added) k_long_order<<<cap((n_long + 255) / 256, w.n_cus), 256, 0, s>>>(w);
  HIPCHK(hipGetLastError());
  HIPCHK(scan_u32(w.long_cnt, w.long_pos, n_long, nullptr, tmp, tmp_cap, s));
  return scan_u32(lwn, w.lw_pos, n_long, nullptr, tmp, tmp_cap, s);
}

// any_gmem: some long piece is longer than the LDS tiers take (launch_long_prep's global-memory
// state total is non-zero); without one the global-memory tier is not launched (it would still
// find every long piece's end to skip it: 0.33 ms on C5)
hipError_t launch_bpe_long(const Work& w, const Tables& t, hipStream_t s, uint32_t n_long, bool any_c3, bool any_gmem) {
  auto cap = [](uint32_t want, uint32_t most) { return std::max(1u, std::min(want, most)); };
  if (t.n_at != 0 || t.dbg == 7) {
    // added tokens can match inside pieces: the linked-list kernel with the added-token split.
    // One wavefront per workgroup (32 KiB of LDS each): a long-piece workgroup fits on a CU next
    // to a merge-pass workgroup (96 KiB), so this pass overlaps them instead of taking CUs away
    if (n_long == 0) return hipSuccess;
    const size_t lds = 4 * kLdsPos * sizeof(uint32_t);
    k_bpe_long<false><<<cap(n_long, 512), 64, lds, s>>>(w, t);
    if (any_gmem) k_bpe_long<true><<<cap((n_long + 3) / 4, 128), 256, 0, s>>>(w, t);
    return hipGetLastError();
  }
  if (n_long) {
    // dense wave tiers: <= 256 B (4 waves per workgroup, Bloom filter only, 43 KiB of LDS: fits
    // next to a merge-pass workgroup), 257..1024 B (segmented, 2 waves per workgroup with the
    // whole image) and 1025..4096 B (segmented, 2 waves with the Bloom filter); longer pieces:
    // GMEM linked list.  Grids: at most one wave per long piece.  (launch_long_prep first: the
    // lengths, the longest-first order of the segmented tiers' pieces, the id places.)
    // The long list holds pieces > kMedMax B and pieces whose end lies past the tile's look-ahead
    // (>= 63 B: they can be shorter than kMedMax), and a tile's class-0 pieces past its list's
    // capacity, so the first tier starts at 1 B.
    // <= 256 B: 16 waves per workgroup, one workgroup per CU (75 KiB of LDS).  A round is a chain
    // of LDS and global round trips, so waves per CU is the lever: C5 31.4 -> 34.5 GB/s against
    // 4 waves x 2 workgroups per CU (which could share a CU with a wide-vocabulary merge pass;
    // profiles/r03/v36_ab_dense_waves.txt)
    if (t.dbg == 12) {  // A/B: the round-2 launch, 4 waves per workgroup, 2 workgroups per CU
      HIPCHK((launch_wave<4, 0, 4, false, false>(w, t, cap((n_long + 3) / 4, 2 * w.n_cus), s)));
    } else {
      HIPCHK((launch_wave<4, 0, 16, false, false>(w, t, cap((n_long + 15) / 16, w.n_cus), s)));
    }
    if (t.dbg == 10) {  // A/B: 257..1024 B four waves per CU
      HIPCHK((launch_wave<16, 256, 4, true, true>(w, t, cap((n_long + 3) / 4, w.n_cus), s)));
    } else if (t.dbg == 15) {  // A/B: 257..1024 B, 8 waves per CU with the Bloom filter only
      HIPCHK((launch_wave<16, 256, 8, false, true>(w, t, cap((n_long + 7) / 8, w.n_cus), s)));
    } else {
      HIPCHK((launch_wave<16, 256, 2, true, true>(w, t, cap((n_long + 1) / 2, w.n_cus), s)));
    }
    // 1025..4096 B: two waves per CU with the Bloom filter only (32 + 2 x 53 KiB) beat one wave
    // with the hot table (96 + 53 KiB): C3 10.3 -> 5.25 ms (profiles/r02/v14_ab_long_tiers.txt)
    if (t.dbg == 9) {  // A/B: the hot-table variant
      HIPCHK((launch_wave<64, 1024, 1, true, true>(w, t, cap(n_long, w.n_cus), s)));
    } else if (t.dbg == 16) {  // A/B: three waves per CU, no Bloom filter (3 x 49 KiB)
      HIPCHK((launch_wave<64, 1024, 3, false, true, true>(w, t, cap((n_long + 2) / 3, w.n_cus), s)));
    } else {
      HIPCHK((launch_wave<64, 1024, 2, false, true>(w, t, cap((n_long + 1) / 2, w.n_cus), s)));
    }
    if (any_gmem) k_bpe_long<true><<<cap((n_long + 3) / 4, 128), 256, 0, s>>>(w, t);
    HIPCHK(hipGetLastError());
  }
  // 33..64 B register pass, side-stream instance (see k_bpe_mid): it shares class 3 with the main
  // instance as the long tiers free CUs; with no long pieces the main instance alone runs it
  if (!any_c3 || n_long == 0) return hipSuccess;
  return t.compact ? launch_mid<true, 3>(w, t, s) : launch_mid<false, 3>(w, t, s);
}


// The call's report (Work::report): k_segment's counters, the class-3 count among them, into
// pinned host words, then the call's sequence number (write_report).  k_bpe_short's first wave
// writes it as that kernel starts (its packet waited for k_segment); this one-wave kernel does it
// when k_bpe_short does not run (added tokens, no tiles).  The host polls the word instead of
// copying the counters on a second stream forked by an event after k_segment; having seen it, it
// knows k_segment has completed, so what it launches next -- on any stream -- needs no fork event.
__global__ __launch_bounds__(64) void k_report(Work w) {
  write_report(w);
}

hipError_t launch_report(const Work& w, hipStream_t s) {
  k_report<<<1, 64, 0, s>>>(w);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// emission.  tile_tok is scanned to each tile's first id (tile_doc to its first document); then
// one wavefront per tile walks the tile's piece records in rounds of 256 pieces: lane l takes
// pieces 256 r + 4 l .. + 3 (one 8- or 16-byte prec load and their pdoc bits), a wave scan
// numbers the round's merged pieces (their mrec slots: consecutive, so the mrec loads are dense
// too), a second scan gives each piece's first id within the tile, and the ids are staged in LDS
// and stored as whole lines: a whole-piece hit's id is its record, a merged piece's ids are
// copied from scratch (or lids).  Loads run ahead: the records two rounds ahead, the merged
// records one round ahead.  A doc-start piece writes tok_off directly when no document is empty,
// else leaves its first id within the tile in tcnt for k_tokoff.

constexpr int kEmitWaves = 4;  // tiles per k_emit workgroup
constexpr uint32_t kEmitStage = 1024;  // ids of one round staged in LDS (4 KiB per wave)

// one lane's four piece records of a round (u16 or u32) and their doc-start bits
template <typename RT>
struct EmitRecs {
  using V = typename std::conditional<sizeof(RT) == 2, uint2, uint4>::type;
  V v;
  uint32_t d;
  __device__ uint32_t rec(int k) const {
    if constexpr (sizeof(RT) == 2) {
      const uint32_t x = k < 2 ? v.x : v.y;
      return (k & 1) ? x >> 16 : x & 0xFFFFu;
    } else {
      return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
    }
  }
};

template <typename RT>
__global__ __launch_bounds__(64 * kEmitWaves) void k_emit(Work w, uint32_t* __restrict__ ids, uint64_t ids_cap,
                                                         uint64_t* __restrict__ tok_off) {
  // (a lean list overflowed: some pieces were never listed, so their merged records were never
  // written -- the host runs the call again with the safe capacities, and this pass must not
  // gather through records no pass wrote)
  if (spec_failed(w) || uni(w.counters[kCtrOverflow]) != 0) return;
  constexpr uint32_t kMerged = sizeof(RT) == 2 ? kRecMerged16 : kRecMerged32;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = uni(blockIdx.x * kEmitWaves + (threadIdx.x >> 6));
  if (tile >= w.n_tiles) return;
  const uint32_t np = uni(w.tile_np[tile]);
  const uint64_t base = uni(w.tile_tok[tile]);
  // no empty documents: the n-th doc-start piece of the tile starts document tile_doc[tile] + n,
  // so tok_off is written here (k_tokoff then only writes tok_off[n_docs])
  const bool direct = uni(w.counters[kCtrEmptyDocs]) == 0;
  const RT* prec = (const RT*)w.prec + (size_t)tile * kTileSlots;
  const uint32_t* mrec = w.mrec + (size_t)tile * kTileSlots;
  const uint32_t* pdoc = w.pdoc + (size_t)tile * (kTileSlots / 32);
  uint32_t* tcnt = w.tcnt + (size_t)tile * kTileSlots;
  const uint32_t* src0 = w.scratch + (size_t)tile * kTileSlots;
  using Recs = EmitRecs<RT>;
  // (no arithmetic on the loaded values here: a use right after the load would wait for it)
  auto load = [&](uint32_t j0) {
    Recs x;
    if (j0 < np) {
      x.v = *reinterpret_cast<const typename Recs::V*>(prec + j0);
      x.d = pdoc[j0 >> 5];
    } else {
      x.v = {};
      x.d = 0;
    }
    return x;
  };
  // the doc-start bits of pieces j0 .. j0 + 3 (j0 % 4 == 0: they share a word)
  auto docs = [&](const Recs& x, uint32_t j0) {
    const uint32_t d = (x.d >> (j0 & 31)) & 15u;
    return j0 + 4 > np ? (j0 < np ? d & ((1u << (np - j0)) - 1u) : 0u) : d;
  };
  __shared__ uint32_t s_stage[kEmitWaves][kEmitStage];
  __shared__ uint32_t s_mrec[kEmitWaves][256];
  lds_u32* stage = (lds_u32*)s_stage[threadIdx.x >> 6];
  lds_u32* smr = (lds_u32*)s_mrec[threadIdx.x >> 6];
  // A round's numbering: one scan of (doc starts << 16 | merged pieces) gives this lane's first
  // merged ordinal and first document; the round's merged records (consecutive in mrec) are
  // loaded by the whole wave, 64 per instruction: the first 64 a round ahead of their use, more
  // (rare on English text) when they are used.
  uint32_t mrun = 0, dnext = uni(w.tile_doc[tile]);  // (wave-uniform)
  struct Ahead {
    uint32_t o, d, nm;  // this lane's first ordinal (within the round) and document; the round's merged pieces
    uint32_t m0;        // the round's first merged ordinal (wave-uniform)
    uint32_t q;         // mrec[m0 + lane]
  };
  auto number = [&](const Recs& x, uint32_t j0) {
    Ahead a;
    uint32_t nm = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) nm += (j0 + k < np && x.rec(k) == kMerged) ? 1u : 0u;
    const uint32_t nd = (uint32_t)__popc(docs(x, j0));
    const uint32_t v = nm | (nd << 16);
    const uint32_t inc = wave_incl_scan(v);
    const uint32_t tot = uni(lane63(inc));
    a.o = (inc - v) & 0xFFFFu;
    a.d = dnext + ((inc - v) >> 16);
    a.nm = tot & 0xFFFFu;
    dnext = uni(dnext + (tot >> 16));
    a.m0 = mrun;
    a.q = lane < a.nm ? mrec[mrun + lane] : 0u;
    mrun = uni(mrun + a.nm);
    return a;
  };
  uint32_t run = 0;  // ids of the earlier rounds (wave-uniform)
  uint32_t r_first = 0;  // the current round's first id within the tile (wave-uniform)
  // (an empty asm reading loaded registers: the compiler waits for those loads there, not at a
  // later use behind the round's stores)
  auto touch = [](const Recs& x) {
    if constexpr (sizeof(RT) == 2) asm volatile("" ::"v"(x.v.x), "v"(x.v.y), "v"(x.d));
    else asm volatile("" ::"v"(x.v.x), "v"(x.v.y), "v"(x.v.z), "v"(x.v.w), "v"(x.d));
  };
  Recs cur = load(4 * lane);
  Ahead acur = number(cur, 4 * lane);
  Recs nx = load(256 + 4 * lane);
  touch(nx);
  if (acur.nm > 0) smr[lane] = acur.q;  // (the first round's; each round writes the next one's)
  for (uint32_t r0 = 0; r0 < np; r0 += 256) {
    const uint32_t j0 = r0 + 4 * lane;
    // this round's merged records into LDS, each lane's four from there
    // Waits: every load of the round is issued before the first wait (the scratch ids), which
    // then also covers the look-ahead loads; the look-ahead values are consumed before the
    // round's stores, so the next round starts without waiting for those stores (vmcnt counts
    // loads and stores together, in issue order).
    if (acur.nm > 64)  // (the round's merged records past the first 64: loaded now)
      for (uint32_t i = 64 + lane; i < acur.nm; i += 64) smr[i] = mrec[acur.m0 + i];
    if (acur.nm > 0) wave_sync_lds();
    uint32_t mv[4];
    {
      uint32_t o = acur.o;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const bool m = j0 + k < np && cur.rec(k) == kMerged;
        mv[k] = m ? smr[o] : 0u;
        o += m ? 1u : 0u;
      }
    }
    // the next round's numbering and merged records, the records of the round after it
    Ahead anx{};
    if (r0 + 256 < np) anx = number(nx, j0 + 256);
    const Recs nx2 = load(j0 + 512);
    // id counts and where the ids are; long pieces' from long_cnt / long_pos, in a wave-uniform
    // branch that waits for those loads itself
    uint32_t c[4];
    const uint32_t* sp[4];
    bool lng = false;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t r = cur.rec(k), v = mv[k];
      const bool merged = j0 + k < np && r == kMerged;
      c[k] = j0 + k >= np ? 0u : !merged ? 1u : (v & 0xFFFFu);
      sp[k] = src0 + (merged ? (v >> 16) & 0xFFFu : 0u);
      lng |= merged && (v & kRecLong);
    }
#ifdef CTOK_CHECK
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t v = mv[k];
      if (j0 + k < np && cur.rec(k) == kMerged) {
        if (v & kRecLong)
          CTOK_CHECK_REC((v & kRecLongMask) < long_count(w), "[ctok check] k_emit tile %u piece %u: long record %08x past %u\n",
                         tile, j0 + k, v, long_count(w));
        else
          CTOK_CHECK_REC((v & 0xFFFFu) <= (uint32_t)kMedMax && ((v >> 16) & 0xFFFu) + (v & 0xFFFFu) <= (uint32_t)kTileSlots,
                         "[ctok check] k_emit tile %u piece %u: merged record %08x out of range\n", tile, j0 + k, v);
      }
    }
#endif
    if (__ballot(lng)) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t v = mv[k];
        if (j0 + k < np && cur.rec(k) == kMerged && (v & kRecLong)) {
          c[k] = w.long_cnt[v & kRecLongMask];
          sp[k] = w.lids + w.long_pos[v & kRecLongMask];
        }
      }
      asm volatile("" ::"v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(sp[0]), "v"(sp[1]), "v"(sp[2]), "v"(sp[3]));
    }
    const uint32_t sum = c[0] + c[1] + c[2] + c[3];
    const uint32_t inc = wave_incl_scan(sum);
    const uint32_t o0 = run + inc - sum;  // this lane's first id within the tile
    run = uni(run + lane63(inc));
    // first ids: all loads of this lane's pieces in flight together
    uint32_t v0[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t r = cur.rec(k);
      v0[k] = r != kMerged ? r : (c[k] != 0 ? sp[k][0] : 0u);
    }
    // the round's ids: staged in LDS when they fit, then written out by the whole wave as 64
    // consecutive dwords per store (whole lines; the lanes' own runs are ~5 ids apart, so direct
    // stores touch a dozen partial lines each); else each lane stores its runs itself
    const uint32_t r_ids = run - r_first;
    const bool staged = r_ids <= kEmitStage;
    if (staged) {
      // first ids into the stage; a merged piece's further ids are copied by the whole wave from a
      // list of (scratch place, count, stage place) descriptors in smr (this round's merged
      // records were read above): one round trip for the round's copies instead of one per piece
      // position k, and the lanes share them evenly (a long piece's ids: its own lane)
      bool sk[4];
      uint32_t nd = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        sk[k] = c[k] > 1 && !(mv[k] & kRecLong);
        nd += sk[k] ? 1u : 0u;
      }
      const uint32_t dinc = wave_incl_scan(nd);
      uint32_t di = dinc - nd;
      const uint32_t n_desc = uni(lane63(dinc));
      uint32_t o = o0 - r_first;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t cj = c[k];
        if (cj > 0) stage[o] = v0[k];
        if (sk[k]) {
          smr[di++] = ((mv[k] >> 16) & 0xFFFu) | (cj << 12) | (o << 19);
        } else if (cj > 1) {
          const uint32_t* spk = sp[k];
          for (uint32_t m = 1; m < cj; m += 4) {
            uint32_t x[4];
#pragma unroll
            for (int i = 0; i < 4; i++) x[i] = m + i < cj ? spk[m + i] : 0u;
#pragma unroll
            for (int i = 0; i < 4; i++)
              if (m + i < cj) stage[o + m + i] = x[i];
          }
        }
        o += cj;
      }
      if (n_desc) {
        wave_sync_lds();
        for (uint32_t q = lane; q < n_desc; q += 64) {
          const uint32_t d = smr[q];
          const uint32_t* spk = src0 + (d & 0xFFFu);
          const uint32_t cj = (d >> 12) & 0x7Fu, so = d >> 19;
          for (uint32_t m = 1; m < cj; m += 4) {
            uint32_t x[4];
#pragma unroll
            for (int i = 0; i < 4; i++) x[i] = m + i < cj ? spk[m + i] : 0u;
#pragma unroll
            for (int i = 0; i < 4; i++)
              if (m + i < cj) stage[so + m + i] = x[i];
          }
        }
      }
    }
    // the look-ahead values in place before any store: the next round's merged records to LDS
    // (this round's were read above), the records it uses waited for here
    if (anx.nm > 0) smr[lane] = anx.q;
    touch(nx2);
    if (staged) {
      wave_sync_lds();
      const uint64_t d0 = base + r_first;
      for (uint32_t i = lane; i < r_ids; i += 64)
        if (d0 + i < ids_cap) ids[d0 + i] = stage[i];
    } else {
      uint32_t o = o0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t cj = c[k];
        const uint64_t dst = base + o;
        if (cj > 0 && dst < ids_cap) ids[dst] = v0[k];
        if (cj > 1) {  // merged / long piece: the rest of its ids, four loads in flight at a time
          const uint32_t* spk = sp[k];
          for (uint32_t m = 1; m < cj; m += 4) {
            uint32_t x[4];
#pragma unroll
            for (int i = 0; i < 4; i++) x[i] = m + i < cj ? spk[m + i] : 0u;
#pragma unroll
            for (int i = 0; i < 4; i++)
              if (m + i < cj && dst + m + i < ids_cap) ids[dst + m + i] = x[i];  // the host reports CTOK_E_CAPACITY when short
          }
        }
        o += cj;
      }
    }
    // document starts / first ids (after the id stores: no load waits behind them)
    {
      const uint32_t dcur = docs(cur, j0);
      uint32_t dord = acur.d;  // this lane's first doc-start piece's document (direct mode)
      uint32_t o = o0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if ((dcur >> k) & 1u) {
          if (direct) tok_off[dord++] = base + o;
          else tcnt[j0 + k] = o;  // read by k_tokoff
        }
        if (w.keep_first && j0 + k < np) tcnt[j0 + k] = o;  // ctok_encode_offsets
        o += c[k];
      }
    }
    r_first = run;
    wave_sync_lds();  // (the next round's staging overwrites the buffer; its smr reads follow)
    cur = nx;
    nx = nx2;
    acur = anx;
  }
}

// tok_off[d] = first id of the piece that starts at doc_off[d] (every non-empty doc starts a
// piece; an empty doc shares the next doc's start, or the end of the text)
__device__ __forceinline__ void tokoff_one(const Work& w, uint64_t* __restrict__ tok_off, uint32_t d) {
  const uint64_t x = w.doc_off[d];
  uint64_t r;
  if (x >= w.n_bytes) {
    r = w.tile_tok[w.n_tiles];
  } else {
    const uint32_t g = (uint32_t)(x >> 6), b = (uint32_t)(x & 63);
    const uint32_t tile = (uint32_t)(x / kTile);
    uint32_t below = __popc(w.pbits[2 * g] & (b >= 32 ? ~0u : ((1u << b) - 1u)));
    if (b > 32) below += __popc(w.pbits[2 * g + 1] & ((1u << (b - 32)) - 1u));
    const uint32_t j = w.wpref[(size_t)tile * 64 + (g - tile * kTileWords)] + below;
    r = (uint64_t)w.tile_tok[tile] + w.tcnt[(size_t)tile * kTileSlots + j];
  }
  tok_off[d] = r;
}

__global__ void k_tokoff(Work w, uint64_t* __restrict__ tok_off) {
  if (w.host_res && blockIdx.x == 0) {  // the call's results into the host's pinned words
    if (threadIdx.x < (uint32_t)kNumCounters) ((uint32_t*)(w.host_res + 1))[threadIdx.x] = w.counters[threadIdx.x];
    if (threadIdx.x == 0) w.host_res[0] = w.tile_tok[w.n_tiles];
    __threadfence_system();
  }
  if (spec_failed(w)) return;
  if (w.counters[kCtrEmptyDocs] == 0) {  // k_emit wrote tok_off[0 .. n_docs)
    if (blockIdx.x == 0 && threadIdx.x == 0) tok_off[w.n_docs] = w.tile_tok[w.n_tiles];
    return;
  }
  for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d <= w.n_docs; d += gridDim.x * blockDim.x)
    tokoff_one(w, tok_off, d);
}

hipError_t launch_emit(const Work& w, uint32_t* ids, uint64_t ids_cap, uint64_t* tok_off, hipStream_t s,
                       bool count_pieces, bool empty_docs, Lx first, Lx last) {
  HIPCHK(scan_tiles(w, s, count_pieces, first));
  if (w.n_tiles) {
    const uint32_t nb = (w.n_tiles + kEmitWaves - 1) / kEmitWaves;
    if (w.rec16) k_emit<uint16_t><<<nb, 64 * kEmitWaves, 0, s>>>(w, ids, ids_cap, tok_off);
    else k_emit<uint32_t><<<nb, 64 * kEmitWaves, 0, s>>>(w, ids, ids_cap, tok_off);
  }
  // (grid-stride: with no empty document only tok_off[n_docs] is left to write)
  launch_lx(last, k_tokoff, empty_docs ? std::min<uint32_t>((w.n_docs + 1 + 255) / 256, 4096) : 1u, 256, 0, s, w,
            tok_off);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// device-wide exclusive scan (4096 elements per 256-thread block, recursive over partials)

constexpr int kScanPer = 16;
constexpr int kScanBlock = 256 * kScanPer;

template <typename T>
__global__ __launch_bounds__(256) void k_scan_reduce(const T* __restrict__ in, uint64_t n_max, const uint32_t* n_dev,
                                                     T* __restrict__ part) {
  __shared__ T s_scan[17];
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_max;
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
  T s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; k++) {
    const uint64_t i = b0 + k;
    if (i < n) s += in[i];
  }
  T total;
  block_excl_scan<T>(s, s_scan, &total);
  if (threadIdx.x == 0) part[blockIdx.x] = total;
}

template <typename T>
__global__ __launch_bounds__(256) void k_scan_apply(const T* in, T* out, uint64_t n_max, const uint32_t* n_dev,
                                                    const T* __restrict__ part_scanned, int write_total) {
  __shared__ T s_scan[17];
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_max;
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
  T v[kScanPer];
  T s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; k++) {
    const uint64_t i = b0 + k;
    v[k] = i < n ? in[i] : T(0);
    s += v[k];
  }
  T total;
  T ex = block_excl_scan<T>(s, s_scan, &total);
  const T base = part_scanned ? part_scanned[blockIdx.x] : T(0);
  ex += base;
#pragma unroll
  for (int k = 0; k < kScanPer; k++) {
    const uint64_t i = b0 + k;
    if (i < n) out[i] = ex;
    ex += v[k];
  }
  if (write_total && threadIdx.x == 0) out[n] = base + total;  // index n is read by no thread
}

template <typename T>
__global__ void k_write_total(T* out, uint64_t n_max, const uint32_t* n_dev, const T* part, uint64_t nb) {
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_max;
  out[n] = part[nb];
}

// exclusive scan of in[0, n) into out[0, n) (in place allowed) and out[n] = total
template <typename T>
static hipError_t scan_impl(const T* in, T* out, uint64_t n_max, const uint32_t* n_dev, T* tmp, uint64_t tmp_cap,
                            hipStream_t s) {
  const uint64_t nb = (n_max + kScanBlock - 1) / kScanBlock;
  if (nb <= 1) {
    k_scan_apply<T><<<1, 256, 0, s>>>(in, out, n_max, n_dev, nullptr, 1);
    return hipGetLastError();
  }
  if (nb + 1 > tmp_cap) return hipErrorInvalidValue;
  T* part = tmp;
  k_scan_reduce<T><<<(unsigned)nb, 256, 0, s>>>(in, n_max, n_dev, part);
  HIPCHK(hipGetLastError());
  HIPCHK(scan_impl<T>(part, part, nb, nullptr, tmp + nb + 1, tmp_cap - nb - 1, s));  // part[nb] = total
  k_scan_apply<T><<<(unsigned)nb, 256, 0, s>>>(in, out, n_max, n_dev, part, 0);
  HIPCHK(hipGetLastError());
  k_write_total<T><<<1, 1, 0, s>>>(out, n_max, n_dev, part, nb);
  return hipGetLastError();
}

uint64_t scan_tmp_elems(uint64_t n_max) {
  uint64_t tot = 0;
  uint64_t n = n_max;
  for (;;) {
    const uint64_t nb = (n + kScanBlock - 1) / kScanBlock;
    if (nb <= 1) break;
    tot += nb + 1;
    n = nb;
  }
  return tot + 16;
}

// Both per-tile scans (tile_tok: the tiles' first ids, tile_doc: their first documents) as ONE
// scan of packed u64 values tok | doc << 32: every partial sum of either array is below 2^32 (ids
// and documents of a call are < 2^32), so the low half never carries into the high one.
// Reduce, scan of the block partials, apply: 3 launches (1 for <= 4096 tiles) instead of 8 (and
// the apply sums the pieces for the statistics, which took a launch of its own).
// The tile scan's blocks: 1024 tiles (4 per thread), so that a call of a few tens of thousands of
// tiles (a 160 MB shard: 40k) spreads its reduce and apply over tens of workgroups instead of ten
// (its 3 launches took 23 us there with 4096-tile blocks)
constexpr int kTileScanPer = 4;
constexpr int kTileScanBlock = 256 * kTileScanPer;

__device__ __forceinline__ uint64_t tile_pair(const Work& w, uint64_t i) {
  return i < w.n_tiles ? (uint64_t)w.tile_tok[i] | ((uint64_t)w.tile_doc[i] << 32) : 0ull;
}

__global__ __launch_bounds__(256) void k_tiles_reduce(Work w, uint64_t* __restrict__ part) {
  __shared__ uint64_t s_scan[17];
  const uint64_t b0 = (uint64_t)blockIdx.x * kTileScanBlock + threadIdx.x * kTileScanPer;
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < kTileScanPer; k++) v += tile_pair(w, b0 + k);
  uint64_t total;
  block_excl_scan<uint64_t>(v, s_scan, &total);
  if (threadIdx.x == 0) part[blockIdx.x] = total;
}

// count: also the batch's pieces (statistics only): the sum of tile_np into counters[5]
__global__ __launch_bounds__(256) void k_tiles_apply(Work w, const uint64_t* __restrict__ part_scanned, uint32_t count) {
  __shared__ uint64_t s_scan[17];
  const uint64_t n = w.n_tiles;
  const uint64_t b0 = (uint64_t)blockIdx.x * kTileScanBlock + threadIdx.x * kTileScanPer;
  uint64_t v[kTileScanPer];
  uint64_t sum = 0;
#pragma unroll
  for (int k = 0; k < kTileScanPer; k++) {
    v[k] = tile_pair(w, b0 + k);
    sum += v[k];
  }
  uint64_t total;
  uint64_t ex = block_excl_scan<uint64_t>(sum, s_scan, &total);
  const uint64_t base = part_scanned ? part_scanned[blockIdx.x] : 0ull;
  ex += base;
#pragma unroll
  for (int k = 0; k < kTileScanPer; k++) {
    const uint64_t i = b0 + k;
    if (i < n) {
      w.tile_tok[i] = (uint32_t)ex;
      w.tile_doc[i] = (uint32_t)(ex >> 32);
    }
    ex += v[k];
  }
  if (count) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kTileScanPer; k++)
      if (b0 + k < n) c += w.tile_np[b0 + k];
    c = wave_sum_full_u32(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&w.counters[5], c);  // (counters are zeroed per call)
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the totals at index n
    w.tile_tok[n] = (uint32_t)(base + total);
    w.tile_doc[n] = (uint32_t)((base + total) >> 32);
  }
}

uint64_t tile_scan_tmp_elems(uint64_t n_tiles) {
  const uint64_t nb = (n_tiles + kTileScanBlock - 1) / kTileScanBlock;
  return nb + 1 + scan_tmp_elems(nb + 1);
}

hipError_t scan_tiles(const Work& w, hipStream_t s, bool count, Lx x) {
  const uint64_t nb = ((uint64_t)w.n_tiles + kTileScanBlock - 1) / kTileScanBlock;
  if (nb <= 1) {
    launch_lx(x, k_tiles_apply, 1, 256, 0, s, w, (const uint64_t*)nullptr, count ? 1u : 0u);
    return hipGetLastError();
  }
  uint64_t* part = reinterpret_cast<uint64_t*>(w.scan_tmp);
  const uint64_t cap = w.scan_tmp_cap / 2;
  if (nb + 1 > cap) return hipErrorInvalidValue;
  launch_lx(x, k_tiles_reduce, (unsigned)nb, 256, 0, s, w, part);
  HIPCHK(hipGetLastError());
  HIPCHK(scan_u64(part, nb, part + nb + 1, cap - nb - 1, s));
  k_tiles_apply<<<(unsigned)nb, 256, 0, s>>>(w, part, count ? 1u : 0u);
  return hipGetLastError();
}

hipError_t scan_u32(const uint32_t* in, uint32_t* out, uint64_t n_max, const uint32_t* n_dev, uint32_t* tmp,
                    uint64_t tmp_cap, hipStream_t s) {
  return scan_impl<uint32_t>(in, out, n_max, n_dev, tmp, tmp_cap, s);
}

hipError_t scan_u64(uint64_t* inout, uint64_t n, uint64_t* tmp, uint64_t tmp_cap, hipStream_t s) {
  return scan_impl<uint64_t>(inout, inout, n, nullptr, tmp, tmp_cap, s);
}

// ------------------------------------------------------------------------------------------
// NFC splice (ctok_host.cpp nfc_splice): after a speculative pass over raw text flagged code
// points NFC may change, only the documents holding them are normalised and encoded again, as a
// sub-batch, and their ids replace the speculative pass's in the output.  rank[d] = flagged docs
// before d (exclusive scan of the NFC-check flags; doc d is flagged when rank[d + 1] > rank[d]).

// flag[d] = 1 when a 64-byte word overlapping doc d holds the start of a code point NFC might
// change (k_segment's nfc_bits; a word shared with a neighbour flags both docs: a superset, and
// NFC leaves an unflagged doc unchanged, so encoding it normalised gives the same ids)
__global__ __launch_bounds__(256) void k_flag_docs(const uint64_t* __restrict__ off, uint64_t n_docs,
                                                   const uint32_t* __restrict__ bits, uint32_t* __restrict__ flag) {
  for (uint64_t d = (uint64_t)blockIdx.x * 256 + threadIdx.x; d < n_docs; d += (uint64_t)gridDim.x * 256) {
    const uint64_t a = off[d], b = off[d + 1];
    uint32_t f = 0;
    if (b > a) {
      const uint64_t g0 = a >> 6, g1 = (b - 1) >> 6;  // words [g0, g1]
      for (uint64_t q = g0 >> 5; q <= (g1 >> 5) && !f; q++) {
        uint32_t m = bits[q];
        if (q == (g0 >> 5)) m &= ~0u << (g0 & 31);
        if (q == (g1 >> 5)) m &= (g1 & 31) == 31 ? ~0u : (2u << (g1 & 31)) - 1u;
        f = m != 0;
      }
    }
    flag[d] = f;
  }
}

// len[d] = bytes of doc d if it is flagged, else 0 (scanned to the sub-batch offsets)
__global__ __launch_bounds__(256) void k_flag_len(const uint64_t* __restrict__ off, const uint32_t* __restrict__ flag,
                                                  uint64_t n_docs, uint64_t* __restrict__ len) {
  for (uint64_t d = (uint64_t)blockIdx.x * 256 + threadIdx.x; d < n_docs; d += (uint64_t)gridDim.x * 256)
    len[d] = flag[d] ? off[d + 1] - off[d] : 0;
}

// one wavefront per flagged doc: its bytes to sub_text at sub_pos[d], its start to sub_off[rank[d]]
__global__ __launch_bounds__(256) void k_gather_flagged(const uint8_t* __restrict__ text, const uint64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ rank, const uint64_t* __restrict__ sub_pos,
                                                        uint64_t n_docs, uint8_t* __restrict__ sub_text,
                                                        uint64_t* __restrict__ sub_off) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t d = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; d < n_docs; d += ((uint64_t)gridDim.x * 256) >> 6) {
    const uint32_t r = rank[d];
    if (rank[d + 1] == r) continue;  // (wave-uniform)
    const uint64_t a = off[d], n = off[d + 1] - a, p = sub_pos[d];
    if (lane == 0) sub_off[r] = p;
    for (uint64_t i = lane; i < n; i += 64) sub_text[p + i] = text[a + i];
  }
}

// cnt[d] = ids of doc d in the spliced output: the sub-batch's for a flagged doc, else the
// speculative pass's (scanned in place to the output tok_off)
__global__ __launch_bounds__(256) void k_splice_count(const uint32_t* __restrict__ rank, const uint64_t* __restrict__ main_off,
                                                      const uint64_t* __restrict__ sub_off, uint64_t n_docs,
                                                      uint64_t* __restrict__ cnt) {
  for (uint64_t d = (uint64_t)blockIdx.x * 256 + threadIdx.x; d < n_docs; d += (uint64_t)gridDim.x * 256) {
    const uint32_t r = rank[d];
    cnt[d] = rank[d + 1] != r ? sub_off[r + 1] - sub_off[r] : main_off[d + 1] - main_off[d];
  }
}

// one wavefront per doc: its ids from the sub-batch or the speculative pass to out_off[d]
__global__ __launch_bounds__(256) void k_splice_copy(const uint32_t* __restrict__ rank, const uint64_t* __restrict__ main_off,
                                                     const uint32_t* __restrict__ main_ids, const uint64_t* __restrict__ sub_off,
                                                     const uint32_t* __restrict__ sub_ids, const uint64_t* __restrict__ out_off,
                                                     uint64_t n_docs, uint32_t* __restrict__ ids, uint64_t ids_cap) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t d = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; d < n_docs; d += ((uint64_t)gridDim.x * 256) >> 6) {
    const uint32_t r = rank[d];
    const bool f = rank[d + 1] != r;
    const uint32_t* src = f ? sub_ids + sub_off[r] : main_ids + main_off[d];
    const uint64_t o = out_off[d], n = out_off[d + 1] - o;
    for (uint64_t i = lane; i < n; i += 64)
      if (o + i < ids_cap) ids[o + i] = src[i];
  }
}

static uint32_t grid_for(uint64_t threads, uint64_t max_blocks = 16384) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((threads + 255) / 256, max_blocks));
}

hipError_t launch_flag_docs(const uint64_t* off, uint64_t n_docs, const uint32_t* nfc_bits, uint32_t* flag, hipStream_t s) {
  if (!n_docs) return hipSuccess;
  k_flag_docs<<<grid_for(n_docs), 256, 0, s>>>(off, n_docs, nfc_bits, flag);
  return hipGetLastError();
}

hipError_t launch_flag_len(const uint64_t* off, const uint32_t* flag, uint64_t n_docs, uint64_t* len, hipStream_t s) {
  if (!n_docs) return hipSuccess;
  k_flag_len<<<grid_for(n_docs), 256, 0, s>>>(off, flag, n_docs, len);
  return hipGetLastError();
}

hipError_t launch_gather_flagged(const uint8_t* text, const uint64_t* off, const uint32_t* rank, const uint64_t* sub_pos,
                                 uint64_t n_docs, uint8_t* sub_text, uint64_t* sub_off, hipStream_t s) {
  if (!n_docs) return hipSuccess;
  k_gather_flagged<<<grid_for(64 * n_docs, 1u << 20), 256, 0, s>>>(text, off, rank, sub_pos, n_docs, sub_text, sub_off);
  return hipGetLastError();
}

hipError_t launch_splice(const uint32_t* rank, const uint64_t* main_off, const uint32_t* main_ids, const uint64_t* sub_off,
                         const uint32_t* sub_ids, uint64_t n_docs, uint32_t* ids, uint64_t ids_cap, uint64_t* out_off,
                         uint64_t* tmp, uint64_t tmp_cap, hipStream_t s) {
  if (!n_docs) return hipSuccess;
  k_splice_count<<<grid_for(n_docs), 256, 0, s>>>(rank, main_off, sub_off, n_docs, out_off);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = scan_u64(out_off, n_docs, tmp, tmp_cap, s);
  if (e != hipSuccess) return e;
  k_splice_copy<<<grid_for(64 * n_docs, 1u << 20), 256, 0, s>>>(rank, main_off, main_ids, sub_off, sub_ids, out_off, n_docs, ids, ids_cap);
  return hipGetLastError();
}

// p[i] += delta (mod 2^64) for i < n: a host-buffer chunk's doc offsets made chunk-relative, its
// tok_off made batch-relative, on the device before the direct copies
__global__ __launch_bounds__(256) void k_shift_u64(uint64_t* __restrict__ p, uint64_t n, uint64_t delta) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) p[i] += delta;
}

// The 16-bit wire format of the host-buffer pipeline (ids16 tokenizers): ids[0, n_ids) as u16
// and tok_off[0, n_off) (chunk-relative, < 2^32) as u32, so the D2H copies move 2 B per id
// instead of 4.  Eight ids per thread: two 16-byte loads, one 16-byte store.
__global__ __launch_bounds__(256) void k_wire16(const uint32_t* __restrict__ ids, uint64_t n_ids, uint16_t* __restrict__ ids16,
                                                const uint64_t* __restrict__ toff, uint64_t n_off,
                                                uint32_t* __restrict__ toff32) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t n8 = n_ids / 8;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
    const uint4 a = reinterpret_cast<const uint4*>(ids)[2 * i], b = reinterpret_cast<const uint4*>(ids)[2 * i + 1];
    reinterpret_cast<uint4*>(ids16)[i] = make_uint4(a.x | (a.y << 16), a.z | (a.w << 16), b.x | (b.y << 16), b.z | (b.w << 16));
  }
  for (uint64_t i = 8 * n8 + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n_ids; i += stride) ids16[i] = (uint16_t)ids[i];
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n_off; i += stride) toff32[i] = (uint32_t)toff[i];
}

hipError_t wire16(const uint32_t* ids, uint64_t n_ids, uint16_t* ids16, const uint64_t* toff, uint64_t n_off,
                  uint32_t* toff32, hipStream_t s) {
  const uint64_t work = std::max<uint64_t>(n_ids / 8, n_off);
  const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((work + 255) / 256, 8192));
  k_wire16<<<g, 256, 0, s>>>(ids, n_ids, ids16, toff, n_off, toff32);
  return hipGetLastError();
}

hipError_t shift_u64(uint64_t* p, uint64_t n, uint64_t delta, hipStream_t s) {
  if (n == 0 || delta == 0) return hipSuccess;
  const uint32_t g = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
  k_shift_u64<<<g, 256, 0, s>>>(p, n, delta);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// NFC (src/normalizers.rs:47): quick check per chunk, exact normalisation per flagged doc.


__device__ __forceinline__ int dev_decode(const uint8_t* s, uint32_t n, uint32_t i, uint32_t* cp) {
  const uint8_t b = s[i];
  if (b < 0x80) { *cp = b; return 1; }
  const int len = u8len(b);
  if (i + len > n) { *cp = 0xFFFD; return 1; }
  if (len == 2) *cp = ((b & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu);
  else if (len == 3) *cp = ((b & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu);
  else *cp = ((b & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu);
  return len;
}

// one thread per 64-byte chunk; a doc is flagged when it holds any code point with
// NFC_QC != Yes or a non-zero combining class (a superset of the docs NFC changes)
__global__ void k_nfc_check(const uint8_t* __restrict__ text, uint64_t n_bytes, const uint64_t* __restrict__ off,
                            uint32_t n_docs, Tables t, uint32_t* doc_flag, uint32_t* counter) {
  const uint64_t c0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 64;
  if (c0 >= n_bytes) return;
  const uint64_t c1 = c0 + 64 < n_bytes ? c0 + 64 : n_bytes;
  bool ascii = true;
  if (c1 - c0 == 64) {
    const uint4* v = reinterpret_cast<const uint4*>(text + c0);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 x = v[k];
      if ((x.x | x.y | x.z | x.w) & 0x80808080u) ascii = false;
    }
  } else {
    for (uint64_t i = c0; i < c1; i++) if (text[i] & 0x80) ascii = false;
  }
  if (ascii) return;
  for (uint64_t i = c0; i < c1;) {
    const uint8_t b = text[i];
    if ((b & 0xC0) == 0x80) { i++; continue; }
    uint32_t cp;
    const int len = dev_decode(text, (uint32_t)(n_bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : n_bytes), (uint32_t)i, &cp);
    const uint16_t f = nfc16(t, cp);
    if (f != 0) {
      // doc of byte i: last d with off[d] <= i and off[d+1] > i
      uint32_t lo = 0, hi = n_docs;  // invariant off[lo] <= i < off[hi]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
      }
      if (atomicOr(&doc_flag[lo], 1u) == 0u) atomicAdd(counter, 1u);
    }
    i += len;
  }
}

hipError_t launch_nfc_check(const uint8_t* text, uint64_t n_bytes, const uint64_t* doc_off, uint32_t n_docs,
                            const Tables& t, uint32_t* doc_flag, uint32_t* counter, hipStream_t s) {
  const uint64_t chunks = (n_bytes + 63) / 64;
  if (chunks) k_nfc_check<<<(unsigned)((chunks + 255) / 256), 256, 0, s>>>(text, n_bytes, doc_off, n_docs, t, doc_flag, counter);
  return hipGetLastError();
}

#define SBASE 0xAC00u
#define LBASE 0x1100u
#define VBASE 0x1161u
#define TBASE 0x11A7u
#define LCOUNT 19u
#define VCOUNT 21u
#define TCOUNT 28u
#define NCOUNT (VCOUNT * TCOUNT)
#define SCOUNT (LCOUNT * NCOUNT)

__device__ int nfc_decompose(const Tables& t, uint32_t cp, uint32_t* o) {
  if (cp >= SBASE && cp < SBASE + SCOUNT) {
    const uint32_t s = cp - SBASE;
    o[0] = LBASE + s / NCOUNT;
    o[1] = VBASE + (s % NCOUNT) / TCOUNT;
    if (s % TCOUNT) { o[2] = TBASE + s % TCOUNT; return 3; }
    return 2;
  }
  int lo = 0, hi = (int)t.n_decomp - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t c = t.decomp_cp[mid];
    if (c == cp) {
      int k = 0;
      for (uint32_t j = t.decomp_off[mid]; j < t.decomp_off[mid + 1]; j++) o[k++] = t.decomp_data[j];
      return k;
    }
    if (c < cp) lo = mid + 1; else hi = mid - 1;
  }
  o[0] = cp;
  return 1;
}

__device__ uint32_t nfc_compose(const Tables& t, uint32_t a, uint32_t b) {
  if (a >= LBASE && a < LBASE + LCOUNT && b >= VBASE && b < VBASE + VCOUNT)
    return SBASE + ((a - LBASE) * VCOUNT + (b - VBASE)) * TCOUNT;
  if (a >= SBASE && a < SBASE + SCOUNT && (a - SBASE) % TCOUNT == 0 && b > TBASE && b < TBASE + TCOUNT)
    return a + (b - TBASE);
  const uint64_t key = ((uint64_t)a << 21) | b;
  int lo = 0, hi = (int)t.n_comp - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint64_t k = t.comp_key[mid];
    if (k == key) return t.comp_val[mid];
    if (k < key) lo = mid + 1; else hi = mid - 1;
  }
  return kNone;
}

// canonical ordering (stable by combining class) then canonical composition of buf[0, k) in place
// (UAX #15); returns the new count
__device__ uint32_t nfc_reorder_compose(const Tables& t, uint32_t* buf, uint32_t k) {
  for (uint32_t i = 1; i < k; i++) {
    const uint32_t c = buf[i];
    const int cc = nfc16(t, c) & 0xFF;
    if (!cc) continue;
    uint32_t j = i;
    while (j > 0) {
      const int pc = nfc16(t, buf[j - 1]) & 0xFF;
      if (pc <= cc || pc == 0) break;
      buf[j] = buf[j - 1];
      j--;
    }
    buf[j] = c;
  }
  if (k == 0) return 0;
  uint32_t starter = 0, comp = 1, sch = buf[0];
  int last = nfc16(t, sch) & 0xFF;
  if (last) last = 256;
  for (uint32_t i = 1; i < k; i++) {
    const uint32_t ch = buf[i];
    const int cc = nfc16(t, ch) & 0xFF;
    const uint32_t c = nfc_compose(t, sch, ch);
    if (c != kNone && (last < cc || last == 0)) { buf[starter] = c; sch = c; continue; }
    if (cc == 0) { starter = comp; sch = ch; }
    last = cc;
    buf[comp++] = ch;
  }
  return comp;
}

__device__ __forceinline__ uint32_t u8size(uint32_t cp) { return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4; }

// NFC of s[0, n) into buf (capacity 4n code points) by one wavefront; returns the code point
// count, *len_out its UTF-8 bytes, *first_out the first code point (0 if none).  A code point
// with nfc16 == 0 (ccc 0 and NFC_QC Yes) is a normalisation boundary: nothing after it combines
// with anything before it, and it is unchanged unless a following code point combines with it.
// So only the segments around unstable code points are normalised -- from the boundary before
// the first (popped back from the output) to the next boundary -- and everything else is copied.
// The wave walks the document in 64-byte windows: every lane decodes the code point starting at
// its byte and looks up its nfc16 (one round of loads per window instead of one per code point),
// the stable code points before the window's first unstable one are appended together, and lane
// 0 normalises the segment there (decomposition / composition table searches for a few code
// points).  Segment workspace in buf[2n ..).
__device__ uint32_t nfc_doc(const Tables& t, const uint8_t* s, uint32_t n, uint32_t* buf, uint64_t* len_out,
                            uint32_t* first_out) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t* tmp = buf + 2 * (size_t)n;
  uint32_t k = 0, first = 0, last = 0;  // wave-uniform: output count, first / last output code point
  uint64_t len = 0;
  bool lb = false;  // the last output code point is a boundary copied through
  for (uint32_t i = 0; i < n;) {
    const uint32_t p = i + lane;
    uint32_t cp = 0;
    bool st = false, un = false;
    if (p < n) {
      st = (s[p] & 0xC0) != 0x80;
      if (st) {
        dev_decode(s, n, p, &cp);
        un = nfc16(t, cp) != 0;
      }
    }
    const uint64_t S = __ballot(st), U = __ballot(st && un);
    const uint64_t keep = U ? S & ((1ull << __builtin_ctzll(U)) - 1ull) : S;  // stable, before the first unstable
    const bool mine = (keep >> lane) & 1ull;
    if (mine) buf[k + __popcll(keep & lanemask_lt())] = cp;
    if (keep) {
      if (k == 0) first = __builtin_amdgcn_readlane(cp, __builtin_ctzll(keep));
      last = __builtin_amdgcn_readlane(cp, 63 - __builtin_clzll(keep));
      k += (uint32_t)__popcll(keep);
      len += wave_sum_full_u32(mine ? u8size(cp) : 0u);  // (phase 1 writes u8size bytes per code point)
      lb = true;
    }
    if (!U) {
      i += 64;
      continue;
    }
    uint32_t j = i + (uint32_t)__builtin_ctzll(U);
    if (lane == 0) {
      uint32_t m = 0;
      if (lb) {  // the boundary before joins the segment
        k--;
        len -= u8size(last);
        m = nfc_decompose(t, last, tmp);
      }
      while (j < n) {
        uint32_t c;
        const int ll = dev_decode(s, n, j, &c);
        if (nfc16(t, c) == 0) break;  // the next boundary ends the segment
        m += nfc_decompose(t, c, tmp + m);
        j += ll;
      }
      m = nfc_reorder_compose(t, tmp, m);
      if (k == 0 && m) first = tmp[0];
      for (uint32_t q = 0; q < m; q++) {
        buf[k++] = tmp[q];
        len += u8size(tmp[q]);
      }
      if (m) last = tmp[m - 1];
    }
    k = __builtin_amdgcn_readlane(k, 0);
    j = __builtin_amdgcn_readlane(j, 0);
    first = __builtin_amdgcn_readlane(first, 0);
    last = __builtin_amdgcn_readlane(last, 0);
    len = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(len >> 32), 0) << 32) | __builtin_amdgcn_readlane((uint32_t)len, 0);
    lb = false;
    i = j;
  }
  *len_out = len;
  *first_out = k ? first : 0u;
  return k;
}


// phase 0: new_len[d] = normalised length (flagged docs: NFC code points left in cp_scratch)
// phase 1: write the normalised text at new_off[d] (new_len scanned into offsets)
// Normalisation (NFC of the flagged documents, optional prefix space), a wavefront per
// document: phase 0 sizes each output document, phase 1 (after a scan) writes it.  An unflagged
// document is copied by the whole wave (consecutive lanes, consecutive bytes); a flagged one is
// normalised by the wave (nfc_doc) into code points, which phase 1 writes as UTF-8.
constexpr int kNormWaves = 4;

__global__ __launch_bounds__(64 * kNormWaves) void k_norm(const uint8_t* __restrict__ text,
                                                          const uint64_t* __restrict__ off, uint32_t n_docs,
                                                          const uint32_t* __restrict__ doc_flag, int add_prefix,
                                                          int nfc, Tables t, uint32_t* cp_scratch, uint32_t* ncp,
                                                          uint64_t* newv, uint8_t* out, int phase) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t d = uni(blockIdx.x * kNormWaves + (threadIdx.x >> 6));
  if (d >= n_docs) return;
  const uint64_t a = off[d];
  const uint32_t n = (uint32_t)(off[d + 1] - a);
  const bool flagged = nfc && uni(doc_flag[d]) != 0;
  uint32_t* buf = cp_scratch + 4 * a;
  if (phase == 0) {
    uint64_t len;
    uint32_t first;
    if (flagged) {
      const uint32_t k = nfc_doc(t, text + a, n, buf, &len, &first);
      if (lane == 0) ncp[d] = k;
    } else {
      len = n;
      first = n ? text[a] : 0;
    }
    if (add_prefix && len > 0 && first != ' ') len += 1;  // src/pretokenizers.rs:163-167
    if (lane == 0) newv[d] = len;
    return;
  }
  uint8_t* o = out + newv[d];
  if (flagged) {  // the code points as UTF-8: a wave scan of their sizes places each lane's bytes
    const uint32_t k = ncp[d];
    const uint32_t pre = (add_prefix && k > 0 && buf[0] != ' ') ? 1u : 0u;
    if (pre && lane == 0) o[0] = ' ';
    uint64_t pos = pre;
    for (uint32_t q0 = 0; q0 < k; q0 += 64) {
      const uint32_t q = q0 + lane;
      const uint32_t c = q < k ? buf[q] : 0u, sz = q < k ? u8size(c) : 0u;
      const uint32_t inc = wave_incl_scan(sz);
      uint8_t* w8 = o + pos + (inc - sz);
      if (sz == 1) {
        w8[0] = (uint8_t)c;
      } else if (sz == 2) {
        w8[0] = (uint8_t)(0xC0 | (c >> 6)); w8[1] = (uint8_t)(0x80 | (c & 0x3F));
      } else if (sz == 3) {
        w8[0] = (uint8_t)(0xE0 | (c >> 12)); w8[1] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); w8[2] = (uint8_t)(0x80 | (c & 0x3F));
      } else if (sz == 4) {
        w8[0] = (uint8_t)(0xF0 | (c >> 18)); w8[1] = (uint8_t)(0x80 | ((c >> 12) & 0x3F));
        w8[2] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); w8[3] = (uint8_t)(0x80 | (c & 0x3F));
      }
      pos += lane63(inc);
    }
    return;
  }
  const uint32_t pre = (add_prefix && n > 0 && text[a] != ' ') ? 1u : 0u;
  if (pre && lane == 0) o[0] = ' ';
  for (uint32_t i = lane; i < n; i += 64) o[pre + i] = text[a + i];
}

hipError_t launch_norm(const uint8_t* text, const uint64_t* doc_off, uint32_t n_docs, const uint32_t* doc_flag,
                       int add_prefix, int nfc, const Tables& t, uint32_t* cp_scratch, uint32_t* ncp,
                       uint64_t* newv, uint8_t* out, int phase, hipStream_t s) {
  if (n_docs)
    k_norm<<<(n_docs + kNormWaves - 1) / kNormWaves, 64 * kNormWaves, 0, s>>>(text, doc_off, n_docs, doc_flag, add_prefix,
                                                                          nfc, t, cp_scratch, ncp, newv, out, phase);
  return hipGetLastError();
}

void upload_done() {}

}  // namespace ctok_dev
