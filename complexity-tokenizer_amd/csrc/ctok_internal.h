// Internal interfaces between the C++ host runtime (ctok_host.cpp) and the HIP kernels
// (kernels.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ctok_dev {

// Merge table entry (u64): bits [0,21) = right id, [21,42) = left id, [42,64) = rank.
// Token ids must be < 2^21 - 1; ranks < 2^22 - 2.  All-ones = empty slot.
constexpr uint64_t kEmpty = ~0ull;
constexpr uint32_t kIdBits = 21;
constexpr uint64_t kKeyMask = (1ull << 42) - 1;
constexpr uint32_t kNoRank = 0x3FFFFFu;      // "no merge" (22-bit all ones)
constexpr uint32_t kMaxId = (1u << kIdBits) - 2;
constexpr uint32_t kPanicVal = kNoRank - 1;  // compact-table value of an entry whose lookup panics

// Error bits written by kernels into Workspace::err (host checks after the call).
constexpr uint32_t kErrPanic = 1u;

// A tile is 62 64-byte bitmap words: one wavefront classifies the previous word, the tile's
// words and the next tile's first word (where the tile's last piece ends) in its 64 lanes.
constexpr int kTileWords = 62;
constexpr int kTile = kTileWords * 64;  // 3968 bytes per pre-tokenizer tile (piece starts are tile-local)
constexpr int kTileSlots = 4096;        // per-tile stride of the piece-indexed arrays (pieces <= kTile)
constexpr int kSegWaves = 4;            // tiles (wavefronts) per k_segment workgroup
constexpr int kSegUnroll = 4;           // pieces per lane per routing round in k_segment
constexpr int kShortMax = 32;      // pieces up to this many bytes: classes 0..2 (and the generic pass)
constexpr int kMedMax = 64;        // class 3: 33..64 B, still thread-per-piece (64 register slots)
// Per-tile piece lists by length class: <= 8 B (whole-piece probe missed), 9..16 B, 17..32 B,
// 33..64 B.  Capacities of classes 1..3 are the most pieces of that class that can start in one
// tile; class 0 holds Work::k0 entries per tile (kCap0Lean normally: a tile's further class-0
// pieces go to the long list, whose dense wave tier merges pieces of any length; kCap0 in the
// safe rerun after a list overflowed).
constexpr uint32_t kCap0 = kTile, kCap1 = (kTile + 8) / 9, kCap2 = (kTile + 16) / 17, kCap3 = (kTile + 32) / 33;
constexpr uint32_t kCap0Lean = 1040;  // (65 lines per tile: a power-of-two stride put every tile's list on one memory channel)
constexpr int kNumClasses = 4;
constexpr int kNumCounters = 32;
// the counters buffer: kNumCounters words, then kC3Shards class-3 counts (k_segment queues tile t's
// class-3 pieces in shard t % kC3Shards; the report sums them into counters[kCtrC3Count])
constexpr int kC3Shards = 64;
constexpr int kCounterWords = kNumCounters + kC3Shards;
// counters[] slots of class pass c: bytes merged / ids produced (statistics), next chunk
__host__ __device__ constexpr int ctr_stat(int c) { return c < 3 ? 6 + 2 * c : 16; }
__host__ __device__ constexpr int ctr_chunk(int c) { return c < 3 ? 13 + c : 18; }
constexpr int kCtrAnyMid = 19;  // counters[19] != 0: some tile has a class-2 piece
constexpr int kCtrAnyC3 = 20;   // counters[20] != 0: some tile has a class-3 piece
constexpr int kCtrEmptyDocs = 21;  // counters[21]: empty documents (k_tilefirst); 0: k_emit writes tok_off
constexpr int kCtrC3Count = 22;    // counters[22] of the report: class-3 pieces (the shards' sum)
constexpr int kCtrC3Take = 23;     // counters[23]: next piece of the sparse class-3 pass
constexpr uint32_t kC3SparseDefault = 65536;  // the most pieces the sparse class-3 path takes by default (ctok_host.cpp)
constexpr uint32_t kWgRecWords = 4 * 1024 * 4;  // Work::wgrec: 4 kernels x 1024 workgroups x 4 words
constexpr int kOverlapDefault = 1;             // merge passes on the side stream without long pieces (CTOK_OVERLAP)
constexpr int kCtrSink = 31;       // counters[31]: panic bits of lookups whose pairs need not exist (discarded)
constexpr int kCtrOverflow = 25;   // counters[25] != 0: a list outgrew its lean capacity (the host reruns the call safe)
constexpr int kCtrLongIds = 26;    // counters[26]: long-piece id slots reserved (k_long_len: a piece's bytes)
constexpr int kCtrLwWords = 27;    // counters[27]: global-memory long-piece state reserved (4 u32 per byte)
constexpr int kCtrRounds = 29;     // counters[29]: rounds of the LDS wave tiers (statistics: ctok_stats.long_rounds)
// Long-piece order (long_hist, u32[kLhWords], zeroed per call): pieces in descending length
// buckets of 64 B (bucket d = 64 - (n - 1) / 64, d = 0 for n > 4096), so every wave tier's pieces
// are a contiguous range of long_ord, longest first.
constexpr int kLhBuckets = 65;
constexpr int kLhHist = 0, kLhScan = 80, kLhFill = 160, kLhTake = 240, kLhWords = 320;
__host__ __device__ inline uint32_t long_bucket(uint32_t n) { return n > 4096 ? 0u : 64u - (n - 1) / 64; }
// List entry (u32): start within the tile [0,12), the piece's ordinal among the tile's merged
// pieces [12,24) (its slot in mrec), length [24,31) (<= kMedMax = 64).
__host__ __device__ inline uint32_t list_entry(uint32_t sl, uint32_t o, uint32_t n) { return sl | (o << 12) | (n << 24); }
__host__ __device__ inline uint32_t ent_len(uint32_t e) { return (e >> 24) & 127u; }
__host__ __device__ inline uint32_t ent_ord(uint32_t e) { return (e >> 12) & 0xFFFu; }
// long_list entry (u64): start byte | ordinal << 32 | n << 44 (n: the piece's length when
// k_segment knows it -- its end lies within the tile's look-ahead --, else 0); mid_list entry:
// start | ordinal << 32 | n << 48.
__host__ __device__ inline uint32_t long_ord(uint64_t e) { return (uint32_t)(e >> 32) & 0xFFFu; }
__host__ __device__ inline uint32_t long_len(uint64_t e) { return (uint32_t)(e >> 44) & 0x7FFFFu; }

// Piece records.  k_segment writes one per piece into prec[tile][j]: the whole-piece probe's id,
// or kRecMerged (all ones) when a later pass produces the piece's ids -- u16 when every id the
// tokenizer emits is below 0xFFFF (Work::rec16), else u32 -- and the piece's doc-start bit into
// pdoc.  The merged pieces of a tile are numbered in piece order (their ordinal, carried by the
// list entries); the pass that finishes the tile's k-th merged piece writes mrec[tile][k] (u32):
//   count | pos << 16       <= 64 B (register passes, generic pass): ids at
//                           scratch[tile * kTileSlots + pos ..] (pos: a slot of the tile's region
//                           for the piece's length class, see tregion)
//   kRecLong | li           long piece li: count long_cnt[li], ids at lids[long_pos[li] ..]
// k_emit reads prec in piece order and mrec in ordinal order: both dense.
constexpr uint32_t kRecLong = 0x40000000u, kRecLongMask = kRecLong - 1u;
constexpr uint32_t kRecMerged32 = 0xFFFFFFFFu, kRecMerged16 = 0xFFFFu;
// Per-tile id regions of the register merge passes in scratch (kTileSlots u32 per tile): class c
// (c = 0..3) starts at the total bytes of the tile's class lists < c (ids <= bytes), packed as
// tregion[tile] = {R1 | R2 << 16, R3}.
__host__ __device__ inline uint32_t region_base(uint2 r, int cls) {
  return cls <= 0 ? 0u : cls == 1 ? (r.x & 0xFFFFu) : cls == 2 ? (r.x >> 16) : r.y;
}
__host__ __device__ inline uint32_t rec_short(uint32_t count, uint32_t sl) { return count | (sl << 16); }

// 24-bit multiply (v_mul_u32_u24: full rate; a 32-bit v_mul_lo_u32 is quarter rate on CDNA)
__host__ __device__ inline uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(a, b);
#else
  return (a & 0xFFFFFFu) * (b & 0xFFFFFFu);
#endif
}

// Merge-table hashes of a pair (a, b) of token ids (< 2^21): mhash picks the global table slot
// (open addressing) and, with mhash2, the two candidate buckets of the LDS hot table and the two
// Bloom-filter bits.  Built from 24-bit multiplies and shift-xors only.
__host__ __device__ inline uint32_t mhash(uint32_t a, uint32_t b) {
  uint32_t h = mul24(a, 0x9E3779u) + mul24(b ^ 0x5A5A5Au, 0x85EBCBu);
  h ^= h >> 15;
  h = mul24(h, 0xC2B2AFu) ^ (h >> 9);
  return h ^ (h >> 16);
}
__host__ __device__ inline uint32_t mhash2(uint32_t h1) {
  uint32_t h = mul24(h1 ^ (h1 >> 24), 0x27D4EBu) + (h1 >> 11);
  h ^= h >> 13;
  h = mul24(h, 0x165667u) ^ (h >> 8);
  return h ^ (h >> 16);
}

// LDS image for the merge passes (loaded once per workgroup): a hot table of the lowest-rank
// mergeable pairs, kHotBuckets buckets of two merge-table entries, a pair in bucket
// mhash & mask or mhash2 & mask; and a Bloom filter over the merge-table entries that are not in
// the hot table (bits (mhash >> 12) and (mhash2 >> 12) mod kBloomBits).  A pair found in neither
// LDS structure goes to the global table only when both Bloom bits are set.  A second filter over
// every entry follows the image in memory, for the kernels that load the filter alone.
constexpr uint32_t kHotBuckets = 4096;                 // 64 KiB
constexpr uint32_t kBloomBits = 1u << 18;              // 32 KiB
constexpr uint32_t kHotU64 = 2 * kHotBuckets;
constexpr uint32_t kBloomWords = kBloomBits / 32;
constexpr uint32_t kLdsImageBytes = kHotU64 * 8 + kBloomWords * 4;
constexpr uint32_t kSortCap = 8192;  // merge-pass chunk entries sorted by length bucket (u16 in LDS)

// Narrow vocabularies (every id < 2^16, Tables::narrow): the register merge passes use a second
// set of pair tables keyed by the 32-bit pair key a << 16 | b, whose lookups cost about half the
// VALU of the 42-bit ones above.  Entries are u64 value << 32 | key; ~0 = empty (no id is 0xFFFF).
//   LDS image (kLdsImageBytes): hot table of kHotBuckets buckets of two entries, a pair in bucket
//   hash16_h >> 20 or hash16_g >> 20; then a Bloom filter (kBloomBits) over the other entries,
//   bits hash16_h & (kBloomBits - 1) and hash16_g >> 14.
//   Global table (merge16, load <= 1/8): open addressing from hash16_h & mask.
__host__ __device__ inline uint32_t key16(uint32_t a, uint32_t b) { return (a << 16) | b; }
__host__ __device__ inline uint32_t hash16_h(uint32_t a, uint32_t b) {
  const uint32_t h = mul24(a, 0x9E3779u) + mul24(b, 0x85EBCBu);
  return h ^ (h >> 13);
}
__host__ __device__ inline uint32_t hash16_g(uint32_t a, uint32_t b) {
  return mul24(b, 0xC2B2AFu) + mul24(a ^ 0x5A5Au, 0x27D4EBu);
}

// Whole-piece table: raw byte strings of <= 8 bytes whose BPE is exactly one token (checked at
// load time by running the merge loop on every vocab entry).  Entry = {lo32, hi32, len, id} of
// the zero-padded bytes; len == 0 marks an empty slot.
__host__ __device__ inline uint32_t piece_hash(uint32_t lo, uint32_t hi, uint32_t len) {
  uint32_t h = mul24(lo, 0x9E3779u) + mul24((lo >> 24) | (hi << 8), 0x85EBCBu) + mul24((hi >> 16) | (len << 16), 0xC2B2AFu);
  h ^= h >> 15;
  h = mul24(h, 0x27D4EBu) ^ (h >> 9);
  return h ^ (h >> 16);
}

// Common non-ASCII blocks classified by range tests instead of the two-level tables (C5: CJK,
// kana, Hangul, emoji): the class (1 = L, 3 = other) when cp lies in one, else -1.  Every code
// point of these ranges has that class and no NFC flag in the generated tables; the host checks
// this once (cp_fast_ok, ctok_host.cpp) and clears Tables::cp_fast otherwise.
__host__ __device__ __forceinline__ int cp_range_class(uint32_t cp) {
  if (cp - 0x4E00u < 0x5200u) return 1;    // CJK Unified Ideographs U+4E00..U+9FFF (Lo)
  if (cp - 0xAC00u < 0x2BA4u) return 1;    // Hangul Syllables U+AC00..U+D7A3 (Lo)
  if (cp - 0x3041u < 0x56u) return 1;      // Hiragana U+3041..U+3096 (Lo)
  if (cp - 0x30A1u < 0x5Au) return 1;      // Katakana U+30A1..U+30FA (Lo)
  if (cp - 0x1F300u < 0x350u) return 3;    // Misc. Symbols and Pictographs, Emoticons U+1F300..U+1F64F (So / Sk)
  return -1;
}

struct Tables {            // device pointers, owned by the host runtime
  const uint64_t* merge_tab;
  uint32_t merge_mask;     // capacity - 1 (power of two)
  const uint4* lds_image;  // hot table + Bloom filter (kLdsImageBytes), copied to LDS by the merge passes;
                           // then the Bloom filter of all pairs (kBloomWords u32)
  const uint32_t* pair0;   // [256 * 256] merge-table value of the byte pair (a, b), kNoRank if none
  const uint4* lds16_image;  // narrow: hot table + Bloom filter of the 32-bit-key tables (see key16)
  const uint64_t* merge16;   // narrow: global table, value << 32 | key16
  uint32_t merge16_mask;
  const uint4* piece_tab;  // whole-piece table (see piece_hash), piece_mask + 2 slots (the last stays empty)
  uint32_t piece_mask;
  const uint32_t* rank_newid;
  uint32_t n_ranks;
  const int32_t* byte2id;  // [256], -1 = byte char missing from vocab (dropped)
  const uint8_t* cls_s1;   // class two-level table (see gen/unicode_data.h)
  const uint8_t* cls_s2;
  const uint8_t* nfc_s1;
  const uint16_t* nfc_s2;
  const uint8_t* cls_bmp;  // [32768] BMP code point c: nibble c & 1 of byte c >> 1 = class | NFC flag << 2
  uint32_t cp_fast;        // 1: the code point ranges of cp_range_class (kernels.hip) hold the class
                           // it gives and no NFC flag in these tables (checked at upload)
  const uint32_t* decomp_cp;
  const uint16_t* decomp_off;
  const uint32_t* decomp_data;
  uint32_t n_decomp;
  const uint64_t* comp_key;
  const uint32_t* comp_val;
  uint32_t n_comp;
  const uint8_t* bytemap_alnum;  // [256]
  // added tokens that can occur inside a piece (raw-byte patterns), usually none
  const uint8_t* at_bytes;
  const uint32_t* at_off;  // [n_at + 1]
  const uint32_t* at_id;
  const uint8_t* at_flags;  // bit0 single_word, bit1 lstrip, bit2 rstrip
  uint32_t n_at;
  uint32_t proper;          // 1: merge table is rank-monotone (parallel same-rank rounds exact)
  const uint32_t* eager;    // bit v: the merge of table value v is "eager" -- a merge consuming its
                            // token ranks before it (only in tables that are not rank-monotone).
                            // A round of a non-eager merge applies all its occurrences at once:
                            // every pair the round makes ranks after it, so the sequential loop
                            // also applies them all, left to right, before any other merge.
  uint32_t window;          // 1: window rounds are exact (every token spans its string's length; a
                            // table that is not rank-monotone also has each eager candidate checked):
                            // the long-piece tiers also merge, in the same round, any pair ranked
                            // below every other pair of its window (kernels.hip bpe_wave_seg)
  const uint32_t* wmeta;    // window: per id, the longest left side of a merge it is the right side of
                            // (bits 0-15) and the longest right side of one it is the left side of
  uint32_t compact;         // 1: entry values are new ids (strictly increasing in rank), else ranks
  uint32_t narrow;          // 1: every vocab id < 2^16 (the merge passes keep the last tier's tokens as u16 in LDS)
  uint32_t dbg;             // debug mode (CTOK_DBG_MODE), 0 in production
  uint32_t all_bytes;       // 1: every byte's char is in the vocab (no piece can have a dropped byte)
};

struct Work {              // device pointers, sized by the host for one call
  const uint8_t* text;     // (normalised) text
  uint32_t n_bytes;
  const uint64_t* doc_off; // (normalised) offsets, n_docs + 1
  uint32_t n_docs;
  uint32_t* tfirst;        // [n_tiles] each tile's first document: the first with doc_off >= its context word
  uint32_t* pbits;         // piece-start bitmap (u32 words), n_words + 8
  uint32_t n_words;
  uint32_t n_tiles;
  uint32_t n_cus;          // compute units of the device (persistent merge-pass grid)
  uint32_t nfc_watch;      // 1, 2: the text was not NFC-checked; k_segment sets counters[12] on a
                           // code point NFC might change; 1: the later passes then stop (the call
                           // runs again normalised), 2: they finish (the flagged docs are spliced)
  uint32_t* nfc_bits;      // nfc_watch: bit g set when 64-byte word g holds the start of a code point
                           // NFC might change (zeroed by the host; nfc_splice flags docs from it)
  uint32_t mid_wide;       // 1: the 17..32 B pass at 768 threads per workgroup (the call has no long pieces)
  uint32_t short_wgs;      // workgroups of k_bpe_short (0: one per CU)
  uint32_t keep_first;     // 1: k_emit leaves every piece's first id within its tile in tcnt (not
                           // only doc-start pieces'), for ctok_encode_offsets
  uint16_t* wpref;         // [n_tiles * 64] pieces of the tile before each 64-byte word
  uint32_t* tile_np;       // [n_tiles] pieces starting in the tile
  uint32_t* tile_tok;      // [n_tiles + 1] tokens per tile, scanned in place to the tile's first id
  uint32_t* tile_doc;      // [n_tiles + 1] documents starting in the tile, scanned to the tile's first doc
  uint32_t* tcls;          // [kNumClasses][n_tiles] entries of each class list
  uint32_t* list0;         // [n_tiles * k0] (also every <= 32 B piece when added tokens can match)
  uint32_t k0;             // class-0 entries per tile (kCap0Lean, or kCap0 in the safe rerun)
  uint32_t* list1;         // [n_tiles * kCap1]
  uint32_t* list2;         // [n_tiles * kCap2]
  uint32_t* list3;         // [n_tiles * kCap3]
  void* prec;              // [n_tiles * kTileSlots] piece record (u16 when rec16, else u32; see kRecLong)
  uint32_t rec16;
  uint32_t* mrec;          // [n_tiles * kTileSlots] merged piece records by ordinal
  uint32_t* pdoc;          // [n_tiles * kTileSlots / 32] bit j: piece j of the tile starts a document
  uint32_t* tcnt;          // [n_tiles * kTileSlots] (k_emit, without direct tok_off or with keep_first)
                           // piece j's first id within the tile
  uint32_t* long_cnt;      // ids of long piece li (its length in bytes until a tier has run it)
  uint32_t* long_ord;      // long-list indices in descending length buckets (k_long_order)
  uint32_t* long_hist;     // [kLhWords] bucket counts | their exclusive scan | fill cursors | per-tier take counters
  uint32_t* scratch;       // [n_tiles * kTileSlots] ids of the register passes' pieces, per tile and class region
  uint32_t* lids;          // ids of the long pieces: piece li's at lids[long_pos[li] ..] (sized after k_long_len)
  uint32_t* long_pos;      // [long capacity] id slot of long piece li (k_long_len: reserved from counters[kCtrLongIds])
  uint32_t* lw_pos;        // [long capacity] global-memory tier state of long piece li at lw + 4 * lw_pos[li]
  uint32_t* rend;          // [kNumClasses][n_tiles] end of the consumed part of each class region (merge passes;
                           // the dropped-byte pass allocates after it)
  uint2* tregion;          // [n_tiles] class region bases of the tile in scratch (region_base)
  uint32_t long_cap, mid_cap;
  uint32_t unit;  // tiles per work unit of the register merge passes (8..64; chunks take 1..KT / unit units)  // long_list / mid_list entries (appends past them set counters[kCtrOverflow])
  uint64_t* long_list;     // pieces > kMedMax B (> kShortMax B in generic mode), or of unknown length
                           // at a tile end: s | j << 32
  uint64_t* mid_list;      // pieces with dropped bytes for the generic kernel: s | j << 32 | n << 48
  uint32_t* counters;      // [kNumCounters] [0] long count, [2] err, [3] nfc docs, [4] mid count,
                           // [5] pieces (stats), [ctr_stat(c)], [ctr_stat(c) + 1]: bytes merged /
                           // ids produced by class pass c (stats), [12] NFC speculation failed,
                           // [ctr_chunk(c)] next chunk of class pass c, [kCtrAnyMid], [kCtrAnyC3]
  uint32_t* lw;            // global-memory long-piece state (4 u32 per byte of the pieces > 4 KiB), sized after k_long_len
  uint32_t* scan_tmp;      // scan partials
  uint64_t scan_tmp_cap;
  uint64_t* stamps;        // diagnostic builds only (CTOK_SEG_STAMPS): 8 u64 per tile, else null
  uint32_t c3_max;         // the sparse path takes class 3 when it holds at most this many pieces (0: never;
                           // a multiple of kC3Shards: each shard of c3q holds c3_max / kC3Shards)
  uint32_t* c3q;           // [c3_max] class-3 pieces as tile << 7 | list index, in kC3Shards shards (k_segment)
  uint32_t* c3pre;         // [kC3Shards + 1] the shards' exclusive prefix (the report writer), for k_bpe_sparse
  uint64_t* host_res;      // pinned host words (device pointer): k_tokoff writes the token count to [0] and
                           // the counters to [1 ..] (null: the host copies them)
  uint64_t* wgrec;         // diagnostic (CTOK_WGREC=1): per-workgroup start / end / CU of the merge passes, else null
  uint32_t* report;        // pinned host words (device pointer): k_report writes the counters to
                           // [0, kNumCounters) and then seq to [kNumCounters] (the host polls it)
  uint32_t seq;            // this call's sequence number (nonzero)
};

// Launch options of one kernel: start / stop events its own dispatch records (hipExtLaunchKernel),
// so a timed call puts no marker packets between its kernels.  (hipExtAnyOrderLaunch was measured
// and left out: such a packet starts only when the previous kernel's first workgroup retires,
// tools/anyorder_check.hip.)
struct Lx {
  hipEvent_t start = nullptr, stop = nullptr;
};

// ---- decode (decode.hip): ids -> UTF-8 text -------------------------------------------
// Per-id decode entry: x = offset of the id's decoded bytes in `bytes`, y = length [0,24) |
// kDecNonAscii (a byte >= 0x80 among them) | kDecSpecial (the id's token is a special added token).
constexpr uint32_t kDecLenMask = 0xFFFFFFu, kDecNonAscii = 1u << 30, kDecSpecial = 1u << 31;
constexpr uint32_t kDecOptSkipSpecial = 1u, kDecOptCleanup = 2u;
constexpr int kDecChunk = 4096;  // ids per workgroup of the gather pass (256 threads x 16)
constexpr int kDecTile = 4096;   // bytes per workgroup of the clean-up passes (256 threads x 16)

struct DecTables {
  const uint2* ent;        // [n_ent]
  uint32_t n_ent;
  const uint8_t* bytes;    // every id's decoded bytes, each entry starting on a 4-byte boundary
};

struct DecWork {
  const uint32_t* ids;     // [n_ids] input
  uint32_t n_ids;
  const uint64_t* tok_off; // [n_docs + 1] input
  uint32_t n_docs;
  uint32_t opts;           // kDecOpt*
  uint32_t n_chunks;
  uint32_t* chunk_off;     // [n_chunks + 1] decoded bytes per id chunk, scanned
  uint8_t* raw;            // [n_raw + 64] decoded bytes before from_utf8_lossy / clean-up
  uint32_t n_raw;
  uint64_t* raw_off;       // [n_docs + 1]
  uint32_t* delbits;       // [n_raw / 32 + 8] units the clean-up deletes (bit at the unit's first byte)
  uint32_t n_tiles;
  uint32_t* tile_cnt;      // [n_tiles + 1] output bytes per tile, scanned
  uint32_t* counters;      // [0] error bits (1: bad offsets), [1] a decoded byte >= 0x80 exists
};

hipError_t launch_dec_len(const DecWork& w, const DecTables& t, uint32_t* tmp, uint64_t tmp_cap, hipStream_t s);
hipError_t launch_dec_gather(const DecWork& w, const DecTables& t, uint8_t* dst, uint64_t* dst_off, hipStream_t s);
hipError_t launch_dec_prepare(const DecWork& w, hipStream_t s);  // clean-up: trimmed and replaced units
hipError_t launch_dec_count(const DecWork& w, uint32_t* tmp, uint64_t tmp_cap, hipStream_t s);
hipError_t launch_dec_write(const DecWork& w, uint8_t* out, uint64_t* out_off, hipStream_t s);

// ---- padded batch encode (pad.hip): Encoding rows as [rows, width] arrays -----------------
// Row r = doc r (or docs 2r, 2r+1 merged as a pair).  Its n ids pass through the post-processor
// items (kPadItemA = the n ids, else one special id), are cut to max_len when truncating, and
// padded to `target` on the right or the left (src/encoding.rs:87-224, src/huggingface/mod.rs:
// 340-392, src/bindings/tokenizer.rs:46-201).
constexpr uint32_t kPadItemA = 0xFFFFFFFFu;
constexpr int kPadMaxItems = 16;

struct PadWork {
  const uint32_t* ids;       // encoded ids of the docs
  const uint64_t* tok_off;   // [n_docs + 1]
  uint32_t n_rows;
  uint32_t pairs;            // 1: row r = docs 2r (type 0) and 2r + 1 (type 1)
  uint32_t use_tpl;          // apply the post-processor items
  uint32_t n_items;
  uint32_t items[kPadMaxItems];
  uint32_t mark;             // special_tokens_mask |= id is a special token (mark_special_tokens)
  const uint32_t* special_ids;  // sorted
  uint32_t n_special;
  uint32_t truncate;
  uint64_t max_len;
  uint64_t target;           // pad to this length (0: no padding)
  uint32_t pad_left;
  uint32_t pad_id;
  uint64_t width;            // columns of the outputs
  uint32_t* out_ids;         // [n_rows * width]; the three masks may be null
  uint32_t* out_attn;
  uint32_t* out_type;
  uint32_t* out_special;
  uint64_t* row_len;         // [n_rows] length of the row (content + padding)
  uint32_t* counters;        // [0..1] longest content (u64, atomicMax), [2] a template dropped ids
};
hipError_t launch_pad_len(const PadWork& w, hipStream_t s);
hipError_t launch_pad_rows(const PadWork& w, hipStream_t s);

// ---- launchers (kernels.hip) -----------------------------------------------------------
void upload_done();
// also zeroes the counters and nfc_bits; x: k_clear's launch options, x2: k_tilefirst's
hipError_t launch_docstart(const Work& w, hipStream_t s, bool zero_counters, Lx x = {}, Lx x2 = {});
uint64_t nfc_bits_words(uint64_t n_bytes);  // nfc_bits size (u32 words)
// tile_tok, tile_doc: exclusive scans + totals at n_tiles; count: pieces into counters[5]; x: the first launch's
hipError_t scan_tiles(const Work& w, hipStream_t s, bool count, Lx x = {});
hipError_t launch_nfc_check(const uint8_t* text, uint64_t n_bytes, const uint64_t* doc_off, uint32_t n_docs,
                            const Tables& t, uint32_t* doc_flag, uint32_t* counter, hipStream_t s);
hipError_t launch_norm(const uint8_t* text, const uint64_t* doc_off, uint32_t n_docs, const uint32_t* doc_flag,
                       int add_prefix, int nfc, const Tables& t, uint32_t* cp_scratch, uint32_t* ncp,
                       uint64_t* new_len_then_off, uint8_t* out_text, int phase, hipStream_t s);
hipError_t launch_segment(const Work& w, const Tables& t, hipStream_t s, Lx x = {});
// cls 0: classes 0 and 1; 2: class 2; 4: class 3 (main instance); 3: dropped-byte pieces (mid_list).
// (With added tokens only cls 0 launches a kernel; cls 3 none when Tables::all_bytes; none without tiles.)
hipError_t launch_bpe_class(const Work& w, const Tables& t, int cls, hipStream_t s, Lx x = {});
// k_report: the counters into Work::report, then Work::seq (one wave, after k_segment; k_bpe_short's
// first wave does the same, so the host launches it only when k_bpe_short does not run)
hipError_t launch_report(const Work& w, hipStream_t s);
// sparse class 3 (k_bpe_sparse): the host launches it instead of the 33..64 B register pass when
// the report's class-3 count is at most Work::c3_max
hipError_t launch_c3_sparse(const Work& w, const Tables& t, uint32_t n_pieces, hipStream_t s, Lx x = {});
// long-piece preparation (side stream): lengths, order, id places (long_pos) and global-memory
// state places (lw_pos); long_pos[n_long] / lw_pos[n_long] = the totals the host sizes lids / lw by
hipError_t launch_long_prep(const Work& w, const Tables& t, hipStream_t s, uint32_t n_long, uint32_t* lwn,
                            uint32_t* tmp, uint64_t tmp_cap);
// long-piece tiers (side stream): n_long = k_segment's long-list length, any_c3 = a class-3
// piece exists (the side instance of the 33..64 B pass); grids sized for them, nothing when empty
hipError_t launch_bpe_long(const Work& w, const Tables& t, hipStream_t s, uint32_t n_long, bool any_c3, bool any_gmem);
// count_pieces: counters[5] = pieces (statistics); empty_docs: some document is empty (k_tokoff
// then writes every tok_off entry; else k_emit wrote them and k_tokoff only the total)
// (first: the tile scan's first launch; last: k_tokoff)
hipError_t launch_emit(const Work& w, uint32_t* ids, uint64_t ids_cap, uint64_t* tok_off, hipStream_t s,
                       bool count_pieces, bool empty_docs = true, Lx first = {}, Lx last = {});
// exclusive scan of n u32 (n read from *n_dev when non-null, else n_max); out[n] = total
hipError_t scan_u32(const uint32_t* in, uint32_t* out, uint64_t n_max, const uint32_t* n_dev,
                    uint32_t* tmp, uint64_t tmp_cap, hipStream_t s);
hipError_t scan_u64(uint64_t* inout, uint64_t n, uint64_t* tmp, uint64_t tmp_cap, hipStream_t s);
uint64_t scan_tmp_elems(uint64_t n_max);
uint64_t tile_scan_tmp_elems(uint64_t n_tiles);  // scan_tmp (u64) that scan_tiles needs
hipError_t shift_u64(uint64_t* p, uint64_t n, uint64_t delta, hipStream_t s);  // p[0, n) += delta
// NFC splice (see kernels.hip): len[d] = flagged doc d's bytes (else 0); flagged docs' bytes
// gathered to the sub-batch; the output's counts, offsets (out_off[0..n_docs]) and ids
hipError_t launch_flag_docs(const uint64_t* off, uint64_t n_docs, const uint32_t* nfc_bits, uint32_t* flag, hipStream_t s);
hipError_t launch_flag_len(const uint64_t* off, const uint32_t* flag, uint64_t n_docs, uint64_t* len, hipStream_t s);
hipError_t launch_gather_flagged(const uint8_t* text, const uint64_t* off, const uint32_t* rank, const uint64_t* sub_pos,
                                 uint64_t n_docs, uint8_t* sub_text, uint64_t* sub_off, hipStream_t s);
hipError_t launch_splice(const uint32_t* rank, const uint64_t* main_off, const uint32_t* main_ids, const uint64_t* sub_off,
                         const uint32_t* sub_ids, uint64_t n_docs, uint32_t* ids, uint64_t ids_cap, uint64_t* out_off,
                         uint64_t* tmp, uint64_t tmp_cap, hipStream_t s);
// ids16[i] = ids[i] (i < n_ids; every id < 2^16), toff32[i] = toff[i] (i < n_off; every value < 2^32);
// ids must be 16-byte aligned (DevBuf allocations are)
hipError_t wire16(const uint32_t* ids, uint64_t n_ids, uint16_t* ids16, const uint64_t* toff, uint64_t n_off,
                  uint32_t* toff32, hipStream_t s);

}  // namespace ctok_dev
