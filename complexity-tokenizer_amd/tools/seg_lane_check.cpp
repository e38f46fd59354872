// Host-side check of k_segment's per-lane piece-start logic (csrc/seg_lane.h): emulates one
// wavefront per tile exactly as the kernel lays it out (lane l = word g0 - 1 + l, lane 0's
// previous word and lane 63's next word read as zero, tile = lanes 1..62, lane 63 = look-ahead
// trusted on bits 0..61) and writes the piece-start bitmap of the whole text.  Built and called
// by tests/test_oracle.py (ctypes), compared there with the `regex` module.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../csrc/seg_lane.h"
#include "../csrc/gen/unicode_data.h"

namespace {

constexpr int kTileWords = 62;

int cls_of(uint32_t cp) {
  if (cp < 0x80) {
    if (cp == 32 || (cp >= 9 && cp <= 13)) return 0;
    if ((cp | 32) >= 'a' && (cp | 32) <= 'z') return 1;
    if (cp >= '0' && cp <= '9') return 2;
    return 3;
  }
  if (cp >= 0x110000) return 3;
  const uint32_t blk = ct_cls_stage1[cp >> 8];
  const uint32_t w = ct_cls_stage2[blk * 64 + ((cp & 255) >> 2)];
  return (w >> ((cp & 3) * 2)) & 3;
}

int u8len(uint8_t b) { return b < 0x80 ? 1 : (b >> 5) == 6 ? 2 : (b >> 4) == 14 ? 3 : 4; }

int cls_at(const uint8_t* t, uint64_t B, uint64_t x) {  // class of the code point byte x is in
  uint64_t j = x;
  for (int k = 0; k < 3 && j > 0 && (t[j] & 0xC0) == 0x80; k++) j--;
  const uint32_t b0 = t[j];
  const int len = u8len((uint8_t)b0);
  auto at = [&](uint64_t i) -> uint32_t { return t[i < B ? i : B - 1] & 0x3Fu; };
  uint32_t c;
  if (len == 1) c = b0;
  else if (len == 2) c = ((b0 & 0x1Fu) << 6) | at(j + 1);
  else if (len == 3) c = ((b0 & 0x0Fu) << 12) | (at(j + 1) << 6) | at(j + 2);
  else c = ((b0 & 0x07u) << 18) | (at(j + 1) << 12) | (at(j + 2) << 6) | at(j + 3);
  return cls_of(c);
}

struct Lane {
  seg::Masks m{};
  seg::Letters lt{};
  uint64_t D = 0, valid = 0, A = 0, C1 = 0, C2 = 0, st = 0;
};

}  // namespace

extern "C" int seg_lane_starts(const uint8_t* text, uint64_t B, const uint8_t* docstart, uint64_t* out_words) {
  const uint64_t n_words = (B + 63) / 64;
  const uint64_t n_tiles = (n_words + kTileWords - 1) / kTileWords;
  std::vector<uint64_t> look(n_tiles + 1, 0);
  for (uint64_t tile = 0; tile < n_tiles; tile++) {
    Lane L[64];
    const int64_t g0 = (int64_t)tile * kTileWords;
    for (int l = 0; l < 64; l++) {
      const int64_t g = g0 - 1 + l;
      uint32_t x[16] = {0};
      Lane& c = L[l];
      if (g < 0 || (uint64_t)g * 64 >= B) {
        c.D = g < 0 ? 0 : ~0ull;
        c.valid = 0;
      } else {
        const uint64_t x0 = (uint64_t)g * 64;
        uint8_t bytes[64] = {0};
        const uint64_t n = B - x0 < 64 ? B - x0 : 64;
        memcpy(bytes, text + x0, n);
        memcpy(x, bytes, 64);
        c.valid = n == 64 ? ~0ull : ((1ull << n) - 1);
        for (uint64_t i = 0; i < n; i++)
          if (docstart[x0 + i]) c.D |= 1ull << i;
        c.D |= ~c.valid;
      }
      c.m = seg::ascii_masks(x);
      for (uint64_t todo = c.m.NA; todo; todo &= todo - 1) {
        const int i = __builtin_ctzll(todo);
        const int k = cls_at(text, B, (uint64_t)g * 64 + i);
        if (k == 0) c.m.W |= 1ull << i;
        if (k == 1) c.m.L |= 1ull << i;
        if (k == 2) c.m.N |= 1ull << i;
      }
      c.lt = seg::letter_masks(x, c.m.NA);
    }
    for (int l = 63; l >= 0; l--) {  // the kernel computes letters only next to an apostrophe
      const uint64_t pQ = l ? L[l - 1].m.Q : 0;
      if (!(L[l].m.Q | (pQ >> 62))) L[l].lt = seg::Letters{};
    }
    for (int l = 0; l < 64; l++) {
      Lane& c = L[l];
      const uint64_t pW = l ? L[l - 1].m.W : 0, nW = l < 63 ? L[l + 1].m.W : 0, nD = l < 63 ? L[l + 1].D : 0;
      c.A = seg::attached(c.m, c.D, pW, nW, nD);
    }
    for (int l = 0; l < 64; l++) {
      Lane& c = L[l];
      const seg::Letters z{};
      const Lane* p = l ? &L[l - 1] : nullptr;
      const Lane* n = l < 63 ? &L[l + 1] : nullptr;
      const uint64_t pP = p ? ~(p->m.W | p->m.L | p->m.N) : ~0ull;  // zero masks: "other"
      seg::contractions(c.m, c.lt, c.D, c.A, p ? p->A : 0, pP, n ? n->m.L : 0, n ? n->D : 0,
                        n ? n->lt : z, c.C1, c.C2);
    }
    for (int l = 0; l < 64; l++) {
      Lane& c = L[l];
      const Lane* p = l ? &L[l - 1] : nullptr;
      c.st = seg::starts(c.m, c.D, p ? p->m.W : 0, p ? p->m.L : 0, p ? p->m.N : 0, c.A, p ? p->A : 0, c.C1, c.C2,
                         p ? p->C1 : 0, p ? p->C2 : 0) & c.valid;
    }
    for (int l = 1; l <= kTileWords; l++) {
      const uint64_t g = (uint64_t)(g0 - 1 + l);
      if (g < n_words) out_words[g] = L[l].st;
    }
    look[tile] = L[63].st & ((1ull << 62) - 1);
  }
  // the look-ahead word must agree with the next tile's first word on its trusted bits
  for (uint64_t tile = 0; tile + 1 < n_tiles; tile++)
    if (look[tile] != (out_words[(tile + 1) * kTileWords] & ((1ull << 62) - 1))) return -1;
  return 0;
}
