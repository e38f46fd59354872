// Piece-start predicate of GPT2_PATTERN on one 64-byte word per lane (k_segment), shared with
// the host-side check in tests (tools/seg_lane_check.cpp): plain integer code, no intrinsics
// except the 32x32->64 high multiply.
//
// A word's bytes become 64-bit masks (bit i = byte i) of the code-point classes White_Space /
// letter / number, of ' ' and '\'', and of the contraction letters, via SWAR tests on 4-byte
// words: every test leaves its answer in bit 7 of each byte, and pack8 gathers the bit-7s of two
// dwords into 8 mask bits with one high multiply.  Non-ASCII bytes are cleared from the ASCII
// masks and classified per code point by the caller (continuation bytes take their lead's
// class).  The predicate itself is then a few dozen 64-bit ops on the
// word's masks and its neighbours' (one word before and after: carried across lanes).
#pragma once
#include <cstdint>

#if defined(__HIP_DEVICE_COMPILE__)
#define SEG_HD __device__ __forceinline__
#else
#define SEG_HD inline
#endif

namespace seg {

constexpr uint32_t kHi = 0x80808080u;
constexpr uint32_t rep(uint32_t c) { return c * 0x01010101u; }

SEG_HD uint32_t mulhi(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(a, b);
#else
  return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

// bit 7 of each byte of r0 then r1 -> 8 bits (byte order).  ((r0 & hi) >> 4) | (r1 & hi) puts
// the eight flags at bits 3,11,19,27 (r0) and 7,15,23,31 (r1); the multiplier's four terms move
// them to bits 32..39 with no two partial products on the same bit (so no carries).
SEG_HD uint32_t pack8(uint32_t r0, uint32_t r1) {
  const uint32_t c = ((r0 & kHi) >> 4) | (r1 & kHi);
  return mulhi(c, 0x20408100u) & 0xFFu;
}

// x7 = x & 0x7f7f7f7f.  Bit 7 of a byte is set iff the byte != c (c < 0x80).
SEG_HD uint32_t ne7(uint32_t x7, uint32_t c) {
  const uint32_t t = x7 ^ rep(c);
  return (t + 0x7F7F7F7Fu) | t;
}
// x80 = x | 0x80808080.  Bit 7 of a byte is set iff (byte & 0x7f) in [lo, hi] (hi < 0x7f).
SEG_HD uint32_t in80(uint32_t x80, uint32_t lo, uint32_t hi) {
  return (x80 - rep(lo)) & ~(x80 - rep(hi + 1));
}

struct Masks {
  uint64_t W, L, N, S, Q, NA;   // White_Space, letter, number, ' ', '\'', byte >= 0x80
};
struct Letters {
  uint64_t T1, R, Le, V, LL;    // s|t|m|d, r, e, v, l
};

// x: the word's 16 little-endian dwords.  W/L/N hold the ASCII bytes only (NA bytes cleared).
SEG_HD Masks ascii_masks(const uint32_t (&x)[16]) {
  uint32_t w[2] = {0, 0}, l[2] = {0, 0}, n[2] = {0, 0}, s[2] = {0, 0}, q[2] = {0, 0}, na[2] = {0, 0};
#pragma unroll
  for (int p = 0; p < 8; p++) {
    const uint32_t a = x[2 * p], b = x[2 * p + 1];
    const uint32_t a7 = a & 0x7F7F7F7Fu, b7 = b & 0x7F7F7F7Fu;
    const uint32_t a80 = a | kHi, b80 = b | kHi;
    const int h = p >> 2, sh = 8 * (p & 3);
    // ' ' and '\'' come out inverted (bit set = not equal); flipped once per mask below
    s[h] |= pack8(ne7(a7, ' '), ne7(b7, ' ')) << sh;
    q[h] |= pack8(ne7(a7, '\''), ne7(b7, '\'')) << sh;
    w[h] |= pack8(in80(a80, 9, 13), in80(b80, 9, 13)) << sh;
    l[h] |= pack8(in80(a80 | rep(0x20), 'a', 'z'), in80(b80 | rep(0x20), 'a', 'z')) << sh;
    n[h] |= pack8(in80(a80, '0', '9'), in80(b80, '0', '9')) << sh;
    na[h] |= pack8(a, b) << sh;
  }
  Masks m;
  m.NA = (uint64_t)na[0] | ((uint64_t)na[1] << 32);
  m.S = ~((uint64_t)s[0] | ((uint64_t)s[1] << 32)) & ~m.NA;
  m.Q = ~((uint64_t)q[0] | ((uint64_t)q[1] << 32)) & ~m.NA;
  m.W = (((uint64_t)w[0] | ((uint64_t)w[1] << 32)) | m.S) & ~m.NA;
  m.L = ((uint64_t)l[0] | ((uint64_t)l[1] << 32)) & ~m.NA;
  m.N = ((uint64_t)n[0] | ((uint64_t)n[1] << 32)) & ~m.NA;
  return m;
}

SEG_HD Letters letter_masks(const uint32_t (&x)[16], uint64_t na) {
  uint32_t t1[2] = {0, 0}, r[2] = {0, 0}, e[2] = {0, 0}, v[2] = {0, 0}, ll[2] = {0, 0};
#pragma unroll
  for (int p = 0; p < 8; p++) {
    const uint32_t a7 = x[2 * p] & 0x7F7F7F7Fu, b7 = x[2 * p + 1] & 0x7F7F7F7Fu;
    const int h = p >> 2, sh = 8 * (p & 3);
    // s|t|m|d: bit 7 clear in all four "not equal" tests
    t1[h] |= pack8(ne7(a7, 's') & ne7(a7, 't') & ne7(a7, 'm') & ne7(a7, 'd'),
                   ne7(b7, 's') & ne7(b7, 't') & ne7(b7, 'm') & ne7(b7, 'd')) << sh;
    r[h] |= pack8(ne7(a7, 'r'), ne7(b7, 'r')) << sh;
    e[h] |= pack8(ne7(a7, 'e'), ne7(b7, 'e')) << sh;
    v[h] |= pack8(ne7(a7, 'v'), ne7(b7, 'v')) << sh;
    ll[h] |= pack8(ne7(a7, 'l'), ne7(b7, 'l')) << sh;
  }
  auto inv = [&](const uint32_t (&y)[2]) { return ~((uint64_t)y[0] | ((uint64_t)y[1] << 32)) & ~na; };
  return Letters{inv(t1), inv(r), inv(e), inv(v), inv(ll)};
}

SEG_HD uint64_t p1(uint64_t c, uint64_t p) { return (c << 1) | (p >> 63); }
SEG_HD uint64_t p2(uint64_t c, uint64_t p) { return (c << 2) | (p >> 62); }
SEG_HD uint64_t p3(uint64_t c, uint64_t p) { return (c << 3) | (p >> 61); }
SEG_HD uint64_t n1(uint64_t c, uint64_t n) { return (c >> 1) | (n << 63); }
SEG_HD uint64_t n2(uint64_t c, uint64_t n) { return (c >> 2) | (n << 62); }

// Step 1: attached space (a single ' ' that begins the following non-space run).
// D = doc starts of the word (and every position past the text); nD, nW = next word's.
SEG_HD uint64_t attached(const Masks& c, uint64_t D, uint64_t pW, uint64_t nW, uint64_t nD) {
  const uint64_t E = n1(D, nD);
  return c.S & ~E & ~n1(c.W, nW) & (D | ~p1(c.W, pW));
}

// Step 2: '\'' starting a 1- or 2-letter contraction.  pA = previous word's attached mask,
// pP = previous word's "other" mask, nl = next word's letters, nL = next word's letter class.
SEG_HD void contractions(const Masks& c, const Letters& lt, uint64_t D, uint64_t A, uint64_t pA, uint64_t pP,
                         uint64_t nL, uint64_t nD, const Letters& nl, uint64_t& C1, uint64_t& C2) {
  const uint64_t E = n1(D, nD);
  const uint64_t P = ~(c.W | c.L | c.N);
  const uint64_t Cb = c.Q & ~E & n1(c.L, nL) & (D | (~p1(P, pP) & ~p1(A, pA)));
  const uint64_t t1 = n1(lt.T1, nl.T1);
  C1 = Cb & t1;
  C2 = Cb & ~t1 & ~n2(D, nD) &
       (((n1(lt.R, nl.R) | n1(lt.V, nl.V)) & n2(lt.Le, nl.Le)) | (n1(lt.LL, nl.LL) & n2(lt.LL, nl.LL)));
}

// Step 3: piece starts.  p* = previous word's masks / derived masks.
SEG_HD uint64_t starts(const Masks& c, uint64_t D, uint64_t pW, uint64_t pL, uint64_t pN, uint64_t A, uint64_t pA,
                       uint64_t C1, uint64_t C2, uint64_t pC1, uint64_t pC2) {
  const uint64_t chg = (c.W ^ p1(c.W, pW)) | (c.L ^ p1(c.L, pL)) | (c.N ^ p1(c.N, pN));
  return D | (chg & ~p1(A, pA) & ~p1(C1 | C2, pC1 | pC2)) | (~chg & c.L & (p2(C1, pC1) | p3(C2, pC2)));
}

}  // namespace seg
