/* TEST INFRASTRUCTURE ONLY -- faithful C restatement of the reference encode path.
 *
 * Role: (1) second oracle beside oracle/ref_py.py (checked against it in tests/), usable on the
 * GPU box where the Python oracle is too slow for large inputs; (2) the CPU baseline timed by
 * bench.py (`cpu_baseline.kind = "port"`).  The product library never links it.
 *
 * It keeps the reference's algorithmic choices (cost model), not just its results:
 *   - NFC of every document (src/normalizers.rs:47; unicode-normalization ^0.1 restated with the
 *     canonical decompose / reorder / compose algorithm of UAX #15 over generated Unicode data);
 *   - bytes_to_unicode() rebuilt for every document with the O(256*188) `contains` loop
 *     (src/pretokenizers.rs:130-153, called from :159);
 *   - leftmost-first matching of GPT2_PATTERN (src/pretokenizers.rs:11-15,170), restated as a
 *     hand-written alternation matcher (try each alternative in order at each position);
 *   - per-word added-token `find`s (src/huggingface/mod.rs:566-675);
 *   - per-character string-keyed vocab lookups (`c.to_string()`, src/bpe.rs:94-97) and the
 *     O(n^2) lowest-rank rescan with Vec::remove (src/bpe.rs:104-153);
 *   - rayon-like parallelism over documents (src/huggingface/mod.rs:694-696).
 * Merge table construction follows src/bpe.rs:52-79 exactly, including the rank/new_id quirk
 * (rank indexes 2-part merges, new_id is read from the list of *valid* merges) and the panic when
 * that index is out of range (reported as return code -3).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdatomic.h>

#include "../complexity-tokenizer_amd/csrc/gen/unicode_data.h"

/* ------------------------------------------------------------------ string-keyed hash map */
typedef struct { char* key; uint32_t klen; uint32_t val; int used; } sent;
typedef struct { sent* e; uint64_t cap; } smap;

static uint64_t fnv(const char* s, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t i = 0; i < n; i++) { h ^= (uint8_t)s[i]; h *= 1099511628211ull; }
  return h;
}
static void smap_init(smap* m, uint64_t n) {
  uint64_t c = 16; while (c < n * 2 + 16) c <<= 1;
  m->cap = c; m->e = (sent*)calloc(c, sizeof(sent));
}
static sent* smap_slot(const smap* m, const char* k, uint32_t n) {
  uint64_t i = fnv(k, n) & (m->cap - 1);
  for (;;) {
    sent* e = &m->e[i];
    if (!e->used || (e->klen == n && memcmp(e->key, k, n) == 0)) return e;
    i = (i + 1) & (m->cap - 1);
  }
}
static void smap_put(smap* m, const char* k, uint32_t n, uint32_t v) {
  sent* e = smap_slot(m, k, n);
  if (!e->used) { e->used = 1; e->key = (char*)malloc(n + 1); memcpy(e->key, k, n); e->klen = n; }
  e->val = v;
}
static int smap_get(const smap* m, const char* k, uint32_t n, uint32_t* v) {
  const sent* e = smap_slot(m, k, n);
  if (!e->used) return 0;
  *v = e->val; return 1;
}

/* ------------------------------------------------------------------ pair -> rank hash map */
typedef struct { uint64_t key; uint64_t rank; } pent;
typedef struct { pent* e; uint64_t cap; } pmap;
#define PEMPTY 0xFFFFFFFFFFFFFFFFull
static uint64_t mix64(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; }
static void pmap_init(pmap* m, uint64_t n) {
  uint64_t c = 16; while (c < n * 2 + 16) c <<= 1;
  m->cap = c; m->e = (pent*)malloc(c * sizeof(pent));
  for (uint64_t i = 0; i < c; i++) m->e[i].key = PEMPTY;
}
static pent* pmap_slot(const pmap* m, uint64_t k) {
  uint64_t i = mix64(k) & (m->cap - 1);
  while (m->e[i].key != PEMPTY && m->e[i].key != k) i = (i + 1) & (m->cap - 1);
  return &m->e[i];
}

/* ------------------------------------------------------------------ tokenizer */
typedef struct {
  char* content; uint32_t len; uint32_t id; int single_word, lstrip, rstrip;
} added_t;

typedef struct ref_tok {
  smap vocab;
  pmap ranks;
  uint32_t* new_ids; uint64_t n_valid;  /* BpeTokenizer.merges[*].new_id */
  added_t* added; int64_t n_added;
  int nfc, add_prefix_space;
} ref_tok;

/* utf-8 */
static int u8dec(const uint8_t* s, uint64_t n, uint64_t i, uint32_t* cp) {
  uint8_t b = s[i];
  if (b < 0x80) { *cp = b; return 1; }
  if ((b & 0xE0) == 0xC0 && i + 1 < n) { *cp = ((b & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu); return 2; }
  if ((b & 0xF0) == 0xE0 && i + 2 < n) { *cp = ((b & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu); return 3; }
  if (i + 3 < n) { *cp = ((b & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu); return 4; }
  *cp = 0xFFFD; return 1;
}
static int u8enc(uint32_t cp, char* o) {
  if (cp < 0x80) { o[0] = (char)cp; return 1; }
  if (cp < 0x800) { o[0] = (char)(0xC0 | (cp >> 6)); o[1] = (char)(0x80 | (cp & 0x3F)); return 2; }
  if (cp < 0x10000) { o[0] = (char)(0xE0 | (cp >> 12)); o[1] = (char)(0x80 | ((cp >> 6) & 0x3F)); o[2] = (char)(0x80 | (cp & 0x3F)); return 3; }
  o[0] = (char)(0xF0 | (cp >> 18)); o[1] = (char)(0x80 | ((cp >> 12) & 0x3F)); o[2] = (char)(0x80 | ((cp >> 6) & 0x3F)); o[3] = (char)(0x80 | (cp & 0x3F)); return 4;
}

static int cls_of(uint32_t cp) {
  if (cp >= 0x110000) return 3;
  uint32_t blk = ct_cls_stage1[cp >> 8];
  uint32_t w = ct_cls_stage2[blk * 64 + ((cp & 255) >> 2)];
  return (w >> ((cp & 3) * 2)) & 3;
}
static uint16_t nfc_of(uint32_t cp) {
  if (cp >= 0x110000) return 0;
  return ct_nfc_stage2[ct_nfc_stage1[cp >> 8] * 256 + (cp & 255)];
}

/* ------------------------------------------------------------------ NFC (UAX #15) */
#define SBASE 0xAC00u
#define LBASE 0x1100u
#define VBASE 0x1161u
#define TBASE 0x11A7u
#define LCOUNT 19u
#define VCOUNT 21u
#define TCOUNT 28u
#define NCOUNT (VCOUNT * TCOUNT)
#define SCOUNT (LCOUNT * NCOUNT)

typedef struct { uint32_t* v; uint64_t n, cap; } u32vec;
static void vpush(u32vec* a, uint32_t x) {
  if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 64; a->v = (uint32_t*)realloc(a->v, a->cap * 4); }
  a->v[a->n++] = x;
}

static void decompose_cp(uint32_t cp, u32vec* out) {
  if (cp >= SBASE && cp < SBASE + SCOUNT) {
    uint32_t s = cp - SBASE;
    vpush(out, LBASE + s / NCOUNT);
    vpush(out, VBASE + (s % NCOUNT) / TCOUNT);
    if (s % TCOUNT) vpush(out, TBASE + s % TCOUNT);
    return;
  }
  int lo = 0, hi = CT_DECOMP_N - 1;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    if (ct_decomp_cp[mid] == cp) {
      for (uint32_t k = ct_decomp_off[mid]; k < ct_decomp_off[mid + 1]; k++) vpush(out, ct_decomp_data[k]);
      return;
    }
    if (ct_decomp_cp[mid] < cp) lo = mid + 1; else hi = mid - 1;
  }
  vpush(out, cp);
}

static uint32_t compose_pair(uint32_t a, uint32_t b) {
  if (a >= LBASE && a < LBASE + LCOUNT && b >= VBASE && b < VBASE + VCOUNT)
    return SBASE + ((a - LBASE) * VCOUNT + (b - VBASE)) * TCOUNT;
  if (a >= SBASE && a < SBASE + SCOUNT && (a - SBASE) % TCOUNT == 0 && b > TBASE && b < TBASE + TCOUNT)
    return a + (b - TBASE);
  uint64_t key = ((uint64_t)a << 21) | b;
  int lo = 0, hi = CT_COMP_N - 1;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    if (ct_comp_key[mid] == key) return ct_comp_val[mid];
    if (ct_comp_key[mid] < key) lo = mid + 1; else hi = mid - 1;
  }
  return 0xFFFFFFFFu;
}

/* text -> NFC(text) (appended to *out, which is a growing byte buffer) */
typedef struct { char* b; uint64_t n, cap; } bbuf;
static void bput(bbuf* o, const char* s, uint64_t n) {
  if (o->n + n > o->cap) { o->cap = (o->n + n) * 2 + 64; o->b = (char*)realloc(o->b, o->cap); }
  memcpy(o->b + o->n, s, n); o->n += n;
}

static void nfc(const uint8_t* s, uint64_t n, bbuf* out) {
  u32vec d = {0};
  for (uint64_t i = 0; i < n;) { uint32_t cp; i += u8dec(s, n, i, &cp); decompose_cp(cp, &d); }
  /* canonical ordering: stable insertion sort of each non-starter run by ccc */
  for (uint64_t i = 1; i < d.n; i++) {
    uint32_t c = d.v[i]; int cc = nfc_of(c) & 0xFF;
    if (!cc) continue;
    uint64_t j = i;
    while (j > 0) { int pc = nfc_of(d.v[j - 1]) & 0xFF; if (pc <= cc || pc == 0) break; d.v[j] = d.v[j - 1]; j--; }
    d.v[j] = c;
  }
  /* canonical composition */
  if (d.n) {
    uint64_t starter = 0, comp = 1;
    uint32_t sch = d.v[0];
    int last = nfc_of(sch) & 0xFF; if (last) last = 256;
    for (uint64_t i = 1; i < d.n; i++) {
      uint32_t ch = d.v[i]; int cc = nfc_of(ch) & 0xFF;
      uint32_t c = compose_pair(sch, ch);
      if (c != 0xFFFFFFFFu && (last < cc || last == 0)) { d.v[starter] = c; sch = c; continue; }
      if (cc == 0) { starter = comp; sch = ch; }
      last = cc;
      d.v[comp++] = ch;
    }
    d.n = comp;
  }
  char tmp[4];
  for (uint64_t i = 0; i < d.n; i++) bput(out, tmp, u8enc(d.v[i], tmp));
  free(d.v);
}

/* ------------------------------------------------------------------ GPT2_PATTERN matcher */
/* returns the end of the leftmost-first match starting at i (the pattern matches at every
 * position of a non-empty string, so find_iter never skips bytes) */
static uint64_t gpt2_match(const uint8_t* s, uint64_t n, uint64_t i) {
  uint32_t c0, c1 = 0, c2 = 0; int l0 = u8dec(s, n, i, &c0), l1 = 0;
  if (i + l0 < n) { l1 = u8dec(s, n, i + l0, &c1); if (i + l0 + l1 < n) u8dec(s, n, i + l0 + l1, &c2); }
  if (c0 == '\'' && l1) {
    if (c1 == 's' || c1 == 't' || c1 == 'm' || c1 == 'd') return i + 2;
    if (i + 2 < n && ((c1 == 'r' && c2 == 'e') || (c1 == 'v' && c2 == 'e') || (c1 == 'l' && c2 == 'l'))) return i + 3;
  }
  for (int want = 1; want <= 3; want++) { /* ' ?\p{L}+', ' ?\p{N}+', ' ?[^\s\p{L}\p{N}]+' */
    uint64_t j = i;
    for (int pass = 0; pass < 2; pass++) {
      j = i;
      if (pass == 0) { if (c0 != ' ') continue; j = i + 1; }
      uint64_t k = j;
      while (k < n) { uint32_t cp; int l = u8dec(s, n, k, &cp); if (cls_of(cp) != want) break; k += l; }
      if (k > j) return k;
    }
  }
  { /* \s+ */
    uint64_t k = i;
    while (k < n) { uint32_t cp; int l = u8dec(s, n, k, &cp); if (cls_of(cp) != 0) break; k += l; }
    if (k > i) return k;
  }
  return i + l0; /* unreachable for valid UTF-8 */
}

/* ------------------------------------------------------------------ BPE (src/bpe.rs:88-153) */
typedef struct { u32vec* out; int panic; } ectx;

static void bpe_encode(const ref_tok* t, const char* w, uint64_t n, ectx* cx) {
  if (!n) return;
  u32vec tok = {0};
  for (uint64_t i = 0; i < n;) { /* chars -> vocab[c.to_string()] (filter_map) */
    uint32_t cp; int l = u8dec((const uint8_t*)w, n, i, &cp);
    char* one = (char*)malloc(l); memcpy(one, w + i, l); /* the per-char String allocation */
    uint32_t id; if (smap_get(&t->vocab, one, l, &id)) vpush(&tok, id);
    free(one); i += l;
  }
  while (tok.n > 1) {
    int64_t bi = -1; uint64_t br = 0; uint32_t bid = 0;
    for (uint64_t i = 0; i + 1 < tok.n; i++) {
      const pent* e = pmap_slot(&t->ranks, ((uint64_t)tok.v[i] << 32) | tok.v[i + 1]);
      if (e->key == PEMPTY) continue;
      if (e->rank >= t->n_valid) { cx->panic = 1; free(tok.v); return; }
      uint32_t nid = t->new_ids[e->rank];
      if (bi < 0 || e->rank < br) { bi = (int64_t)i; br = e->rank; bid = nid; }
    }
    if (bi < 0) break;
    tok.v[bi] = bid;
    memmove(tok.v + bi + 1, tok.v + bi + 2, (tok.n - bi - 2) * 4); /* Vec::remove */
    tok.n--;
  }
  for (uint64_t i = 0; i < tok.n; i++) vpush(cx->out, tok.v[i]);
  free(tok.v);
}

/* ------------------------------------------------------------------ added tokens */
static int utf8_last(const char* s, uint64_t pos, uint32_t* cp) { /* char before pos */
  uint64_t k = pos - 1; while (k > 0 && ((uint8_t)s[k] & 0xC0) == 0x80) k--;
  u8dec((const uint8_t*)s, pos, k, cp); return 1;
}
static int rust_ws(uint32_t c) { return cls_of(c) == 0; }
static int rust_alnum(uint32_t c) {
  /* Rust char::is_alphanumeric.  Only ever called on GPT-2 byte-map characters (U+0021..U+0143),
   * where Alphabetic||Numeric coincides with \p{L}||\p{N}. */
  int k = cls_of(c); return k == 1 || k == 2;
}

static int64_t find_added(const char* text, uint64_t n, const added_t* a) {
  if (a->len > n) return -1;
  const char* p = (const char*)memmem(text, n, a->content, a->len);
  if (!p) return -1;
  uint64_t pos = (uint64_t)(p - text);
  if (a->single_word) {
    int before_ok = 1, after_ok = 1; uint32_t c;
    if (pos > 0) { utf8_last(text, pos, &c); before_ok = !rust_alnum(c); }
    if (pos + a->len < n) { u8dec((const uint8_t*)text, n, pos + a->len, &c); after_ok = !rust_alnum(c); }
    if (!before_ok || !after_ok) return -1;
  }
  if (a->lstrip && pos > 0) { uint32_t c; utf8_last(text, pos, &c); if (!rust_ws(c)) return -1; }
  if (a->rstrip && pos + a->len < n) { uint32_t c; u8dec((const uint8_t*)text, n, pos + a->len, &c); if (!rust_ws(c)) return -1; }
  return (int64_t)pos;
}

static void encode_word(const ref_tok* t, const char* w, uint64_t n, ectx* cx) {
  while (n > 0 && !cx->panic) {
    int64_t best = -1;
    for (int64_t k = 0; k < t->n_added; k++) {
      if (find_added(w, n, &t->added[k]) == 0 && (best < 0 || t->added[k].len > t->added[best].len)) best = k;
    }
    if (best >= 0) { vpush(cx->out, t->added[best].id); w += t->added[best].len; n -= t->added[best].len; continue; }
    uint64_t nxt = n;
    for (int64_t k = 0; k < t->n_added; k++) {
      int64_t p = find_added(w, n, &t->added[k]);
      if (p > 0 && (uint64_t)p < nxt) nxt = (uint64_t)p;
    }
    bpe_encode(t, w, nxt, cx);
    w += nxt; n -= nxt;
  }
}

static void encode_doc(const ref_tok* t, const uint8_t* text, uint64_t n, ectx* cx) {
  bbuf norm = {0};
  if (t->nfc) nfc(text, n, &norm); else bput(&norm, (const char*)text, n);
  /* byte_level_pretokenize, src/pretokenizers.rs:158-185 */
  uint32_t bmap[256]; { /* bytes_to_unicode() rebuilt per call */
    uint8_t bs[256]; uint32_t cs[256]; int nb = 0, nn = 0;
    for (int b = '!'; b <= '~'; b++) { bs[nb] = (uint8_t)b; cs[nb++] = (uint32_t)b; }
    for (int b = 0xA1; b <= 0xAC; b++) { bs[nb] = (uint8_t)b; cs[nb++] = (uint32_t)b; }
    for (int b = 0xAE; b <= 0xFF; b++) { bs[nb] = (uint8_t)b; cs[nb++] = (uint32_t)b; }
    for (int b = 0; b < 256; b++) {
      int found = 0; for (int k = 0; k < nb; k++) if (bs[k] == b) { found = 1; break; }
      if (!found) { bs[nb] = (uint8_t)b; cs[nb++] = 256u + (uint32_t)nn++; }
    }
    for (int k = 0; k < 256; k++) bmap[bs[k]] = cs[k];
  }
  bbuf txt = {0};
  if (t->add_prefix_space && norm.n > 0 && norm.b[0] != ' ') bput(&txt, " ", 1);
  bput(&txt, norm.b, norm.n);
  bbuf word = {0};
  for (uint64_t i = 0; i < txt.n && !cx->panic;) {
    uint64_t e = gpt2_match((const uint8_t*)txt.b, txt.n, i);
    word.n = 0;
    char tmp[4];
    for (uint64_t k = i; k < e; k++) bput(&word, tmp, u8enc(bmap[(uint8_t)txt.b[k]], tmp));
    if (word.n) encode_word(t, word.b, word.n, cx);
    i = e;
  }
  free(norm.b); free(txt.b); free(word.b);
}

/* ------------------------------------------------------------------ public C ABI (ctypes) */
ref_tok* ref_create(const char* const* vtok, const uint32_t* vtok_len, const uint32_t* vid, int64_t nv,
                    const char* const* merges, const uint32_t* merges_len, int64_t nm,
                    const char* const* added, const uint32_t* added_len, const uint32_t* added_id,
                    const uint8_t* added_flags, int64_t na, int nfc_on, int add_prefix_space) {
  ref_tok* t = (ref_tok*)calloc(1, sizeof(ref_tok));
  smap_init(&t->vocab, (uint64_t)nv);
  for (int64_t i = 0; i < nv; i++) smap_put(&t->vocab, vtok[i], vtok_len[i], vid[i]);
  pmap_init(&t->ranks, (uint64_t)nm);
  t->new_ids = (uint32_t*)malloc(((uint64_t)nm + 1) * 4);
  uint64_t rank = 0;
  for (int64_t m = 0; m < nm; m++) {   /* src/huggingface/mod.rs:252-264: split(' ') == 2 parts */
    const char* s = merges[m]; uint32_t L = merges_len[m];
    int spaces = 0; uint32_t sp = 0;
    for (uint32_t k = 0; k < L; k++) if (s[k] == ' ') { if (!spaces) sp = k; spaces++; }
    if (spaces != 1) continue;
    uint32_t ia, ib, inew;
    int ok = smap_get(&t->vocab, s, sp, &ia) && smap_get(&t->vocab, s + sp + 1, L - sp - 1, &ib);
    if (ok) {
      char* cat = (char*)malloc(L); memcpy(cat, s, sp); memcpy(cat + sp, s + sp + 1, L - sp - 1);
      if (smap_get(&t->vocab, cat, L - 1, &inew)) {
        pent* e = pmap_slot(&t->ranks, ((uint64_t)ia << 32) | ib);
        e->key = ((uint64_t)ia << 32) | ib; e->rank = rank;   /* insert: last duplicate wins */
        t->new_ids[t->n_valid++] = inew;
      }
      free(cat);
    }
    rank++;
  }
  /* added tokens: HashMap<String, _> semantics, a later duplicate content replaces the earlier */
  t->added = (added_t*)calloc((size_t)na + 1, sizeof(added_t));
  for (int64_t i = 0; i < na; i++) {
    int64_t slot = t->n_added;
    for (int64_t k = 0; k < t->n_added; k++)
      if (t->added[k].len == added_len[i] && memcmp(t->added[k].content, added[i], added_len[i]) == 0) { slot = k; break; }
    if (slot == t->n_added) {
      t->n_added++;
      t->added[slot].content = (char*)malloc(added_len[i] + 1);
      memcpy(t->added[slot].content, added[i], added_len[i]);
      t->added[slot].len = added_len[i];
    }
    t->added[slot].id = added_id[i];
    t->added[slot].single_word = added_flags[i] & 1;
    t->added[slot].lstrip = (added_flags[i] >> 1) & 1;
    t->added[slot].rstrip = (added_flags[i] >> 2) & 1;
  }
  t->nfc = nfc_on; t->add_prefix_space = add_prefix_space;
  return t;
}

void ref_destroy(ref_tok* t) {
  if (!t) return;
  for (uint64_t i = 0; i < t->vocab.cap; i++) free(t->vocab.e[i].key);
  free(t->vocab.e); free(t->ranks.e); free(t->new_ids);
  for (int64_t i = 0; i < t->n_added; i++) free(t->added[i].content);
  free(t->added); free(t);
}

typedef struct {
  const ref_tok* t; const uint8_t* text; const uint64_t* off; int64_t nd;
  u32vec* per_doc; atomic_long next; atomic_int panic;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (;;) {
    long d0 = atomic_fetch_add(&j->next, 16);
    if (d0 >= j->nd) break;
    long d1 = d0 + 16 < j->nd ? d0 + 16 : j->nd;
    for (long d = d0; d < d1; d++) {
      ectx cx = { &j->per_doc[d], 0 };
      encode_doc(j->t, j->text + j->off[d], j->off[d + 1] - j->off[d], &cx);
      if (cx.panic) atomic_store(&j->panic, 1);
    }
  }
  return NULL;
}

/* Encode n_docs docs (flat UTF-8 + n_docs+1 offsets).  ids must hold ids_cap u32.
 * Returns 0 ok, -2 ids_cap too small (tok_off[n_docs] holds the needed size), -3 panic. */
int ref_encode_batch(const ref_tok* t, const uint8_t* text, const uint64_t* off, int64_t nd,
                     uint32_t* ids, uint64_t ids_cap, uint64_t* tok_off, int threads) {
  job_t j; j.t = t; j.text = text; j.off = off; j.nd = nd;
  j.per_doc = (u32vec*)calloc((size_t)nd + 1, sizeof(u32vec));
  atomic_init(&j.next, 0); atomic_init(&j.panic, 0);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, worker, &j);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  free(th);
  int rc = 0;
  uint64_t acc = 0;
  for (int64_t d = 0; d < nd; d++) { tok_off[d] = acc; acc += j.per_doc[d].n; }
  tok_off[nd] = acc;
  if (atomic_load(&j.panic)) rc = -3;
  else if (acc > ids_cap) rc = -2;
  else for (int64_t d = 0; d < nd; d++) memcpy(ids + tok_off[d], j.per_doc[d].v, j.per_doc[d].n * 4);
  for (int64_t d = 0; d < nd; d++) free(j.per_doc[d].v);
  free(j.per_doc);
  return rc;
}

/* NFC of one string, for tests. out must hold 3*n+4 bytes; returns output length. */
int64_t ref_nfc(const uint8_t* s, uint64_t n, uint8_t* out) {
  bbuf b = {0}; nfc(s, n, &b);
  memcpy(out, b.b, b.n); int64_t r = (int64_t)b.n; free(b.b); return r;
}

/* GPT2_PATTERN piece boundaries of one string (after optional prefix space), for tests.
 * ends must hold n+2 entries; returns the number of pieces. */
int64_t ref_pieces(const uint8_t* s, uint64_t n, uint64_t* ends) {
  int64_t k = 0;
  for (uint64_t i = 0; i < n;) { uint64_t e = gpt2_match(s, n, i); ends[k++] = e; i = e; }
  return k;
}

/* ================================================================== decode
 * decode_batch_with_options (src/huggingface/mod.rs:771-785) -> decode_impl (:710-747) per doc,
 * with the reference's cost model: a filtered id Vec when skipping special tokens (a string-keyed
 * HashMap probe per id, :716-726), one String clone per id (:729-732), the ByteLevel decoder's
 * unicode_to_bytes() HashMap rebuilt per doc with the O(256*188) `contains` loop
 * (src/decoders.rs:74-92, called from :96), a char-keyed HashMap probe per char (:101-116),
 * from_utf8_lossy (:118), then the 15 allocating `replace` passes and split_whitespace/join of
 * clean_up_tokenization_spaces (:749-767); rayon-like doc parallelism. */
typedef struct ref_dec {
  char** tok; uint32_t* tok_len; uint64_t n_ids;   /* Vocab::id_to_token (model.vocab only) */
  smap special;                                    /* special added tokens by content */
  int kind;                                        /* 1 ByteLevel, 0 raw concatenation */
} ref_dec;

ref_dec* ref_dec_create(const char* const* tok, const uint32_t* tok_len, const uint8_t* has_tok, uint64_t n_ids,
                        const char* const* special, const uint32_t* special_len, int64_t n_special, int kind) {
  ref_dec* d = (ref_dec*)calloc(1, sizeof(ref_dec));
  d->n_ids = n_ids; d->kind = kind;
  d->tok = (char**)calloc(n_ids + 1, sizeof(char*));
  d->tok_len = (uint32_t*)calloc(n_ids + 1, 4);
  for (uint64_t i = 0; i < n_ids; i++)
    if (has_tok[i]) {
      d->tok[i] = (char*)malloc(tok_len[i] + 1);
      memcpy(d->tok[i], tok[i], tok_len[i]);
      d->tok_len[i] = tok_len[i];
    }
  smap_init(&d->special, (uint64_t)n_special);
  for (int64_t i = 0; i < n_special; i++) smap_put(&d->special, special[i], special_len[i], 1);
  return d;
}

void ref_dec_destroy(ref_dec* d) {
  if (!d) return;
  for (uint64_t i = 0; i < d->n_ids; i++) free(d->tok[i]);
  free(d->tok); free(d->tok_len);
  for (uint64_t i = 0; i < d->special.cap; i++) free(d->special.e[i].key);
  free(d->special.e); free(d);
}

/* char -> byte HashMap of unicode_to_bytes (open addressing on the code point) */
typedef struct { uint32_t key[512]; uint8_t val[512]; uint8_t used[512]; } cmap;
static uint32_t chash(uint32_t c) { return (uint32_t)(mix64(c) & 511); }
static void cmap_put(cmap* m, uint32_t c, uint8_t b) {
  uint32_t i = chash(c);
  while (m->used[i] && m->key[i] != c) i = (i + 1) & 511;
  m->used[i] = 1; m->key[i] = c; m->val[i] = b;
}
static int cmap_get(const cmap* m, uint32_t c, uint8_t* b) {
  uint32_t i = chash(c);
  while (m->used[i]) { if (m->key[i] == c) { *b = m->val[i]; return 1; } i = (i + 1) & 511; }
  return 0;
}
static void unicode_to_bytes(cmap* m) {  /* src/decoders.rs:74-92, the Vec::contains loop kept */
  uint8_t bs[256]; uint32_t cs[256]; int nb = 0;
  for (int b = '!'; b <= '~'; b++) bs[nb++] = (uint8_t)b;
  for (int b = 0xA1; b <= 0xAC; b++) bs[nb++] = (uint8_t)b;
  for (int b = 0xAE; b <= 0xFF; b++) bs[nb++] = (uint8_t)b;
  for (int i = 0; i < nb; i++) cs[i] = bs[i];
  uint32_t n = 0; int base = nb;
  for (int b = 0; b < 256; b++) {
    int found = 0;
    for (int k = 0; k < nb; k++) if (bs[k] == b) { found = 1; break; }
    if (!found) { bs[nb] = (uint8_t)b; cs[nb] = 256 + n; nb++; n++; }
  }
  (void)base;
  memset(m, 0, sizeof(*m));
  for (int i = 0; i < nb; i++) cmap_put(m, cs[i], bs[i]);
}

/* String::from_utf8_lossy (core::str::lossy::Utf8Chunks) */
static void utf8_lossy(const uint8_t* v, uint64_t n, bbuf* out) {
  uint64_t i = 0;
  while (i < n) {
    uint64_t start = i;
    uint8_t c = v[i++];
    if (c < 0x80) { bput(out, (const char*)&c, 1); continue; }
#define NX(k) ((k) < n ? v[k] : 0)
#define CONT(x) ((x) >= 0x80 && (x) <= 0xBF)
    int ok = 0;
    if (c >= 0xC2 && c <= 0xDF) {
      if (CONT(NX(i))) { i++; ok = 1; }
    } else if (c >= 0xE0 && c <= 0xEF) {
      uint8_t c1 = NX(i);
      if ((c == 0xE0 && c1 >= 0xA0 && c1 <= 0xBF) || (c >= 0xE1 && c <= 0xEC && CONT(c1)) ||
          (c == 0xED && c1 >= 0x80 && c1 <= 0x9F) || (c >= 0xEE && CONT(c1))) {
        i++;
        if (CONT(NX(i))) { i++; ok = 1; }
      }
    } else if (c >= 0xF0 && c <= 0xF4) {
      uint8_t c1 = NX(i);
      if ((c == 0xF0 && c1 >= 0x90 && c1 <= 0xBF) || (c >= 0xF1 && c <= 0xF3 && CONT(c1)) ||
          (c == 0xF4 && c1 >= 0x80 && c1 <= 0x8F)) {
        i++;
        if (CONT(NX(i))) { i++; if (CONT(NX(i))) { i++; ok = 1; } }
      }
    }
#undef NX
#undef CONT
    if (ok) bput(out, (const char*)v + start, i - start);
    else bput(out, "\xEF\xBF\xBD", 3);
  }
}

/* str::replace: leftmost non-overlapping matches, a new String every call */
static void str_replace(bbuf* s, const char* pat, uint64_t pn, const char* rep, uint64_t rn) {
  bbuf o = {0};
  uint64_t i = 0, last = 0;
  while (i + pn <= s->n) {
    if (memcmp(s->b + i, pat, pn) == 0) {
      bput(&o, s->b + last, i - last); bput(&o, rep, rn);
      i += pn; last = i;
    } else i++;
  }
  bput(&o, s->b + last, s->n - last);
  free(s->b); *s = o;
}

static int ws_len_at(const uint8_t* s, uint64_t n, uint64_t i) {  /* White_Space char at i: its length, else 0 */
  uint8_t b = s[i];
  if ((b >= 0x09 && b <= 0x0D) || b == 0x20) return 1;
  if (b < 0x80) return 0;
  uint32_t cp; int l = u8dec(s, n, i, &cp);
  return cls_of(cp) == 0 && cp != 0xFFFD ? l : 0;
}

static void clean_up(bbuf* s) {  /* src/huggingface/mod.rs:749-767 */
  static const char* pats[15][2] = {{" .", "."}, {" ,", ","}, {" !", "!"}, {" ?", "?"}, {" :", ":"}, {" ;", ";"},
                                    {"\" ", "\""}, {" \"", "\""}, {"' ", "'"}, {" '", "'"}, {"( ", "("},
                                    {" )", ")"}, {"[ ", "["}, {" ]", "]"}, {" - ", "-"}};
  for (int k = 0; k < 15; k++) str_replace(s, pats[k][0], strlen(pats[k][0]), pats[k][1], strlen(pats[k][1]));
  bbuf o = {0};
  const uint8_t* t = (const uint8_t*)s->b;
  uint64_t i = 0; int first = 1;
  while (i < s->n) {
    int w;
    while (i < s->n && (w = ws_len_at(t, s->n, i)) > 0) i += (uint64_t)w;
    if (i >= s->n) break;
    uint64_t st = i;
    while (i < s->n && ws_len_at(t, s->n, i) == 0) {
      uint32_t cp; i += (uint64_t)u8dec(t, s->n, i, &cp);
    }
    if (!first) bput(&o, " ", 1);
    bput(&o, s->b + st, i - st); first = 0;
  }
  free(s->b); *s = o;
}

static void decode_doc(const ref_dec* d, const uint32_t* ids, uint64_t n, int skip, int cleanup, bbuf* out) {
  uint32_t* keep = (uint32_t*)malloc((n + 1) * 4); uint64_t nk = 0;
  for (uint64_t i = 0; i < n; i++) {
    uint32_t id = ids[i];
    if (skip && id < d->n_ids && d->tok[id]) {
      uint32_t v;
      if (smap_get(&d->special, d->tok[id], d->tok_len[id], &v)) continue;
    }
    keep[nk++] = id;
  }
  char** toks = (char**)malloc((nk + 1) * sizeof(char*)); uint32_t* tl = (uint32_t*)malloc((nk + 1) * 4);
  uint64_t nt = 0;
  for (uint64_t i = 0; i < nk; i++) {
    uint32_t id = keep[i];
    if (id >= d->n_ids || !d->tok[id]) continue;
    toks[nt] = (char*)malloc(d->tok_len[id] + 1); memcpy(toks[nt], d->tok[id], d->tok_len[id]);
    tl[nt++] = d->tok_len[id];
  }
  bbuf text = {0};
  if (d->kind == 1) {
    cmap m; unicode_to_bytes(&m);
    bbuf joined = {0};
    for (uint64_t i = 0; i < nt; i++) bput(&joined, toks[i], tl[i]);
    bbuf raw = {0};
    for (uint64_t i = 0; i < joined.n;) {
      uint32_t cp; i += (uint64_t)u8dec((const uint8_t*)joined.b, joined.n, i, &cp);
      uint8_t b;
      if (cp == 0x120) { b = 0x20; bput(&raw, (const char*)&b, 1); }
      else if (cmap_get(&m, cp, &b)) bput(&raw, (const char*)&b, 1);
      else if (cp < 0x80) { b = (uint8_t)cp; bput(&raw, (const char*)&b, 1); }
    }
    utf8_lossy((const uint8_t*)raw.b, raw.n, &text);
    free(joined.b); free(raw.b);
  } else {
    for (uint64_t i = 0; i < nt; i++) bput(&text, toks[i], tl[i]);
  }
  for (uint64_t i = 0; i < nt; i++) free(toks[i]);
  free(toks); free(tl); free(keep);
  if (cleanup) clean_up(&text);
  *out = text;
}

typedef struct {
  const ref_dec* d; const uint32_t* ids; const uint64_t* off; int64_t nd; int skip, cleanup;
  bbuf* per_doc; atomic_long next;
} djob_t;

static void* dworker(void* arg) {
  djob_t* j = (djob_t*)arg;
  for (;;) {
    long d0 = atomic_fetch_add(&j->next, 16);
    if (d0 >= j->nd) break;
    long d1 = d0 + 16 < j->nd ? d0 + 16 : j->nd;
    for (long k = d0; k < d1; k++)
      decode_doc(j->d, j->ids + j->off[k], j->off[k + 1] - j->off[k], j->skip, j->cleanup, &j->per_doc[k]);
  }
  return NULL;
}

/* Decode n_docs id sequences (flat ids + n_docs+1 offsets) into UTF-8 strings packed in out
 * (out_off[n_docs+1]).  Returns 0, or -2 when out_cap is too small (out_off[n_docs] = needed). */
int ref_decode_batch(const ref_dec* d, const uint32_t* ids, const uint64_t* off, int64_t nd, int skip, int cleanup,
                     uint8_t* out, uint64_t out_cap, uint64_t* out_off, int threads) {
  djob_t j; j.d = d; j.ids = ids; j.off = off; j.nd = nd; j.skip = skip; j.cleanup = cleanup;
  j.per_doc = (bbuf*)calloc((size_t)nd + 1, sizeof(bbuf));
  atomic_init(&j.next, 0);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, dworker, &j);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  free(th);
  uint64_t acc = 0;
  for (int64_t k = 0; k < nd; k++) { out_off[k] = acc; acc += j.per_doc[k].n; }
  out_off[nd] = acc;
  int rc = acc > out_cap ? -2 : 0;
  if (!rc) for (int64_t k = 0; k < nd; k++) if (j.per_doc[k].n) memcpy(out + out_off[k], j.per_doc[k].b, j.per_doc[k].n);
  for (int64_t k = 0; k < nd; k++) free(j.per_doc[k].b);
  free(j.per_doc);
  return rc;
}
