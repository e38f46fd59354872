// C++ host runtime behind the C ABI (include/ctok.h): tokenizer.json loader, table compiler,
// per-device workspace and the stream-ordered encode pipeline.
//
// Reference counterparts (Complexity-ML/complexity-tokenizer v0.3.3):
//   loader            src/huggingface/mod.rs:32-116 (schema), :159-166 (from_file), :247-334
//   merge table       src/bpe.rs:52-79 (BpeTokenizer::new)
//   normaliser choice src/huggingface/parsing.rs:10-90 (NFC default at :89)
//   pre-tokenizer     src/huggingface/parsing.rs:92-190; src/pretokenizers.rs:71-126, :298-302
//   vocab getters     src/vocab.rs:34-100, src/huggingface/mod.rs:856-866
//   decode            src/huggingface/mod.rs:698-785, src/decoders.rs:74-119, parsing.rs:272-364
#include <emmintrin.h>
#include <sched.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <exception>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <thread>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/ctok.h"
#include "ctok_internal.h"
#include "gen/regex_props.h"
#include "gen/unicode_data.h"
#include "json.hpp"

using namespace ctok_dev;

namespace {

thread_local std::string g_err;

// CPUs this process may run on: the affinity mask capped by the cgroup v2 quota (cpu.max), as
// Rust's available_parallelism (rayon's default pool, reference src/huggingface/mod.rs:695)
// counts them on Linux.  Cached: read once per process.
unsigned usable_cpus_once() {
  static const unsigned n = [] {
    unsigned c = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) c = std::max(1, CPU_COUNT(&set));
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      unsigned long long period = 0;
      if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
        const unsigned long long quota = strtoull(q, nullptr, 10);
        c = std::min<unsigned>(c, (unsigned)std::max<unsigned long long>(1, quota / period));
      }
      fclose(f);
    }
    return c;
  }();
  return n;
}

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct CtokError {
  int code;
  std::string msg;
};

[[noreturn]] void throw_err(int code, const std::string& msg) { throw CtokError{code, msg}; }

#define HIPTRY(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw_err(CTOK_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ----------------------------------------------------------------------------- byte map
// GPT-2 bytes_to_unicode (src/pretokenizers.rs:130-153): byte -> code point
std::vector<uint32_t> byte_map() {
  std::vector<int> bs;
  for (int b = '!'; b <= '~'; b++) bs.push_back(b);
  for (int b = 0xA1; b <= 0xAC; b++) bs.push_back(b);
  for (int b = 0xAE; b <= 0xFF; b++) bs.push_back(b);
  std::vector<uint32_t> cs(bs.begin(), bs.end());
  uint32_t n = 0;
  std::vector<bool> in(256, false);
  for (int b : bs) in[b] = true;
  for (int b = 0; b < 256; b++)
    if (!in[b]) { bs.push_back(b); cs.push_back(256 + n++); }
  std::vector<uint32_t> m(256);
  for (size_t i = 0; i < 256; i++) m[bs[i]] = cs[i];
  return m;
}

std::string utf8(uint32_t cp) {
  std::string o;
  if (cp < 0x80) o += (char)cp;
  else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  return o;
}

bool decode_utf8(const std::string& s, std::vector<uint32_t>& out) {
  out.clear();
  for (size_t i = 0; i < s.size();) {
    uint8_t b = (uint8_t)s[i];
    int len = b < 0x80 ? 1 : (b >> 5) == 6 ? 2 : (b >> 4) == 14 ? 3 : (b >> 3) == 30 ? 4 : 0;
    if (!len || i + len > s.size()) return false;
    uint32_t cp = len == 1 ? b : len == 2 ? (b & 0x1Fu) : len == 3 ? (b & 0x0Fu) : (b & 0x07u);
    for (int k = 1; k < len; k++) cp = (cp << 6) | ((uint8_t)s[i + k] & 0x3Fu);
    out.push_back(cp);
    i += len;
  }
  return true;
}

int host_cls(uint32_t cp) {
  if (cp >= 0x110000) return 3;
  uint32_t w = ct_cls_stage2[ct_cls_stage1[cp >> 8] * 64 + ((cp & 255) >> 2)];
  return (w >> ((cp & 3) * 2)) & 3;
}

// Can the raw byte string `pat` occur inside one GPT2_PATTERN piece?  Pieces are: a run of
// White_Space; an optional leading U+0020 plus a run of one class among {L, N, other}; or a
// contraction 's 't 're 've 'm 'll 'd.  Conservative: true unless provably impossible.
bool can_occur_in_piece(const std::string& pat) {
  if (pat.empty()) return true;
  static const char* con[] = {"'s", "'t", "'re", "'ve", "'m", "'ll", "'d"};
  for (const char* c : con)
    if (std::string(c).find(pat) != std::string::npos) return true;
  size_t i = 0;
  bool lead_partial = false;
  while (i < pat.size() && ((uint8_t)pat[i] & 0xC0) == 0x80) { i++; lead_partial = true; }
  std::vector<int> cls;
  std::vector<uint32_t> cps;
  while (i < pat.size()) {
    uint8_t b = (uint8_t)pat[i];
    int len = b < 0x80 ? 1 : (b >> 5) == 6 ? 2 : (b >> 4) == 14 ? 3 : 4;
    if (i + len > pat.size()) break;  // trailing partial code point: class unknown
    uint32_t cp = len == 1 ? b : len == 2 ? (b & 0x1Fu) : len == 3 ? (b & 0x0Fu) : (b & 0x07u);
    for (int k = 1; k < len; k++) cp = (cp << 6) | ((uint8_t)pat[i + k] & 0x3Fu);
    cps.push_back(cp);
    cls.push_back(host_cls(cp));
    i += len;
  }
  if (cls.empty()) return true;
  bool all_ws = std::all_of(cls.begin(), cls.end(), [](int c) { return c == 0; });
  if (all_ws) return true;
  size_t k = 0;
  if (!lead_partial && cps[0] == ' ') k = 1;
  int want = -1;
  for (; k < cls.size(); k++) {
    if (cls[k] == 0) return false;
    if (want < 0) want = cls[k];
    else if (cls[k] != want) return false;
  }
  return true;
}

// ----------------------------------------------------------------------------- device state

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  void ensure(size_t n) {
    if (n <= cap && p) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    size_t want = std::max<size_t>(n + n / 16, 1024);  // (grow-only; a little slack for the next call)
    HIPTRY(hipMalloc((void**)&p, want * sizeof(T)));
    cap = want;
  }
  ~DevBuf() { if (p) (void)hipFree(p); }
};

// Pinned (page-locked) host buffer: the landing side of the 16-bit id copies.
template <typename T>
struct PinBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  void ensure(size_t n) {
    if (n <= cap && p) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    size_t want = std::max<size_t>(n + n / 8, 1024);
    HIPTRY(hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocDefault));
    cap = want;
  }
  ~PinBuf() { if (p) (void)hipHostFree(p); }
};

// Double-buffered host-buffer pipeline of one device (ctok_encode_batch): chunk c's text is
// copied from the caller's buffer to d_in[c & 1] on the up stream while chunk c - 1 is encoded;
// its ids come back from d_ids[c & 1] into the caller's buffer while chunk c + 1 is encoded.
struct HostPipe {
  hipStream_t up = nullptr, down = nullptr;  // H2D and D2H copy streams (both directions at once)
  hipEvent_t ev_h2d[2] = {}, ev_enc[2] = {}, ev_d2h[2] = {};
  hipEvent_t ev_t[4] = {};  // timing of the first chunk's H2D and the last chunk's D2H
  DevBuf<uint16_t> d_ids16[2];    // 16-bit wire format (ids16 tokenizers): ids, and tok_off as u32
  DevBuf<uint32_t> d_toff32[2];
  PinBuf<uint16_t> pin_ids16[2];
  PinBuf<uint32_t> pin_toff32[2];
  DevBuf<uint8_t> d_in[2];
  DevBuf<uint64_t> d_off[2], d_tokoff[2];
  DevBuf<uint32_t> d_ids[2];
};

struct DeviceState {
  int device = -1;
  uint32_t n_cus = 1;
  std::recursive_mutex mu;  // serialises calls on this device; recursive: ctok_encode_padded holds it
                            // across its nested ctok_encode_padded_device call
  hipStream_t stream = nullptr;
  hipEvent_t ev[12] = {};
  hipEvent_t ev_sync = nullptr;   // spin-waited completion marker (no blocking-wait wakeup latency)
  hipStream_t side = nullptr;     // long-piece pass, overlapped with the short merge passes
  hipEvent_t ev_tot = nullptr;    // the long pieces' totals are in the host words
  hipEvent_t ev_join = nullptr;   // the side stream's long tiers are done
  uint32_t seq = 0;               // encode calls (attempts) on this device: Work::seq
  uint64_t* host = nullptr;       // pinned host words for small device->host readbacks
  uint64_t* host_dev = nullptr;   // the same words as a device pointer (k_tokoff writes the results there)
  // tables
  DevBuf<uint64_t> merge_tab, lds_image, lds16_image, merge16;
  DevBuf<uint32_t> pair0;
  DevBuf<uint32_t> piece_tab;
  DevBuf<uint32_t> rank_newid, eager, wmeta;
  DevBuf<int32_t> byte2id;
  DevBuf<uint8_t> cls_s1, cls_s2, nfc_s1, alnum, at_bytes, at_flags, cls_bmp;
  DevBuf<uint16_t> nfc_s2, decomp_off;
  DevBuf<uint32_t> decomp_cp, decomp_data, comp_val, at_off, at_id;
  DevBuf<uint64_t> comp_key;
  Tables t{};
  // workspace
  DevBuf<uint32_t> tfirst, pbits, tile_np, tile_tok, tile_doc, tcls, list0, list1, list2, list3, tcnt, scratch, counters;
  DevBuf<uint16_t> prec;  // piece records (u16, or pairs of them as u32)
  DevBuf<uint32_t> mrec, pdoc;
  DevBuf<uint32_t> lids, lw, long_pos, lw_pos, lwn, rend, cps;
  DevBuf<uint64_t> tregion;
  DevBuf<uint64_t> stamps;  // diagnostic builds (CTOK_SEG_STAMPS) with CTOK_STAMPS=1
  DevBuf<uint64_t> wgrec;   // diagnostic: CTOK_WGREC=1
  DevBuf<uint16_t> wpref;
  DevBuf<uint32_t> long_cnt, long_ord, long_hist, c3q, c3pre;
  DevBuf<uint64_t> long_list, mid_list, scan_tmp, scan_tmp2;
  DevBuf<uint32_t> doc_flag, ncp;
  // NFC splice (nfc_splice): flagged-doc ranks / sub-batch positions, the speculative pass's
  // output, the sub-batch and its output
  DevBuf<uint32_t> spl_rank, spl_ids, sub_ids;
  DevBuf<uint64_t> spl_pos, spl_toff, sub_off, sub_toff;
  DevBuf<uint8_t> sub_text;
  DevBuf<uint32_t> nfc_bits;  // k_segment's NFC word flags (speculative passes)
  DevBuf<uint64_t> norm_off;
  DevBuf<uint8_t> norm_text;
  bool last_norm = false;  // the last encode ran on norm_text / norm_off (last_B bytes)
  bool last_mid_side = false;  // the last encode ran the 17..32 B pass on the side stream
  uint64_t last_B = 0;
  // decode: tables (uploaded on first use), workspace, events
  bool dec_ready = false;
  DevBuf<uint32_t> dec_ent;
  DevBuf<uint8_t> dec_bytes;
  DevBuf<uint32_t> dec_chunk, dec_del, dec_tile, dec_cnt;
  DevBuf<uint8_t> dec_raw, dec_out;
  DevBuf<uint64_t> dec_rawoff, dec_outoff, dec_tokoff;
  DevBuf<uint32_t> dec_ids;
  hipEvent_t dev_ev[8] = {};
  // host-API staging
  std::unique_ptr<HostPipe> pipe;
  // padded encode: encoded ids, special ids, counters; host-API input / outputs
  DevBuf<uint32_t> pad_ids, pad_special, pad_ctr, pad_out[4];
  DevBuf<uint64_t> pad_tokoff, pad_rowlen, pad_in_off;
  DevBuf<uint8_t> pad_in_text;
  // bytes of device memory held for encode calls (the workspace, not the tokenizer tables)
  uint64_t workspace_bytes() const {
    uint64_t b = 0;
    auto add = [&](const auto& x) { b += (uint64_t)x.cap * sizeof(*x.p); };
    add(tfirst), add(pbits), add(tile_np), add(tile_tok), add(tile_doc), add(tcls), add(list0), add(list1);
    add(list2), add(list3), add(tcnt), add(prec), add(mrec), add(pdoc), add(scratch), add(counters), add(lids), add(lw), add(tregion), add(rend);
    add(wpref), add(long_cnt), add(long_ord), add(long_hist), add(long_pos), add(lw_pos), add(lwn), add(long_list), add(c3q), add(c3pre);
    add(mid_list), add(scan_tmp), add(scan_tmp2), add(cps);
    add(doc_flag), add(ncp), add(norm_off), add(norm_text);
    add(nfc_bits), add(spl_rank), add(spl_ids), add(sub_ids), add(spl_pos), add(spl_toff), add(sub_off), add(sub_toff), add(sub_text);
    return b;
  }
  ~DeviceState() {
    if (device >= 0) {
      (void)hipSetDevice(device);
      if (pipe) {
        for (int i = 0; i < 2; i++) {
          if (pipe->ev_h2d[i]) (void)hipEventDestroy(pipe->ev_h2d[i]);
          if (pipe->ev_enc[i]) (void)hipEventDestroy(pipe->ev_enc[i]);
          if (pipe->ev_d2h[i]) (void)hipEventDestroy(pipe->ev_d2h[i]);
        }
        for (auto& e : pipe->ev_t) if (e) (void)hipEventDestroy(e);
        if (pipe->up) (void)hipStreamDestroy(pipe->up);
        if (pipe->down) (void)hipStreamDestroy(pipe->down);
        pipe.reset();
      }
      for (auto& e : ev) if (e) (void)hipEventDestroy(e);
      for (auto& e : dev_ev) if (e) (void)hipEventDestroy(e);
      if (ev_sync) (void)hipEventDestroy(ev_sync);
      if (ev_join) (void)hipEventDestroy(ev_join);
      if (side) (void)hipStreamDestroy(side);
      if (ev_tot) (void)hipEventDestroy(ev_tot);
      if (host) (void)hipHostFree(host);
      if (stream) (void)hipStreamDestroy(stream);
    }
  }
};

}  // namespace

// ----------------------------------------------------------------------------- tokenizer

struct ctok {
  // host-side model (immutable after load)
  std::unordered_map<std::string, uint32_t> vocab;          // model.vocab
  std::unordered_map<uint32_t, std::string> id_to_token;    // Vocab::id_to_token
  std::vector<std::pair<std::string, uint32_t>> special;    // special added tokens
  bool nfc = true;
  bool add_prefix_space = false;
  // compiled tables
  std::vector<uint64_t> merge_tab;
  uint32_t merge_mask = 0;
  std::vector<uint64_t> lds_image;  // kLdsImageBytes: hot table + Bloom filter
  std::vector<uint64_t> lds16_image, merge16;  // narrow vocabularies: the 32-bit-key tables (key16)
  uint32_t merge16_mask = 0;
  std::vector<uint32_t> pair0;      // 256 x 256 byte-pair merge values
  size_t hot_entries = 0;
  std::vector<uint32_t> piece_tab;  // 4 u32 per slot (see ctok_internal.h piece_hash)
  uint32_t piece_mask = 0;
  std::vector<uint32_t> rank_newid;
  std::vector<uint32_t> eager_bits;  // bit v: the merge of table value v is eager (see Tables::eager)
  std::vector<uint32_t> wmeta;       // window rounds (Tables::wmeta): per id, max left | max right << 16
  bool window = false;               // window rounds exact for this table (see Tables::window)
  int32_t byte2id[256];
  std::string at_bytes;
  std::vector<uint32_t> at_off{0}, at_id;
  std::vector<uint8_t> at_flags;
  bool proper = true;
  bool compact = false;
  bool narrow = false;  // every vocab id < 2^16
  bool ids16 = false;   // every id encode can emit (vocab and added tokens) < 2^16: 16-bit ids on PCIe
  // decode (src/huggingface/mod.rs:710-747): decoder kind, per-id decoded bytes
  int decoder = 1;                  // 1 ByteLevel, 0 raw concatenation (unknown decoder type), -1 unsupported
  std::string decoder_name;         // for the unsupported message
  std::vector<uint32_t> dec_ent;    // 2 u32 per id: byte offset, length | kDecNonAscii | kDecSpecial
  std::vector<uint8_t> dec_bytes;   // each id's bytes, 4-byte aligned, + 8 bytes of padding
  // post-processor, compiled to the items of PostProcessor::process(ids, None)
  // (src/postprocessors.rs:34-55): kPadItemA = the row's ids, else one special id
  bool has_pp = false;
  std::vector<uint32_t> pp_items;
  int pp_kind = 0;                   // 1 TemplateProcessing, 2 RobertaProcessing, 3 BertProcessing
  std::string pp_single, pp_pair;    // template strings (num_special_tokens_to_add)
  bool pp_has_pair = false;
  uint64_t model_max_length = 512;  // from_file / from_str: src/huggingface/mod.rs:243-245
  // per device
  std::mutex dev_mu;
  std::map<int, std::unique_ptr<DeviceState>> devs;
};

namespace {

bool get_bool_field(const ctj::Value& o, const char* k, bool dflt, const char* ctx) {
  const ctj::Value* v = o.get(k);
  if (!v) return dflt;
  if (v->kind != ctj::Value::Bool) throw_err(CTOK_E_PARSE, std::string("invalid type for `") + k + "` in " + ctx + ", expected a boolean");
  return v->b;
}

// parse_normalizer (src/huggingface/parsing.rs:10-90): 1 = NFC, 0 = none
int parse_normalizer(const ctj::Value* v) {
  if (v && v->kind == ctj::Value::Object) {
    const ctj::Value* t = v->get("type");
    if (t) {
      std::string ty = t->kind == ctj::Value::String ? t->s : "";
      if (ty == "NFC") return 1;
      if (ty == "Sequence") {
        const ctj::Value* ns = v->get("normalizers");
        if (!ns || ns->kind != ctj::Value::Array) return 0;
        int any = 0;
        for (const auto& n : ns->arr) any |= parse_normalizer(&n);  // NFC is idempotent
        return any;
      }
      static const char* unsup[] = {"NFD", "NFKC", "NFKD", "Lowercase", "Strip", "StripAccents", "Replace",
                                    "Prepend", "BertNormalizer", "Precompiled"};
      for (const char* u : unsup)
        if (ty == u) throw_err(CTOK_E_UNSUPPORTED, "normalizer `" + ty + "` is outside the encode hot path (only NFC / none)");
      return 0;
    }
  }
  return 1;  // null, absent, or an object without "type": NFC (parsing.rs:89)
}

bool is_white_space(uint32_t c) {  // Unicode White_Space (Rust char::is_whitespace)
  return (c >= 9 && c <= 13) || c == 32 || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
         c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

std::string encode_utf8(const std::vector<uint32_t>& cps, size_t a, size_t b) {
  std::string s;
  for (size_t i = a; i < b; i++) {
    const uint32_t c = cps[i];
    if (c < 0x80) {
      s += (char)c;
    } else if (c < 0x800) {
      s += (char)(0xC0 | (c >> 6));
      s += (char)(0x80 | (c & 63));
    } else if (c < 0x10000) {
      s += (char)(0xE0 | (c >> 12));
      s += (char)(0x80 | ((c >> 6) & 63));
      s += (char)(0x80 | (c & 63));
    } else {
      s += (char)(0xF0 | (c >> 18));
      s += (char)(0x80 | ((c >> 12) & 63));
      s += (char)(0x80 | ((c >> 6) & 63));
      s += (char)(0x80 | (c & 63));
    }
  }
  return s;
}

// parse_post_processor (src/huggingface/parsing.rs:193-253) and PostProcessor::process(ids, None)
// (src/postprocessors.rs:34-147), compiled to a list of items: kPadItemA = the sequence's ids,
// anything else = one special id.  The encode paths only ever call process(ids, None), so a
// template's $B and the pair template are never used.  "Sequence" and other types -> None.
void parse_post_processor(ctok* t, const ctj::Value* v) {
  t->has_pp = false;
  t->pp_items.clear();
  t->pp_kind = 0;
  if (!v || v->kind != ctj::Value::Object) return;
  const ctj::Value* ty = v->get("type");
  if (!ty) return;
  const std::string kind = ty->kind == ctj::Value::String ? ty->s : "";
  auto special = [&](const std::string& name, bool* found) -> uint32_t {
    for (const auto& e : t->special)
      if (e.first == name) {
        *found = true;
        return e.second;
      }
    *found = false;
    return 0;
  };
  if (kind == "TemplateProcessing") {
    std::string tpl = "<s> $A </s>";
    const ctj::Value* single = v->get("single");
    if (single && single->kind == ctj::Value::Array) {  // template_from_array (parsing.rs:236-253)
      std::vector<std::string> parts;
      for (const auto& item : single->arr) {
        if (item.kind != ctj::Value::Object) continue;
        if (const ctj::Value* sp = item.get("SpecialToken")) {
          const ctj::Value* id = sp->get("id");
          if (id && id->kind == ctj::Value::String) parts.push_back(id->s);
          continue;
        }
        if (const ctj::Value* sq = item.get("Sequence")) {
          const ctj::Value* id = sq->get("id");
          if (id && id->kind == ctj::Value::String) parts.push_back("$" + id->s);
        }
      }
      tpl.clear();
      for (size_t i = 0; i < parts.size(); i++) tpl += (i ? " " : "") + parts[i];
    }
    t->pp_single = tpl;
    if (const ctj::Value* pair = v->get("pair")) {
      if (pair->kind == ctj::Value::Array) {
        std::string ps;
        bool first = true;
        for (const auto& item : pair->arr) {
          if (item.kind != ctj::Value::Object) continue;
          std::string part;
          bool ok = false;
          if (const ctj::Value* sp = item.get("SpecialToken")) {
            const ctj::Value* id = sp->get("id");
            if (id && id->kind == ctj::Value::String) part = id->s, ok = true;
          } else if (const ctj::Value* sq = item.get("Sequence")) {
            const ctj::Value* id = sq->get("id");
            if (id && id->kind == ctj::Value::String) part = "$" + id->s, ok = true;
          }
          if (ok) {
            ps += (first ? "" : " ") + part;
            first = false;
          }
        }
        t->pp_pair = ps;
        t->pp_has_pair = true;
      }
    }
    t->pp_kind = 1;
    std::vector<uint32_t> ch;
    if (!decode_utf8(tpl, ch)) throw_err(CTOK_E_PARSE, "post_processor template is not valid UTF-8");
    size_t i = 0;  // template_process's walk (postprocessors.rs:103-144)
    while (i < ch.size()) {
      if (ch[i] == '$' && i + 1 < ch.size()) {
        if (ch[i + 1] == 'A') t->pp_items.push_back(kPadItemA);
        if (ch[i + 1] == 'A' || ch[i + 1] == 'B') i += 2;  // $B: the pair, absent in process(ids, None)
        else i += 1;
      } else if (ch[i] == '<' || ch[i] == '[') {
        const uint32_t end = ch[i] == '<' ? '>' : ']';
        const size_t a = i;
        while (i < ch.size() && ch[i] != end) i++;
        if (i < ch.size()) i++;  // include the end char
        size_t b = i;
        while (b > a && is_white_space(ch[b - 1])) b--;  // str::trim (the start is '<' or '[')
        bool found;
        const uint32_t id = special(encode_utf8(ch, a, b), &found);
        if (found) t->pp_items.push_back(id);
      } else {
        i++;
      }
    }
    t->has_pp = true;
  } else if (kind == "RobertaProcessing" || kind == "BertProcessing") {  // parsing.rs:221-236
    const bool roberta = kind == "RobertaProcessing";
    bool f;
    uint32_t a = special(roberta ? "<s>" : "[CLS]", &f);
    if (!f) a = roberta ? 0 : 101;
    uint32_t b = special(roberta ? "</s>" : "[SEP]", &f);
    if (!f) b = roberta ? 2 : 102;
    t->pp_items = {a, kPadItemA, b};  // roberta_process / bert_process with no pair
    t->has_pp = true;
    t->pp_kind = roberta ? 2 : 3;
  }
}

// Does the Rust regex crate compile pattern p?  The reference compiles a Split's pattern and, when
// Regex::new fails, leaves the text unsplit (src/pretokenizers.rs:277-302): the Split is a no-op.
// The crate (regex ^1.10, Cargo.toml:19; the regex-syntax grammar) has no look-around,
// backreferences, atomic groups, branch resets, comments or conditionals, rejects unknown escapes,
// a repetition with nothing to repeat, an inverted {n,m}, unbalanced groups / classes, unknown ASCII
// classes and \p{..} names that are not Unicode property names or values (UAX #44 loose matching;
// gen/regex_props.h, from the `regex` module's tables: a superset of the crate's).  This walks the
// pattern with that grammar and returns the first construct the crate rejects, "" when there is
// none.  It errs one way only: what it cannot decide counts as compiling (verbose-mode patterns,
// hex escapes, Age=), and a compiling Split is refused by the loader (CTOK_E_UNSUPPORTED), never
// silently dropped.  Possessive quantifiers (a++) are a repetition of a repetition to regex-syntax:
// they compile.  Restated for the tests by oracle/rust_regex.py.
namespace rxs {

std::string canon(std::string_view s) {
  std::string o;
  for (char c : s)
    if (c != ' ' && c != '_' && c != '-' && c != '\t' && c != '\n') o += (char)toupper((unsigned char)c);
  return o;
}

template <size_t N>
bool in_table(const char* const (&tab)[N], const std::string& k) {
  return std::binary_search(tab, tab + N, k.c_str(), [](const char* a, const char* b) { return strcmp(a, b) < 0; });
}

bool single_known(const std::string& c) {
  if (in_table(ct_prop_single, c)) return true;
  return c.size() > 2 && c.compare(0, 2, "IS") == 0 && in_table(ct_prop_single, c.substr(2));  // "is" prefix
}

// \p{body}: a property the crate may know (name=value for gc / sc / scx / gcb / wb / sb, age
// taken as known; other properties the tables know: taken as known, a name they do not: unknown)
bool property_known(std::string_view body) {
  for (std::string_view sep : {std::string_view("!="), std::string_view("="), std::string_view(":")}) {
    const size_t at = body.find(sep);
    if (at == std::string_view::npos) continue;
    std::string k = canon(body.substr(0, at)), v = canon(body.substr(at + sep.size()));
    if (k == "AGE") return true;
    static const std::map<std::string, std::string> kv = {
        {"GC", "GC"}, {"GENERALCATEGORY", "GC"}, {"SC", "SC"}, {"SCRIPT", "SC"}, {"SCX", "SCX"},
        {"SCRIPTEXTENSIONS", "SCX"}, {"GCB", "GCB"}, {"GRAPHEMECLUSTERBREAK", "GCB"}, {"WB", "WB"},
        {"WORDBREAK", "WB"}, {"SB", "SB"}, {"SENTENCEBREAK", "SB"}};
    auto it = kv.find(k);
    if (it != kv.end()) return in_table(ct_prop_kv, it->second + "=" + v);
    return in_table(ct_prop_other, k);
  }
  return single_known(canon(body));
}

}  // namespace rxs

std::string rust_regex_rejects(const std::string& p) {
  const size_t n = p.size();
  size_t i = 0;
  int depth = 0;
  std::vector<bool> empty{true};  // per open group: nothing to repeat yet
  auto is_alnum = [](char c) { return isalnum((unsigned char)c) != 0; };
  // at p[j] == '\\' (inside or outside a class): "" or the reason; j moves past the escape
  auto escape = [&](size_t& j) -> std::string {
    if (j + 1 >= n) return "trailing backslash";
    const char c = p[j + 1];
    if (c >= '1' && c <= '9') return std::string("backreference \\") + c;
    if (c == 'k') return "named backreference \\k";
    if (c == 'g') return "backreference \\g";
    if (c == 'p' || c == 'P') {
      if (j + 2 >= n) return "incomplete \\p escape";
      if (p[j + 2] == '{') {
        const size_t e = p.find('}', j + 3);
        if (e == std::string::npos) return "unclosed \\p{";
        const std::string body = p.substr(j + 3, e - j - 3);
        j = e + 1;
        return rxs::property_known(body) ? "" : "unknown Unicode property \\p{" + body + "}";
      }
      const std::string body(1, p[j + 2]);
      j += 3;
      return rxs::property_known(body) ? "" : "unknown Unicode property \\p" + body;
    }
    j += 2;
    if (c == 'x' || c == 'u' || c == 'U') return "";  // (hex escapes: taken as valid)
    if (is_alnum(c) && !strchr("aftnrvAzbBdDsSwW", c)) return std::string("unrecognized escape \\") + c;
    return "";
  };
  while (i < n) {
    const char c = p[i];
    if (c == '\\') {
      const std::string why = escape(i);
      if (!why.empty()) return why;
      empty.back() = false;
      continue;
    }
    if (c == '[') {  // class: nested classes, escapes, [:name:]; a leading ']' is literal
      size_t j = i + 1;
      if (j < n && p[j] == '^') j++;
      if (j < n && p[j] == ']') j++;
      int cd = 1;
      while (j < n && cd) {
        const char d = p[j];
        if (d == '\\') {
          const std::string why = escape(j);
          if (!why.empty()) return why;
          continue;
        }
        if (d == '[' && j + 1 < n && p[j + 1] == ':') {
          // [:name:] with a known name is an ASCII class; with any other name regex-syntax
          // (maybe_parse_ascii_class) backtracks and reads the '[' as a nested class
          const size_t e = p.find(":]", j + 2);
          if (e != std::string::npos) {
            std::string nm = p.substr(j + 2, e - j - 2);
            if (!nm.empty() && nm[0] == '^') nm.erase(0, 1);
            static const char* const kAscii[] = {"alnum", "alpha", "ascii", "blank", "cntrl", "digit", "graph",
                                                 "lower", "print", "punct", "space", "upper", "word", "xdigit"};
            if (std::find_if(std::begin(kAscii), std::end(kAscii), [&](const char* a) { return nm == a; }) != std::end(kAscii)) {
              j = e + 2;
              continue;
            }
          }
        }
        if (d == '[') {
          cd++;
          j++;
          if (j < n && p[j] == '^') j++;
          if (j < n && p[j] == ']') j++;
          continue;
        }
        if (d == ']') cd--;
        j++;
      }
      if (cd) return "unclosed character class";
      i = j;
      empty.back() = false;
      continue;
    }
    if (c == '(') {
      if (i + 1 < n && p[i + 1] == '?') {
        const std::string_view rest = std::string_view(p).substr(i + 2);
        auto starts = [&](const char* s) { return rest.compare(0, strlen(s), s) == 0; };
        if (starts("=") || starts("!")) return std::string("look-ahead (?") + rest[0];
        if (starts("<=") || starts("<!")) return "look-behind (?" + std::string(rest.substr(0, 2));
        if (starts(">")) return "atomic group (?>";
        if (starts("P=")) return "named backreference (?P=";
        if (!rest.empty() && (strchr("|#('&+0", rest[0]) || isdigit((unsigned char)rest[0])))
          return std::string("unsupported group (?") + rest[0];
        if (starts("P<") || starts("<")) {
          const size_t k = i + 2 + (starts("P<") ? 2 : 1);
          const size_t e = p.find('>', k);
          if (e == std::string::npos) return "unclosed group name";
          const std::string name = p.substr(k, e - k);
          bool ok = !name.empty() && (isalpha((unsigned char)name[0]) || name[0] == '_');
          for (char ch : name) ok = ok && (is_alnum(ch) || ch == '_' || ch == '.' || ch == '[' || ch == ']');
          if (!ok) return "invalid group name " + name;
          i = e + 1;
        } else {  // flags: (?flags) or (?flags:...)
          size_t k = i + 2;
          while (k < n && strchr("imsxuUR-", p[k])) {
            if (p[k] == 'x') return "";  // verbose mode (comments, ignored space): not walked; taken as compiling
            k++;
          }
          if (k >= n || (p[k] != ':' && p[k] != ')')) return std::string("unrecognized flag ") + (k < n ? p.substr(k, 1) : "(end)");
          i = k + 1;
          if (p[k] == ')') continue;
        }
      } else {
        i++;
      }
      depth++;
      empty.push_back(true);
      continue;
    }
    if (c == ')') {
      if (--depth < 0) return "unbalanced ')'";
      empty.pop_back();
      empty.back() = false;
      i++;
      continue;
    }
    if (c == '|') {
      empty.back() = true;
      i++;
      continue;
    }
    if (c == '*' || c == '+' || c == '?') {
      if (empty.back()) return "repetition operator missing expression";
      i++;
      continue;
    }
    if (c == '{') {  // counted repetition {n}, {n,}, {n,m}; anything else is not walked further
      const size_t e = p.find('}', i);
      if (e != std::string::npos) {
        const std::string body = p.substr(i + 1, e - i - 1);
        const size_t comma = body.find(',');
        const std::string a = body.substr(0, comma), b = comma == std::string::npos ? "" : body.substr(comma + 1);
        auto digits = [](const std::string& s) { return !s.empty() && std::all_of(s.begin(), s.end(), ::isdigit); };
        // a count is a u32 (regex-syntax parse_decimal): a longer one is an invalid decimal
        auto count = [](const std::string& s) -> uint64_t {
          uint64_t v = 0;
          for (char ch : s) {
            v = v * 10 + (uint64_t)(ch - '0');
            if (v > 0xFFFFFFFFull) return ~(uint64_t)0;
          }
          return v;
        };
        if (digits(a) && (comma == std::string::npos || b.empty() || digits(b))) {
          if (empty.back()) return "repetition operator missing expression";
          if (count(a) == ~(uint64_t)0 || (!b.empty() && count(b) == ~(uint64_t)0)) return "repetition count overflows u32 {" + body + "}";
          if (!b.empty() && count(b) < count(a)) return "invalid repetition range {" + body + "}";
          i = e + 1;
          continue;
        }
      }
      empty.back() = false;
      i++;
      continue;
    }
    empty.back() = false;
    i++;
  }
  if (depth) return "unclosed group";
  return "";
}

// flattens parse_pre_tokenizer (src/huggingface/parsing.rs:92-190) into the supported chain:
// no-op Splits (patterns the Rust regex crate rejects, src/pretokenizers.rs:298-302) around
// exactly one ByteLevel.  kinds: 'B' ByteLevel, 'S' no-op split
void parse_pre_tokenizer(const ctj::Value* v, std::vector<std::pair<char, bool>>& chain, int depth) {
  if (!(v && v->kind == ctj::Value::Object && v->get("type"))) {
    if (depth == 0) { chain.push_back({'B', false}); return; }  // default ByteLevel(false)
    throw_err(CTOK_E_UNSUPPORTED, "pre_tokenizer entry without a type");
  }
  const ctj::Value* t = v->get("type");
  std::string ty = t->kind == ctj::Value::String ? t->s : "";
  if (ty == "ByteLevel") {
    const ctj::Value* a = v->get("add_prefix_space");
    chain.push_back({'B', a && a->kind == ctj::Value::Bool ? a->b : false});
  } else if (ty == "Split") {
    std::string pat;
    const ctj::Value* p = v->get("pattern");
    if (p && p->kind == ctj::Value::Object) {
      const ctj::Value* r = p->get("Regex");
      if (r && r->kind == ctj::Value::String) pat = r->s;
    }
    if (rust_regex_rejects(pat).empty())
      throw_err(CTOK_E_UNSUPPORTED, "Split pre-tokenizer with a pattern the Rust regex crate compiles is outside the "
                                    "encode hot path: nothing the crate rejects (look-around, backreference, atomic "
                                    "group, unknown escape or \\p{..} name, unbalanced group / class) was found, so "
                                    "the pattern is taken as compiling (pattern: " + pat + ")");
    chain.push_back({'S', false});
  } else if (ty == "Sequence" && depth == 0) {
    const ctj::Value* ps = v->get("pretokenizers");
    if (!ps || ps->kind != ctj::Value::Array || ps->arr.empty())
      throw_err(CTOK_E_UNSUPPORTED, "empty pre_tokenizer Sequence (no byte-level split)");
    for (const auto& e : ps->arr) parse_pre_tokenizer(&e, chain, depth + 1);
  } else {
    throw_err(CTOK_E_UNSUPPORTED, "pre_tokenizer `" + ty + "` is outside the encode hot path (ByteLevel only)");
  }
}


// parse_decoder (src/huggingface/parsing.rs:272-364) reduced to what decode needs: 1 = ByteLevel
// (also the default for a null / absent / non-object value or an object without "type"),
// 0 = None (an unknown type string: BpeTokenizer::decode joins the raw vocab strings,
// src/huggingface/mod.rs:737-740), -1 = a decoder outside the ByteLevel-BPE path.  In a
// Sequence, entries that parse to None are dropped (filter_map), Fuse is the identity on the
// one-string list the previous decoder leaves, and one ByteLevel is the whole effect.
int parse_decoder(const ctj::Value* v, std::string& name) {
  if (!v || v->kind != ctj::Value::Object) return 1;
  const ctj::Value* ty = v->get("type");
  if (!ty) return 1;
  const std::string t = ty->kind == ctj::Value::String ? ty->s : "";
  if (t == "ByteLevel") return 1;
  if (t == "Fuse") return 0;
  if (t == "Metaspace" || t == "WordPiece" || t == "BPE" || t == "CTC" || t == "Strip") { name = t; return -1; }
  if (t != "Sequence") return 0;
  const ctj::Value* decs = v->get("decoders");
  if (!decs || decs->kind != ctj::Value::Array || decs->arr.empty()) return 0;
  int nbl = 0, kept = 0;
  for (const auto& d : decs->arr) {
    std::string sub;
    const int k = parse_decoder(&d, sub);
    if (k < 0) { name = sub; return -1; }
    const ctj::Value* dt = d.kind == ctj::Value::Object ? d.get("type") : nullptr;
    const bool fuse = dt && dt->kind == ctj::Value::String && dt->s == "Fuse";
    if (k == 0 && !fuse) continue;  // None: dropped by filter_map
    kept++;
    if (k == 1) nbl++;
  }
  if (!kept) return 0;
  if (nbl > 1) { name = "Sequence with more than one ByteLevel"; return -1; }
  return nbl;
}

// Per-id decoded bytes: the ByteLevel decoder maps every char of the token back to a byte ('Ġ'
// and the 255 other GPT-2 chars, src/decoders.rs:74-92,101-107), keeps other ASCII chars
// (:108-110) and drops the rest; the raw decoder keeps the token's UTF-8 bytes.
void build_decode_table(ctok* t) {
  uint32_t n_ent = 0;
  for (const auto& kv : t->id_to_token) n_ent = std::max(n_ent, kv.first + 1);
  if (n_ent > (1u << 26)) throw_err(CTOK_E_UNSUPPORTED, "token ids above 2^26 are not supported by the decode table");
  std::vector<int> inv(0x144, -1);  // GPT-2 char -> byte
  {
    std::vector<uint32_t> bm = byte_map();
    for (int b = 0; b < 256; b++) inv[bm[b]] = b;
  }
  std::unordered_set<std::string> special;
  for (const auto& sp : t->special) special.insert(sp.first);
  t->dec_ent.assign(2 * (size_t)n_ent, 0);
  t->dec_bytes.clear();
  std::vector<uint32_t> cps;
  std::string out;
  for (uint32_t id = 0; id < n_ent; id++) {
    auto it = t->id_to_token.find(id);
    if (it == t->id_to_token.end()) continue;
    const std::string& tok = it->second;
    out.clear();
    if (t->decoder == 1) {
      if (!decode_utf8(tok, cps)) throw_err(CTOK_E_PARSE, "vocab entry is not valid UTF-8");
      for (uint32_t c : cps) {
        if (c < inv.size() && inv[c] >= 0) out += (char)inv[c];
        else if (c < 0x80) out += (char)c;
      }
    } else {
      out = tok;
    }
    if (out.size() > kDecLenMask) throw_err(CTOK_E_UNSUPPORTED, "vocab entry longer than 16 MiB");
    uint32_t y = (uint32_t)out.size();
    for (unsigned char c : out)
      if (c >= 0x80) { y |= kDecNonAscii; break; }
    if (special.count(tok)) y |= kDecSpecial;
    while (t->dec_bytes.size() & 3) t->dec_bytes.push_back(0);
    t->dec_ent[2 * id] = (uint32_t)t->dec_bytes.size();
    t->dec_ent[2 * id + 1] = y;
    t->dec_bytes.insert(t->dec_bytes.end(), out.begin(), out.end());
  }
  for (int k = 0; k < 8; k++) t->dec_bytes.push_back(0);
}

void load_root(ctok* t, const ctj::Value& root);

void load(ctok* t, const char* buf, size_t len) {
  // CTOK_LOAD_TIMING=1: per-phase load times on stderr
  const bool lt = getenv("CTOK_LOAD_TIMING") != nullptr;
  auto lt0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!lt) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[ctok load] %-12s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - lt0).count());
    lt0 = now;
  };
  ctj::Value root;
  try {
    root = ctj::parse(buf, len);
  } catch (const ctj::ParseError& e) {
    throw_err(CTOK_E_PARSE, e.what());
  }
  lap("json");
  load_root(t, root);
}

// The tokenizer from its parsed tokenizer.json value (from a file, a buffer, or built from tables
// by ctok_create_from_tables).
void load_root(ctok* t, const ctj::Value& root) {
  const bool lt = getenv("CTOK_LOAD_TIMING") != nullptr;
  auto lt0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!lt) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[ctok load] %-12s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - lt0).count());
    lt0 = now;
  };
  if (root.kind != ctj::Value::Object) throw_err(CTOK_E_PARSE, "invalid type: expected struct TokenizerJson");
  const ctj::Value* model = root.get("model");
  if (!model) throw_err(CTOK_E_PARSE, "missing field `model`");
  if (model->kind != ctj::Value::Object) throw_err(CTOK_E_PARSE, "invalid type for `model`, expected struct ModelJson");
  const ctj::Value* vocab = model->get("vocab");
  if (!vocab) throw_err(CTOK_E_PARSE, "missing field `vocab`");
  if (vocab->kind != ctj::Value::Object) throw_err(CTOK_E_PARSE, "invalid type for `vocab`, expected a map");
  t->vocab.reserve(vocab->obj.size() * 2);
  std::vector<const std::string*> first_keys;  // first occurrence of each key, in file order
  first_keys.reserve(vocab->obj.size());
  for (const auto& m : vocab->obj) {
    if (!m.second.is_u32()) throw_err(CTOK_E_PARSE, "invalid value for vocab entry `" + m.first + "`, expected u32");
    auto ins = t->vocab.try_emplace(m.first, (uint32_t)m.second.u);
    if (ins.second) first_keys.push_back(&m.first);
    else ins.first->second = (uint32_t)m.second.u;  // HashMap insert: a later duplicate key wins
  }
  // Vocab::id_to_token (src/vocab.rs:47-52).  Several tokens sharing one id make the reference's
  // choice depend on HashMap order; here the later entry of the file wins (first occurrence of a
  // key, final value) -- parity for such files is unpinned.
  t->id_to_token.reserve(first_keys.size() * 2);
  for (const std::string* k : first_keys) t->id_to_token[t->vocab.find(*k)->second] = *k;

  lap("vocab");
  // merges: deserialize_merges (mod.rs:56-101) then split(' ') == 2 parts (mod.rs:252-264)
  std::vector<std::pair<std::string, std::string>> merges;
  if (const ctj::Value* mv = model->get("merges")) {
    if (mv->kind != ctj::Value::Array) throw_err(CTOK_E_PARSE, "invalid type for `merges`, expected a sequence of strings or arrays of two strings");
    merges.reserve(mv->arr.size());
    for (const auto& it : mv->arr) {
      std::string s;
      if (it.kind == ctj::Value::String) s = it.s;
      else if (it.kind == ctj::Value::Array && it.arr.size() == 2 && it.arr[0].kind == ctj::Value::String &&
               it.arr[1].kind == ctj::Value::String) s = it.arr[0].s + " " + it.arr[1].s;
      else continue;
      size_t sp = s.find(' ');
      if (sp == std::string::npos || s.find(' ', sp + 1) != std::string::npos) continue;
      merges.emplace_back(s.substr(0, sp), s.substr(sp + 1));
    }
  }
  // BpeTokenizer::new (src/bpe.rs:52-79)
  std::unordered_map<uint64_t, uint32_t> ranks;  // (a<<32|b) -> rank, last duplicate wins
  ranks.reserve(merges.size() * 2);
  std::vector<uint32_t> valid_new;
  for (size_t r = 0; r < merges.size(); r++) {
    auto ia = t->vocab.find(merges[r].first);
    auto ib = t->vocab.find(merges[r].second);
    if (ia == t->vocab.end() || ib == t->vocab.end()) continue;
    auto in = t->vocab.find(merges[r].first + merges[r].second);
    if (in == t->vocab.end()) continue;
    ranks[((uint64_t)ia->second << 32) | ib->second] = (uint32_t)r;
    valid_new.push_back(in->second);
  }
  lap("ranks");
  if (merges.size() >= (size_t)kNoRank - 2) throw_err(CTOK_E_UNSUPPORTED, "more than 4M merges");
  t->rank_newid = valid_new;
  {
    uint32_t max_id = 0;
    for (const auto& kv : t->vocab) max_id = std::max(max_id, kv.second);
    t->narrow = max_id < 0xFFFFu;
  }
  // compact table: values are the new ids themselves when new id is strictly increasing in rank
  {
    std::vector<std::pair<uint32_t, uint32_t>> rv;  // (rank, new id) of the entries that can merge
    rv.reserve(ranks.size());
    for (const auto& kv : ranks)
      if (kv.second < valid_new.size()) rv.push_back({kv.second, valid_new[kv.second]});
    std::sort(rv.begin(), rv.end());
    t->compact = true;
    for (size_t i = 1; i < rv.size(); i++)
      if (rv[i].second <= rv[i - 1].second) { t->compact = false; break; }
    if (getenv("CTOK_FORCE_WIDE")) t->compact = false;
  }
  size_t cap = 1024;
  // load factor <= 1/8: a lookup the Bloom filter lets through is often a pair with no merge,
  // whose linear probe runs to an empty slot (C2 k_bpe_short 0.54 -> 0.48 ms against 1/2)
  const size_t f42 = getenv("CTOK_MERGE_SLACK") ? (size_t)atoi(getenv("CTOK_MERGE_SLACK")) : 8;  // A/B knob
  while (cap < ranks.size() * f42 + 16) cap <<= 1;
  t->merge_tab.assign(cap, kEmpty);
  t->merge_mask = (uint32_t)(cap - 1);
  // inserted in rank order: the low-rank (frequent) pairs sit in their home slots, so their
  // lookups end at the first probe (the same reason the whole-piece table is filled in id order)
  std::vector<std::pair<uint32_t, uint64_t>> by_rank_key;
  by_rank_key.reserve(ranks.size());
  for (const auto& kv : ranks) by_rank_key.push_back({kv.second, kv.first});
  std::sort(by_rank_key.begin(), by_rank_key.end());
  for (const auto& rk : by_rank_key) {
    const std::pair<uint64_t, uint32_t> kv{rk.second, rk.first};
    uint32_t a = (uint32_t)(kv.first >> 32), b = (uint32_t)kv.first;
    if (a > kMaxId || b > kMaxId) throw_err(CTOK_E_UNSUPPORTED, "token ids above 2^21-2 are not supported by the device merge table");
    uint64_t val = kv.second;
    if (t->compact) val = kv.second < valid_new.size() ? valid_new[kv.second] : kPanicVal;
    uint64_t e = (val << 42) | ((uint64_t)a << kIdBits) | b;
    uint32_t h = mhash(a, b) & t->merge_mask;
    while (t->merge_tab[h] != kEmpty) h = (h + 1) & t->merge_mask;
    t->merge_tab[h] = e;
  }
  for (uint32_t id : valid_new)
    if (id > kMaxId) throw_err(CTOK_E_UNSUPPORTED, "token ids above 2^21-2 are not supported by the device merge table");
  lap("merge_tab");
  // byte-level initial ids: vocab[bytes_to_unicode[b]] (src/bpe.rs:94-97), -1 = dropped
  std::vector<uint32_t> bm = byte_map();
  for (int b = 0; b < 256; b++) {
    auto it = t->vocab.find(utf8(bm[b]));
    t->byte2id[b] = it == t->vocab.end() ? -1 : (int32_t)it->second;
  }

  // LDS image: hot table filled greedily in rank order (a pair whose two buckets are full stays
  // global-only), Bloom filter over every entry (including the ones whose lookup panics).
  // Byte-pair merges are left out of both: the merge passes look a pair up in LDS only after a
  // merge, when one side is a merged (multi-byte) token; initial byte pairs use pair0.
  {
    std::vector<uint8_t> is_byte_tok(kMaxId + 2, 0);
    for (int b = 0; b < 256; b++)
      if (t->byte2id[b] >= 0 && (uint32_t)t->byte2id[b] <= kMaxId) is_byte_tok[t->byte2id[b]] = 1;
    // image = hot table | Bloom filter of the pairs not in the hot table (the merge passes ask
    // the filter only after a hot-table miss), then, outside the image, the Bloom filter of all
    // pairs for the kernels that load the filter alone (k_bpe_wave without HOT)
    t->lds_image.assign(kLdsImageBytes / 8 + kBloomWords / 2, 0);
    uint64_t* hot = t->lds_image.data();
    std::fill(hot, hot + kHotU64, kEmpty);
    uint32_t* bloom = reinterpret_cast<uint32_t*>(hot + kHotU64);
    uint32_t* bloom_all = reinterpret_cast<uint32_t*>(t->lds_image.data() + kLdsImageBytes / 8);
    std::vector<std::pair<uint32_t, uint64_t>> by_rank;  // (rank, entry)
    by_rank.reserve(ranks.size());
    for (uint64_t e : t->merge_tab) {
      if (e == kEmpty) continue;
      const uint32_t a = (uint32_t)((e >> kIdBits) & ((1u << kIdBits) - 1)), b = (uint32_t)(e & ((1u << kIdBits) - 1));
      if (is_byte_tok[a] && is_byte_tok[b]) continue;
      by_rank.push_back({ranks.at(((uint64_t)a << 32) | b), e});
    }
    std::sort(by_rank.begin(), by_rank.end());
    size_t placed = 0;
    const bool use_hot = !getenv("CTOK_NO_HOT_TABLE");
    for (const auto& re : by_rank) {
      const uint64_t e = re.second;
      const uint32_t a = (uint32_t)((e >> kIdBits) & ((1u << kIdBits) - 1)), b = (uint32_t)(e & ((1u << kIdBits) - 1));
      const uint32_t h1 = mhash(a, b), h2 = mhash2(h1);
      const uint32_t b1 = (h1 >> 12) & (kBloomBits - 1), b2 = (h2 >> 12) & (kBloomBits - 1);
      bloom_all[b1 >> 5] |= 1u << (b1 & 31);
      bloom_all[b2 >> 5] |= 1u << (b2 & 31);
      uint64_t* slot = nullptr;
      if (use_hot && re.first < valid_new.size()) {  // never cache an entry that panics
        for (uint32_t c : {h1 & (kHotBuckets - 1), h2 & (kHotBuckets - 1)})
          for (int k = 0; k < 2 && !slot; k++)
            if (hot[2 * c + k] == kEmpty) slot = &hot[2 * c + k];
      }
      if (slot) {
        *slot = e;
        placed++;
        continue;  // a hot pair is found in the hot table before the filter is asked
      }
      bloom[b1 >> 5] |= 1u << (b1 & 31);
      bloom[b2 >> 5] |= 1u << (b2 & 31);
    }
    t->hot_entries = placed;
    // narrow vocabularies: the same tables keyed by key16 (ctok_internal.h), for the register
    // merge passes.  Global table: every entry, in rank order; hot table / Bloom filter: as above.
    if (t->narrow) {
      size_t cap16 = 1024;
      // load <= 1/64: a lookup that reaches this table (a hot-table miss passing the Bloom filter)
      // stops at its first slot almost always, and a wavefront waits for its slowest lane's
      // probe chain -- C2 k_bpe_short 0.414 ms at 1/8, 0.391 at 1/32, 0.385 at 1/128 (A/B on one
      // box, profiles/r02/v9_ab_merge16_load.txt); 32 MB for 50k merges
      const size_t f16 = getenv("CTOK_MERGE16_SLACK") ? (size_t)atoi(getenv("CTOK_MERGE16_SLACK")) : 64;
      while (cap16 < ranks.size() * f16 + 16) cap16 <<= 1;
      t->merge16.assign(cap16, kEmpty);
      t->merge16_mask = (uint32_t)(cap16 - 1);
      for (const auto& rk : by_rank_key) {
        const uint32_t a = (uint32_t)(rk.second >> 32), b = (uint32_t)rk.second;
        uint64_t val = rk.first;
        if (t->compact) val = rk.first < valid_new.size() ? valid_new[rk.first] : kPanicVal;
        uint32_t h = hash16_h(a, b) & t->merge16_mask;
        while (t->merge16[h] != kEmpty) h = (h + 1) & t->merge16_mask;
        t->merge16[h] = (val << 32) | key16(a, b);
      }
      t->lds16_image.assign(kLdsImageBytes / 8, 0);
      uint64_t* hot16 = t->lds16_image.data();
      std::fill(hot16, hot16 + kHotU64, kEmpty);
      uint32_t* bloom16 = reinterpret_cast<uint32_t*>(hot16 + kHotU64);
      for (const auto& re : by_rank) {
        const uint64_t e = re.second;
        const uint32_t a = (uint32_t)((e >> kIdBits) & ((1u << kIdBits) - 1)), b = (uint32_t)(e & ((1u << kIdBits) - 1));
        const uint32_t h = hash16_h(a, b), g = hash16_g(a, b);
        uint64_t* slot = nullptr;
        if (use_hot && re.first < valid_new.size())
          for (uint32_t c : {h >> 20, g >> 20})
            for (int k = 0; k < 2 && !slot; k++)
              if (hot16[2 * c + k] == kEmpty) slot = &hot16[2 * c + k];
        if (slot) {
          *slot = ((e >> 42) << 32) | key16(a, b);
          continue;
        }
        const uint32_t b1 = h & (kBloomBits - 1), b2 = g >> 14;
        bloom16[b1 >> 5] |= 1u << (b1 & 31);
        bloom16[b2 >> 5] |= 1u << (b2 & 31);
      }
    }
  }
  lap("lds_image");
  // rank monotonicity ("proper"): every merge consuming z ranks after every merge producing z
  {
    // per id (ids <= kMaxId, checked above): the latest rank producing it, the earliest consuming it
    constexpr uint32_t kUnset = UINT32_MAX;
    std::vector<uint32_t> maxprod(kMaxId + 2, kUnset), mincons(kMaxId + 2, kUnset);
    for (const auto& kv : ranks) {
      uint32_t r = kv.second;
      if (r >= valid_new.size()) continue;  // panics on lookup anyway
      uint32_t z = valid_new[r];
      if (maxprod[z] == kUnset || maxprod[z] < r) maxprod[z] = r;
      for (uint32_t c : {(uint32_t)(kv.first >> 32), (uint32_t)kv.first})
        if (mincons[c] == kUnset || mincons[c] > r) mincons[c] = r;
    }
    t->proper = true;
    for (size_t z = 0; z < maxprod.size(); z++)
      if (maxprod[z] != kUnset && mincons[z] != kUnset && mincons[z] <= maxprod[z]) { t->proper = false; break; }
    // per merge (bit at its table value: the rank, or the new id in a compact table): "eager"
    // when a merge consuming its token ranks before it.  Only an eager merge can be followed at
    // once by a merge of lower rank, so the long-piece rounds apply every occurrence of a
    // non-eager merge together even when the table as a whole is not rank-monotone (tiktoken-
    // style lists), and the leftmost one alone for an eager merge (ctok_internal.h Tables::eager).
    t->eager_bits.assign(((t->compact ? kMaxId + 2 : valid_new.size()) + 31) / 32 + 1, 0u);
    if (!t->proper) {
      for (const auto& kv : ranks) {
        const uint32_t r = kv.second;
        if (r >= valid_new.size()) continue;
        const uint32_t z = valid_new[r];
        if (mincons[z] != kUnset && mincons[z] < r) {
          const uint32_t v = t->compact ? z : r;
          t->eager_bits[v >> 5] |= 1u << (v & 31);
        }
      }
    }
  }


  // window rounds of the long-piece tiers (Tables::window, kernels.hip bpe_wave_seg): exact when
  // every token instance spans exactly its string's length -- each byte's initial token is one
  // char, and every merge that can apply makes the token its two sides spell (no rank shift from
  // an invalid merge before it, src/bpe.rs:60-69); on a table that is not rank-monotone the
  // kernels add a check for candidates whose merge is eager.
  // Per id: the longest left side of a merge whose right side it is, and the longest right side
  // of a merge whose left side it is (chars = bytes; 0xFFFF when longer).
  {
    auto nchars = [&](uint32_t id, bool& ok) -> uint32_t {
      auto it = t->id_to_token.find(id);
      if (it == t->id_to_token.end()) { ok = false; return 0; }
      uint32_t c = 0;
      for (unsigned char ch : it->second) c += (ch & 0xC0) != 0x80;
      return c;
    };
    // (not rank-monotone: the kernels check each candidate whose merge is eager, bpe_wave_seg)
    bool ok = !getenv("CTOK_NO_WINDOW");
    for (int b = 0; b < 256 && ok; b++)
      if (t->byte2id[b] >= 0 && nchars((uint32_t)t->byte2id[b], ok) != 1) ok = false;
    uint32_t max_id = 0;
    for (const auto& kv : t->vocab) max_id = std::max(max_id, kv.second);
    std::vector<uint32_t> ml, mr;
    if (ok) {
      ml.assign((size_t)max_id + 1, 0);
      mr.assign((size_t)max_id + 1, 0);
    }
    for (const auto& kv : ranks) {
      if (!ok) break;
      const uint32_t r = kv.second;
      if (r >= valid_new.size()) continue;  // panics when looked up: never merges
      const uint32_t a = (uint32_t)(kv.first >> 32), b = (uint32_t)kv.first;
      const uint32_t la = nchars(a, ok), lb = nchars(b, ok), lz = nchars(valid_new[r], ok);
      if (!ok || lz != la + lb || a > max_id || b > max_id) { ok = false; break; }
      ml[b] = std::max(ml[b], la);
      mr[a] = std::max(mr[a], lb);
    }
    t->window = ok;
    if (ok) {
      t->wmeta.resize((size_t)max_id + 1);
      for (size_t i = 0; i <= max_id; i++) t->wmeta[i] = std::min(ml[i], 0xFFFFu) | std::min(mr[i], 0xFFFFu) << 16;
    }
  }
  lap("window");

  // byte-pair table: the merge-table value of (byte2id[a], byte2id[b]) for every byte pair a, b
  // (the initial pairs of every piece are byte pairs), kNoRank where the pair has no merge
  t->pair0.assign(65536, kNoRank);
  for (uint32_t a = 0; a < 256; a++)
    for (uint32_t b = 0; b < 256; b++) {
      if (t->byte2id[a] < 0 || t->byte2id[b] < 0) continue;
      auto it = ranks.find(((uint64_t)(uint32_t)t->byte2id[a] << 32) | (uint32_t)t->byte2id[b]);
      if (it == ranks.end()) continue;
      const uint32_t r = it->second;
      t->pair0[a * 256 + b] = t->compact ? (r < valid_new.size() ? valid_new[r] : kPanicVal) : r;
    }

  lap("proper+pair0");
  // whole-piece table: every vocab entry of <= 8 raw bytes whose own BPE is that single token
  {
    std::vector<int> inv0(0x144, -1);  // mapped code point (< U+0144) -> byte
    for (int b = 0; b < 256; b++) inv0[bm[b]] = b;
    // the merge table probed as the kernels probe it: value = rank, or (compact) the new id,
    // both increasing in rank; kPanicVal / a rank past the valid merges would panic
    auto tab_value = [&](uint32_t a, uint32_t b) -> uint64_t {
      const uint64_t key = ((uint64_t)a << kIdBits) | b;
      for (uint32_t h = mhash(a, b) & t->merge_mask;; h = (h + 1) & t->merge_mask) {
        const uint64_t e = t->merge_tab[h];
        if (e == kEmpty) return UINT64_MAX;
        if ((e & ((1ull << 42) - 1)) == key) return e >> 42;
      }
    };
    const uint64_t n_valid = valid_new.size();
    auto panics = [&](uint64_t v) { return t->compact ? v == kPanicVal : v >= n_valid; };
    std::vector<std::pair<const std::string*, uint32_t>> items;
    items.reserve(t->vocab.size());
    for (const auto& kv : t->vocab) items.push_back({&kv.first, kv.second});
    // the reference merge loop (src/bpe.rs:88-153) on each entry's bytes, vocab split over threads
    const unsigned nth = std::min(16u, usable_cpus_once());
    std::vector<std::vector<std::pair<std::string, uint32_t>>> part(nth);
    auto work = [&](unsigned w) {
      std::vector<uint32_t> cps, tk;
      for (size_t i = w; i < items.size(); i += nth) {
        const std::string& key = *items[i].first;
        if (!decode_utf8(key, cps) || cps.empty() || cps.size() > 8) continue;
        std::string raw;
        bool ok = true;
        for (uint32_t c : cps) {
          if (c >= inv0.size() || inv0[c] < 0) { ok = false; break; }
          raw += (char)inv0[c];
        }
        if (!ok) continue;
        tk.clear();
        for (unsigned char c : raw) {
          if (t->byte2id[c] < 0) { ok = false; break; }
          tk.push_back((uint32_t)t->byte2id[c]);
        }
        if (!ok) continue;
        for (;;) {
          size_t bi = 0;
          uint64_t best = UINT64_MAX;
          for (size_t j = 0; j + 1 < tk.size(); j++) {
            const uint64_t v = tab_value(tk[j], tk[j + 1]);
            if (v == UINT64_MAX) continue;
            if (panics(v)) { ok = false; break; }  // would panic: leave to the kernels
            if (v < best) { best = v; bi = j; }
          }
          if (!ok || best == UINT64_MAX) break;
          tk[bi] = t->compact ? (uint32_t)best : valid_new[best];
          tk.erase(tk.begin() + bi + 1);
        }
        if (ok && tk.size() == 1 && tk[0] == items[i].second) part[w].push_back({raw, items[i].second});
      }
    };
    {
      std::vector<std::thread> th;
      for (unsigned w = 1; w < nth; w++) th.emplace_back(work, w);
      work(0);
      for (auto& x : th) x.join();
    }
    std::vector<std::pair<std::string, uint32_t>> ents;
    for (auto& p : part)
      for (auto& e : p) ents.push_back(std::move(e));
    // id order (BPE ids grow with merge order, roughly inverse frequency): frequent pieces are
    // inserted first and sit in their home slots -- k_segment's probes mostly end at the first
    // slot (C2 k_segment 0.42 -> 0.32 ms against the hash-map order used before)
    std::sort(ents.begin(), ents.end(), [](const auto& x, const auto& y) { return x.second < y.second; });
    size_t pcap = 1024;
    const size_t fp = getenv("CTOK_PIECE_SLACK") ? (size_t)atoi(getenv("CTOK_PIECE_SLACK")) : 8;  // A/B knob
    while (pcap < ents.size() * fp + 16) pcap <<= 1;  // load <= 1/8: misses end early (C2 k_segment -10%)
    t->piece_tab.assign((pcap + 1) * 4, 0);  // + one slot that stays empty (k_segment's no-probe lanes)
    t->piece_mask = (uint32_t)(pcap - 1);
    for (const auto& e : ents) {
      uint64_t v = 0;
      for (size_t i = 0; i < e.first.size(); i++) v |= (uint64_t)(uint8_t)e.first[i] << (8 * i);
      const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32), len = (uint32_t)e.first.size();
      uint32_t h = piece_hash(lo, hi, len) & t->piece_mask;
      while (t->piece_tab[4 * h + 2] != 0) h = (h + 1) & t->piece_mask;
      t->piece_tab[4 * h] = lo;
      t->piece_tab[4 * h + 1] = hi;
      t->piece_tab[4 * h + 2] = len;
      t->piece_tab[4 * h + 3] = e.second;
    }
    if (getenv("CTOK_NO_PIECE_TABLE")) std::fill(t->piece_tab.begin(), t->piece_tab.end(), 0u);
  }

  lap("piece_tab");
  // added tokens (mod.rs:103-116 schema, :274-305 maps)
  std::vector<std::pair<std::string, std::pair<uint32_t, uint8_t>>> added;  // content -> (id, flags)
  if (const ctj::Value* at = root.get("added_tokens")) {
    if (at->kind != ctj::Value::Array) throw_err(CTOK_E_PARSE, "invalid type for `added_tokens`, expected a sequence");
    for (const auto& a : at->arr) {
      if (a.kind != ctj::Value::Object) throw_err(CTOK_E_PARSE, "invalid type: expected struct AddedToken");
      const ctj::Value* id = a.get("id");
      const ctj::Value* content = a.get("content");
      const ctj::Value* special = a.get("special");
      if (!id) throw_err(CTOK_E_PARSE, "missing field `id`");
      if (!content) throw_err(CTOK_E_PARSE, "missing field `content`");
      if (!special) throw_err(CTOK_E_PARSE, "missing field `special`");
      if (!id->is_u32()) throw_err(CTOK_E_PARSE, "invalid type for added token `id`, expected u32");
      if (content->kind != ctj::Value::String) throw_err(CTOK_E_PARSE, "invalid type for added token `content`, expected a string");
      if (special->kind != ctj::Value::Bool) throw_err(CTOK_E_PARSE, "invalid type for added token `special`, expected a boolean");
      uint8_t flags = (get_bool_field(a, "single_word", false, "AddedToken") ? 1 : 0) |
                      (get_bool_field(a, "lstrip", false, "AddedToken") ? 2 : 0) |
                      (get_bool_field(a, "rstrip", false, "AddedToken") ? 4 : 0);
      (void)get_bool_field(a, "normalized", false, "AddedToken");
      bool replaced = false;
      for (auto& e : added)
        if (e.first == content->s) { e.second = {(uint32_t)id->u, flags}; replaced = true; }
      if (!replaced) added.push_back({content->s, {(uint32_t)id->u, flags}});
      if (special->b) {
        bool rep = false;
        for (auto& e : t->special)
          if (e.first == content->s) { e.second = (uint32_t)id->u; rep = true; }
        if (!rep) t->special.push_back({content->s, (uint32_t)id->u});
      }
    }
  }
  // added tokens that can match inside a byte-mapped word, as raw-byte patterns
  std::unordered_map<uint32_t, int> inv;  // mapped code point -> byte
  for (int b = 0; b < 256; b++) inv[bm[b]] = b;
  for (const auto& e : added) {
    if (e.first.empty()) throw_err(CTOK_E_UNSUPPORTED, "added token with empty content: the reference's word loop never terminates (src/huggingface/mod.rs:569-610)");
    std::vector<uint32_t> cps;
    if (!decode_utf8(e.first, cps)) continue;
    std::string raw;
    bool ok = true;
    for (uint32_t c : cps) {
      auto it = inv.find(c);
      if (it == inv.end()) { ok = false; break; }
      raw += (char)it->second;
    }
    if (!ok || !can_occur_in_piece(raw)) continue;  // provably never matches inside a piece
    t->at_bytes += raw;
    t->at_off.push_back((uint32_t)t->at_bytes.size());
    t->at_id.push_back(e.second.first);
    t->at_flags.push_back(e.second.second);
  }

  t->ids16 = t->narrow;
  for (uint32_t id : t->at_id) t->ids16 = t->ids16 && id < 0xFFFFu;
  t->nfc = parse_normalizer(root.get("normalizer")) != 0;
  std::vector<std::pair<char, bool>> chain;
  parse_pre_tokenizer(root.get("pre_tokenizer"), chain, 0);
  int nbl = 0;
  for (auto& c : chain)
    if (c.first == 'B') { nbl++; t->add_prefix_space = c.second; }
  if (nbl != 1) throw_err(CTOK_E_UNSUPPORTED, "pre_tokenizer must contain exactly one ByteLevel");

  // decoder (parsing.rs:272-364) and the per-id decode table
  parse_post_processor(t, root.get("post_processor"));
  t->decoder = parse_decoder(root.get("decoder"), t->decoder_name);
  build_decode_table(t);
  lap("rest");
}

template <typename T>
void upload(DevBuf<T>& b, const T* src, size_t n, hipStream_t s) {
  b.ensure(n ? n : 1);
  if (n) HIPTRY(hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, s));
}

// Tables::cp_fast: every code point of cp_range_class's ranges has the class it gives and no NFC
// flag in the generated tables (gen/unicode_data.h), so k_segment may skip their lookups.
bool cp_fast_ok() {
  static const bool ok = [] {
    if (getenv("CTOK_NO_CP_RANGES")) return false;
    for (uint32_t cp = 0x3000; cp < 0x1F700; cp++) {
      const int rc = cp_range_class(cp);
      if (rc < 0) continue;
      const int cl = (ct_cls_stage2[ct_cls_stage1[cp >> 8] * 64 + ((cp & 255) >> 2)] >> ((cp & 3) * 2)) & 3;
      if (cl != rc || ct_nfc_stage2[ct_nfc_stage1[cp >> 8] * 256 + (cp & 255)] != 0) return false;
    }
    return true;
  }();
  return ok;
}

DeviceState* device_state(ctok* t, int device) {
  std::lock_guard<std::mutex> lk(t->dev_mu);
  auto it = t->devs.find(device);
  if (it != t->devs.end()) return it->second.get();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw_err(CTOK_E_DEVICE, "no HIP device visible (the encode path has no CPU fallback)");
  if (device < 0 || device >= n) throw_err(CTOK_E_ARG, "device ordinal out of range");
  HIPTRY(hipSetDevice(device));
  auto ds = std::make_unique<DeviceState>();
  ds->device = device;
  HIPTRY(hipStreamCreateWithFlags(&ds->stream, hipStreamNonBlocking));
  {
    int cus = 0;
    HIPTRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    ds->n_cus = cus > 0 ? (uint32_t)cus : 1u;
  }
  for (auto& e : ds->ev) HIPTRY(hipEventCreate(&e));
  for (auto& e : ds->dev_ev) HIPTRY(hipEventCreate(&e));
  HIPTRY(hipEventCreateWithFlags(&ds->ev_sync, hipEventDisableTiming));
  HIPTRY(hipEventCreateWithFlags(&ds->ev_join, hipEventDisableTiming));
  HIPTRY(hipStreamCreateWithFlags(&ds->side, hipStreamNonBlocking));
  HIPTRY(hipEventCreateWithFlags(&ds->ev_tot, hipEventDisableTiming));
  // (coherent: the host polls words k_report writes while the call runs -- Work::report)
  HIPTRY(hipHostMalloc((void**)&ds->host, 4096, hipHostMallocCoherent));
  HIPTRY(hipHostGetDevicePointer((void**)&ds->host_dev, ds->host, 0));
  hipStream_t s = ds->stream;
  upload(ds->merge_tab, t->merge_tab.data(), t->merge_tab.size(), s);
  upload(ds->lds_image, t->lds_image.data(), t->lds_image.size(), s);
  if (t->narrow) {
    upload(ds->lds16_image, t->lds16_image.data(), t->lds16_image.size(), s);
    upload(ds->merge16, t->merge16.data(), t->merge16.size(), s);
  }
  upload(ds->pair0, t->pair0.data(), t->pair0.size(), s);
  upload(ds->rank_newid, t->rank_newid.data(), t->rank_newid.size(), s);
  upload(ds->eager, t->eager_bits.data(), t->eager_bits.size(), s);
  if (t->window) upload(ds->wmeta, t->wmeta.data(), t->wmeta.size(), s);
  upload(ds->piece_tab, t->piece_tab.data(), t->piece_tab.size(), s);
  upload(ds->byte2id, t->byte2id, 256, s);
  upload(ds->cls_s1, ct_cls_stage1, sizeof(ct_cls_stage1), s);
  upload(ds->cls_s2, ct_cls_stage2, sizeof(ct_cls_stage2), s);
  upload(ds->nfc_s1, ct_nfc_stage1, sizeof(ct_nfc_stage1), s);
  upload(ds->nfc_s2, ct_nfc_stage2, sizeof(ct_nfc_stage2) / 2, s);
  {  // the BMP's classes and NFC flags as one direct table: a nibble per code point
    static const std::vector<uint8_t> bmp = [] {
      std::vector<uint8_t> b(32768, 0);
      for (uint32_t cp = 0; cp < 0x10000; cp++) {
        const uint32_t cl = (ct_cls_stage2[ct_cls_stage1[cp >> 8] * 64 + ((cp & 255) >> 2)] >> ((cp & 3) * 2)) & 3;
        const uint32_t nf = ct_nfc_stage2[ct_nfc_stage1[cp >> 8] * 256 + (cp & 255)] != 0 ? 4u : 0u;
        b[cp >> 1] |= (uint8_t)((cl | nf) << ((cp & 1) * 4));
      }
      return b;
    }();
    upload(ds->cls_bmp, bmp.data(), bmp.size(), s);
  }
  upload(ds->decomp_cp, ct_decomp_cp, CT_DECOMP_N, s);
  upload(ds->decomp_off, ct_decomp_off, CT_DECOMP_N + 1, s);
  upload(ds->decomp_data, ct_decomp_data, CT_DECOMP_DATA_N, s);
  upload(ds->comp_key, (const uint64_t*)ct_comp_key, CT_COMP_N, s);
  upload(ds->comp_val, ct_comp_val, CT_COMP_N, s);
  upload(ds->alnum, ct_bytemap_alnum, 256, s);
  upload(ds->at_bytes, (const uint8_t*)t->at_bytes.data(), t->at_bytes.size(), s);
  upload(ds->at_off, t->at_off.data(), t->at_off.size(), s);
  upload(ds->at_id, t->at_id.data(), t->at_id.size(), s);
  upload(ds->at_flags, t->at_flags.data(), t->at_flags.size(), s);
  HIPTRY(hipStreamSynchronize(s));
  Tables& tb = ds->t;
  tb.merge_tab = ds->merge_tab.p;
  tb.merge_mask = t->merge_mask;
  tb.lds_image = (const uint4*)ds->lds_image.p;
  tb.pair0 = ds->pair0.p;
  tb.lds16_image = (const uint4*)ds->lds16_image.p;
  tb.merge16 = ds->merge16.p;
  tb.merge16_mask = t->merge16_mask;
  tb.piece_tab = (const uint4*)ds->piece_tab.p;
  tb.piece_mask = t->piece_mask;
  tb.rank_newid = ds->rank_newid.p;
  tb.eager = ds->eager.p;
  tb.wmeta = ds->wmeta.p;
  tb.window = t->window ? 1 : 0;
  tb.n_ranks = (uint32_t)t->rank_newid.size();
  tb.byte2id = ds->byte2id.p;
  tb.cls_s1 = ds->cls_s1.p;
  tb.cls_s2 = ds->cls_s2.p;
  tb.nfc_s1 = ds->nfc_s1.p;
  tb.nfc_s2 = ds->nfc_s2.p;
  tb.cls_bmp = ds->cls_bmp.p;
  tb.cp_fast = cp_fast_ok() ? 1u : 0u;
  tb.decomp_cp = ds->decomp_cp.p;
  tb.decomp_off = ds->decomp_off.p;
  tb.decomp_data = ds->decomp_data.p;
  tb.n_decomp = CT_DECOMP_N;
  tb.comp_key = ds->comp_key.p;
  tb.comp_val = ds->comp_val.p;
  tb.n_comp = CT_COMP_N;
  tb.bytemap_alnum = ds->alnum.p;
  tb.at_bytes = ds->at_bytes.p;
  tb.at_off = ds->at_off.p;
  tb.at_id = ds->at_id.p;
  tb.at_flags = ds->at_flags.p;
  tb.n_at = (uint32_t)t->at_id.size();
  tb.proper = (t->proper && !getenv("CTOK_FORCE_IMPROPER")) ? 1 : 0;
  tb.compact = t->compact ? 1 : 0;
  tb.narrow = (t->narrow && !getenv("CTOK_FORCE_WIDE_SLOTS")) ? 1 : 0;
  tb.all_bytes = std::all_of(t->byte2id, t->byte2id + 256, [](int32_t v) { return v >= 0; }) ? 1 : 0;
  tb.dbg = getenv("CTOK_DBG_MODE") ? (uint32_t)atoi(getenv("CTOK_DBG_MODE")) : 0;
  DeviceState* r = ds.get();
  t->devs[device] = std::move(ds);
  return r;
}

bool debug_sync() {
  static int v = -1;
  if (v < 0) v = getenv("CTOK_DEBUG_SYNC") ? 1 : 0;
  return v == 1;
}

#define STEP(name, x)                                                                    \
  do {                                                                                   \
    HIPTRY(x);                                                                           \
    if (debug_sync()) {                                                                  \
      fprintf(stderr, "[ctok] %s launched\n", name);                                     \
      HIPTRY(hipStreamSynchronize(s));                                                   \
      fprintf(stderr, "[ctok] %s done\n", name);                                         \
    }                                                                                    \
  } while (0)

// Wait for all work on s by spinning on an event: a blocking stream synchronise can add
// hundreds of microseconds of wake-up latency per call on this path's few sync points.
// (idle: called between polls -- the timed calls read their event pairs there, see Laps)
template <class Idle>
void spin_sync(DeviceState* ds, hipStream_t s, Idle idle) {
  HIPTRY(hipEventRecord(ds->ev_sync, s));
  for (;;) {
    hipError_t e = hipEventQuery(ds->ev_sync);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) throw_err(CTOK_E_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(e));
    idle();
  }
}
void spin_sync(DeviceState* ds, hipStream_t s) {
  spin_sync(ds, s, [] {});
}

// The elapsed times of a timed call's event pairs, each read as soon as its later event has
// completed, while the host waits for the rest of the call: a read costs a few microseconds, and
// the ten of an encode call, read after its final wait, added ~40 us to every timed call
// (C4S8 1.20 -> 1.16 ms untimed, profiles/r06).
struct Laps {
  struct Lap {
    hipEvent_t a, b;
    double v;
    bool done;
  };
  Lap l[12];
  int n = 0;
  int add(hipEvent_t a, hipEvent_t b) {
    l[n] = {a, b, 0.0, false};
    return n++;
  }
  void read(Lap& p) {
    float v = 0;
    HIPTRY(hipEventElapsedTime(&v, p.a, p.b));
    p.v = v;
    p.done = true;
  }
  void poll() {  // reads the first pair whose events have both completed, if any
    for (int k = 0; k < n; k++) {
      if (l[k].done) continue;
      // (both: the events can be on two streams, the "later" one done first)
      if (!done(l[k].b) || !done(l[k].a)) continue;
      read(l[k]);
      return;
    }
  }
  static bool done(hipEvent_t ev) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipErrorNotReady) return false;
    if (e != hipSuccess) throw_err(CTOK_E_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(e));
    return true;
  }
  void finish() {
    for (int k = 0; k < n; k++)
      if (!l[k].done) read(l[k]);
  }
  double operator[](int k) const { return k < 0 ? 0.0 : l[k].v; }  // (-1: a pair not timed)
};

// Waits for k_report's report of this call (Work::report: the counters, then the sequence number);
// a device error, or the stream running dry without it, ends the wait
void wait_report(hipStream_t s, volatile uint32_t* rep, uint32_t seq) {
  for (uint32_t i = 1;; i++) {
    if (rep[kNumCounters] == seq) return;
    if ((i & 4095) == 0) {
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess && rep[kNumCounters] != seq) throw_err(CTOK_E_DEVICE, "k_report: the call's report never came");
      if (e != hipSuccess && e != hipErrorNotReady)
        throw_err(CTOK_E_DEVICE, std::string("hipStreamQuery: ") + hipGetErrorString(e));
    }
  }
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

uint64_t encode_device(ctok* t, DeviceState* ds, const uint8_t* d_text, const uint64_t* d_off, uint64_t n_docs,
                       uint64_t n_bytes, uint32_t* d_ids, uint64_t ids_cap, uint64_t* d_tok_off, hipStream_t s,
                       bool timing, ctok_stats* st, bool split_added = true, bool segment_only = false,
                       bool keep_first = false, bool all_nfc = false);

// NFC splice: the speculative pass over the raw text finished but flagged a code point NFC may
// change (src/normalizers.rs:45-47 normalises every document).  Only the documents holding such
// code points (k_nfc_check's flags, a superset of those NFC changes) are gathered into a
// sub-batch, encoded normalised, and their ids replace the pass's in d_ids / d_tok_off; the
// others' ids are already right (NFC leaves them unchanged, and pieces never cross documents).
// Returns the token count; *n_flagged = the flagged documents.
uint64_t nfc_splice(ctok* t, DeviceState* ds, const uint8_t* d_text, const uint64_t* d_off, uint64_t n_docs,
                    uint64_t n_bytes, uint32_t* d_ids, uint64_t ids_cap, uint64_t* d_tok_off, uint64_t ntok_main,
                    hipStream_t s, uint64_t* n_flagged, bool split_added) {
  (void)n_bytes;
  ds->doc_flag.ensure(n_docs + 1);
  HIPTRY(launch_flag_docs(d_off, n_docs, ds->nfc_bits.p, ds->doc_flag.p, s));
  // ranks of the flagged docs, their places in the sub-batch
  ds->spl_rank.ensure(n_docs + 1);
  ds->spl_pos.ensure(n_docs + 1);
  ds->scan_tmp.ensure(scan_tmp_elems(n_docs + 1) + 64);
  HIPTRY(scan_u32(ds->doc_flag.p, ds->spl_rank.p, n_docs, nullptr, (uint32_t*)ds->scan_tmp.p, ds->scan_tmp.cap * 2, s));
  HIPTRY(launch_flag_len(d_off, ds->doc_flag.p, n_docs, ds->spl_pos.p, s));
  HIPTRY(scan_u64(ds->spl_pos.p, n_docs, ds->scan_tmp.p, ds->scan_tmp.cap, s));
  volatile uint64_t* h = (volatile uint64_t*)(ds->host + 100);
  HIPTRY(hipMemcpyAsync((void*)h, ds->spl_pos.p + n_docs, 8, hipMemcpyDeviceToHost, s));
  HIPTRY(hipMemcpyAsync((void*)(h + 1), ds->spl_rank.p + n_docs, 4, hipMemcpyDeviceToHost, s));
  spin_sync(ds, s);
  const uint64_t SB = h[0], F = (uint32_t)h[1];
  *n_flagged = F;
  if (F == 0) return ntok_main;
  // the flagged docs' raw text as a sub-batch (16-byte aligned, zero padded)
  ds->sub_text.ensure(SB + 16);
  ds->sub_off.ensure(F + 1);
  HIPTRY(launch_gather_flagged(d_text, d_off, ds->spl_rank.p, ds->spl_pos.p, n_docs, ds->sub_text.p, ds->sub_off.p, s));
  HIPTRY(hipMemcpyAsync(ds->sub_off.p + F, ds->spl_pos.p + n_docs, 8, hipMemcpyDeviceToDevice, s));
  HIPTRY(hipMemsetAsync(ds->sub_text.p + SB, 0, 16, s));
  // the pass's output, read by the splice
  ds->spl_ids.ensure(ntok_main + 1);
  ds->spl_toff.ensure(n_docs + 1);
  if (ntok_main) HIPTRY(hipMemcpyAsync(ds->spl_ids.p, d_ids, ntok_main * 4, hipMemcpyDeviceToDevice, s));
  HIPTRY(hipMemcpyAsync(ds->spl_toff.p, d_tok_off, (n_docs + 1) * 8, hipMemcpyDeviceToDevice, s));
  // the sub-batch: NFC check + normalise + encode (no speculation: every doc in it is flagged),
  // with the outer call's added-token rule (encode_to_encoding's words skip the split,
  // src/huggingface/mod.rs:395-420)
  ds->sub_ids.ensure(ctok_ids_bound(t, SB, F));
  ds->sub_toff.ensure(F + 1);
  encode_device(t, ds, ds->sub_text.p, ds->sub_off.p, F, SB, ds->sub_ids.p, ds->sub_ids.cap, ds->sub_toff.p, s, false,
                nullptr, split_added, false, false, true);  // (all_nfc: every doc of the sub-batch is normalised)
  ds->scan_tmp.ensure(scan_tmp_elems(n_docs + 1) + 64);
  HIPTRY(launch_splice(ds->spl_rank.p, ds->spl_toff.p, ds->spl_ids.p, ds->sub_toff.p, ds->sub_ids.p, n_docs, d_ids,
                       ids_cap, d_tok_off, ds->scan_tmp.p, ds->scan_tmp.cap, s));
  HIPTRY(hipMemcpyAsync((void*)h, d_tok_off + n_docs, 8, hipMemcpyDeviceToHost, s));
  spin_sync(ds, s);
  return h[0];
}

// The pipeline on device-resident buffers.  Returns the token count.
uint64_t encode_device(ctok* t, DeviceState* ds, const uint8_t* d_text, const uint64_t* d_off, uint64_t n_docs,
                       uint64_t n_bytes, uint32_t* d_ids, uint64_t ids_cap, uint64_t* d_tok_off, hipStream_t s,
                       bool timing, ctok_stats* st, bool split_added, bool segment_only, bool keep_first, bool all_nfc) {
  if (n_bytes >= 0xF0000000ull) throw_err(CTOK_E_ARG, "a single call is limited to < 3.75 GiB of text; split the batch");
  if (n_docs >= 0xF0000000ull) throw_err(CTOK_E_ARG, "too many documents in one call");
  // split_added = false: encode_to_encoding's words go straight to BpeTokenizer::encode, with
  // no added-token split (src/huggingface/mod.rs:395-420)
  Tables tb_call = ds->t;
  if (!split_added) tb_call.n_at = 0;
  const Tables& tb = tb_call;
  // NFC speculation: when NFC is the only normalisation, run the pipeline on the raw text and
  // let k_segment flag any code point that NFC might change (NFC_QC != Yes or a non-zero
  // combining class; ASCII never is).  Only a flagged batch pays for the check + normalise
  // passes and a second run.
  // all_nfc (nfc_splice's sub-batch of flagged docs): no speculation and no check, every doc is
  // normalised
  bool speculate = t->nfc && !t->add_prefix_space && n_bytes && !all_nfc && !getenv("CTOK_NO_NFC_SPECULATION");
  // a flagged pass is finished and only its flagged docs are encoded again (nfc_splice), except
  // where the whole batch's pass state is read afterwards (offsets, the trainer's pre-tokenizer)
  const bool splice = d_ids && !keep_first && !segment_only && !getenv("CTOK_NFC_RERUN");
  // lean list capacities first; a call whose lists outgrow them runs again with the safe ones
  static const bool always_safe = getenv("CTOK_SAFE_CAPACITIES") != nullptr;
  bool safe = always_safe;
  // diagnostic (CTOK_HOSTPROF=1): host time at points of the call, printed at its end
  static const bool hostprof = getenv("CTOK_HOSTPROF") != nullptr;
  double hp[10] = {};
#define HP(i) \
  if (hostprof) hp[i] = now_ms()
  HP(0);
  for (;;) {
  // (timing: ev[0] is k_clear's start event, or a marker here when normalising work comes first)
  const bool ev0_marker = timing && (t->add_prefix_space || (t->nfc && n_bytes && (all_nfc || !speculate)));
  if (ev0_marker) HIPTRY(hipEventRecord(ds->ev[0], s));

  ds->counters.ensure(kCounterWords);
  bool ctr_zeroed = false;  // (else launch_docstart zeroes them, in the bitmap's clearing launch)
  const uint8_t* text = d_text;
  const uint64_t* off = d_off;
  uint64_t B = n_bytes;
  uint64_t nfc_docs = 0;
  bool norm = t->add_prefix_space;
  if (t->nfc && n_bytes && all_nfc) {
    ds->doc_flag.ensure(n_docs + 1);
    HIPTRY(hipMemsetD32Async((hipDeviceptr_t)ds->doc_flag.p, 1, n_docs + 1, s));
    nfc_docs = n_docs;
    norm = true;
  } else if (t->nfc && n_bytes && !speculate) {
    ds->doc_flag.ensure(n_docs + 1);
    HIPTRY(hipMemsetAsync(ds->doc_flag.p, 0, (n_docs + 1) * 4, s));
    HIPTRY(hipMemsetAsync(ds->counters.p, 0, kCounterWords * 4, s));
    ctr_zeroed = true;
    STEP("nfc_check", launch_nfc_check(d_text, n_bytes, d_off, (uint32_t)n_docs, tb, ds->doc_flag.p, ds->counters.p + 3, s));
    HIPTRY(hipMemcpyAsync(ds->host, ds->counters.p + 3, 4, hipMemcpyDeviceToHost, s));
    spin_sync(ds, s);
    const uint32_t cnt = *(volatile uint32_t*)ds->host;
    nfc_docs = cnt;
    if (cnt) norm = true;
  }
  if (norm) {
    ds->doc_flag.ensure(n_docs + 1);
    if (!t->nfc) HIPTRY(hipMemsetAsync(ds->doc_flag.p, 0, (n_docs + 1) * 4, s));
    ds->ncp.ensure(n_docs + 1);
    ds->norm_off.ensure(n_docs + 2);
    ds->cps.ensure(4 * n_bytes + 64);
    STEP("norm0", launch_norm(d_text, d_off, (uint32_t)n_docs, ds->doc_flag.p, t->add_prefix_space, t->nfc && nfc_docs, tb,
                       ds->cps.p, ds->ncp.p, ds->norm_off.p, nullptr, 0, s));
    ds->scan_tmp.ensure(scan_tmp_elems(n_docs + 1) + 64);
    HIPTRY(scan_u64(ds->norm_off.p, n_docs, ds->scan_tmp.p, ds->scan_tmp.cap, s));
    HIPTRY(hipMemcpyAsync(ds->host, ds->norm_off.p + n_docs, 8, hipMemcpyDeviceToHost, s));
    spin_sync(ds, s);
    const uint64_t nb = *(volatile uint64_t*)ds->host;
    if (nb >= 0xF0000000ull) throw_err(CTOK_E_ARG, "normalised batch exceeds 3.75 GiB; split the batch");
    ds->norm_text.ensure(nb + 16);
    STEP("norm1", launch_norm(d_text, d_off, (uint32_t)n_docs, ds->doc_flag.p, t->add_prefix_space, t->nfc && nfc_docs, tb,
                       ds->cps.p, ds->ncp.p, ds->norm_off.p, ds->norm_text.p, 1, s));
    text = ds->norm_text.p;
    off = ds->norm_off.p;
    B = nb;
  }
  if (B > 0 && ((uintptr_t)text & 15)) throw_err(CTOK_E_ARG, "device text buffer must be 16-byte aligned");
  ds->last_norm = norm;
  ds->last_B = B;

  Work w{};
  w.text = text;
  w.n_bytes = (uint32_t)B;
  w.doc_off = off;
  w.n_docs = (uint32_t)n_docs;
  w.n_words = (uint32_t)((B + 31) / 32);
  w.n_tiles = (uint32_t)((B + kTile - 1) / kTile);
  w.n_cus = ds->n_cus;
  w.nfc_watch = speculate ? (splice ? 2u : 1u) : 0u;
  if (w.nfc_watch == 2) {
    ds->nfc_bits.ensure(nfc_bits_words(B));  // (zeroed by launch_docstart)
    w.nfc_bits = ds->nfc_bits.p;
  }
  w.keep_first = keep_first ? 1u : 0u;
  {
    const char* v = getenv("CTOK_SHORT_WGS");
    w.short_wgs = v ? (uint32_t)atoi(v) : 0u;
  }
  const size_t nt = w.n_tiles;
  ds->tfirst.ensure(nt + 8);
  ds->pbits.ensure(w.n_words + 8);
  ds->wpref.ensure(nt * 64 + 8);
  ds->tile_np.ensure(nt + 8);
  ds->tile_tok.ensure(nt + 8);
  ds->tile_doc.ensure(nt + 8);
  // Workspace sized from what the call needs (ctok_stats.workspace_bytes): the class-0 lists lean
  // (kCap0Lean per tile, the rest of a tile's class-0 pieces spill to the long list), the
  // dropped-byte list small (it only fills when the vocab lacks some byte chars), the long pieces'
  // ids and global-memory state sized from launch_long_prep's totals (none without long pieces).
  // A list that outgrows its lean capacity sets counters[kCtrOverflow]: the call runs again with
  // the safe capacities (every class-0 piece listed, a dropped-byte entry per byte).
  w.k0 = safe ? kCap0 : kCap0Lean;
  // merge-pass work units: 64 tiles, or 16 for batches under 8192 tiles (32 MB), which 64-tile
  // units spread over too few CUs (3.8 MB: 0.41 -> 0.30 ms per call; from 16 MB up 64 is faster,
  // profiles/r03/v16_ab_unit.txt)
  static const uint32_t unit_env = getenv("CTOK_UNIT") ? (uint32_t)atoi(getenv("CTOK_UNIT")) : 0u;
  w.unit = unit_env == 8 || unit_env == 16 || unit_env == 32 || unit_env == 64 ? unit_env
           : nt >= 8192                                                        ? 64u
                                                                               : 16u;
  w.long_cap = (uint32_t)(B / kShortMax + nt + 8);
  w.mid_cap = (uint32_t)(safe ? B + 8 : std::min<uint64_t>(B + 8, std::max<uint64_t>(65536, B / 256)));
  ds->tcls.ensure(kNumClasses * nt + 8);
  ds->list0.ensure(nt * w.k0 + 8);
  ds->rend.ensure(kNumClasses * nt + 8);
  if (tb.n_at == 0) {
    ds->list1.ensure(nt * kCap1 + 8);
    ds->list2.ensure(nt * kCap2 + 8);
    ds->list3.ensure(nt * kCap3 + 8);
  }
  ds->tcnt.ensure(nt * kTileSlots + 8);
  // piece records: u16 when every id a whole-piece probe can return is below 0xFFFF
  static const bool rec32_env = getenv("CTOK_REC32") != nullptr;
  w.rec16 = (t->narrow && !rec32_env) ? 1u : 0u;
  ds->prec.ensure(nt * kTileSlots * (w.rec16 ? 1 : 2) + 16);
  ds->mrec.ensure(nt * kTileSlots + 8);
  ds->pdoc.ensure(nt * (kTileSlots / 32) + 8);
  ds->scratch.ensure(nt * kTileSlots + 8);  // per tile: the class regions of the register passes
  ds->tregion.ensure(nt + 8);
  ds->long_list.ensure(w.long_cap + 8);
  ds->long_cnt.ensure(w.long_cap + 8);
  ds->long_ord.ensure(w.long_cap + 8);
  ds->long_hist.ensure(kLhWords);
  ds->mid_list.ensure(w.mid_cap + 8);
  ds->scan_tmp.ensure(std::max(scan_tmp_elems(std::max<uint64_t>(nt + 1, n_docs + 1)), tile_scan_tmp_elems(nt)) + 64);
  w.tfirst = ds->tfirst.p;
  w.pbits = ds->pbits.p;
  w.wpref = ds->wpref.p;
  w.tile_np = ds->tile_np.p;
  w.tile_tok = ds->tile_tok.p;
  w.tile_doc = ds->tile_doc.p;
  w.tcls = ds->tcls.p;
  w.list0 = ds->list0.p;
  w.list1 = ds->list1.p;
  w.list2 = ds->list2.p;
  w.list3 = ds->list3.p;
  w.long_cnt = ds->long_cnt.p;
  w.long_ord = ds->long_ord.p;
  w.long_hist = ds->long_hist.p;
  w.tcnt = ds->tcnt.p;
  w.prec = ds->prec.p;
  w.mrec = ds->mrec.p;
  w.pdoc = ds->pdoc.p;
  w.scratch = ds->scratch.p;
  w.rend = ds->rend.p;
  w.tregion = (uint2*)ds->tregion.p;
  w.long_list = ds->long_list.p;
  w.mid_list = ds->mid_list.p;
  w.counters = ds->counters.p;
  w.scan_tmp = (uint32_t*)ds->scan_tmp.p;
  w.scan_tmp_cap = ds->scan_tmp.cap * 2;
  // sparse class 3 (k_bpe_sparse): at most c3_limit pieces of 33..64 B are merged a wavefront
  // each instead of by the register pass -- by default the class is sparse at <= 1 piece per 16
  // tiles (English text: C4 ~600 in 322k tiles; C5-NFC's sub-batch of CJK-heavy documents, ~17
  // per tile, is faster in the register pass), up to kC3SparseDefault; CTOK_C3_SPARSE=n sets the
  // bound (0 disables), read per call (the GPU tests switch it within one process).  k_segment
  // queues the pieces in c3q's 64 shards (shard = tile % 64): capacity the bound rounded up to
  // whole shards, at most what a shard's tiles can hold (kCap3 each) -- a bound that large never
  // overflows; a smaller one overflows when the pieces crowd into a few tiles, and the call then
  // takes the register pass (locally dense: the faster one there).
  const char* c3_var = getenv("CTOK_C3_SPARSE");
  const uint64_t c3_limit = tb.n_at != 0 ? 0ull
                            : c3_var     ? strtoull(c3_var, nullptr, 10)
                                         : std::min<uint64_t>(kC3SparseDefault, std::max<uint64_t>(64, nt / 16));
  const uint64_t c3_most = (uint64_t)kCap3 * ((nt + kC3Shards - 1) / kC3Shards) * kC3Shards;
  w.c3_max = c3_limit ? (uint32_t)std::min<uint64_t>((c3_limit + kC3Shards - 1) / kC3Shards * kC3Shards, c3_most) : 0u;
  if (w.c3_max) {
    ds->c3q.ensure(w.c3_max + 8);
    ds->c3pre.ensure(kC3Shards + 8);
    w.c3q = ds->c3q.p;
    w.c3pre = ds->c3pre.p;
  }
#ifdef CTOK_CHECK
  // (range-checking build: every merged record starts out of range, so one no pass wrote traps)
  HIPTRY(hipMemsetAsync(ds->mrec.p, 0xFF, (size_t)nt * kTileSlots * 4, s));
#endif
  static const bool wgrec_on = getenv("CTOK_WGREC") != nullptr;
  if (wgrec_on) {  // diagnostic: per-workgroup records of the merge passes (kernels.hip WgRec)
    ds->wgrec.ensure(kWgRecWords);
    HIPTRY(hipMemsetAsync(ds->wgrec.p, 0, kWgRecWords * 8, s));
    w.wgrec = ds->wgrec.p;
  }
  static const bool stamps_on = getenv("CTOK_STAMPS") != nullptr;
  if (stamps_on && nt) {  // (k_segment writes them only in a -DCTOK_SEG_STAMPS build)
    ds->stamps.ensure(nt * 8 + 8);
    HIPTRY(hipMemsetAsync(ds->stamps.p, 0, nt * 8 * 8, s));
    w.stamps = ds->stamps.p;
  }

  // Streams and ordering.  The main stream s runs k_clear, k_tilefirst, k_segment, k_bpe_short,
  // whose first wave writes the report the host polls (k_segment's counters, the class-3 count
  // among them, into pinned host words, then the call's sequence number; k_report does it when
  // k_bpe_short does not run).  Having seen it, the host knows k_segment has completed, so it
  // launches what reads k_segment's output on the side stream with no fork event: the 17..32 B
  // pass when the call has no long pieces (its workgroups take the CUs k_bpe_short's free at its
  // end, beside the 33..64 B pass -- register or sparse -- on the main stream), else the
  // long-piece preparation and tiers; one join before the tail (dropped-byte pass, tile scan,
  // k_emit, k_tokoff).  The round-5 flow forked the side stream with an event after k_segment
  // (the counter copy and, in round 6's first build, the class-3 list there), and the sparse pass
  // waited for the list's event: ~3 us per event marker on the main stream and ~10 us per
  // cross-stream wait (tools/queue_gaps.hip, profiles/r06).  Any-order packets
  // (hipExtAnyOrderLaunch) do not help here: one starts when the previous kernel's first
  // workgroup retires, and k_bpe_short's persistent workgroups retire together at its end
  // (tools/anyorder_check.hip).
  // Timing (stats): events recorded by the kernels' own dispatches (Lx), no marker packets, and
  // none on the launches the device waits for at the call's start (an event costs the host ~3 us
  // per launch there; later launches run ahead of the device): 0 k_clear start (a marker when
  //   normalising work precedes it) | 7 k_tilefirst end | 1 k_segment end | 2 k_bpe_short end |
  //   8, 10 the 17..32 B pass | 9 the 33..64 B pass's end | 5 the dropped-byte pass start | 3 the
  //   tile scan start | 6 k_tokoff end
  const bool tm = timing && st && nt;  // (no tiles: no merge pass to time)
  auto lx = [&](int a, int b) {
    Lx x;
    if (tm && a >= 0) x.start = ds->ev[a];
    if (tm && b >= 0) x.stop = ds->ev[b];
    return x;
  };
  HP(1);
  STEP("docstart", launch_docstart(w, s, !ctr_zeroed, lx(ev0_marker ? -1 : 0, -1), lx(-1, 7)));
  STEP("segment", launch_segment(w, tb, s, lx(-1, 1)));
  if (segment_only) {  // pre-tokenization only (the trainer's word counting): pbits of the text
    HIPTRY(hipMemcpyAsync(ds->host + 1, ds->counters.p, kNumCounters * 4, hipMemcpyDeviceToHost, s));
    spin_sync(ds, s);
    if (speculate && ((volatile uint32_t*)(ds->host + 1))[12]) {
      speculate = false;
      continue;
    }
    return 0;
  }
  if (++ds->seq == 0) ds->seq = 1;
  w.seq = ds->seq;
  w.report = (uint32_t*)(ds->host_dev + 64);
  volatile uint32_t* seg_cnt = (volatile uint32_t*)(ds->host + 64);
  // (k_bpe_short's first wave writes the report; without it -- added tokens, no tiles -- k_report)
  HP(2);
  if (tb.n_at != 0 || !nt) STEP("report", launch_report(w, s));
  STEP("bpe_short", launch_bpe_class(w, tb, 0, s, lx(-1, 2)));
  HP(3);
  wait_report(s, seg_cnt, w.seq);
  HP(4);
  // the 17..32 B pass takes 768 threads per workgroup when there are no long pieces
  w.mid_wide = (seg_cnt[0] == 0 && !getenv("CTOK_MID512")) ? 1u : 0u;
  // long pieces: their lengths, order and places first (side stream, before the host waits for
  // anything else: the long tiers after them are the side stream's critical path on C5 / C3);
  // lids / lw are sized from the totals read back below, once the merge passes are launched
  const bool spec_fail1 = w.nfc_watch == 1 && seg_cnt[12];  // (a failed NFC speculation: nothing to launch)
  const uint32_t n_long = spec_fail1 ? 0u : std::min<uint32_t>((uint32_t)seg_cnt[0], w.long_cap);
  volatile uint32_t* tot = (volatile uint32_t*)(ds->host + 96);
  if (n_long) {
    ds->long_pos.ensure(n_long + 8);
    ds->lw_pos.ensure(n_long + 8);
    ds->lwn.ensure(n_long + 8);
    ds->scan_tmp2.ensure(scan_tmp_elems(n_long + 1) + 64);
    w.long_pos = ds->long_pos.p;
    w.lw_pos = ds->lw_pos.p;
    STEP("long_prep", launch_long_prep(w, tb, ds->side, n_long, ds->lwn.p, (uint32_t*)ds->scan_tmp2.p,
                                       ds->scan_tmp2.cap * 2));
    HIPTRY(hipMemcpyAsync((void*)tot, ds->long_pos.p + n_long, 4, hipMemcpyDeviceToHost, ds->side));
    HIPTRY(hipMemcpyAsync((void*)(tot + 1), ds->lw_pos.p + n_long, 4, hipMemcpyDeviceToHost, ds->side));
    HIPTRY(hipEventRecord(ds->ev_tot, ds->side));
  }
  const uint32_t c3n = seg_cnt[kCtrC3Count];
  const bool c3_sparse = c3n != 0 && c3n <= c3_limit && c3n <= w.c3_max;  // (all ones: a shard overflowed)
  // Without long pieces the side stream is idle: the 17..32 B pass goes there (CTOK_OVERLAP=0: on
  // the main stream after k_bpe_short), so its workgroups take the CUs k_bpe_short's free at its
  // end, beside the 33..64 B pass on the main stream (the classes' pieces, regions and records are
  // disjoint); no fork event -- the report orders it after k_segment --, one join before the tail
  const char* ov_var = getenv("CTOK_OVERLAP");
  const int overlap = ov_var ? atoi(ov_var) : kOverlapDefault;
  const bool mid_side = overlap >= 1 && seg_cnt[0] == 0;
  ds->last_mid_side = mid_side;
  STEP("bpe_mid", launch_bpe_class(w, tb, 2, mid_side ? ds->side : s, lx(8, 10)));
  if (c3_sparse) STEP("bpe_c3_sparse", launch_c3_sparse(w, tb, c3n, s, lx(-1, 9)));
  else STEP("bpe_c3", launch_bpe_class(w, tb, 4, s, lx(-1, 9)));
  if (!spec_fail1 && n_long) {
    for (;;) {  // the long pieces' totals (launch_long_prep above)
      const hipError_t e = hipEventQuery(ds->ev_tot);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) throw_err(CTOK_E_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(e));
    }
    const bool any_gmem = tot[1] != 0;  // a long piece for the global-memory tier (its state words reserved)
    ds->lids.ensure((uint64_t)tot[0] + 64);
    ds->lw.ensure(4 * (uint64_t)tot[1] + 64);
    w.lids = ds->lids.p;
    w.lw = ds->lw.p;
    STEP("bpe_long", launch_bpe_long(w, tb, ds->side, n_long, seg_cnt[kCtrAnyC3] != 0 && !c3_sparse, any_gmem));
  }
  if (n_long || mid_side) {
    HIPTRY(hipEventRecord(ds->ev_join, ds->side));
    HIPTRY(hipStreamWaitEvent(s, ds->ev_join, 0));
  }
  const bool dropped_pass = tb.n_at == 0 && !tb.all_bytes;
  STEP("bpe_dropped", launch_bpe_class(w, tb, 3, s, lx(5, -1)));
  // the token count and the counters: written by k_tokoff straight into the pinned host words
  // (two copy launches fewer at the end of every call), or copied
  static const bool copy_res = getenv("CTOK_COPY_RESULTS") != nullptr;
  w.host_res = copy_res ? nullptr : ds->host_dev;
  STEP("emit", launch_emit(w, d_ids, ids_cap, d_tok_off, s, st != nullptr, seg_cnt[kCtrEmptyDocs] != 0,
                           lx(3, -1), lx(-1, 6)));
  if (!w.host_res) {
    HIPTRY(hipMemcpyAsync(ds->host, d_tok_off + n_docs, 8, hipMemcpyDeviceToHost, s));
    HIPTRY(hipMemcpyAsync(ds->host + 1, ds->counters.p, kNumCounters * 4, hipMemcpyDeviceToHost, s));
  }
  Laps laps;
  int lap[11];
  if (tm) {
    hipEvent_t* e = ds->ev;
    const bool passes = tb.n_at == 0;  // (with added tokens one kernel merges every <= 32 B piece)
    lap[0] = laps.add(e[0], e[1]);  // pretok
    lap[1] = laps.add(e[7], e[1]);  // segment (from k_tilefirst's end)
    lap[2] = laps.add(e[1], e[2]);  // <= 16 B pass (from k_segment's end)
    // class 2; on the side stream its events span the wait for k_bpe_short's CUs, so the time it
    // adds after k_bpe_short's end is reported
    lap[3] = !passes ? -1 : mid_side ? laps.add(e[2], e[10]) : laps.add(e[8], e[10]);
    lap[4] = passes ? laps.add(e[2], e[9]) : -1;  // class 3 (register or sparse pass; after k_bpe_short)
    lap[5] = laps.add(e[1], e[2]);  // k_segment's end to the merge passes' ends
    lap[6] = passes ? laps.add(e[1], e[10]) : -1;
    lap[7] = passes ? laps.add(e[1], e[9]) : -1;
    lap[8] = laps.add(e[1], e[dropped_pass ? 5 : 3]);  // ... to the tail's start
    lap[9] = laps.add(e[3], e[6]);  // tile scan + emit
    lap[10] = laps.add(e[0], e[6]);  // device
  }
  HP(5);
  spin_sync(ds, s, [&] { laps.poll(); });
  HP(6);
  laps.finish();
  HP(7);
  uint64_t ntok = ((volatile uint64_t*)ds->host)[0];
  if (w.wgrec) {  // per kernel: workgroups, distinct CUs, start / end spread (us from the first start)
    std::vector<uint64_t> r(kWgRecWords);
    HIPTRY(hipMemcpy(r.data(), w.wgrec, kWgRecWords * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (size_t i = 0; i < kWgRecWords; i += 4)
      if (r[i]) t0 = std::min(t0, r[i]);
    static const char* names[4] = {"k_bpe_short", "k_bpe_mid<2>", "k_bpe_mid<3>", "k_bpe_sparse"};
    for (int k = 0; k < 4; k++) {
      std::vector<uint64_t> cus;
      double s0 = 1e30, s1 = 0, e0 = 1e30, e1 = 0;
      int n = 0, busy = 0;
      for (int b = 0; b < 1024; b++) {
        const uint64_t* q = &r[((size_t)k * 1024 + b) * 4];
        if (!q[0] || !q[1]) continue;
        n++;
        busy += q[3] != 0;
        cus.push_back(q[2]);
        const double a = (q[0] - t0) / 100.0, e = (q[1] - t0) / 100.0;  // (100 MHz clock)
        s0 = std::min(s0, a), s1 = std::max(s1, a), e0 = std::min(e0, e), e1 = std::max(e1, e);
      }
      if (!n) continue;
      std::sort(cus.begin(), cus.end());
      const size_t ncu = std::unique(cus.begin(), cus.end()) - cus.begin();
      fprintf(stderr, "[ctok wgrec] %-13s wgs %4d (working %4d) on %3zu CUs  start %8.1f .. %8.1f  end %8.1f .. %8.1f us\n",
              names[k], n, busy, ncu, s0, s1, e0, e1);
    }
  }
  if (w.stamps) {  // diagnostic: k_segment's mean cycles per phase over the tiles that stamped
    std::vector<uint64_t> st8((size_t)w.n_tiles * 8);
    HIPTRY(hipMemcpy(st8.data(), w.stamps, st8.size() * 8, hipMemcpyDeviceToHost));
    double acc[6] = {0, 0, 0, 0, 0, 0}, np_sum = 0;
    uint64_t n = 0;
    for (size_t i = 0; i < w.n_tiles; i++) {
      const uint64_t* r = &st8[i * 8];
      if (!r[0] || !r[5]) continue;
      for (int k = 0; k < 5; k++) acc[k] += (double)(r[k + 1] - r[k]);
      acc[5] += (double)(r[5] - r[0]);
      np_sum += (double)r[6];
      n++;
    }
    if (n)
      fprintf(stderr, "[ctok stamps] k_segment cycles per tile (mean of %llu): loads %.0f  non-ascii %.0f  starts %.0f  "
              "routing %.0f  tail %.0f  total %.0f  pieces %.1f\n", (unsigned long long)n, acc[0] / n, acc[1] / n,
              acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n, np_sum / n);
  }
  uint32_t cnt[kNumCounters];
  for (int i = 0; i < kNumCounters; i++) cnt[i] = ((volatile uint32_t*)(ds->host + 1))[i];
  if (w.nfc_watch == 1 && cnt[12]) {  // a code point NFC may change: check, normalise, run again
    speculate = false;
    continue;
  }
  if ((cnt[kCtrOverflow] || cnt[0] > w.long_cap) && !safe) {  // a lean list overflowed: run again safe
    safe = true;
    continue;
  }
  if (w.nfc_watch == 2 && cnt[12]) {
    // the pass's ids did not all fit the output, or its panic flag may come from a flagged doc's
    // raw (unnormalised) pairs, which the reference never sees (it normalises first): run again
    // normalised
    if (ntok > ids_cap || (cnt[2] & kErrPanic)) {
      speculate = false;
      continue;
    }
    ntok = nfc_splice(t, ds, d_text, d_off, n_docs, n_bytes, d_ids, ids_cap, d_tok_off, ntok, s, &nfc_docs, split_added);
    if (timing) {
      HIPTRY(hipEventRecord(ds->ev[11], s));
      HIPTRY(hipEventSynchronize(ds->ev[11]));
    }
  }
  const uint32_t P = cnt[5];
  if (cnt[2] & kErrPanic)
    throw_err(CTOK_E_PANIC, "index out of bounds: a merge rank points past the list of valid merges (reference src/bpe.rs:141 panics)");
  if (ntok > ids_cap) throw_err(CTOK_E_CAPACITY, "ids_cap too small: tok_off[n_docs] holds the number of ids needed");
  if (st) {
    st->bytes_in = n_bytes;
    st->bytes_norm = B;
    st->docs = n_docs;
    st->pieces = w.n_tiles ? P : 0;
    st->long_pieces = cnt[0];
    st->tokens = ntok;
    st->workspace_bytes = ds->workspace_bytes();
    st->long_rounds = cnt[kCtrRounds];
    st->nfc_docs = nfc_docs;
    for (int c = 0; c < kNumClasses; c++) {
      st->class_bytes[c] = cnt[ctr_stat(c)];
      st->class_ids[c] = cnt[ctr_stat(c) + 1];
    }
    if (tm) {
      st->ms_pretok = laps[lap[0]];
      st->ms_segment = laps[lap[1]];
      st->ms_bpe_lo = laps[lap[2]];
      st->ms_bpe_hi = std::max(0.0, laps[lap[3]]);
      st->ms_bpe_med = laps[lap[4]];
      // the merge passes (k_segment's end to the last one's end) and the side stream's long tiers
      // past them (the tail's start waits for the join)
      st->ms_bpe_short = std::max(laps[lap[5]], std::max(laps[lap[6]], laps[lap[7]]));
      st->ms_bpe_long = std::max(0.0, laps[lap[8]] - st->ms_bpe_short);
      st->ms_emit = laps[lap[9]];
      st->ms_device = laps[lap[10]];
      if (w.nfc_watch == 2 && cnt[12]) {  // (the NFC splice ran after the main call: ev[11] ends it)
        float v = 0;
        HIPTRY(hipEventElapsedTime(&v, ds->ev[0], ds->ev[11]));
        st->ms_device = v;
      }
    }
  }
  HP(8);
  if (hostprof)
    fprintf(stderr, "[ctok hostprof] us from entry: prep %.1f  clear..segment launched %.1f  short launched %.1f  report %.1f  "
            "all launched %.1f  synced %.1f  laps %.1f  end %.1f\n", (hp[1] - hp[0]) * 1e3, (hp[2] - hp[0]) * 1e3,
            (hp[3] - hp[0]) * 1e3, (hp[4] - hp[0]) * 1e3, (hp[5] - hp[0]) * 1e3, (hp[6] - hp[0]) * 1e3,
            (hp[7] - hp[0]) * 1e3, (hp[8] - hp[0]) * 1e3);
#undef HP
  return ntok;
  }
}

// ----------------------------------------------------------------------------- decode

void ensure_decode_tables(ctok* t, DeviceState* ds, hipStream_t s) {
  if (ds->dec_ready) return;
  upload(ds->dec_ent, t->dec_ent.data(), t->dec_ent.size(), s);
  upload(ds->dec_bytes, t->dec_bytes.data(), t->dec_bytes.size(), s);
  HIPTRY(hipStreamSynchronize(s));
  ds->dec_ready = true;
}

// decode_batch_with_options on device-resident ids (src/huggingface/mod.rs:771-785).  Returns
// the output byte count; get_out(n) supplies an output buffer of >= n bytes (or throws).
uint64_t decode_device(ctok* t, DeviceState* ds, const uint32_t* d_ids, const uint64_t* d_tok_off, uint64_t n_docs,
                       uint64_t n_ids, uint32_t opts, const std::function<uint8_t*(uint64_t)>& get_out,
                       uint64_t* d_out_off, hipStream_t s, bool timing, ctok_decode_stats* st) {
  if (t->decoder < 0)
    throw_err(CTOK_E_UNSUPPORTED, "decoder " + t->decoder_name + " is outside the ByteLevel-BPE decode path");
  if (n_ids >= 0xF0000000ull || n_docs >= 0xF0000000ull)
    throw_err(CTOK_E_ARG, "a single decode call is limited to < 3.75 G ids and docs; split the batch");
  if (n_ids && ((uintptr_t)d_ids & 3)) throw_err(CTOK_E_ARG, "device ids buffer must be 4-byte aligned");
  ensure_decode_tables(t, ds, s);
  DecTables tb{(const uint2*)ds->dec_ent.p, (uint32_t)(t->dec_ent.size() / 2), ds->dec_bytes.p};
  DecWork w{};
  w.ids = d_ids;
  w.n_ids = (uint32_t)n_ids;
  w.tok_off = d_tok_off;
  w.n_docs = (uint32_t)n_docs;
  w.opts = opts & (kDecOptSkipSpecial | kDecOptCleanup);
  w.n_chunks = (uint32_t)((n_ids + kDecChunk - 1) / kDecChunk);
  ds->dec_chunk.ensure(w.n_chunks + 8);
  ds->dec_cnt.ensure(8);
  ds->scan_tmp.ensure(scan_tmp_elems(w.n_chunks + 1) + 64);
  w.chunk_off = ds->dec_chunk.p;
  w.counters = ds->dec_cnt.p;
  if (timing) HIPTRY(hipEventRecord(ds->dev_ev[0], s));
  HIPTRY(hipMemsetAsync(ds->dec_cnt.p, 0, 32, s));
  HIPTRY(launch_dec_len(w, tb, (uint32_t*)ds->scan_tmp.p, ds->scan_tmp.cap * 2, s));
  if (timing) HIPTRY(hipEventRecord(ds->dev_ev[1], s));
  HIPTRY(hipMemcpyAsync(ds->host, ds->dec_cnt.p, 16, hipMemcpyDeviceToHost, s));
  spin_sync(ds, s);
  const uint32_t err = ((volatile uint32_t*)ds->host)[0], nonascii = ((volatile uint32_t*)ds->host)[1];
  const uint64_t R = ((volatile uint64_t*)ds->host)[1];
  if (err) throw_err(CTOK_E_ARG, "tok_off must start at 0, be non-decreasing and end at the number of ids");
  if (R >= 0xF0000000ull) throw_err(CTOK_E_ARG, "decoded batch exceeds 3.75 GiB; split the batch");
  const bool direct = !(w.opts & kDecOptCleanup) && !nonascii;
  uint64_t n_out = R;
  if (direct) {  // every unit is a valid ASCII byte and nothing is cleaned: the gather is the output
    uint8_t* d_out = get_out(R);
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[2], s));
    HIPTRY(launch_dec_gather(w, tb, d_out, d_out_off, s));
    if (!n_ids) HIPTRY(hipMemsetAsync(d_out_off, 0, (n_docs + 1) * 8, s));
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[3], s));
  } else {
    ds->dec_raw.ensure(R + 64);
    ds->dec_rawoff.ensure(n_docs + 1);
    w.raw = ds->dec_raw.p;
    w.n_raw = (uint32_t)R;
    w.raw_off = ds->dec_rawoff.p;
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[2], s));
    HIPTRY(launch_dec_gather(w, tb, w.raw, w.raw_off, s));
    if (!n_ids) HIPTRY(hipMemsetAsync(w.raw_off, 0, (n_docs + 1) * 8, s));
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[3], s));
    w.n_tiles = (uint32_t)((R + kDecTile - 1) / kDecTile);
    ds->dec_tile.ensure(w.n_tiles + 8);
    ds->dec_del.ensure(R / 32 + 8);
    ds->scan_tmp.ensure(scan_tmp_elems(w.n_tiles + 1) + 64);
    w.tile_cnt = ds->dec_tile.p;
    w.delbits = ds->dec_del.p;
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[4], s));
    if (w.opts & kDecOptCleanup) HIPTRY(hipMemsetAsync(w.delbits, 0, (R / 32 + 8) * 4, s));
    HIPTRY(launch_dec_prepare(w, s));
    HIPTRY(launch_dec_count(w, (uint32_t*)ds->scan_tmp.p, ds->scan_tmp.cap * 2, s));
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[5], s));
    HIPTRY(hipMemcpyAsync(ds->host, w.tile_cnt + w.n_tiles, 4, hipMemcpyDeviceToHost, s));
    spin_sync(ds, s);
    n_out = ((volatile uint32_t*)ds->host)[0];
    uint8_t* d_out = get_out(n_out);
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[6], s));
    HIPTRY(launch_dec_write(w, d_out, d_out_off, s));
    if (!R) HIPTRY(hipMemsetAsync(d_out_off, 0, (n_docs + 1) * 8, s));
    if (timing) HIPTRY(hipEventRecord(ds->dev_ev[7], s));
  }
  if (st) {
    st->ids = n_ids;
    st->docs = n_docs;
    st->bytes_raw = R;
    st->bytes_out = n_out;
    st->direct = direct ? 1 : 0;
    if (timing) {
      HIPTRY(hipEventSynchronize(ds->dev_ev[direct ? 3 : 7]));
      auto el = [&](int i, int j) {
        float v = 0;
        HIPTRY(hipEventElapsedTime(&v, ds->dev_ev[i], ds->dev_ev[j]));
        return (double)v;
      };
      st->ms_len = el(0, 1);
      st->ms_gather = el(2, 3);
      st->ms_clean = direct ? 0.0 : el(4, 5) + el(6, 7);
      st->ms_device = st->ms_len + st->ms_gather + st->ms_clean;
    }
  }
  return n_out;
}

// ----------------------------------------------------------------------------- host-buffer pipeline
//
// ctok_encode_batch on host memory.  The batch is cut into chunks of about `chunk` text bytes
// (whole documents); per chunk c (slot c & 1):
//   stage   the up stream copies the chunk's text from the caller's buffer to d_in and its
//           offsets to d_off, made chunk-relative on the device                  (ev_h2d)
//   encode  the encode stream waits for ev_h2d (and for the D2H of chunk c - 2, which used the
//           same d_ids), runs encode_device, adds the running token base to tok_off (ev_enc)
//   drain   the down stream copies ids / tok_off straight into the caller's ids (at the running
//           token base) and tok_off                                              (ev_d2h)
// stage(c + 1) and drain(c - 1) run on helper threads while encode(c) runs, so PCIe traffic in
// both directions overlaps the kernels.  The copies touch the caller's pageable memory directly:
// the runtime pins it in place at the link's rate (56-57 GB/s each way on the MI355X box, the same
// as from hipHostMalloc memory; profiles/r03/pcie_probe.txt), so staging through pinned buffers
// only added two host memcpys per byte (round 2: 16.3 GB/s E2E on C2).

// dst[i] = src[i] for i < n, with non-temporal 16-byte stores (the caller's ids are written once
// and not read back here: no read-for-ownership of their lines)
void widen16(uint32_t* dst, const uint16_t* src, size_t n) {
  size_t i = 0;
  for (; i < n && ((uintptr_t)(dst + i) & 15u); i++) dst[i] = src[i];
  const __m128i z = _mm_setzero_si128();
  for (; i + 8 <= n; i += 8) {
    const __m128i v = _mm_loadu_si128((const __m128i*)(src + i));
    _mm_stream_si128((__m128i*)(dst + i), _mm_unpacklo_epi16(v, z));
    _mm_stream_si128((__m128i*)(dst + i + 4), _mm_unpackhi_epi16(v, z));
  }
  for (; i < n; i++) dst[i] = src[i];
  _mm_sfence();
}

HostPipe* host_pipe(DeviceState* ds) {
  if (ds->pipe) return ds->pipe.get();
  auto p = std::make_unique<HostPipe>();
  HIPTRY(hipStreamCreateWithFlags(&p->up, hipStreamNonBlocking));
  HIPTRY(hipStreamCreateWithFlags(&p->down, hipStreamNonBlocking));
  for (int i = 0; i < 2; i++) {
    HIPTRY(hipEventCreateWithFlags(&p->ev_h2d[i], hipEventDisableTiming));
    HIPTRY(hipEventCreateWithFlags(&p->ev_enc[i], hipEventDisableTiming));
    HIPTRY(hipEventCreateWithFlags(&p->ev_d2h[i], hipEventDisableTiming));
  }
  for (auto& e : p->ev_t) HIPTRY(hipEventCreate(&e));
  ds->pipe = std::move(p);
  return ds->pipe.get();
}

struct RangeOut {
  uint64_t ntok = 0;     // ids of the range
  bool overflow = false;  // ntok > cap: nothing past cap was written
};

// Encode docs [d0, d1) of a host batch on one device; ids go to ids[0, cap), tok_off[i] (i in
// [1, d1 - d0]) = ids of docs d0 .. d0 + i - 1 (tok_off[0] is not written: with several shards
// it is the previous shard's last entry).  The device lock is held by the caller.
RangeOut encode_host_range(ctok* t, DeviceState* ds, const uint8_t* text, const uint64_t* off, uint64_t d0,
                           uint64_t d1, uint32_t* ids, uint64_t cap, uint64_t* tok_off, uint64_t chunk,
                           unsigned nthreads, bool timing, ctok_stats* st) {
  RangeOut r;
  if (d1 <= d0) return r;
  HostPipe* P = host_pipe(ds);
  hipStream_t s = ds->stream;
  // chunk boundaries: whole docs, about `chunk` bytes each (a longer doc is a chunk by itself),
  // ramped: the first chunks grow from chunk / 8 and the last ones shrink to it, so the first
  // upload and the last download, which nothing overlaps, are short
  static const bool no_ramp = getenv("CTOK_NO_CHUNK_RAMP") != nullptr;
  const uint64_t c_min = std::max<uint64_t>(chunk / 8, 1u << 20);
  uint64_t want = no_ramp ? chunk : c_min;
  std::vector<uint64_t> cut{d0};
  while (cut.back() < d1) {
    const uint64_t a = cut.back(), left = off[d1] - off[a];
    uint64_t sz = no_ramp ? chunk : std::min(std::min(want, chunk), std::max(c_min, left / 2));
    if (left < sz + c_min) sz = left;  // no small remainder
    want = std::min(2 * want, chunk);
    const uint64_t* e = std::upper_bound(off + a + 1, off + d1 + 1, off[a] + sz);
    uint64_t b = (uint64_t)(e - off) - 1;  // last doc end <= off[a] + chunk
    if (b <= a) b = a + 1;
    cut.push_back(std::min(b, d1));
  }
  const size_t C = cut.size() - 1;
  std::vector<uint64_t> ntok(C, 0), base(C + 1, 0);
  double ms_h2d = 0, ms_d2h = 0, ms_dev = 0, ms_pre = 0, ms_bs = 0, ms_bl = 0, ms_em = 0, ms_seg = 0, ms_lo = 0, ms_hi = 0;
  double ms_med = 0;

  // stage / drain run on helper threads: each makes the shard's device current first (the HIP
  // current device is per thread).  Both copy straight between the caller's (pageable) buffers
  // and the device: the runtime pins the pages in place and copies at the link's rate, as fast as
  // from pinned memory (profiles/r03/pcie_probe.txt), so there is no staging copy on the host.
  static const bool trace = getenv("CTOK_PIPE_TRACE") != nullptr;
  const double tr0 = now_ms();
  auto TR = [&](const char* what, size_t c) { if (trace) fprintf(stderr, "[pipe] %8.3f %s %zu\n", now_ms() - tr0, what, c); };
  auto stage = [&](size_t c) {
    TR("stage<", c);
    HIPTRY(hipSetDevice(ds->device));
    const int k = (int)(c & 1);
    const uint64_t a = cut[c], b = cut[c + 1], n = b - a, B = off[b] - off[a];
    // (d_in[k] / d_off[k] were last read by chunk c - 2's encode, which has returned)
    if (timing && c == 0) HIPTRY(hipEventRecord(P->ev_t[0], P->up));
    if (B) HIPTRY(hipMemcpyAsync(P->d_in[k].p, text + off[a], B, hipMemcpyHostToDevice, P->up));
    HIPTRY(hipMemsetAsync(P->d_in[k].p + B, 0, 16, P->up));
    HIPTRY(hipMemcpyAsync(P->d_off[k].p, off + a, (n + 1) * 8, hipMemcpyHostToDevice, P->up));
    HIPTRY(shift_u64(P->d_off[k].p, n + 1, (uint64_t)0 - off[a], P->up));  // chunk-relative offsets
    if (timing && c == 0) HIPTRY(hipEventRecord(P->ev_t[1], P->up));
    HIPTRY(hipEventRecord(P->ev_h2d[k], P->up));
    if (trace) { HIPTRY(hipEventSynchronize(P->ev_h2d[k])); TR("stage>", c); }
  };
  // ids16 tokenizers: the ids cross the link as u16 and tok_off as u32 (k_wire16), into pinned
  // buffers, and host threads widen them into the caller's buffers (which also first-touches
  // fresh output pages on several threads); the link is the E2E bound (56 GB/s for both
  // directions together), and this moves 2 B per id instead of 4
  const bool w16 = t->ids16 && !getenv("CTOK_WIRE32");
  auto drain = [&](size_t c) {
    HIPTRY(hipSetDevice(ds->device));
    const int k = (int)(c & 1);
    const uint64_t a = cut[c], n = cut[c + 1] - a;
    const uint64_t b0 = base[c], nt = ntok[c];
    const uint64_t nc = b0 < cap ? std::min(nt, cap - b0) : 0;  // ids that fit the caller's buffer
    uint64_t* dst_off = tok_off + (a - d0);
    HIPTRY(hipStreamWaitEvent(P->down, P->ev_enc[k], 0));  // chunk c's ids and tok_off
    if (timing && c + 1 == C) HIPTRY(hipEventRecord(P->ev_t[2], P->down));
    if (w16) {
      P->pin_ids16[k].ensure(nt + 8);
      P->pin_toff32[k].ensure(n + 1);
      if (nc) HIPTRY(hipMemcpyAsync(P->pin_ids16[k].p, P->d_ids16[k].p, nc * 2, hipMemcpyDeviceToHost, P->down));
      HIPTRY(hipMemcpyAsync(P->pin_toff32[k].p, P->d_toff32[k].p, (n + 1) * 4, hipMemcpyDeviceToHost, P->down));
    } else {
      if (nc) HIPTRY(hipMemcpyAsync(ids + b0, P->d_ids[k].p, nc * 4, hipMemcpyDeviceToHost, P->down));
      if (n) HIPTRY(hipMemcpyAsync(dst_off + 1, P->d_tokoff[k].p + 1, n * 8, hipMemcpyDeviceToHost, P->down));
    }
    if (timing && c + 1 == C) HIPTRY(hipEventRecord(P->ev_t[3], P->down));
    HIPTRY(hipEventRecord(P->ev_d2h[k], P->down));
    TR("drain<", c);
    HIPTRY(hipEventSynchronize(P->ev_d2h[k]));
    TR("d2h>", c);
  };
  // widen(c) (w16): chunk c's 16-bit ids / 32-bit tok_off from the pinned slot into the caller's
  // buffers, on up to nthreads threads.  Runs on its own thread, overlapping the next chunks'
  // copies; joined before the slot is drained into again (wid[c & 1]) and at the end.
  auto widen = [&](size_t c) {
    const int k = (int)(c & 1);
    const uint64_t a = cut[c], n = cut[c + 1] - a;
    const uint64_t b0 = base[c], nt = ntok[c];
    const uint64_t nc = b0 < cap ? std::min(nt, cap - b0) : 0;
    const uint16_t* src = P->pin_ids16[k].p;
    uint32_t* dst = ids + b0;
    const unsigned nw = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nthreads, nc >> 20));
    const uint64_t per = (nc + nw - 1) / nw;
    std::vector<std::thread> th;
    for (unsigned i = 1; i < nw; i++)
      th.emplace_back([=] { const uint64_t lo = std::min(nc, i * per); widen16(dst + lo, src + lo, std::min(nc, lo + per) - lo); });
    widen16(dst, src, std::min(nc, per));
    const uint32_t* to = P->pin_toff32[k].p;
    uint64_t* dst_off = tok_off + (a - d0);
    for (uint64_t i = 1; i <= n; i++) dst_off[i] = b0 + to[i];
    for (auto& x : th) x.join();
    TR("widen>", c);
  };
  std::thread wid[2];
  std::exception_ptr ex_wid[2];
  struct WidJoiner {
    std::thread* w;
    ~WidJoiner() {
      for (int i = 0; i < 2; i++)
        if (w[i].joinable()) w[i].join();
    }
  } wid_joiner{wid};
  auto start_widen = [&](size_t c) {
    wid[c & 1] = std::thread([&, c] {
      try { widen(c); } catch (...) { ex_wid[c & 1] = std::current_exception(); }
    });
  };
  auto join_widen = [&](int k) {
    if (wid[k].joinable()) wid[k].join();
    if (ex_wid[k]) std::rethrow_exception(ex_wid[k]);
  };
  // device buffers sized for the largest chunk up front (no reallocation while copies are in flight)
  {
    uint64_t maxB = 0, maxD = 0;
    for (size_t c = 0; c < C; c++) {
      maxB = std::max(maxB, off[cut[c + 1]] - off[cut[c]]);
      maxD = std::max(maxD, cut[c + 1] - cut[c]);
    }
    for (int k = 0; k < 2; k++) {
      P->d_in[k].ensure(maxB + 16);
      P->d_off[k].ensure(maxD + 1);
      P->d_tokoff[k].ensure(maxD + 1);
      P->d_ids[k].ensure(ctok_ids_bound(t, maxB, maxD));
      if (w16) {
        P->d_ids16[k].ensure(ctok_ids_bound(t, maxB, maxD));
        P->d_toff32[k].ensure(maxD + 1);
      }
    }
  }
  stage(0);
  for (size_t c = 0; c < C; c++) {
    const int k = (int)(c & 1);
    const uint64_t a = cut[c], n = cut[c + 1] - a, B = off[cut[c + 1]] - off[a];
    // helper threads: chunk c + 1 goes up and chunk c - 1 comes down while chunk c is encoded;
    // an exception inside one is rethrown here after the join
    std::exception_ptr ex_stage, ex_drain;
    std::thread th_stage, th_drain;
    if (c + 1 < C)
      th_stage = std::thread([&, c] {
        try { stage(c + 1); } catch (...) { ex_stage = std::current_exception(); }
      });
    if (c >= 1) join_widen((int)((c - 1) & 1));  // (widen(c - 3) read the pinned slot drain(c - 1) fills)
    if (c >= 1)
      th_drain = std::thread([&, c] {
        try { drain(c - 1); } catch (...) { ex_drain = std::current_exception(); }
      });
    struct Joiner {
      std::thread& a;
      std::thread& b;
      ~Joiner() {
        if (a.joinable()) a.join();
        if (b.joinable()) b.join();
      }
    } joiner{th_stage, th_drain};
    HIPTRY(hipStreamWaitEvent(s, P->ev_h2d[k], 0));
    HIPTRY(hipStreamWaitEvent(s, P->ev_d2h[k], 0));  // chunk c - 2's ids have left d_ids[k]
    ctok_stats cs{};
    TR("enc<", c);
    ntok[c] = encode_device(t, ds, P->d_in[k].p, P->d_off[k].p, n, B, P->d_ids[k].p, P->d_ids[k].cap,
                            P->d_tokoff[k].p, s, timing, &cs);
    base[c + 1] = base[c] + ntok[c];
    TR("enc>", c);
    if (st) {
      st->pieces += cs.pieces;
      st->long_pieces += cs.long_pieces;
      st->long_rounds += cs.long_rounds;
      st->nfc_docs += cs.nfc_docs;
      st->workspace_bytes = std::max(st->workspace_bytes, cs.workspace_bytes);
      st->bytes_norm += cs.bytes_norm;
      for (int q = 0; q < kNumClasses; q++) {
        st->class_bytes[q] += cs.class_bytes[q];
        st->class_ids[q] += cs.class_ids[q];
      }
      ms_dev += cs.ms_device, ms_pre += cs.ms_pretok, ms_bs += cs.ms_bpe_short, ms_bl += cs.ms_bpe_long;
      ms_em += cs.ms_emit, ms_seg += cs.ms_segment, ms_lo += cs.ms_bpe_lo, ms_hi += cs.ms_bpe_hi;
      ms_med += cs.ms_bpe_med;
    }
    if (w16)
      HIPTRY(wire16(P->d_ids[k].p, ntok[c], P->d_ids16[k].p, P->d_tokoff[k].p, n + 1, P->d_toff32[k].p, s));
    else
      HIPTRY(shift_u64(P->d_tokoff[k].p + 1, n, base[c], s));  // batch-relative tok_off
    HIPTRY(hipEventRecord(P->ev_enc[k], s));
    if (th_drain.joinable()) th_drain.join();
    if (ex_drain) std::rethrow_exception(ex_drain);
    if (c >= 1 && w16) start_widen(c - 1);
    if (th_stage.joinable()) th_stage.join();
    if (ex_stage) std::rethrow_exception(ex_stage);
  }
  join_widen((int)((C - 1) & 1));
  drain(C - 1);
  if (w16) widen(C - 1);
  join_widen(0);
  join_widen(1);
  r.ntok = base[C];
  r.overflow = r.ntok > cap;
  if (st && timing) {
    float v = 0;
    HIPTRY(hipEventElapsedTime(&v, P->ev_t[0], P->ev_t[1]));
    ms_h2d = v;
    HIPTRY(hipEventElapsedTime(&v, P->ev_t[2], P->ev_t[3]));
    ms_d2h = v;
    st->ms_h2d += ms_h2d, st->ms_d2h += ms_d2h, st->ms_device += ms_dev, st->ms_pretok += ms_pre;
    st->ms_bpe_short += ms_bs, st->ms_bpe_long += ms_bl, st->ms_emit += ms_em, st->ms_segment += ms_seg;
    st->ms_bpe_lo += ms_lo, st->ms_bpe_hi += ms_hi, st->ms_bpe_med += ms_med;
  }
  return r;
}

}  // namespace

// ----------------------------------------------------------------------------- internal API
// for trainer_host.cpp (host_common.h): errors, and the GPU pre-tokenizer of a host batch

namespace {
int run(const std::function<void()>& f);
}

namespace ctok_host {
[[noreturn]] void throw_error(int code, const std::string& msg) { throw_err(code, msg); }
int run_guarded(const std::function<void()>& f) { return run(f); }
unsigned usable_cpus() { return usable_cpus_once(); }

// NFC (when the tokenizer normalises) + ByteLevel pre-tokenization of n_docs host texts on device
// dev: the text the pieces index (normalised when normalisation ran), its doc offsets, and the
// piece-start bitmap (bit g = a piece starts at byte g).
void pretokenize(ctok* t, int dev, const uint8_t* utf8, const uint64_t* doc_off, uint64_t n_docs,
                 std::vector<uint8_t>& text, std::vector<uint64_t>& off, std::vector<uint32_t>& pbits) {
  if (doc_off[0] != 0) throw_err(CTOK_E_ARG, "offsets[0] must be 0");
  for (uint64_t d = 0; d < n_docs; d++)
    if (doc_off[d + 1] < doc_off[d]) throw_err(CTOK_E_ARG, "offsets must be non-decreasing");
  const uint64_t n_in = doc_off[n_docs];
  if (n_in && !utf8) throw_err(CTOK_E_ARG, "null text");
  DeviceState* ds = device_state(t, dev);
  std::lock_guard<std::recursive_mutex> lk(ds->mu);
  HIPTRY(hipSetDevice(dev));
  hipStream_t s = ds->stream;
  ds->pad_in_text.ensure(n_in + 16);
  ds->pad_in_off.ensure(n_docs + 1);
  if (n_in) HIPTRY(hipMemcpyAsync(ds->pad_in_text.p, utf8, n_in, hipMemcpyHostToDevice, s));
  HIPTRY(hipMemsetAsync(ds->pad_in_text.p + n_in, 0, 16, s));
  HIPTRY(hipMemcpyAsync(ds->pad_in_off.p, doc_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, s));
  encode_device(t, ds, ds->pad_in_text.p, ds->pad_in_off.p, n_docs, n_in, nullptr, 0, nullptr, s, false, nullptr, true,
                true);
  const uint64_t B = ds->last_B;
  pbits.assign((B + 31) / 32, 0);
  off.resize(n_docs + 1);
  text.resize(B);
  if (!pbits.empty()) HIPTRY(hipMemcpyAsync(pbits.data(), ds->pbits.p, pbits.size() * 4, hipMemcpyDeviceToHost, s));
  if (ds->last_norm) {
    if (B) HIPTRY(hipMemcpyAsync(text.data(), ds->norm_text.p, B, hipMemcpyDeviceToHost, s));
    HIPTRY(hipMemcpyAsync(off.data(), ds->norm_off.p, (n_docs + 1) * 8, hipMemcpyDeviceToHost, s));
  }
  HIPTRY(hipStreamSynchronize(s));
  if (!ds->last_norm) {
    if (B) std::memcpy(text.data(), utf8, B);
    std::memcpy(off.data(), doc_off, (n_docs + 1) * 8);
  }
}
}  // namespace ctok_host

// ----------------------------------------------------------------------------- C ABI

namespace {
int run(const std::function<void()>& f) {
  try {
    f();
    g_err.clear();
    return CTOK_OK;
  } catch (const CtokError& e) {
    return fail(e.code, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(CTOK_E_DEVICE, "out of host memory");
  } catch (const std::exception& e) {
    return fail(CTOK_E_ARG, e.what());
  }
}
}  // namespace

extern "C" {

const char* ctok_last_error(void) { return g_err.c_str(); }
const char* ctok_version(void) { return "0.3.3+mi355x.1"; }

int ctok_create_from_buffer(const char* json, size_t len, ctok** out) {
  if (!out || (!json && len)) return fail(CTOK_E_ARG, "null argument");
  *out = nullptr;
  return run([&] {
    std::unique_ptr<ctok> t(new ctok());
    load(t.get(), json, len);
    *out = t.release();
  });
}

int ctok_create_from_tables(const ctok_tables* tb, ctok** out) {
  if (!tb || !out) return fail(CTOK_E_ARG, "null argument");
  *out = nullptr;
  return run([&] {
    if ((tb->n_vocab && (!tb->vocab || !tb->vocab_off || !tb->vocab_id)) ||
        (tb->n_merges && (!tb->merge_left || !tb->merge_right)) ||
        (tb->n_added && (!tb->added || !tb->added_off || !tb->added_id || !tb->added_flags)))
      throw_err(CTOK_E_ARG, "null table");
    // the value tree tokenizer.json would parse to (no JSON text): model.vocab, model.merges as
    // "a b" strings of the vocab's tokens, added_tokens, normalizer, ByteLevel pre-tokenizer/decoder
    auto str = [](std::string v) { ctj::Value x; x.kind = ctj::Value::String; x.s = std::move(v); return x; };
    auto num = [](uint64_t v) { ctj::Value x; x.kind = ctj::Value::Int; x.u = v; return x; };
    auto boo = [](bool v) { ctj::Value x; x.kind = ctj::Value::Bool; x.b = v; return x; };
    auto obj = [] { ctj::Value x; x.kind = ctj::Value::Object; return x; };
    ctj::Value vocab = obj(), merges, added;
    merges.kind = added.kind = ctj::Value::Array;
    std::unordered_map<uint32_t, std::string> by_id;
    vocab.obj.reserve(tb->n_vocab);
    for (uint64_t i = 0; i < tb->n_vocab; i++) {
      std::string k(tb->vocab + tb->vocab_off[i], tb->vocab_off[i + 1] - tb->vocab_off[i]);
      by_id[tb->vocab_id[i]] = k;
      vocab.obj.emplace_back(std::move(k), num(tb->vocab_id[i]));
    }
    merges.arr.reserve(tb->n_merges);
    for (uint64_t r = 0; r < tb->n_merges; r++) {
      auto a = by_id.find(tb->merge_left[r]), b = by_id.find(tb->merge_right[r]);
      if (a == by_id.end() || b == by_id.end())
        throw_err(CTOK_E_ARG, "merge " + std::to_string(r) + " names an id that is not in the vocab");
      // the reference joins every merge to "a b" and keeps it only when it splits on ' ' into
      // exactly two parts (src/huggingface/mod.rs:252-264, array form :87-94): a token holding a
      // space would be dropped silently and shift every later rank, so the table is refused
      if (a->second.find(' ') != std::string::npos || b->second.find(' ') != std::string::npos)
        throw_err(CTOK_E_ARG, "merge " + std::to_string(r) +
                                  " joins a token that contains ' ': the reference's merge format cannot express it");
      merges.arr.push_back(str(a->second + " " + b->second));
    }
    for (uint64_t i = 0; i < tb->n_added; i++) {
      ctj::Value e = obj();
      const uint8_t f = tb->added_flags[i];
      e.obj.emplace_back("id", num(tb->added_id[i]));
      e.obj.emplace_back("content", str(std::string(tb->added + tb->added_off[i], tb->added_off[i + 1] - tb->added_off[i])));
      e.obj.emplace_back("special", boo(f & CTOK_ADDED_SPECIAL));
      e.obj.emplace_back("single_word", boo(f & CTOK_ADDED_SINGLE_WORD));
      e.obj.emplace_back("lstrip", boo(f & CTOK_ADDED_LSTRIP));
      e.obj.emplace_back("rstrip", boo(f & CTOK_ADDED_RSTRIP));
      e.obj.emplace_back("normalized", boo(f & CTOK_ADDED_NORMALIZED));
      added.arr.push_back(std::move(e));
    }
    ctj::Value model = obj(), root = obj(), norm = obj(), pre = obj(), dec = obj();
    model.obj.emplace_back("type", str("BPE"));
    model.obj.emplace_back("vocab", std::move(vocab));
    model.obj.emplace_back("merges", std::move(merges));
    if (tb->nfc) {
      norm.obj.emplace_back("type", str("NFC"));
    } else {  // no normalisation (a null normalizer would mean NFC, src/huggingface/parsing.rs:89)
      ctj::Value none;
      none.kind = ctj::Value::Array;
      norm.obj.emplace_back("type", str("Sequence"));
      norm.obj.emplace_back("normalizers", std::move(none));
    }
    pre.obj.emplace_back("type", str("ByteLevel"));
    pre.obj.emplace_back("add_prefix_space", boo(tb->add_prefix_space != 0));
    dec.obj.emplace_back("type", str("ByteLevel"));
    root.obj.emplace_back("model", std::move(model));
    root.obj.emplace_back("added_tokens", std::move(added));
    root.obj.emplace_back("normalizer", std::move(norm));
    root.obj.emplace_back("pre_tokenizer", std::move(pre));
    root.obj.emplace_back("decoder", std::move(dec));
    auto t = std::make_unique<ctok>();
    load_root(t.get(), root);
    *out = t.release();
  });
}

int ctok_create_from_file(const char* path, ctok** out) {
  if (!path || !out) return fail(CTOK_E_ARG, "null argument");
  *out = nullptr;
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(CTOK_E_IO, std::string("No such file or directory (os error 2): ") + path);
  std::stringstream ss;
  ss << f.rdbuf();
  if (f.bad()) return fail(CTOK_E_IO, std::string("read error: ") + path);
  std::string s = ss.str();
  return ctok_create_from_buffer(s.data(), s.size(), out);
}

void ctok_destroy(ctok* t) { delete t; }

uint64_t ctok_vocab_size(const ctok* t) { return t ? t->vocab.size() : 0; }

int ctok_token_to_id(const ctok* t, const char* tok, size_t len, uint32_t* id) {
  if (!t || (!tok && len) || !id) return fail(CTOK_E_ARG, "null argument");
  auto it = t->vocab.find(std::string(tok, len));
  if (it == t->vocab.end()) return CTOK_E_NOTFOUND;
  *id = it->second;
  return CTOK_OK;
}

int ctok_id_to_token(const ctok* t, uint32_t id, char* buf, size_t cap, size_t* len) {
  if (!t || !len) return fail(CTOK_E_ARG, "null argument");
  auto it = t->id_to_token.find(id);
  if (it == t->id_to_token.end()) return CTOK_E_NOTFOUND;
  *len = it->second.size();
  if (buf && cap) memcpy(buf, it->second.data(), std::min(cap, it->second.size()));
  return CTOK_OK;
}

uint64_t ctok_num_special_tokens(const ctok* t) { return t ? t->special.size() : 0; }

int ctok_special_token(const ctok* t, uint64_t i, char* buf, size_t cap, size_t* len, uint32_t* id) {
  if (!t || !len || !id) return fail(CTOK_E_ARG, "null argument");
  if (i >= t->special.size()) return fail(CTOK_E_ARG, "index out of range");
  const auto& e = t->special[i];
  *len = e.first.size();
  *id = e.second;
  if (buf && cap) memcpy(buf, e.first.data(), std::min(cap, e.first.size()));
  return CTOK_OK;
}

uint64_t ctok_num_piece_added_tokens(const ctok* t) { return t ? t->at_id.size() : 0; }

int ctok_piece_can_contain(const uint8_t* raw, size_t len) {
  if (!raw && len) return fail(CTOK_E_ARG, "null argument");
  return can_occur_in_piece(std::string((const char*)raw, len)) ? 1 : 0;
}

uint64_t ctok_ids_bound(const ctok*, uint64_t n_bytes, uint64_t n_docs) { return 3 * n_bytes + n_docs + 16; }

int ctok_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int ctok_encode_batch_device(const ctok* tc, const uint8_t* d_utf8, const uint64_t* d_doc_off, uint64_t n_docs,
                             uint64_t n_bytes, uint32_t* d_ids, uint64_t ids_cap, uint64_t* d_tok_off,
                             uint64_t* n_tokens_out, const ctok_exec* exec, ctok_stats* stats) {
  if (!tc || !d_doc_off || !d_tok_off || (n_bytes && (!d_utf8 || !d_ids))) return fail(CTOK_E_ARG, "null argument");
  ctok* t = const_cast<ctok*>(tc);
  return run([&] {
    double t0 = now_ms();
    int dev = exec ? exec->device : 0;
    DeviceState* ds = device_state(t, dev);
    std::lock_guard<std::recursive_mutex> lk(ds->mu);
    HIPTRY(hipSetDevice(dev));
    hipStream_t s = exec && exec->stream ? (hipStream_t)exec->stream : ds->stream;
    bool timing = exec && (exec->flags & CTOK_F_TIMING);
    uint64_t n = encode_device(t, ds, d_utf8, d_doc_off, n_docs, n_bytes, d_ids, ids_cap, d_tok_off, s, timing, stats);
    if (n_tokens_out) *n_tokens_out = n;
    if (stats) stats->ms_total = now_ms() - t0;
  });
}

int ctok_decode_batch_device(const ctok* tc, const uint32_t* d_ids, const uint64_t* d_tok_off, uint64_t n_docs,
                             uint64_t n_ids, uint32_t options, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off,
                             uint64_t* n_bytes_out, const ctok_exec* exec, ctok_decode_stats* stats) {
  if (!tc || !d_tok_off || !d_out_off || (n_ids && !d_ids)) return fail(CTOK_E_ARG, "null argument");
  ctok* t = const_cast<ctok*>(tc);
  return run([&] {
    double t0 = now_ms();
    int dev = exec ? exec->device : 0;
    DeviceState* ds = device_state(t, dev);
    std::lock_guard<std::recursive_mutex> lk(ds->mu);
    HIPTRY(hipSetDevice(dev));
    hipStream_t s = exec && exec->stream ? (hipStream_t)exec->stream : ds->stream;
    bool timing = exec && (exec->flags & CTOK_F_TIMING);
    auto get_out = [&](uint64_t n) -> uint8_t* {
      if (n_bytes_out) *n_bytes_out = n;
      if (n > out_cap) throw_err(CTOK_E_CAPACITY, "out_cap too small: *n_bytes_out holds the number of bytes needed");
      if (n && !d_out) throw_err(CTOK_E_ARG, "null output buffer");
      return d_out;
    };
    uint64_t n = decode_device(t, ds, d_ids, d_tok_off, n_docs, n_ids, options, get_out, d_out_off, s, timing, stats);
    if (n_bytes_out) *n_bytes_out = n;
    if (stats) stats->ms_total = now_ms() - t0;
  });
}

int ctok_decode_batch(const ctok* tc, const uint32_t* ids, const uint64_t* tok_off, uint64_t n_docs, uint32_t options,
                      uint8_t* out, uint64_t out_cap, uint64_t* out_off, const ctok_exec* exec,
                      ctok_decode_stats* stats) {
  if (!tc || !tok_off || !out_off) return fail(CTOK_E_ARG, "null argument");
  ctok* t = const_cast<ctok*>(tc);
  return run([&] {
    double t0 = now_ms();
    if (tok_off[0] != 0) throw_err(CTOK_E_ARG, "tok_off[0] must be 0");
    for (uint64_t d = 0; d < n_docs; d++)
      if (tok_off[d + 1] < tok_off[d]) throw_err(CTOK_E_ARG, "tok_off must be non-decreasing");
    const uint64_t T = tok_off[n_docs];
    if (T && !ids) throw_err(CTOK_E_ARG, "null ids");
    int dev = exec ? exec->device : 0;
    DeviceState* ds = device_state(t, dev);
    std::lock_guard<std::recursive_mutex> lk(ds->mu);
    HIPTRY(hipSetDevice(dev));
    hipStream_t s = exec && exec->stream ? (hipStream_t)exec->stream : ds->stream;
    bool timing = exec && (exec->flags & CTOK_F_TIMING);
    double h0 = now_ms();
    ds->dec_ids.ensure(T + 4);
    ds->dec_tokoff.ensure(n_docs + 1);
    ds->dec_outoff.ensure(n_docs + 1);
    if (T) HIPTRY(hipMemcpyAsync(ds->dec_ids.p, ids, T * 4, hipMemcpyHostToDevice, s));
    HIPTRY(hipMemcpyAsync(ds->dec_tokoff.p, tok_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, s));
    HIPTRY(hipStreamSynchronize(s));
    double h1 = now_ms();
    auto get_out = [&](uint64_t n) -> uint8_t* {
      ds->dec_out.ensure(n + 16);
      return ds->dec_out.p;
    };
    uint64_t n = decode_device(t, ds, ds->dec_ids.p, ds->dec_tokoff.p, n_docs, T, options, get_out, ds->dec_outoff.p,
                               s, timing, stats);
    double d0 = now_ms();
    HIPTRY(hipMemcpyAsync(out_off, ds->dec_outoff.p, (n_docs + 1) * 8, hipMemcpyDeviceToHost, s));
    if (n <= out_cap && n) HIPTRY(hipMemcpyAsync(out, ds->dec_out.p, n, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    if (n > out_cap) throw_err(CTOK_E_CAPACITY, "out_cap too small: out_off[n_docs] holds the number of bytes needed");
    if (stats) {
      stats->ms_h2d = h1 - h0;
      stats->ms_d2h = now_ms() - d0;
      stats->ms_total = now_ms() - t0;
    }
  });
}

int ctok_encode_batch(const ctok* tc, const uint8_t* utf8_in, const uint64_t* doc_off, uint64_t n_docs, uint32_t* ids,
                      uint64_t ids_cap, uint64_t* tok_off, const ctok_exec* exec, ctok_stats* stats) {
  if (!tc || !doc_off || !tok_off) return fail(CTOK_E_ARG, "null argument");
  ctok* t = const_cast<ctok*>(tc);
  return run([&] {
    double t0 = now_ms();
    if (doc_off[0] != 0) throw_err(CTOK_E_ARG, "doc_off[0] must be 0");
    for (uint64_t d = 0; d < n_docs; d++)
      if (doc_off[d + 1] < doc_off[d]) throw_err(CTOK_E_ARG, "doc_off must be non-decreasing");
    const uint64_t B = doc_off[n_docs];
    if (B && !utf8_in) throw_err(CTOK_E_ARG, "null text");
    if (ids_cap && !ids) throw_err(CTOK_E_ARG, "null ids");
    std::vector<int> devs;
    if (exec && exec->devices && exec->n_devices > 0) devs.assign(exec->devices, exec->devices + exec->n_devices);
    else devs.push_back(exec ? exec->device : 0);
    const bool timing = exec && (exec->flags & CTOK_F_TIMING);
    const uint64_t chunk = (uint64_t)(exec && exec->chunk_mb ? exec->chunk_mb : 64u) << 20;
    const unsigned hw = usable_cpus_once();
    const unsigned nthr = exec && exec->host_threads ? exec->host_threads
                                                     : std::max(1u, std::min(8u, hw / (unsigned)devs.size()));  // (widening threads: 4 / 8 / 16 within run-to-run noise on C2, profiles/r03/v22_e2e_probe.txt, v27_*; 8 + the pipeline threads stay inside a 16-CPU quota)
    if (stats) *stats = ctok_stats{};
    // shards: contiguous doc ranges balanced by bytes (cut at the first doc start >= k * B / G)
    const size_t G = devs.size();
    std::vector<uint64_t> cut(G + 1, 0);
    for (size_t g = 1; g < G; g++) {
      const uint64_t target = B / G * g;
      cut[g] = (uint64_t)(std::lower_bound(doc_off, doc_off + n_docs, target) - doc_off);
      cut[g] = std::max(cut[g], cut[g - 1]);
    }
    cut[G] = n_docs;
    // output placement: shard g writes its ids at region[g] of the caller's buffer, sized for
    // ids <= bytes + docs (true unless NFC grows the text or a prefix space is added) when the
    // regions fit, else into a private buffer; a shard that outgrows its region runs again
    std::vector<uint64_t> region(G + 1, 0);
    for (size_t g = 0; g < G; g++)
      region[g + 1] = region[g] + (doc_off[cut[g + 1]] - doc_off[cut[g]]) + (cut[g + 1] - cut[g]);
    std::vector<std::unique_ptr<uint32_t[]>> priv(G);
    std::vector<RangeOut> res(G);
    std::vector<ctok_stats> sst(G);
    // one pass over all shards; in_place: shard g writes at region[g] of the caller's ids, else
    // into priv[g] of priv_size[g] ids
    auto attempt = [&](bool in_place, const std::vector<uint64_t>& priv_size) {
      std::vector<std::exception_ptr> err(G);
      auto shard = [&](size_t g) {
        try {
          DeviceState* ds = device_state(t, devs[g]);
          std::lock_guard<std::recursive_mutex> lk(ds->mu);
          HIPTRY(hipSetDevice(devs[g]));
          uint32_t* out = ids;
          uint64_t cap = ids_cap;
          if (G > 1) {
            if (in_place) {
              out = ids + region[g];
              cap = region[g + 1] - region[g];
            } else {
              priv[g].reset(new uint32_t[priv_size[g] + 1]);  // no zero fill: ids[0, ntok) are written
              out = priv[g].get();
              cap = priv_size[g] + 1;
            }
          }
          sst[g] = ctok_stats{};
          res[g] = encode_host_range(t, ds, utf8_in, doc_off, cut[g], cut[g + 1], out, cap, tok_off + cut[g], chunk,
                                     nthr, timing, stats ? &sst[g] : nullptr);
        } catch (...) {
          err[g] = std::current_exception();
        }
      };
      if (G == 1) {
        shard(0);
      } else {
        std::vector<std::thread> th;
        for (size_t g = 0; g < G; g++) th.emplace_back(shard, g);
        for (auto& x : th) x.join();
      }
      for (size_t g = 0; g < G; g++)
        if (err[g]) std::rethrow_exception(err[g]);
    };
    tok_off[0] = 0;
    bool in_place = G == 1 || region[G] <= ids_cap;
    {
      std::vector<uint64_t> sz(G);
      for (size_t g = 0; g < G; g++) sz[g] = region[g + 1] - region[g];
      attempt(in_place, sz);
    }
    uint64_t total = 0;
    bool overflow = false;
    for (size_t g = 0; g < G; g++) total += res[g].ntok, overflow |= res[g].overflow;
    if (G > 1 && overflow && total <= ids_cap) {
      // a shard outgrew its id bound region (NFC growth): again, into private buffers of the
      // now known sizes
      std::vector<uint64_t> sz(G);
      for (size_t g = 0; g < G; g++) sz[g] = res[g].ntok;
      in_place = false;
      attempt(false, sz);
    }
    if (G > 1) {
      // rebase: tok_off of shard g gets the ids of shards < g added; its ids move from
      // region[g] (or priv[g]) to that base.  In place, the regions start at or after their
      // destinations, so moving in shard order never overwrites ids not yet moved.
      uint64_t basev = 0;
      for (size_t g = 0; g < G; g++) {
        const uint64_t n = res[g].ntok;
        if (g > 0)
          for (uint64_t d = cut[g] + 1; d <= cut[g + 1]; d++) tok_off[d] += basev;
        if (total <= ids_cap && n) {
          if (in_place) {
            if (region[g] != basev) std::memmove(ids + basev, ids + region[g], n * 4);
          } else {
            std::memcpy(ids + basev, priv[g].get(), n * 4);
          }
        }
        basev += n;
      }
    }
    tok_off[n_docs] = total;
    if (total > ids_cap) throw_err(CTOK_E_CAPACITY, "ids_cap too small: tok_off[n_docs] holds the number of ids needed");
    if (stats) {
      for (size_t g = 0; g < G; g++) {
        const ctok_stats& q = sst[g];
        stats->pieces += q.pieces, stats->long_pieces += q.long_pieces, stats->nfc_docs += q.nfc_docs;
        stats->long_rounds += q.long_rounds;
        stats->workspace_bytes += q.workspace_bytes;  // (shards on one device report it once each)
        stats->bytes_norm += q.bytes_norm;
        for (int c = 0; c < kNumClasses; c++)
          stats->class_bytes[c] += q.class_bytes[c], stats->class_ids[c] += q.class_ids[c];
        // device times: the slowest shard
        stats->ms_device = std::max(stats->ms_device, q.ms_device);
        stats->ms_pretok = std::max(stats->ms_pretok, q.ms_pretok);
        stats->ms_segment = std::max(stats->ms_segment, q.ms_segment);
        stats->ms_bpe_short = std::max(stats->ms_bpe_short, q.ms_bpe_short);
        stats->ms_bpe_lo = std::max(stats->ms_bpe_lo, q.ms_bpe_lo);
        stats->ms_bpe_hi = std::max(stats->ms_bpe_hi, q.ms_bpe_hi);
        stats->ms_bpe_med = std::max(stats->ms_bpe_med, q.ms_bpe_med);
        stats->ms_bpe_long = std::max(stats->ms_bpe_long, q.ms_bpe_long);
        stats->ms_emit = std::max(stats->ms_emit, q.ms_emit);
        stats->ms_h2d = std::max(stats->ms_h2d, q.ms_h2d);
        stats->ms_d2h = std::max(stats->ms_d2h, q.ms_d2h);
      }
      stats->bytes_in = B;
      stats->docs = n_docs;
      stats->tokens = total;
      stats->ms_total = now_ms() - t0;
    }
  });
}

uint64_t ctok_model_max_length(const ctok* t) { return t ? t->model_max_length : 0; }

int ctok_post_processor(const ctok* t, uint32_t* items, uint64_t cap, int64_t* n_items) {
  if (!t || !n_items) return fail(CTOK_E_ARG, "null argument");
  if (!t->has_pp) {
    *n_items = -1;
    return CTOK_OK;
  }
  *n_items = (int64_t)t->pp_items.size();
  for (uint64_t i = 0; i < t->pp_items.size() && i < cap && items; i++) items[i] = t->pp_items[i];
  return CTOK_OK;
}

// pad id: special_tokens["[PAD]"], else ["<pad>"], else 0 (src/huggingface/mod.rs:500-504)
uint32_t ctok_pad_id(const ctok* t) {
  if (!t) return 0;
  for (const char* name : {"[PAD]", "<pad>"})
    for (const auto& e : t->special)
      if (e.first == name) return e.second;
  return 0;
}

// src/huggingface/mod.rs:915-932
uint64_t ctok_num_special_tokens_to_add(const ctok* t, int is_pair) {
  if (!t) return 0;
  if (t->pp_kind == 3) return is_pair ? 3 : 2;
  if (t->pp_kind == 2) return is_pair ? 4 : 2;
  if (t->pp_kind != 1) return 0;
  const std::string& tpl = (is_pair && t->pp_has_pair) ? t->pp_pair : t->pp_single;
  std::vector<uint32_t> ch;
  if (!decode_utf8(tpl, ch)) return 0;
  uint64_t n = 0;
  size_t i = 0;
  while (i < ch.size()) {  // split_whitespace, parts not starting with '$'
    while (i < ch.size() && is_white_space(ch[i])) i++;
    if (i >= ch.size()) break;
    if (ch[i] != '$') n++;
    while (i < ch.size() && !is_white_space(ch[i])) i++;
  }
  return n;
}

int ctok_encode_padded_device(const ctok* tc, const uint8_t* d_utf8, const uint64_t* d_doc_off, uint64_t n_docs,
                              uint64_t n_bytes, const ctok_pad_opts* o, uint32_t* d_ids, uint32_t* d_attn,
                              uint32_t* d_type, uint32_t* d_special, uint64_t cap, uint64_t* d_row_len,
                              uint64_t* width_out, const ctok_exec* exec, ctok_stats* stats) {
  if (!tc || !o || !d_doc_off || !d_row_len || !width_out || (n_bytes && !d_utf8))
    return fail(CTOK_E_ARG, "null argument");
  ctok* t = const_cast<ctok*>(tc);
  return run([&] {
    double t0 = now_ms();
    const uint32_t f = o->flags;
    const bool pairs = f & CTOK_P_PAIRS;
    if (pairs && (n_docs & 1)) throw_err(CTOK_E_ARG, "CTOK_P_PAIRS needs an even number of documents");
    const uint64_t rows = pairs ? n_docs / 2 : n_docs;
    if (rows >= 0xFFFFFFFFull) throw_err(CTOK_E_ARG, "too many rows");
    const bool add_special = f & CTOK_P_ADD_SPECIAL;
    if (add_special && t->pp_items.size() > (size_t)kPadMaxItems)
      throw_err(CTOK_E_UNSUPPORTED, "post-processor template with more than 16 items");
    int dev = exec ? exec->device : 0;
    DeviceState* ds = device_state(t, dev);
    std::lock_guard<std::recursive_mutex> lk(ds->mu);
    HIPTRY(hipSetDevice(dev));
    hipStream_t s = exec && exec->stream ? (hipStream_t)exec->stream : ds->stream;
    const bool timing = exec && (exec->flags & CTOK_F_TIMING);
    // 1. encode (encode_to_encoding flavour: no added-token split)
    const uint64_t cap_ids = ctok_ids_bound(t, n_bytes, n_docs);
    ds->pad_ids.ensure(cap_ids);
    ds->pad_tokoff.ensure(n_docs + 1);
    ctok_stats st{};
    encode_device(t, ds, d_utf8, d_doc_off, n_docs, n_bytes, ds->pad_ids.p, ds->pad_ids.cap, ds->pad_tokoff.p, s,
                  timing, &st, !add_special);
    // 2. row lengths and the longest row
    std::vector<uint32_t> sp;
    for (const auto& e : t->special) sp.push_back(e.second);
    std::sort(sp.begin(), sp.end());
    sp.erase(std::unique(sp.begin(), sp.end()), sp.end());
    ds->pad_special.ensure(sp.size() + 1);
    if (!sp.empty()) HIPTRY(hipMemcpyAsync(ds->pad_special.p, sp.data(), sp.size() * 4, hipMemcpyHostToDevice, s));
    ds->pad_ctr.ensure(4);
    HIPTRY(hipMemsetAsync(ds->pad_ctr.p, 0, 16, s));
    PadWork w{};
    w.ids = ds->pad_ids.p;
    w.tok_off = ds->pad_tokoff.p;
    w.n_rows = (uint32_t)rows;
    w.pairs = pairs ? 1 : 0;
    w.use_tpl = (add_special && t->has_pp && !(f & CTOK_P_NO_POSTPROCESS)) ? 1 : 0;
    w.n_items = w.use_tpl ? (uint32_t)t->pp_items.size() : 0;
    for (uint32_t k = 0; k < w.n_items; k++) w.items[k] = t->pp_items[k];
    w.mark = (add_special && !(f & CTOK_P_NO_POSTPROCESS)) ? 1 : 0;
    w.special_ids = ds->pad_special.p;
    w.n_special = (uint32_t)sp.size();
    w.truncate = (f & CTOK_P_TRUNCATE) ? 1 : 0;
    w.max_len = o->max_length;
    w.target = 0;
    if (f & CTOK_P_PAD_TO_MAX) w.target = o->max_length;
    w.pad_left = (f & CTOK_P_PAD_LEFT) ? 1 : 0;
    w.pad_id = (f & CTOK_P_PAD_ID) ? o->pad_id : ctok_pad_id(t);
    w.row_len = d_row_len;
    w.counters = ds->pad_ctr.p;
    HIPTRY(launch_pad_len(w, s));
    HIPTRY(hipMemcpyAsync(ds->host, ds->pad_ctr.p, 16, hipMemcpyDeviceToHost, s));
    spin_sync(ds, s);
    const uint64_t longest = ((volatile uint64_t*)ds->host)[0];
    const uint32_t dropped = ((volatile uint32_t*)ds->host)[2];
    if (w.use_tpl && dropped)
      throw_err(CTOK_E_PANIC, "attempt to subtract with overflow: the post-processor template drops ids (reference src/huggingface/mod.rs:378)");
    if ((f & CTOK_P_PAD_LONGEST) && !(f & CTOK_P_PAD_TO_MAX)) {
      w.target = longest;  // every row padded to the longest: row_len again
      HIPTRY(launch_pad_len(w, s));
    }
    const uint64_t width = std::max<uint64_t>(longest, w.target);
    *width_out = width;
    w.width = width;
    if (rows * width > cap) {
      HIPTRY(hipStreamSynchronize(s));
      throw_err(CTOK_E_CAPACITY, "cap too small: *width_out holds the row width needed");
    }
    if (rows * width && !d_ids) throw_err(CTOK_E_ARG, "null ids");
    w.out_ids = d_ids;
    w.out_attn = d_attn;
    w.out_type = d_type;
    w.out_special = d_special;
    HIPTRY(launch_pad_rows(w, s));
    spin_sync(ds, s);
    if (stats) {
      *stats = st;
      stats->ms_total = now_ms() - t0;
    }
  });
}

int ctok_encode_padded(const ctok* tc, const uint8_t* utf8, const uint64_t* doc_off, uint64_t n_docs,
                       const ctok_pad_opts* o, uint32_t* ids, uint32_t* attn, uint32_t* type, uint32_t* special,
                       uint64_t cap, uint64_t* row_len, uint64_t* width_out, const ctok_exec* exec, ctok_stats* stats) {
  if (!tc || !o || !doc_off || !row_len || !width_out) return fail(CTOK_E_ARG, "null argument");
  ctok* t = const_cast<ctok*>(tc);
  return run([&] {
    if (doc_off[0] != 0) throw_err(CTOK_E_ARG, "doc_off[0] must be 0");
    for (uint64_t d = 0; d < n_docs; d++)
      if (doc_off[d + 1] < doc_off[d]) throw_err(CTOK_E_ARG, "doc_off must be non-decreasing");
    const uint64_t B = doc_off[n_docs];
    if (B && !utf8) throw_err(CTOK_E_ARG, "null text");
    const uint64_t rows = (o->flags & CTOK_P_PAIRS) ? n_docs / 2 : n_docs;
    int dev = exec ? exec->device : 0;
    DeviceState* ds = device_state(t, dev);
    // held from staging to readback: another thread's call on this device cannot overwrite the
    // staged inputs or the outputs in between (the nested device call locks again, recursively)
    std::lock_guard<std::recursive_mutex> lk(ds->mu);
    HIPTRY(hipSetDevice(dev));
    hipStream_t s = exec && exec->stream ? (hipStream_t)exec->stream : ds->stream;
    ds->pad_in_text.ensure(B + 16);
    ds->pad_in_off.ensure(n_docs + 1);
    ds->pad_rowlen.ensure(rows + 1);
    for (auto& b : ds->pad_out) b.ensure(cap ? cap : 1);
    if (B) HIPTRY(hipMemcpyAsync(ds->pad_in_text.p, utf8, B, hipMemcpyHostToDevice, s));
    HIPTRY(hipMemsetAsync(ds->pad_in_text.p + B, 0, 16, s));
    HIPTRY(hipMemcpyAsync(ds->pad_in_off.p, doc_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, s));
    ctok_exec ex = exec ? *exec : ctok_exec{};
    ex.stream = s;
    uint64_t width = 0;
    const int rc = ctok_encode_padded_device(t, ds->pad_in_text.p, ds->pad_in_off.p, n_docs, B, o, ds->pad_out[0].p,
                                             attn ? ds->pad_out[1].p : nullptr, type ? ds->pad_out[2].p : nullptr,
                                             special ? ds->pad_out[3].p : nullptr, cap, ds->pad_rowlen.p, &width, &ex,
                                             stats);
    *width_out = width;
    if (rc != CTOK_OK && rc != CTOK_E_CAPACITY) throw_err(rc, g_err);
    HIPTRY(hipMemcpyAsync(row_len, ds->pad_rowlen.p, rows * 8, hipMemcpyDeviceToHost, s));
    if (rc == CTOK_OK && rows * width) {
      const size_t nb = rows * width * 4;
      HIPTRY(hipMemcpyAsync(ids, ds->pad_out[0].p, nb, hipMemcpyDeviceToHost, s));
      if (attn) HIPTRY(hipMemcpyAsync(attn, ds->pad_out[1].p, nb, hipMemcpyDeviceToHost, s));
      if (type) HIPTRY(hipMemcpyAsync(type, ds->pad_out[2].p, nb, hipMemcpyDeviceToHost, s));
      if (special) HIPTRY(hipMemcpyAsync(special, ds->pad_out[3].p, nb, hipMemcpyDeviceToHost, s));
    }
    HIPTRY(hipStreamSynchronize(s));
    if (rc == CTOK_E_CAPACITY) throw_err(CTOK_E_CAPACITY, "cap too small: *width_out holds the row width needed");
  });
}

// Offsets and word ids of encode_to_encoding (src/huggingface/mod.rs:395-480).  The ids and the
// piece starts (the pre-tokenizer's words) come from the GPU encode; the walk that places each
// word in the original text by str::find and each token inside its word is a sequential host
// pass per document, as in the reference.  A word's ids are its piece's ids on the device (k_emit
// leaves every piece's first id for this call), not a sum of token string lengths: with the
// rank-shift quirk (src/bpe.rs:60-69) an id's token string need not be its piece's bytes.
int ctok_encode_offsets(const ctok* tc, const uint8_t* utf8, const uint64_t* doc_off, uint64_t n_docs,
                        uint32_t* ids, uint64_t* offsets, uint32_t* word_ids, uint64_t cap, uint64_t* tok_off,
                        const ctok_exec* exec) {
  if (!tc || !doc_off || !tok_off) return fail(CTOK_E_ARG, "null argument");
  ctok* t = const_cast<ctok*>(tc);
  return run([&] {
    if (doc_off[0] != 0) throw_err(CTOK_E_ARG, "doc_off[0] must be 0");
    for (uint64_t d = 0; d < n_docs; d++)
      if (doc_off[d + 1] < doc_off[d]) throw_err(CTOK_E_ARG, "doc_off must be non-decreasing");
    const uint64_t n_in = doc_off[n_docs];
    if (n_in && !utf8) throw_err(CTOK_E_ARG, "null text");
    const int dev = exec ? exec->device : 0;
    DeviceState* ds = device_state(t, dev);
    std::lock_guard<std::recursive_mutex> lk(ds->mu);
    HIPTRY(hipSetDevice(dev));
    hipStream_t s = exec && exec->stream ? (hipStream_t)exec->stream : ds->stream;
    ds->pad_in_text.ensure(n_in + 16);
    ds->pad_in_off.ensure(n_docs + 1);
    if (n_in) HIPTRY(hipMemcpyAsync(ds->pad_in_text.p, utf8, n_in, hipMemcpyHostToDevice, s));
    HIPTRY(hipMemsetAsync(ds->pad_in_text.p + n_in, 0, 16, s));
    HIPTRY(hipMemcpyAsync(ds->pad_in_off.p, doc_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, s));
    ds->pad_ids.ensure(ctok_ids_bound(t, n_in, n_docs));
    ds->pad_tokoff.ensure(n_docs + 1);
    const uint64_t ntok = encode_device(t, ds, ds->pad_in_text.p, ds->pad_in_off.p, n_docs, n_in, ds->pad_ids.p,
                                        ds->pad_ids.cap, ds->pad_tokoff.p, s, false, nullptr, false, false, true);
    const uint64_t B = ds->last_B;
    const bool norm = ds->last_norm;
    // each piece's first id: tile_tok[tile] (scanned) + tcnt[tile][j] (k_emit with keep_first)
    const uint64_t n_tiles = (B + kTile - 1) / kTile;
    std::vector<uint32_t> hid(ntok), pb((B + 31) / 32), pfirst(n_tiles * kTileSlots), tfirst(n_tiles + 1);
    std::vector<uint64_t> toff(n_docs + 1), noff;
    std::vector<uint8_t> ntext;
    HIPTRY(hipMemcpyAsync(toff.data(), ds->pad_tokoff.p, (n_docs + 1) * 8, hipMemcpyDeviceToHost, s));
    if (ntok) HIPTRY(hipMemcpyAsync(hid.data(), ds->pad_ids.p, ntok * 4, hipMemcpyDeviceToHost, s));
    if (!pb.empty()) HIPTRY(hipMemcpyAsync(pb.data(), ds->pbits.p, pb.size() * 4, hipMemcpyDeviceToHost, s));
    if (n_tiles) {
      HIPTRY(hipMemcpyAsync(pfirst.data(), ds->tcnt.p, pfirst.size() * 4, hipMemcpyDeviceToHost, s));
      HIPTRY(hipMemcpyAsync(tfirst.data(), ds->tile_tok.p, tfirst.size() * 4, hipMemcpyDeviceToHost, s));
    }
    if (norm) {
      ntext.resize(B + 1);
      noff.resize(n_docs + 1);
      if (B) HIPTRY(hipMemcpyAsync(ntext.data(), ds->norm_text.p, B, hipMemcpyDeviceToHost, s));
      HIPTRY(hipMemcpyAsync(noff.data(), ds->norm_off.p, (n_docs + 1) * 8, hipMemcpyDeviceToHost, s));
    }
    HIPTRY(hipStreamSynchronize(s));
    for (uint64_t d = 0; d <= n_docs; d++) tok_off[d] = toff[d];
    if (ntok > cap) throw_err(CTOK_E_CAPACITY, "cap too small: tok_off[n_docs] holds the number of ids needed");
    if (ntok && (!ids || !offsets || !word_ids)) throw_err(CTOK_E_ARG, "null output");
    std::memcpy(ids, hid.data(), ntok * 4);
    // bytes_to_unicode (src/pretokenizers.rs:130-153): the UTF-8 of each byte's char
    std::string benc[256];
    {
      int n = 0;
      for (int b = 0; b < 256; b++) {
        const bool keep = (b >= 0x21 && b <= 0x7E) || (b >= 0xA1 && b <= 0xAC) || (b >= 0xAE && b <= 0xFF);
        const std::vector<uint32_t> cp{keep ? (uint32_t)b : 256u + (uint32_t)n++};
        benc[b] = encode_utf8(cp, 0, 1);
      }
    }
    auto is_start = [&](uint64_t g) { return (pb[g >> 5] >> (g & 31)) & 1u; };
    // first id of the piece starting at byte g, the j-th piece of its tile
    auto first_id = [&](uint64_t g, uint32_t j) { return (uint64_t)tfirst[g / kTile] + pfirst[(g / kTile) * kTileSlots + j]; };
    // documents are independent: contiguous ranges over host threads, each with its own cache
    auto walk = [&](uint64_t d_begin, uint64_t d_end) {
    std::unordered_map<uint32_t, std::pair<uint32_t, uint32_t>> tlen;  // id -> (bytes, chars) of its token string
    auto token_len = [&](uint32_t id) {
      auto it = tlen.find(id);
      if (it != tlen.end()) return it->second;
      auto jt = t->id_to_token.find(id);
      uint32_t nb = 0, nc = 0;
      if (jt != t->id_to_token.end()) {
        nb = (uint32_t)jt->second.size();
        for (unsigned char c : jt->second) nc += (c & 0xC0) != 0x80;
      }
      return tlen.emplace(id, std::make_pair(nb, nc)).first->second;
    };
    std::string word;
    uint64_t jpos = ~0ull;  // the next piece's start and its index in its tile
    uint32_t jcur = 0;
    for (uint64_t d = d_begin; d < d_end; d++) {
      const uint8_t* o = utf8 + doc_off[d];
      const uint64_t olen = doc_off[d + 1] - doc_off[d];
      const uint64_t g0 = norm ? noff[d] : doc_off[d], g1 = norm ? noff[d + 1] : doc_off[d + 1];
      const uint8_t* nt = norm ? ntext.data() + g0 : o;
      const std::string_view orig((const char*)o, olen);
      uint64_t search = 0, k = toff[d], widx = 0;
      // j: the piece's index within its tile (pieces start in text order; a tile's first piece is
      // 0), carried over from the previous document's last piece
      uint32_t j = 0;
      if (g0 < g1) {
        if (jpos == g0) j = jcur;
        else
          for (uint64_t x = (g0 / kTile) * kTile; x < g0; x++) j += is_start(x);
      }
      for (uint64_t p = g0; p < g1;) {
        uint64_t q = p + 1;
        while (q < g1 && !is_start(q)) q++;
        // the piece's ids: up to the next piece's first id (the next doc's first piece, or the end)
        uint64_t nq = q;
        while (nq < B && !is_start(nq)) nq++;
        const uint32_t jn = nq < B && nq / kTile == p / kTile ? j + 1 : 0;
        const uint64_t k_end = nq < B ? first_id(nq, jn) : ntok;
        if (first_id(p, j) != k) throw_err(CTOK_E_DEVICE, "offsets: piece ids out of order");
        word.clear();
        uint64_t kept = 0;  // bytes whose char is in the vocab (the others are dropped, src/bpe.rs:94-97)
        for (uint64_t i = p; i < q; i++) {
          const uint8_t b = nt[i - g0];
          word += benc[b];
          kept += t->byte2id[b] >= 0;
        }
        size_t lead = 0;  // trim_start_matches('Ġ' | '▁')
        while (true) {
          if (word.compare(lead, 2, "\xC4\xA0") == 0) lead += 2;
          else if (word.compare(lead, 3, "\xE2\x96\x81") == 0) lead += 3;
          else break;
        }
        const std::string_view find = lead < word.size() ? std::string_view(word).substr(lead) : std::string_view(word);
        if (search < olen && (o[search] & 0xC0) == 0x80)
          throw_err(CTOK_E_PANIC, "byte index " + std::to_string(search) +
                                      " is not a char boundary (reference src/huggingface/mod.rs:464 slices the text there)");
        const size_t pos = orig.substr(search).find(find);
        uint64_t ws, we;
        if (pos != std::string_view::npos) {
          ws = search + pos;
          we = ws + find.size();
        } else {
          ws = search;
          we = std::min<uint64_t>(ws + word.size(), olen);
        }
        search = we;
        uint64_t at = ws;
        (void)kept;
        if (k_end > toff[d + 1]) throw_err(CTOK_E_DEVICE, "offsets: ids and words disagree");
        for (; k < k_end; k++) {
          const auto L = token_len(hid[k]);
          const uint64_t e = std::min<uint64_t>(at + L.first, we);
          offsets[2 * k] = at;
          offsets[2 * k + 1] = e;
          word_ids[k] = (uint32_t)widx;
          at = e;
        }
        widx++;
        p = q;
        j = jn;
        jpos = nq;
        jcur = jn;
      }
      if (k != toff[d + 1]) throw_err(CTOK_E_DEVICE, "offsets: ids and words disagree");
    }
    };
    const unsigned nth = n_docs < 256 ? 1u : std::min(16u, usable_cpus_once());
    std::vector<std::exception_ptr> errs(nth);
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nth; w++) {
      const uint64_t a = n_docs * w / nth, b = n_docs * (w + 1) / nth;
      auto job = [&, w, a, b] {
        try {
          walk(a, b);
        } catch (...) {
          errs[w] = std::current_exception();
        }
      };
      if (w + 1 < nth) th.emplace_back(job);
      else job();
    }
    for (auto& x : th) x.join();
    for (auto& e : errs)  // the error of the lowest document range
      if (e) std::rethrow_exception(e);
  });
}

}  // extern "C"
