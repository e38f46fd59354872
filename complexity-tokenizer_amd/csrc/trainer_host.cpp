// Host runtime of the INL-BPE trainer behind include/ctok_trainer.h.
//
// Reference: InlBpeTrainer, src/trainer.rs (Complexity-ML/complexity-tokenizer v0.3.3).  This file
// restates its control flow step by step; the O(words) work of every step runs on the GPU:
//   count_batch / count_words (:207-285)   NFC + ByteLevel pre-tokenization on the GPU (the encode
//                                          path's k_segment), word histogram on host threads
//   init_vocab_bytelevel (:288-339)        host (alphabet ids in ascending code point order: the
//                                          reference's HashSet order is randomly seeded)
//   compute_initial_pairs (:341-367)       GPU pair histogram (trainer.hip k_count_pairs)
//   build_heap / learn_merges_heap         host, f32 arithmetic as the reference (this file is
//     (:369-520)                           compiled with -ffp-contract=off); equal scores pop in
//                                          ascending (token_a, token_b) byte order, then ids
//   apply_merge_incremental (:522-590)     GPU pass over all words + per-merge pair-count deltas
//                                          (k_apply_merge, k_drain); the host map takes the deltas
//   save (:600-645)                        serde_json's pretty, key-sorted output
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/ctok_trainer.h"
#include "host_common.h"
#include "trainer_internal.h"

using namespace ctok_train;
using ctok_host::throw_error;

#define HIPT(x)                                                                                         \
  do {                                                                                                  \
    hipError_t e_ = (x);                                                                                \
    if (e_ != hipSuccess) throw_error(CTOK_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace {

template <typename T>
struct DBuf {  // device buffer, grown on demand
  T* p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    HIPT(hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T)));
    cap = n;
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};

// GPT-2 bytes_to_unicode (src/pretokenizers.rs:130-153, src/trainer.rs:20-44): byte -> code point
std::vector<uint32_t> byte_cps() {
  std::vector<uint32_t> cp(256);
  int n = 0;
  for (int b = 0; b < 256; b++) {
    const bool keep = (b >= 0x21 && b <= 0x7E) || (b >= 0xA1 && b <= 0xAC) || (b >= 0xAE && b <= 0xFF);
    cp[b] = keep ? (uint32_t)b : 256u + (uint32_t)n++;
  }
  return cp;
}

std::string utf8_of(uint32_t c) {
  std::string s;
  if (c < 0x80) s += (char)c;
  else if (c < 0x800) { s += (char)(0xC0 | (c >> 6)); s += (char)(0x80 | (c & 63)); }
  else if (c < 0x10000) { s += (char)(0xE0 | (c >> 12)); s += (char)(0x80 | ((c >> 6) & 63)); s += (char)(0x80 | (c & 63)); }
  else { s += (char)(0xF0 | (c >> 18)); s += (char)(0x80 | ((c >> 12) & 63)); s += (char)(0x80 | ((c >> 6) & 63)); s += (char)(0x80 | (c & 63)); }
  return s;
}

// serde_json string escaping (only '"', '\\' and control characters)
void json_str(std::string& o, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) { o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15]; }
        else o += (char)c;
    }
  }
  o += '"';
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct ctok_trainer {
  // TrainerConfig (src/trainer.rs:66-110)
  uint64_t vocab_size = 32000;
  uint32_t min_frequency = 2;
  uint64_t min_word_length = 1;
  float alpha = 0.9f, beta = 0.3f, gate = 0.5f, mu_target = 0.01f, vmax = 10.0f, beta_max = 2.0f;
  std::vector<std::string> specials;
  int device = 0;
  // InlBpeTrainer fields (src/trainer.rs:139-149); they persist across trainings, as there
  std::unordered_map<std::string, uint32_t> vocab;
  std::unordered_map<uint32_t, std::string> vocab_r;
  std::vector<std::pair<std::string, std::string>> merges;
  std::unordered_map<uint32_t, uint64_t> token_freqs;
  std::unordered_map<uint32_t, float> velocity;
  std::unordered_map<uint64_t, int64_t> pair_freqs;  // a << 32 | b
  std::unordered_map<std::string, uint32_t> acc;     // word_freqs_accumulator (raw-byte words)
  std::unordered_map<std::string, uint32_t> local;   // count_words / count_words_from_iter
  std::vector<std::pair<uint64_t, int64_t>> initial; // compute_initial_pairs, sorted (for tests)
  double ms_pairs = 0, ms_merges = 0, ms_heap = 0;
  ctok* pretok = nullptr;  // NFC + ByteLevel pre-tokenizer (its k_segment does the splitting)
  std::vector<uint32_t> cp = byte_cps();
  // device state
  hipStream_t s = nullptr;
  DBuf<uint32_t> tok, wstart, wlen, wfreq, used, n_used;
  DBuf<uint64_t> keys, out_keys;
  DBuf<int64_t> vals, out_vals;
  DBuf<unsigned long long> tok_freq;
  uint32_t mask = 0;

  ~ctok_trainer() {
    if (pretok) ctok_destroy(pretok);
    if (s) (void)hipStreamDestroy(s);
  }

  std::string mapped(const std::string& raw) const {
    std::string m;
    for (unsigned char c : raw) m += utf8_of(cp[c]);
    return m;
  }

  void ensure_pretok() {
    if (pretok) return;
    // the trainer's fixed pipeline: normalizer NFC, pre_tokenizer ByteLevel{add_prefix_space: false}
    // (src/trainer.rs:90-109); the byte alphabet as vocab so that the loader accepts the model
    std::string j = "{\"model\":{\"type\":\"BPE\",\"merges\":[],\"vocab\":{";
    for (int b = 0; b < 256; b++) {
      if (b) j += ',';
      json_str(j, utf8_of(cp[b]));
      j += ':' + std::to_string(b);
    }
    j += "}},\"normalizer\":{\"type\":\"NFC\"},\"pre_tokenizer\":{\"type\":\"ByteLevel\",\"add_prefix_space\":false}}";
    if (ctok_create_from_buffer(j.data(), j.size(), &pretok) != CTOK_OK)
      throw_error(CTOK_E_DEVICE, std::string("trainer pre-tokenizer: ") + ctok_last_error());
  }

  // count_batch / count_words: every word (raw bytes of a piece) of >= min_word_length chars.
  // The texts go to the GPU pre-tokenizer in doc-aligned chunks of about kCountChunk bytes (a
  // longer text is a chunk by itself): one encode call is limited to 3.75 GiB and sizes its
  // workspace from its text, while count_words streams any amount (src/trainer.rs:265-285).
  void count(const uint8_t* utf8, const uint64_t* off, uint64_t n, std::unordered_map<std::string, uint32_t>& into) {
    if (!n) return;
    if (off[0] != 0) throw_error(CTOK_E_ARG, "offsets[0] must be 0");
    ensure_pretok();
    uint64_t chunk = 256ull << 20;
    if (const char* e = getenv("CTOK_TRAIN_CHUNK_BYTES")) chunk = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    std::vector<uint64_t> coff;
    for (uint64_t d0 = 0; d0 < n;) {
      uint64_t d1 = d0 + 1;  // at least one text per chunk
      while (d1 < n && off[d1 + 1] - off[d0] <= chunk) d1++;
      coff.resize(d1 - d0 + 1);
      for (uint64_t i = d0; i <= d1; i++) coff[i - d0] = off[i] - off[d0];
      count_chunk(utf8 + off[d0], coff.data(), d1 - d0, into);
      d0 = d1;
    }
  }

  void count_chunk(const uint8_t* utf8, const uint64_t* off, uint64_t n, std::unordered_map<std::string, uint32_t>& into) {
    std::vector<uint8_t> text;
    std::vector<uint64_t> noff;
    std::vector<uint32_t> pb;
    ctok_host::pretokenize(pretok, device, utf8, off, n, text, noff, pb);
    auto is_start = [&](uint64_t g) { return (pb[g >> 5] >> (g & 31)) & 1u; };
    const unsigned nth = n < 64 ? 1u : std::min(16u, ctok_host::usable_cpus());
    std::vector<std::unordered_map<std::string, uint32_t>> part(nth);
    auto walk = [&](unsigned w) {
      auto& m = part[w];
      for (uint64_t d = n * w / nth; d < n * (w + 1) / nth; d++) {
        for (uint64_t p = noff[d]; p < noff[d + 1];) {
          uint64_t q = p + 1;
          while (q < noff[d + 1] && !is_start(q)) q++;
          if (q - p >= min_word_length) m[std::string((const char*)text.data() + p, q - p)]++;  // chars == bytes
          p = q;
        }
      }
    };
    std::vector<std::thread> th;
    for (unsigned w = 1; w < nth; w++) th.emplace_back(walk, w);
    walk(0);
    for (auto& x : th) x.join();
    for (auto& m : part)
      for (auto& kv : m) into[kv.first] += kv.second;
  }

  // train_from_word_freqs (src/trainer.rs:231-243) on raw-byte words
  void train(const std::vector<std::pair<std::string, uint32_t>>& wf) {
    ms_pairs = ms_merges = ms_heap = 0;
    if (!s) {
      HIPT(hipSetDevice(device));
      HIPT(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    HIPT(hipSetDevice(device));
    // init_vocab_bytelevel (:288-339)
    uint32_t next_id = 0;
    for (const auto& t : specials) {
      vocab[t] = next_id;
      vocab_r[next_id] = t;
      next_id++;
    }
    bool seen[256] = {false};
    for (const auto& w : wf)
      for (unsigned char c : w.first) seen[c] = true;
    std::vector<uint32_t> chars;
    for (int b = 0; b < 256; b++)
      if (seen[b]) chars.push_back(cp[b]);
    std::sort(chars.begin(), chars.end());
    for (uint32_t c : chars) {
      const std::string t = utf8_of(c);
      if (!vocab.count(t)) {
        vocab[t] = next_id;
        vocab_r[next_id] = t;
        next_id++;
      }
    }
    uint32_t byte_id[256];
    for (int b = 0; b < 256; b++) {
      auto it = vocab.find(utf8_of(cp[b]));
      byte_id[b] = it == vocab.end() ? ~0u : it->second;
    }
    std::vector<uint32_t> h_tok, h_start{0}, h_len, h_freq;
    for (const auto& w : wf) {
      for (unsigned char c : w.first) {
        h_tok.push_back(byte_id[c]);
        token_freqs[byte_id[c]] += w.second;
      }
      h_len.push_back((uint32_t)w.first.size());
      h_start.push_back((uint32_t)h_tok.size());
      h_freq.push_back(w.second);
    }
    if (h_tok.size() >= 0xFFFFFFF0ull) throw_error(CTOK_E_ARG, "more than 2^32 word tokens");
    for (const auto& kv : vocab) velocity[kv.second] = 0.0f;
    const uint64_t T = h_tok.size(), W = wf.size();
    // device words and the pair table (capacity > every key set a pass can insert: <= T initial
    // pairs, <= 4 keys per merged occurrence)
    tok.ensure(T + 1);
    wstart.ensure(W + 1);
    wlen.ensure(W + 1);
    wfreq.ensure(W + 1);
    uint64_t cap = 1024;
    while (cap < 4 * T + 1024) cap <<= 1;
    if (cap > (1ull << 31)) throw_error(CTOK_E_ARG, "training set too large for one device pair table");
    keys.ensure(cap);
    vals.ensure(cap);
    used.ensure(cap);
    out_keys.ensure(cap);
    out_vals.ensure(cap);
    n_used.ensure(1);
    tok_freq.ensure(1);
    mask = (uint32_t)(cap - 1);
    if (T) HIPT(hipMemcpyAsync(tok.p, h_tok.data(), T * 4, hipMemcpyHostToDevice, s));
    HIPT(hipMemcpyAsync(wstart.p, h_start.data(), (W + 1) * 4, hipMemcpyHostToDevice, s));
    if (W) HIPT(hipMemcpyAsync(wlen.p, h_len.data(), W * 4, hipMemcpyHostToDevice, s));
    if (W) HIPT(hipMemcpyAsync(wfreq.p, h_freq.data(), W * 4, hipMemcpyHostToDevice, s));
    HIPT(hipMemsetAsync(keys.p, 0xFF, cap * 8, s));
    HIPT(hipMemsetAsync(vals.p, 0, cap * 8, s));
    HIPT(hipMemsetAsync(n_used.p, 0, 4, s));
    HIPT(hipMemsetAsync(tok_freq.p, 0, 8, s));
    Words Wd{tok.p, wstart.p, wlen.p, wfreq.p, (uint32_t)W};
    PairTable Td{keys.p, vals.p, mask, used.p, n_used.p};
    // compute_initial_pairs (:341-367)
    double t0 = now_ms();
    HIPT(launch_count_pairs(Wd, Td, s));
    std::vector<std::pair<uint64_t, int64_t>> got;
    drain(Td, got);
    pair_freqs.clear();
    for (const auto& kv : got) pair_freqs[kv.first] = kv.second;
    initial = got;
    std::sort(initial.begin(), initial.end());
    ms_pairs = now_ms() - t0;
    learn_merges(Wd, Td);
  }

  // used slots -> host (key, count) list; the table is left empty
  void drain(const PairTable& Td, std::vector<std::pair<uint64_t, int64_t>>& out) {
    HIPT(launch_drain(Td, (uint64_t)mask + 1, out_keys.p, out_vals.p, s));
    uint32_t n = 0;
    unsigned long long tf = 0;
    HIPT(hipMemcpyAsync(&n, n_used.p, 4, hipMemcpyDeviceToHost, s));
    HIPT(hipMemcpyAsync(&tf, tok_freq.p, 8, hipMemcpyDeviceToHost, s));
    HIPT(hipStreamSynchronize(s));
    last_tok_freq = tf;
    std::vector<uint64_t> k(n);
    std::vector<int64_t> v(n);
    if (n) {
      HIPT(hipMemcpyAsync(k.data(), out_keys.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
      HIPT(hipMemcpyAsync(v.data(), out_vals.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    }
    HIPT(hipMemsetAsync(n_used.p, 0, 4, s));
    HIPT(hipMemsetAsync(tok_freq.p, 0, 8, s));
    HIPT(hipStreamSynchronize(s));
    out.resize(n);
    for (uint32_t i = 0; i < n; i++) out[i] = {k[i], v[i]};
  }
  unsigned long long last_tok_freq = 0;

  struct Cand {
    float score;
    uint32_t a, b;
  };

  // build_heap (:369-405): the pairs with freq > 0 in pop order
  std::vector<Cand> build_heap() {
    uint64_t total = 0;
    for (const auto& kv : token_freqs) total += kv.second;
    const float mu = mu_target * (float)total;
    const float beta_c = std::fmax(std::fmin(beta, beta_max), 0.0f);
    std::vector<Cand> h;
    h.reserve(pair_freqs.size());
    auto tf = [&](uint32_t id) {
      auto it = token_freqs.find(id);
      return it == token_freqs.end() ? 0.0f : (float)it->second;
    };
    auto vel = [&](uint32_t id) {
      auto it = velocity.find(id);
      return it == velocity.end() ? 0.0f : it->second;
    };
    for (const auto& kv : pair_freqs) {
      if (kv.second <= 0) continue;
      const uint32_t a = (uint32_t)(kv.first >> 32), b = (uint32_t)kv.first;
      const float base = (float)kv.second;
      const float ea = tf(a) - mu, eb = tf(b) - mu;
      const float t_a = alpha * vel(a), u_a = beta_c * ea;
      const float t_b = alpha * vel(b), u_b = beta_c * eb;
      const float van = std::fmin(std::fmax(t_a - u_a, -vmax), vmax);
      const float vbn = std::fmin(std::fmax(t_b - u_b, -vmax), vmax);
      const float adj = gate * (van + vbn);
      h.push_back({base - adj, a, b});
    }
    std::sort(h.begin(), h.end(), [&](const Cand& x, const Cand& y) {
      if (x.score != y.score) return x.score > y.score;
      const std::string &xa = vocab_r[x.a], &ya = vocab_r[y.a];
      if (xa != ya) return xa < ya;
      const std::string &xb = vocab_r[x.b], &yb = vocab_r[y.b];
      if (xb != yb) return xb < yb;
      return x.a != y.a ? x.a < y.a : x.b < y.b;
    });
    return h;
  }

  // learn_merges_heap (:407-520)
  void learn_merges(const Words& Wd, const PairTable& Td) {
    std::vector<std::pair<uint64_t, int64_t>> deltas;
    while (vocab.size() < vocab_size) {
      double t0 = now_ms();
      const std::vector<Cand> heap = build_heap();
      ms_heap += now_ms() - t0;
      size_t hi = 0;
      for (int it = 0; it < 100; it++) {
        if (vocab.size() >= vocab_size) break;
        const Cand* best = nullptr;
        while (hi < heap.size()) {  // pop, skipping stale entries
          const Cand& c = heap[hi++];
          auto f = pair_freqs.find(((uint64_t)c.a << 32) | c.b);
          if (f != pair_freqs.end() && f->second > 0) {
            best = &c;
            break;
          }
        }
        if (!best) break;
        const uint32_t a = best->a, b = best->b;
        const std::string ta = vocab_r.at(a), tb = vocab_r.at(b);
        const std::string merged = ta + tb;
        const uint32_t new_id = (uint32_t)vocab.size();
        vocab[merged] = new_id;
        vocab_r[new_id] = merged;
        merges.emplace_back(ta, tb);
        // apply_merge_incremental (:522-590): GPU pass + deltas
        t0 = now_ms();
        pair_freqs.erase(((uint64_t)a << 32) | b);
        HIPT(launch_apply_merge(Wd, Td, a, b, new_id, tok_freq.p, s));
        drain(Td, deltas);
        const uint64_t new_tf = last_tok_freq;
        for (const auto& kv : deltas) pair_freqs[kv.first] += kv.second;
        auto sat = [&](uint32_t id) {
          auto f = token_freqs.find(id);
          if (f != token_freqs.end()) f->second = f->second > new_tf ? f->second - new_tf : 0;
        };
        sat(a);
        sat(b);
        token_freqs[new_id] = new_tf;
        for (const auto& kv : deltas) {  // retain(v > 0): only the touched entries can change
          auto f = pair_freqs.find(kv.first);
          if (f != pair_freqs.end() && f->second <= 0) pair_freqs.erase(f);
        }
        ms_merges += now_ms() - t0;
        const float va = velocity.count(a) ? velocity[a] : 0.0f, vb = velocity.count(b) ? velocity[b] : 0.0f;
        velocity[new_id] = (va + vb) / 2.0f;
      }
      bool any = false;
      for (const auto& kv : pair_freqs)
        if (kv.second > 0) { any = true; break; }
      if (!any) break;
    }
  }

  // save (:600-645): serde_json::to_string_pretty of a json! value (maps are key-sorted)
  std::string to_json() const {
    std::string o = "{\n  \"added_tokens\": [";
    for (size_t i = 0; i < specials.size(); i++) {
      o += i ? ",\n    {\n" : "\n    {\n";
      o += "      \"content\": ";
      json_str(o, specials[i]);
      o += ",\n      \"id\": " + std::to_string(i) +
           ",\n      \"lstrip\": false,\n      \"normalized\": false,\n      \"rstrip\": false,\n"
           "      \"single_word\": false,\n      \"special\": true\n    }";
    }
    o += specials.empty() ? "]" : "\n  ]";
    o += ",\n  \"decoder\": {\n    \"type\": \"ByteLevel\"\n  },\n  \"model\": {\n    \"merges\": [";
    for (size_t i = 0; i < merges.size(); i++) {
      o += i ? ",\n      " : "\n      ";
      json_str(o, merges[i].first + " " + merges[i].second);
    }
    o += merges.empty() ? "]" : "\n    ]";
    o += ",\n    \"type\": \"BPE\",\n    \"vocab\": {";
    std::map<std::string, uint32_t> sorted(vocab.begin(), vocab.end());
    bool first = true;
    for (const auto& kv : sorted) {
      o += first ? "\n      " : ",\n      ";
      first = false;
      json_str(o, kv.first);
      o += ": " + std::to_string(kv.second);
    }
    o += sorted.empty() ? "}" : "\n    }";
    o += "\n  },\n  \"pre_tokenizer\": {\n    \"add_prefix_space\": false,\n    \"type\": \"ByteLevel\",\n"
         "    \"use_regex\": true\n  },\n  \"version\": \"1.0\"\n}";
    return o;
  }
};

namespace {
std::vector<std::pair<std::string, uint32_t>> retained(std::unordered_map<std::string, uint32_t>& m, uint32_t min_f) {
  std::vector<std::pair<std::string, uint32_t>> v;
  for (auto& kv : m)
    if (kv.second >= min_f) v.emplace_back(kv.first, kv.second);
  std::sort(v.begin(), v.end());  // (the reference's order is HashMap order; results do not depend on it)
  m.clear();
  return v;
}
}  // namespace

extern "C" {

int ctok_trainer_create(const ctok_trainer_config* cfg, ctok_trainer** out) {
  if (!cfg || !out) return ctok_host::run_guarded([] { throw_error(CTOK_E_ARG, "null argument"); });
  *out = nullptr;
  return ctok_host::run_guarded([&] {
    auto tr = std::make_unique<ctok_trainer>();
    tr->vocab_size = cfg->vocab_size;
    tr->min_frequency = cfg->min_frequency;
    tr->min_word_length = cfg->min_word_length;
    tr->alpha = cfg->inl_alpha;
    tr->beta = cfg->inl_beta;
    tr->gate = cfg->inl_gate;
    tr->mu_target = cfg->inl_mu_target;
    tr->vmax = cfg->inl_velocity_max;
    tr->beta_max = cfg->inl_beta_max;
    tr->device = cfg->device;
    if (cfg->n_special && !cfg->special_off) throw_error(CTOK_E_ARG, "null special_off");
    if (cfg->n_special && cfg->special_off[cfg->n_special] && !cfg->special) throw_error(CTOK_E_ARG, "null special");
    for (uint64_t i = 0; i < cfg->n_special; i++)
      tr->specials.emplace_back(cfg->special + cfg->special_off[i], cfg->special_off[i + 1] - cfg->special_off[i]);
    *out = tr.release();
  });
}

void ctok_trainer_destroy(ctok_trainer* tr) { delete tr; }

int ctok_trainer_count(ctok_trainer* tr, const uint8_t* utf8, const uint64_t* off, uint64_t n_texts,
                       int into_accumulator) {
  return ctok_host::run_guarded([&] {
    if (!tr || (n_texts && !off)) throw_error(CTOK_E_ARG, "null argument");
    tr->count(utf8, off, n_texts, into_accumulator ? tr->acc : tr->local);
  });
}

int ctok_trainer_clear_counts(ctok_trainer* tr, int accumulator) {
  return ctok_host::run_guarded([&] {
    if (!tr) throw_error(CTOK_E_ARG, "null argument");
    (accumulator ? tr->acc : tr->local).clear();
  });
}

int ctok_trainer_train(ctok_trainer* tr, int from_accumulator) {
  return ctok_host::run_guarded([&] {
    if (!tr) throw_error(CTOK_E_ARG, "null argument");
    tr->train(retained(from_accumulator ? tr->acc : tr->local, tr->min_frequency));
  });
}

int ctok_trainer_train_words(ctok_trainer* tr, const uint8_t* words, const uint64_t* word_off, const uint32_t* freqs,
                             uint64_t n_words) {
  return ctok_host::run_guarded([&] {
    if (!tr || (n_words && (!word_off || !freqs))) throw_error(CTOK_E_ARG, "null argument");
    std::unordered_map<std::string, uint32_t> m;
    for (uint64_t i = 0; i < n_words; i++)
      m[std::string((const char*)words + word_off[i], word_off[i + 1] - word_off[i])] += freqs[i];
    std::vector<std::pair<std::string, uint32_t>> v(m.begin(), m.end());
    std::sort(v.begin(), v.end());
    tr->train(v);
  });
}

uint64_t ctok_trainer_vocab_size(const ctok_trainer* tr) { return tr ? tr->vocab.size() : 0; }
uint64_t ctok_trainer_num_merges(const ctok_trainer* tr) { return tr ? tr->merges.size() : 0; }

int ctok_trainer_json(const ctok_trainer* tr, char* buf, size_t cap, size_t* len) {
  return ctok_host::run_guarded([&] {
    if (!tr || !len || (cap && !buf)) throw_error(CTOK_E_ARG, "null argument");
    const std::string j = tr->to_json();
    *len = j.size();
    if (buf) std::memcpy(buf, j.data(), std::min(cap, j.size()));
  });
}

int ctok_trainer_save(const ctok_trainer* tr, const char* path) {
  return ctok_host::run_guarded([&] {
    if (!tr || !path) throw_error(CTOK_E_ARG, "null argument");
    std::ofstream f(path, std::ios::binary);
    if (!f) throw_error(CTOK_E_IO, std::string("cannot create ") + path);
    const std::string j = tr->to_json();
    f.write(j.data(), (std::streamsize)j.size());
    if (!f) throw_error(CTOK_E_IO, std::string("cannot write ") + path);
  });
}

int ctok_trainer_initial_pairs(const ctok_trainer* tr, uint32_t* a, uint32_t* b, int64_t* count, uint64_t cap,
                               uint64_t* n) {
  return ctok_host::run_guarded([&] {
    if (!tr || !n || (cap && (!a || !b || !count))) throw_error(CTOK_E_ARG, "null argument");
    *n = tr->initial.size();
    for (uint64_t i = 0; i < std::min<uint64_t>(cap, tr->initial.size()); i++) {
      a[i] = (uint32_t)(tr->initial[i].first >> 32);
      b[i] = (uint32_t)tr->initial[i].first;
      count[i] = tr->initial[i].second;
    }
  });
}

int ctok_trainer_timing(const ctok_trainer* tr, double* ms_pairs, double* ms_merges, double* ms_heap) {
  return ctok_host::run_guarded([&] {
    if (!tr) throw_error(CTOK_E_ARG, "null argument");
    if (ms_pairs) *ms_pairs = tr->ms_pairs;
    if (ms_merges) *ms_merges = tr->ms_merges;
    if (ms_heap) *ms_heap = tr->ms_heap;
  });
}

}  // extern "C"
