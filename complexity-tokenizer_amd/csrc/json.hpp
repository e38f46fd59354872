// Minimal strict JSON reader for tokenizer.json (RFC 8259 subset that serde_json accepts).
//
// The reference deserialises tokenizer.json with serde_json into `TokenizerJson`
// (src/huggingface/mod.rs:32-51).  This DOM keeps what the loader needs to reproduce serde's
// accept/reject decisions on the fields the encode path reads: integer vs float numbers
// (u32 fields reject floats and negatives), \uXXXX escapes with surrogate pairs (a lone
// surrogate is an error, as in serde_json), and object member order.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ctj {

struct Value;
using Member = std::pair<std::string, Value>;

struct Value {
  enum Kind { Null, Bool, Int, Float, String, Array, Object } kind = Null;
  bool b = false;
  bool neg = false;       // Int: sign
  uint64_t u = 0;         // Int: magnitude (saturates; `big` set when it does)
  bool big = false;
  double f = 0;
  std::string s;
  std::vector<Value> arr;
  std::vector<Member> obj;

  const Value* get(const char* key) const {  // last occurrence wins (HashMap semantics)
    const Value* r = nullptr;
    for (const auto& m : obj)
      if (m.first == key) r = &m.second;
    return r;
  }
  bool is_u32() const { return kind == Int && !neg && !big && u <= 0xFFFFFFFFull; }
};

class ParseError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), e_(p + n), b_(p) {}

  Value parse() {
    Value v;
    ws();
    value(v, 0);
    ws();
    if (p_ != e_) fail("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  const char* b_;

  [[noreturn]] void fail(const char* what) {
    size_t line = 1, col = 1;
    for (const char* q = b_; q < p_ && q < e_; ++q) {
      if (*q == '\n') { ++line; col = 1; } else { ++col; }
    }
    throw ParseError(std::string(what) + " at line " + std::to_string(line) + " column " + std::to_string(col));
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e_ - p_) >= n && memcmp(p_, s, n) == 0) { p_ += n; return true; }
    return false;
  }
  void value(Value& v, int depth) {
    if (depth > 128) fail("recursion limit exceeded");
    if (p_ >= e_) fail("EOF while parsing a value");
    char c = *p_;
    if (c == '{') {
      v.kind = Value::Object; ++p_; ws();
      if (p_ < e_ && *p_ == '}') { ++p_; return; }
      for (;;) {
        ws();
        if (p_ >= e_ || *p_ != '"') fail("key must be a string");
        Member m;
        string(m.first);
        ws();
        if (p_ >= e_ || *p_ != ':') fail("expected `:`");
        ++p_; ws();
        value(m.second, depth + 1);
        v.obj.push_back(std::move(m));
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; return; }
        fail("expected `,` or `}`");
      }
    } else if (c == '[') {
      v.kind = Value::Array; ++p_; ws();
      if (p_ < e_ && *p_ == ']') { ++p_; return; }
      for (;;) {
        ws();
        v.arr.emplace_back();
        value(v.arr.back(), depth + 1);
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; return; }
        fail("expected `,` or `]`");
      }
    } else if (c == '"') {
      v.kind = Value::String;
      string(v.s);
    } else if (lit("null")) {
      v.kind = Value::Null;
    } else if (lit("true")) {
      v.kind = Value::Bool; v.b = true;
    } else if (lit("false")) {
      v.kind = Value::Bool; v.b = false;
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      number(v);
    } else {
      fail("expected value");
    }
  }
  void number(Value& v) {
    const char* s = p_;
    bool neg = false;
    if (*p_ == '-') { neg = true; ++p_; }
    if (p_ >= e_ || !(*p_ >= '0' && *p_ <= '9')) fail("invalid number");
    if (*p_ == '0' && p_ + 1 < e_ && p_[1] >= '0' && p_[1] <= '9') fail("invalid number");
    uint64_t u = 0;
    bool big = false;
    while (p_ < e_ && *p_ >= '0' && *p_ <= '9') {
      uint64_t d = (uint64_t)(*p_ - '0');
      if (u > (UINT64_MAX - d) / 10) big = true; else u = u * 10 + d;
      ++p_;
    }
    bool isf = false;
    if (p_ < e_ && *p_ == '.') {
      isf = true; ++p_;
      if (p_ >= e_ || !(*p_ >= '0' && *p_ <= '9')) fail("invalid number");
      while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    }
    if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
      isf = true; ++p_;
      if (p_ < e_ && (*p_ == '+' || *p_ == '-')) ++p_;
      if (p_ >= e_ || !(*p_ >= '0' && *p_ <= '9')) fail("invalid number");
      while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    }
    if (isf) {
      v.kind = Value::Float;
      v.f = strtod(std::string(s, p_).c_str(), nullptr);
    } else {
      v.kind = Value::Int; v.neg = neg && u != 0; v.u = u; v.big = big;
    }
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) { o += (char)cp; }
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) fail("EOF while parsing a string");
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("invalid escape");
    }
    return v;
  }
  void string(std::string& out) {
    ++p_;  // opening quote
    for (;;) {
      const char* run = p_;
      while (p_ < e_ && *p_ != '"' && *p_ != '\\' && (unsigned char)*p_ >= 0x20) ++p_;
      out.append(run, p_);
      if (p_ >= e_) fail("EOF while parsing a string");
      char c = *p_;
      if (c == '"') { ++p_; break; }
      if ((unsigned char)c < 0x20) fail("control character (\\u0000-\\u001F) found while parsing a string");
      ++p_;  // backslash
      if (p_ >= e_) fail("EOF while parsing a string");
      char k = *p_++;
      switch (k) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (e_ - p_ < 6 || p_[0] != '\\' || p_[1] != 'u') fail("lone leading surrogate in hex escape");
            p_ += 2;
            uint32_t lo = hex4();
            if (lo < 0xDC00 || lo > 0xDFFF) fail("lone leading surrogate in hex escape");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            fail("lone leading surrogate in hex escape");
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("invalid escape");
      }
    }
  }
};

inline Value parse(const char* p, size_t n) { return Parser(p, n).parse(); }

}  // namespace ctj
