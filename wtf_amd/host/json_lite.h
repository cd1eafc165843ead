// json_lite.h — a small JSON reader/writer for the files this path consumes
// (bdump regs.json, symbol-store.json) and for testcase payloads (tlv packets).
// Values: null, bool, number (kept as double and as the literal text), string,
// array, object (insertion-ordered).
#pragma once
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace jsonl {

struct Value {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;  // String, or the literal of a Number
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  // a key given twice: the last one counts (nlohmann's parser overwrites)
  const Value *find(const std::string &k) const {
    for (auto it = obj.rbegin(); it != obj.rend(); ++it)
      if (it->first == k) return &it->second;
    return nullptr;
  }
  const Value &at(const std::string &k) const {
    const Value *v = find(k);
    if (!v) throw std::runtime_error("json: missing key " + k);
    return *v;
  }
  // nlohmann's get<unsigned integer>: numbers (cast) and booleans, nothing else
  uint64_t num_u64() const {
    if (kind == Number) return str.empty() ? (uint64_t)num : (uint64_t)std::strtoull(str.c_str(), nullptr, 10);
    if (kind == Bool) return b ? 1 : 0;
    throw std::runtime_error("json: not a number");
  }
  const std::vector<Value> &array() const {
    if (kind != Array) throw std::runtime_error("json: not an array");
    return arr;
  }
  // integer view: numbers (exact when written as integers) or "0x.." strings
  uint64_t u64() const {
    if (kind == Number) return str.empty() ? (uint64_t)num : (uint64_t)std::strtoull(str.c_str(), nullptr, 0);
    if (kind == String) return std::strtoull(str.c_str(), nullptr, 0);
    if (kind == Bool) return b ? 1 : 0;
    throw std::runtime_error("json: not an integer");
  }
};

class Parser {
  const char *p_, *e_;

  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) p_++;
  }
  [[noreturn]] void fail(const char *what) { throw std::runtime_error(std::string("json: ") + what); }
  char peek() {
    ws();
    if (p_ >= e_) fail("unexpected end");
    return *p_;
  }
  void expect(char c) {
    if (peek() != c) fail("unexpected character");
    p_++;
  }
  std::string string() {
    expect('"');
    std::string s;
    while (p_ < e_ && *p_ != '"') {
      char c = *p_++;
      if (c != '\\') {
        s += c;
        continue;
      }
      if (p_ >= e_) fail("bad escape");
      c = *p_++;
      switch (c) {
        case 'n': s += '\n'; break;
        case 't': s += '\t'; break;
        case 'r': s += '\r'; break;
        case 'b': s += '\b'; break;
        case 'f': s += '\f'; break;
        case 'u': {
          if (e_ - p_ < 4) fail("bad \\u");
          const unsigned cp = (unsigned)std::strtoul(std::string(p_, 4).c_str(), nullptr, 16);
          p_ += 4;
          if (cp < 0x80) {
            s += (char)cp;
          } else if (cp < 0x800) {
            s += (char)(0xc0 | (cp >> 6));
            s += (char)(0x80 | (cp & 0x3f));
          } else {
            s += (char)(0xe0 | (cp >> 12));
            s += (char)(0x80 | ((cp >> 6) & 0x3f));
            s += (char)(0x80 | (cp & 0x3f));
          }
          break;
        }
        default: s += c; break;
      }
    }
    expect('"');
    return s;
  }
  Value value() {
    Value v;
    const char c = peek();
    if (c == '{') {
      p_++;
      v.kind = Value::Object;
      if (peek() == '}') {
        p_++;
        return v;
      }
      for (;;) {
        std::string k = string();
        expect(':');
        v.obj.emplace_back(std::move(k), value());
        if (peek() == ',') {
          p_++;
          continue;
        }
        expect('}');
        return v;
      }
    }
    if (c == '[') {
      p_++;
      v.kind = Value::Array;
      if (peek() == ']') {
        p_++;
        return v;
      }
      for (;;) {
        v.arr.push_back(value());
        if (peek() == ',') {
          p_++;
          continue;
        }
        expect(']');
        return v;
      }
    }
    if (c == '"') {
      v.kind = Value::String;
      v.str = string();
      return v;
    }
    if (e_ - p_ >= 4 && std::string(p_, 4) == "true") {
      p_ += 4;
      v.kind = Value::Bool;
      v.b = true;
      return v;
    }
    if (e_ - p_ >= 5 && std::string(p_, 5) == "false") {
      p_ += 5;
      v.kind = Value::Bool;
      return v;
    }
    if (e_ - p_ >= 4 && std::string(p_, 4) == "null") {
      p_ += 4;
      return v;
    }
    // RFC 8259 number: -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)? (nlohmann's
    // lexer rejects anything else, leading zeros included)
    const char *s = p_;
    auto digits = [&]() {
      const char *d = p_;
      while (p_ < e_ && std::isdigit((unsigned char)*p_)) p_++;
      return p_ > d;
    };
    if (p_ < e_ && *p_ == '-') p_++;
    if (p_ < e_ && *p_ == '0') {
      p_++;
    } else if (!digits()) {
      fail("bad value");
    }
    if (p_ < e_ && *p_ == '.') {
      p_++;
      if (!digits()) fail("bad number");
    }
    if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
      p_++;
      if (p_ < e_ && (*p_ == '+' || *p_ == '-')) p_++;
      if (!digits()) fail("bad number");
    }
    v.kind = Value::Number;
    v.str.assign(s, p_);
    v.num = std::strtod(v.str.c_str(), nullptr);
    const bool integral = v.str.find_first_of(".eE") == std::string::npos;
    if (!integral) v.str.clear();
    return v;
  }

 public:
  Parser(const char *p, size_t n) : p_(p), e_(p + n) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != e_) fail("trailing characters");
    return v;
  }
};

inline Value parse(const std::string &s) { return Parser(s.data(), s.size()).parse(); }
inline Value parse(const uint8_t *p, size_t n) { return Parser((const char *)p, n).parse(); }

}  // namespace jsonl
