// Minimal JSON value + recursive-descent parser (no third-party deps in the image). Enough for the
// reference's substitution rule collections (substitutions/*.json, ~2 MB) and our strategy files.
#pragma once
#include <cctype>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ffcore {

struct Json {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;

  const Json& at(const std::string& k) const {
    for (auto& kv : obj)
      if (kv.first == k) return kv.second;
    throw std::runtime_error("json: missing key " + k);
  }
  const Json* find(const std::string& k) const {
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  int as_int() const { return (int)num; }
  double as_num() const { return num; }
  const std::string& as_str() const { return str; }
};

class JsonParser {
 public:
  explicit JsonParser(const std::string& s) : s_(s) {}
  Json parse() {
    Json v = value();
    ws();
    if (i_ != s_.size()) throw err("trailing data");
    return v;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;

  std::runtime_error err(const char* m) const {
    return std::runtime_error(std::string("json parse error: ") + m + " at " + std::to_string(i_));
  }
  void ws() {
    while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) ++i_;
  }
  Json value() {
    ws();
    if (i_ >= s_.size()) throw err("eof");
    char c = s_[i_];
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') {
      Json j;
      j.kind = Json::STR;
      j.str = string();
      return j;
    }
    if (c == 't' || c == 'f') {
      Json j;
      j.kind = Json::BOOL;
      if (s_.compare(i_, 4, "true") == 0) { j.b = true; i_ += 4; }
      else if (s_.compare(i_, 5, "false") == 0) { j.b = false; i_ += 5; }
      else throw err("bad literal");
      return j;
    }
    if (c == 'n') {
      if (s_.compare(i_, 4, "null") != 0) throw err("bad literal");
      i_ += 4;
      return Json();
    }
    return number();
  }
  Json number() {
    size_t st = i_;
    if (s_[i_] == '-' || s_[i_] == '+') ++i_;
    while (i_ < s_.size() && (std::isdigit((unsigned char)s_[i_]) || s_[i_] == '.' || s_[i_] == 'e' ||
                              s_[i_] == 'E' || s_[i_] == '-' || s_[i_] == '+'))
      ++i_;
    if (st == i_) throw err("expected value");
    Json j;
    j.kind = Json::NUM;
    j.num = std::strtod(s_.c_str() + st, nullptr);
    return j;
  }
  std::string string() {
    std::string out;
    ++i_;  // opening quote
    while (i_ < s_.size() && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\' && i_ < s_.size()) {
        char e = s_[i_++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': i_ += 4; out += '?'; break;
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    if (i_ >= s_.size()) throw err("unterminated string");
    ++i_;
    return out;
  }
  Json array() {
    Json j;
    j.kind = Json::ARR;
    ++i_;
    ws();
    if (s_[i_] == ']') { ++i_; return j; }
    while (true) {
      j.arr.push_back(value());
      ws();
      if (s_[i_] == ',') { ++i_; continue; }
      if (s_[i_] == ']') { ++i_; break; }
      throw err("expected , or ]");
    }
    return j;
  }
  Json object() {
    Json j;
    j.kind = Json::OBJ;
    ++i_;
    ws();
    if (s_[i_] == '}') { ++i_; return j; }
    while (true) {
      ws();
      if (s_[i_] != '"') throw err("expected key");
      std::string k = string();
      ws();
      if (s_[i_] != ':') throw err("expected :");
      ++i_;
      j.obj.emplace_back(k, value());
      ws();
      if (s_[i_] == ',') { ++i_; continue; }
      if (s_[i_] == '}') { ++i_; break; }
      throw err("expected , or }");
    }
    return j;
  }
};

inline Json parse_json(const std::string& s) { return JsonParser(s).parse(); }

}  // namespace ffcore
