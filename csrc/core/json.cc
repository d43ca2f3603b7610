#include "core/json.h"

#include <cmath>
#include <cstdio>
#include <stdexcept>

#include "core/util.h"

namespace gcsb {

class JsonParser {
 public:
  explicit JsonParser(std::string_view s) : s_(s) {}
  Json parse_value() {
    ws();
    if (p_ >= s_.size()) fail("unexpected end");
    char c = s_[p_];
    if (c == '{') return parse_object();
    if (c == '[') return parse_array();
    if (c == '"') return Json::str(parse_string());
    if (c == 't' && s_.substr(p_, 4) == "true") { p_ += 4; return Json::boolean(true); }
    if (c == 'f' && s_.substr(p_, 5) == "false") { p_ += 5; return Json::boolean(false); }
    if (c == 'n' && s_.substr(p_, 4) == "null") { p_ += 4; return Json(); }
    return parse_number();
  }
  void finish() {
    ws();
    if (p_ != s_.size()) fail("trailing characters");
  }

 private:
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() {
    while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\n' || s_[p_] == '\r' || s_[p_] == '\t')) ++p_;
  }
  Json parse_object() {
    Json j = Json::object();
    ++p_;
    ws();
    if (p_ < s_.size() && s_[p_] == '}') { ++p_; return j; }
    for (;;) {
      ws();
      if (p_ >= s_.size() || s_[p_] != '"') fail("expected key");
      std::string k = parse_string();
      ws();
      if (p_ >= s_.size() || s_[p_] != ':') fail("expected ':'");
      ++p_;
      j.obj_.emplace_back(std::move(k), parse_value());
      ws();
      if (p_ < s_.size() && s_[p_] == ',') { ++p_; continue; }
      if (p_ < s_.size() && s_[p_] == '}') { ++p_; return j; }
      fail("expected ',' or '}'");
    }
  }
  Json parse_array() {
    Json j = Json::array();
    ++p_;
    ws();
    if (p_ < s_.size() && s_[p_] == ']') { ++p_; return j; }
    for (;;) {
      j.arr_.push_back(parse_value());
      ws();
      if (p_ < s_.size() && s_[p_] == ',') { ++p_; continue; }
      if (p_ < s_.size() && s_[p_] == ']') { ++p_; return j; }
      fail("expected ',' or ']'");
    }
  }
  std::string parse_string() {
    ++p_;
    std::string out;
    while (p_ < s_.size()) {
      char c = s_[p_++];
      if (c == '"') return out;
      if (c != '\\') { out += c; continue; }
      if (p_ >= s_.size()) break;
      char e = s_[p_++];
      switch (e) {
        case 'n': out += '\n'; break;
        case 't': out += '\t'; break;
        case 'r': out += '\r'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'u': {
          if (p_ + 4 > s_.size()) fail("bad \\u");
          unsigned cp = static_cast<unsigned>(std::stoul(std::string(s_.substr(p_, 4)), nullptr, 16));
          p_ += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && p_ + 6 <= s_.size() && s_[p_] == '\\' && s_[p_ + 1] == 'u') {
            unsigned lo = static_cast<unsigned>(std::stoul(std::string(s_.substr(p_ + 2, 4)), nullptr, 16));
            p_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          if (cp < 0x80) out += static_cast<char>(cp);
          else if (cp < 0x800) { out += static_cast<char>(0xC0 | (cp >> 6)); out += static_cast<char>(0x80 | (cp & 0x3F)); }
          else if (cp < 0x10000) {
            out += static_cast<char>(0xE0 | (cp >> 12));
            out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
            out += static_cast<char>(0x80 | (cp & 0x3F));
          } else {
            out += static_cast<char>(0xF0 | (cp >> 18));
            out += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
            out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
            out += static_cast<char>(0x80 | (cp & 0x3F));
          }
          break;
        }
        default: out += e;
      }
    }
    fail("unterminated string");
  }
  Json parse_number() {
    size_t st = p_;
    while (p_ < s_.size() && (std::isdigit(static_cast<unsigned char>(s_[p_])) || s_[p_] == '-' || s_[p_] == '+' ||
                              s_[p_] == '.' || s_[p_] == 'e' || s_[p_] == 'E'))
      ++p_;
    if (st == p_) fail("unexpected character");
    return Json::num(std::stod(std::string(s_.substr(st, p_ - st))));
  }
  std::string_view s_;
  size_t p_ = 0;
};

Json Json::parse(std::string_view s) {
  JsonParser p(s);
  Json j = p.parse_value();
  p.finish();
  return j;
}

const Json* Json::get(std::string_view key) const {
  for (const auto& kv : obj_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

std::string Json::get_string(std::string_view key, const std::string& dflt) const {
  const Json* j = get(key);
  if (!j) return dflt;
  if (j->type_ == kString) return j->s_;
  if (j->type_ == kNumber) return std::to_string(static_cast<int64_t>(j->d_));
  return dflt;
}

int64_t Json::get_int(std::string_view key, int64_t dflt) const {
  const Json* j = get(key);
  if (!j) return dflt;
  if (j->type_ == kNumber) return static_cast<int64_t>(j->d_);
  if (j->type_ == kString && !j->s_.empty()) {
    try {
      return std::stoll(j->s_);
    } catch (...) {
      return dflt;
    }
  }
  return dflt;
}

Json& Json::set(const std::string& key, Json v) {
  type_ = kObject;
  for (auto& kv : obj_)
    if (kv.first == key) {
      kv.second = std::move(v);
      return kv.second;
    }
  obj_.emplace_back(key, std::move(v));
  return obj_.back().second;
}

Json& Json::push(Json v) {
  type_ = kArray;
  arr_.push_back(std::move(v));
  return arr_.back();
}

std::string Json::dump() const {
  switch (type_) {
    case kNull: return "null";
    case kBool: return b_ ? "true" : "false";
    case kNumber: {
      if (std::floor(d_) == d_ && std::fabs(d_) < 9e15) return std::to_string(static_cast<int64_t>(d_));
      char b[64];
      std::snprintf(b, sizeof(b), "%.17g", d_);
      return b;
    }
    case kString: return "\"" + json_escape(s_) + "\"";
    case kArray: {
      std::string o = "[";
      for (size_t i = 0; i < arr_.size(); ++i) {
        if (i) o += ",";
        o += arr_[i].dump();
      }
      return o + "]";
    }
    case kObject: {
      std::string o = "{";
      for (size_t i = 0; i < obj_.size(); ++i) {
        if (i) o += ",";
        o += "\"" + json_escape(obj_[i].first) + "\":" + obj_[i].second.dump();
      }
      return o + "}";
    }
  }
  return "null";
}

}  // namespace gcsb
