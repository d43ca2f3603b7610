// Minimal JSON DOM (parse + serialize) for the JSON API (list / metadata /
// upload initiation) on both client and fake-server sides.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace gcsb {

class Json {
 public:
  enum Type { kNull, kBool, kNumber, kString, kArray, kObject };
  Json() = default;
  static Json parse(std::string_view s);  // throws std::runtime_error
  static Json object() { Json j; j.type_ = kObject; return j; }
  static Json array() { Json j; j.type_ = kArray; return j; }
  static Json str(std::string s) { Json j; j.type_ = kString; j.s_ = std::move(s); return j; }
  static Json num(double d) { Json j; j.type_ = kNumber; j.d_ = d; return j; }
  static Json boolean(bool b) { Json j; j.type_ = kBool; j.b_ = b; return j; }

  Type type() const { return type_; }
  bool is_object() const { return type_ == kObject; }
  bool is_array() const { return type_ == kArray; }
  bool is_string() const { return type_ == kString; }
  const std::string& as_string() const { return s_; }
  double as_number() const { return d_; }
  bool as_bool() const { return b_; }
  const std::vector<Json>& items() const { return arr_; }
  const std::vector<std::pair<std::string, Json>>& members() const { return obj_; }
  const Json* get(std::string_view key) const;
  std::string get_string(std::string_view key, const std::string& dflt = "") const;
  // GCS encodes int64 fields as decimal strings.
  int64_t get_int(std::string_view key, int64_t dflt = 0) const;

  Json& set(const std::string& key, Json v);
  Json& push(Json v);
  std::string dump() const;

 private:
  Type type_ = kNull;
  bool b_ = false;
  double d_ = 0;
  std::string s_;
  std::vector<Json> arr_;
  std::vector<std::pair<std::string, Json>> obj_;
  friend class JsonParser;
};

}  // namespace gcsb
