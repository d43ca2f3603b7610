// Go `flag` package compatible command-line parsing for the native tools.
//
// The reference tools are Go binaries using the standard `flag` package
// (e.g. reference benchmark-script/ssd_test/main.go:18-38), which accepts
// -name value, -name=value, --name value, --name=value, and bare -b / -b=false
// for booleans, stops at the first non-flag argument or "--", exits 2 with
// "flag provided but not defined: -x" for unknown flags and 0 for -h/-help.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <string>
#include <vector>

namespace gcsb {

class GoFlags {
 public:
  explicit GoFlags(std::string prog) : prog_(std::move(prog)) {}

  std::string* String(const std::string& name, const std::string& dflt, const std::string& usage) {
    auto* p = new std::string(dflt);
    add(name, usage, "string", "\"" + dflt + "\"", false, [p](const std::string& v) { *p = v; return true; });
    return p;
  }
  int64_t* Int(const std::string& name, int64_t dflt, const std::string& usage) {
    auto* p = new int64_t(dflt);
    add(name, usage, "int", std::to_string(dflt), false, [p](const std::string& v) { return parse_int(v, p); });
    return p;
  }
  double* Float(const std::string& name, double dflt, const std::string& usage) {
    auto* p = new double(dflt);
    char b[64];
    std::snprintf(b, sizeof(b), "%g", dflt);
    add(name, usage, "float", b, false, [p](const std::string& v) {
      char* end = nullptr;
      *p = std::strtod(v.c_str(), &end);
      return end && *end == '\0' && !v.empty();
    });
    return p;
  }
  bool* Bool(const std::string& name, bool dflt, const std::string& usage) {
    auto* p = new bool(dflt);
    add(name, usage, "", dflt ? "true" : "false", true, [p](const std::string& v) {
      if (v == "1" || v == "t" || v == "T" || v == "true" || v == "TRUE" || v == "True") *p = true;
      else if (v == "0" || v == "f" || v == "F" || v == "false" || v == "FALSE" || v == "False") *p = false;
      else return false;
      return true;
    });
    return p;
  }

  // Parses argv; exits like Go's flag.ExitOnError.
  void Parse(int argc, char** argv) {
    int i = 1;
    for (; i < argc; ++i) {
      std::string a = argv[i];
      if (a.size() < 2 || a[0] != '-') break;
      if (a == "--") {
        ++i;
        break;
      }
      std::string body = a.substr(a[1] == '-' ? 2 : 1);
      if (body.empty() || body[0] == '-' || body[0] == '=') fail("bad flag syntax: " + a);
      std::string name = body, value;
      bool has_value = false;
      size_t eq = body.find('=');
      if (eq != std::string::npos) {
        name = body.substr(0, eq);
        value = body.substr(eq + 1);
        has_value = true;
      }
      if (name == "h" || name == "help") {
        if (!flags_.count(name)) {
          usage();
          std::exit(0);
        }
      }
      auto it = flags_.find(name);
      if (it == flags_.end()) fail("flag provided but not defined: -" + name);
      Flag& f = it->second;
      if (f.is_bool) {
        if (!has_value) value = "true";
      } else if (!has_value) {
        if (i + 1 >= argc) fail("flag needs an argument: -" + name);
        value = argv[++i];
      }
      if (!f.set(value))
        fail("invalid value \"" + value + "\" for flag -" + name + ": parse error");
    }
    for (; i < argc; ++i) args_.push_back(argv[i]);
  }
  const std::vector<std::string>& Args() const { return args_; }

  void usage() const {
    std::fprintf(stderr, "Usage of %s:\n", prog_.c_str());
    for (const auto& kv : flags_) {
      const Flag& f = kv.second;
      std::fprintf(stderr, "  -%s%s%s\n    \t%s", kv.first.c_str(), f.type.empty() ? "" : " ", f.type.c_str(),
                   f.usage.c_str());
      if (!(f.is_bool && f.dflt == "false") && f.dflt != "\"\"" && f.dflt != "0")
        std::fprintf(stderr, " (default %s)", f.dflt.c_str());
      std::fprintf(stderr, "\n");
    }
  }

 private:
  struct Flag {
    std::string usage, type, dflt;
    bool is_bool;
    std::function<bool(const std::string&)> set;
  };
  static bool parse_int(const std::string& v, int64_t* out) {
    if (v.empty()) return false;
    char* end = nullptr;
    long long x = std::strtoll(v.c_str(), &end, 0);  // Go accepts 0x / 0 prefixes
    if (!end || *end != '\0') return false;
    *out = x;
    return true;
  }
  void add(const std::string& name, const std::string& usage, const std::string& type, const std::string& dflt,
           bool is_bool, std::function<bool(const std::string&)> set) {
    flags_[name] = Flag{usage, type, dflt, is_bool, std::move(set)};
  }
  [[noreturn]] void fail(const std::string& msg) const {
    std::fprintf(stderr, "%s\n", msg.c_str());
    usage();
    std::exit(2);
  }
  std::string prog_;
  std::map<std::string, Flag> flags_;
  std::vector<std::string> args_;
};

}  // namespace gcsb
