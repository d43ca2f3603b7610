#include "core/util.h"

#include <algorithm>
#include <cstring>

#include <openssl/evp.h>

#include <cctype>
#include <cstring>

namespace gcsb {



static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(const void* data, size_t n) {
  const auto* p = static_cast<const uint8_t*>(data);
  std::string out;
  out.reserve((n + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 2 < n; i += 3) {
    uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
    out += kB64[v >> 18];
    out += kB64[(v >> 12) & 63];
    out += kB64[(v >> 6) & 63];
    out += kB64[v & 63];
  }
  if (i + 1 == n) {
    uint32_t v = p[i] << 16;
    out += kB64[v >> 18];
    out += kB64[(v >> 12) & 63];
    out += "==";
  } else if (i + 2 == n) {
    uint32_t v = (p[i] << 16) | (p[i + 1] << 8);
    out += kB64[v >> 18];
    out += kB64[(v >> 12) & 63];
    out += kB64[(v >> 6) & 63];
    out += '=';
  }
  return out;
}

std::string base64_encode(std::string_view s) { return base64_encode(s.data(), s.size()); }

bool base64_decode(std::string_view in, std::string* out) {
  int8_t rev[256];
  std::memset(rev, -1, sizeof(rev));
  for (int i = 0; i < 64; ++i) rev[static_cast<uint8_t>(kB64[i])] = static_cast<int8_t>(i);
  rev[static_cast<uint8_t>('-')] = 62;  // url-safe alphabet accepted too
  rev[static_cast<uint8_t>('_')] = 63;
  out->clear();
  uint32_t acc = 0;
  int bits = 0;
  for (char c : in) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ') continue;
    int8_t v = rev[static_cast<uint8_t>(c)];
    if (v < 0) return false;
    acc = (acc << 6) | static_cast<uint32_t>(v);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out->push_back(static_cast<char>((acc >> bits) & 0xff));
    }
  }
  return true;
}

std::string base64url_encode(std::string_view s) {
  std::string b = base64_encode(s);
  while (!b.empty() && b.back() == '=') b.pop_back();
  for (char& c : b) {
    if (c == '+') c = '-';
    else if (c == '/') c = '_';
  }
  return b;
}

std::string url_encode(std::string_view s, bool keep_slash) {
  static const char hex[] = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~' || (keep_slash && c == '/')) {
      out += static_cast<char>(c);
    } else {
      out += '%';
      out += hex[c >> 4];
      out += hex[c & 15];
    }
  }
  return out;
}

std::string url_decode(std::string_view s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && std::isxdigit(static_cast<unsigned char>(s[i + 1])) &&
        std::isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out += static_cast<char>(std::stoi(std::string(s.substr(i + 1, 2)), nullptr, 16));
      i += 2;
    } else if (s[i] == '+') {
      out += ' ';
    } else {
      out += s[i];
    }
  }
  return out;
}

std::string to_lower(std::string_view s) {
  std::string o(s);
  for (char& c : o) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return o;
}

std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t' || s.front() == '\r' || s.front() == '\n'))
    s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r' || s.back() == '\n'))
    s.remove_suffix(1);
  return s;
}

std::vector<std::string_view> split(std::string_view s, char sep) {
  std::vector<std::string_view> out;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || s[i] == sep) {
      out.push_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  return out;
}

bool starts_with(std::string_view s, std::string_view p) { return s.substr(0, p.size()) == p; }

bool iequals(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i])))
      return false;
  return true;
}

std::vector<std::pair<std::string, std::string>> parse_query(std::string_view q) {
  std::vector<std::pair<std::string, std::string>> out;
  if (q.empty()) return out;
  for (auto kv : split(q, '&')) {
    if (kv.empty()) continue;
    size_t eq = kv.find('=');
    if (eq == std::string_view::npos)
      out.emplace_back(url_decode(kv), "");
    else
      out.emplace_back(url_decode(kv.substr(0, eq)), url_decode(kv.substr(eq + 1)));
  }
  return out;
}

uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
void put_be32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 24);
  p[1] = uint8_t(v >> 16);
  p[2] = uint8_t(v >> 8);
  p[3] = uint8_t(v);
}

std::string md5_digest(const void* data, size_t n) {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_Digest(data, n, md, &len, EVP_md5(), nullptr);
  return std::string(reinterpret_cast<char*>(md), len);
}

std::string json_escape(std::string_view s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          o += buf;
        } else {
          o += c;
        }
    }
  }
  return o;
}

static size_t json_find_value(std::string_view json, std::string_view key) {
  std::string pat = "\"" + std::string(key) + "\"";
  size_t p = 0;
  while ((p = json.find(pat, p)) != std::string_view::npos) {
    size_t q = p + pat.size();
    while (q < json.size() && (json[q] == ' ' || json[q] == '\n' || json[q] == '\t' || json[q] == '\r')) ++q;
    if (q < json.size() && json[q] == ':') {
      ++q;
      while (q < json.size() && (json[q] == ' ' || json[q] == '\n' || json[q] == '\t' || json[q] == '\r')) ++q;
      return q;
    }
    p = q;
  }
  return std::string_view::npos;
}

bool json_get_string(std::string_view json, std::string_view key, std::string* out) {
  size_t q = json_find_value(json, key);
  if (q == std::string_view::npos || q >= json.size() || json[q] != '"') return false;
  out->clear();
  for (size_t i = q + 1; i < json.size(); ++i) {
    char c = json[i];
    if (c == '"') return true;
    if (c == '\\' && i + 1 < json.size()) {
      char e = json[++i];
      switch (e) {
        case 'n': *out += '\n'; break;
        case 't': *out += '\t'; break;
        case 'r': *out += '\r'; break;
        case 'u':
          if (i + 4 < json.size()) {
            int cp = std::stoi(std::string(json.substr(i + 1, 4)), nullptr, 16);
            if (cp < 0x80) *out += static_cast<char>(cp);
            else if (cp < 0x800) {
              *out += static_cast<char>(0xC0 | (cp >> 6));
              *out += static_cast<char>(0x80 | (cp & 0x3F));
            } else {
              *out += static_cast<char>(0xE0 | (cp >> 12));
              *out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
              *out += static_cast<char>(0x80 | (cp & 0x3F));
            }
            i += 4;
          }
          break;
        default: *out += e;
      }
    } else {
      *out += c;
    }
  }
  return false;
}

bool json_get_int(std::string_view json, std::string_view key, int64_t* out) {
  size_t q = json_find_value(json, key);
  if (q == std::string_view::npos) return false;
  bool quoted = q < json.size() && json[q] == '"';
  if (quoted) ++q;
  size_t e = q;
  while (e < json.size() && (std::isdigit(static_cast<unsigned char>(json[e])) || json[e] == '-')) ++e;
  if (e == q) return false;
  *out = std::stoll(std::string(json.substr(q, e - q)));
  return true;
}

}  // namespace gcsb
