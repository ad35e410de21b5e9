// Go flag-package value parsing (see mi355x/goflag.h).
#include "mi355x/goflag.h"

#include <cctype>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdlib>

namespace mi355x::goflag {

bool parse_bool(const std::string& s, bool* out) {
  if (s == "1" || s == "t" || s == "T" || s == "TRUE" || s == "true" || s == "True") return *out = true, true;
  if (s == "0" || s == "f" || s == "F" || s == "FALSE" || s == "false" || s == "False") return *out = false, true;
  return false;
}

namespace {

int digit_value(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'z') return c - 'a' + 10;
  if (c >= 'A' && c <= 'Z') return c - 'A' + 10;
  return 99;
}

// strconv's underscoreOK: '_' only between digits, or between a base prefix and
// a digit (base 0 parsing)
bool underscores_ok(const std::string& s) {
  char saw = '^';  // '^' start, '0' digit or prefix, '_' underscore, '!' other
  size_t i = 0;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
  bool hex = false;
  if (s.size() - i >= 2 && s[i] == '0') {
    const char b = static_cast<char>(s[i + 1] | 0x20);
    if (b == 'x' || b == 'o' || b == 'b') {
      hex = b == 'x';
      i += 2;
      saw = '0';
    }
  }
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if ((c >= '0' && c <= '9') || (hex && digit_value(c) < 16)) {
      saw = '0';
      continue;
    }
    if (c == '_') {
      if (saw != '0') return false;
      saw = '_';
      continue;
    }
    if (saw == '_') return false;
    saw = '!';
  }
  return saw != '_';
}

}  // namespace

bool parse_int(const std::string& s0, int base0, int bits, int64_t* out) {
  if (s0.empty()) return false;
  const std::string& s = s0;
  bool neg = false;
  size_t i = 0;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  int base = 10;
  if (base0 == 0 && s.size() - i >= 2 && s[i] == '0') {
    const char b = static_cast<char>(s[i + 1] | 0x20);
    if (b == 'x') base = 16, i += 2;
    else if (b == 'o') base = 8, i += 2;
    else if (b == 'b') base = 2, i += 2;
    else base = 8, i += 1;  // leading 0: octal
  }
  bool underscores = false;
  uint64_t v = 0;
  bool any = false;
  const uint64_t limit = bits >= 64 ? (neg ? uint64_t(1) << 63 : (uint64_t(1) << 63) - 1)
                                    : (neg ? uint64_t(1) << (bits - 1) : (uint64_t(1) << (bits - 1)) - 1);
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c == '_' && base0 == 0) {  // base 0: Go literal syntax, checked below
      underscores = true;
      continue;
    }
    const int d = digit_value(c);
    if (d >= base) return false;
    any = true;
    if (v > (limit - static_cast<uint64_t>(d)) / static_cast<uint64_t>(base)) return false;  // out of range
    v = v * static_cast<uint64_t>(base) + static_cast<uint64_t>(d);
  }
  if (!any) return false;  // "", "-", "0x"
  if (underscores && !underscores_ok(s)) return false;
  *out = neg ? static_cast<int64_t>(0 - v) : static_cast<int64_t>(v);
  return true;
}

bool parse_int_flag(const std::string& s, int* out) {
  int64_t v = 0;
  if (!parse_int(s, 0, 64, &v) || v < INT_MIN || v > INT_MAX) return false;
  *out = static_cast<int>(v);
  return true;
}

bool parse_float(const std::string& s, double* out) {
  if (s.empty() || std::isspace(static_cast<unsigned char>(s[0]))) return false;  // strtod would skip these
  if (s.find('_') != std::string::npos) return false;  // only legal in hex floats, which flags never need
  char* end = nullptr;
  errno = 0;
  const double v = std::strtod(s.c_str(), &end);
  if (end == s.c_str() || *end) return false;
  if (errno == ERANGE && std::isinf(v)) return false;  // ParseFloat: value out of range
  *out = v;
  return true;
}

}  // namespace mi355x::goflag
