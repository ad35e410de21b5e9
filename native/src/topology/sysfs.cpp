#include "mi355x/sysfs.h"

#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace mi355x {

std::string path_join(const std::string& a, const std::string& b) {
  if (a.empty()) return b;
  if (b.empty()) return a;
  if (a.back() == '/') return b.front() == '/' ? a + b.substr(1) : a + b;
  return b.front() == '/' ? a + b : a + "/" + b;
}

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

std::string to_lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

std::string basename(const std::string& p) {
  std::string s = p;
  while (s.size() > 1 && s.back() == '/') s.pop_back();
  auto pos = s.find_last_of('/');
  return pos == std::string::npos ? s : s.substr(pos + 1);
}

std::optional<std::string> read_file(const std::string& path) {
  // sysfs attributes report st_size 4096 regardless of content, so read in a
  // loop rather than trusting the size.
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return std::nullopt;
  std::string out;
  char buf[4096];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, n);
  bool err = std::ferror(f);
  std::fclose(f);
  if (err) return std::nullopt;
  return out;
}

std::optional<std::string> read_trimmed(const std::string& path) {
  auto r = read_file(path);
  if (!r) return std::nullopt;
  return trim(*r);
}

std::optional<std::string> read_link(const std::string& path) {
  char buf[4096];
  ssize_t n = ::readlink(path.c_str(), buf, sizeof(buf) - 1);
  if (n < 0) return std::nullopt;
  buf[n] = 0;
  return std::string(buf);
}

bool path_exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0;
}

bool is_dir(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> out;
  DIR* d = ::opendir(path.c_str());
  if (!d) return out;
  while (auto* e = ::readdir(d)) {
    if (std::strcmp(e->d_name, ".") == 0 || std::strcmp(e->d_name, "..") == 0) continue;
    out.emplace_back(e->d_name);
  }
  ::closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<std::string> list_dir_prefix(const std::string& path, const std::string& prefix) {
  std::vector<std::string> out;
  for (auto& n : list_dir(path))
    if (n.compare(0, prefix.size(), prefix) == 0) out.push_back(n);
  return out;
}

std::optional<KeyValues> parse_kv_file(const std::string& path) {
  auto content = read_file(path);
  if (!content) return std::nullopt;
  KeyValues kv;
  const std::string& s = *content;
  size_t pos = 0;
  while (pos < s.size()) {
    size_t eol = s.find('\n', pos);
    if (eol == std::string::npos) eol = s.size();
    size_t b = pos;
    while (b < eol && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
    size_t k = b;
    while (k < eol && !std::isspace(static_cast<unsigned char>(s[k]))) ++k;
    if (k > b) {
      size_t v = k;
      while (v < eol && std::isspace(static_cast<unsigned char>(s[v]))) ++v;
      size_t ve = eol;
      while (ve > v && std::isspace(static_cast<unsigned char>(s[ve - 1]))) --ve;
      kv.emplace(s.substr(b, k - b), s.substr(v, ve - v));
    }
    pos = eol + 1;
  }
  return kv;
}

bool is_all_digits(const std::string& s) {
  if (s.empty()) return false;
  for (char c : s)
    if (!std::isdigit(static_cast<unsigned char>(c))) return false;
  return true;
}

int64_t parse_i64(const std::string& s, int64_t fallback) {
  if (s.empty()) return fallback;
  errno = 0;
  char* end = nullptr;
  long long v = std::strtoll(s.c_str(), &end, 0);
  if (errno != 0 || end == s.c_str() || *end != 0) return fallback;
  return static_cast<int64_t>(v);
}

uint64_t parse_u64(const std::string& s, uint64_t fallback) {
  if (s.empty() || s[0] == '-') return fallback;
  errno = 0;
  char* end = nullptr;
  unsigned long long v = std::strtoull(s.c_str(), &end, 0);
  if (errno != 0 || end == s.c_str() || *end != 0) return fallback;
  return static_cast<uint64_t>(v);
}

int64_t kv_i64(const KeyValues& kv, const char* key, int64_t fallback) {
  auto it = kv.find(key);
  return it == kv.end() ? fallback : parse_i64(it->second, fallback);
}

uint64_t kv_u64(const KeyValues& kv, const char* key, uint64_t fallback) {
  auto it = kv.find(key);
  return it == kv.end() ? fallback : parse_u64(it->second, fallback);
}

std::string kv_str(const KeyValues& kv, const char* key, const std::string& fallback) {
  auto it = kv.find(key);
  return it == kv.end() ? fallback : it->second;
}

}  // namespace mi355x
