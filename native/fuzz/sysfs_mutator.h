// Rewrites a private copy of a generated sysfs tree from a fuzz input and
// restores it afterwards (fuzz_sysfs, fuzz_labels). Input: records of
// [u16 file index][u16 length][bytes]; length 0xFFFF removes the file.
#pragma once

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <map>
#include <optional>
#include <sstream>
#include <string>
#include <vector>

#include "fuzz_common.h"
#include "mi355x/sysfs.h"

namespace mi355x::fuzz {

class SysfsMutator {
 public:
  // every regular file under `root` but the CPU / NUMA trees (views only)
  explicit SysfsMutator(std::string root) : root_(std::move(root)) {
    walk("");
    std::sort(files_.begin(), files_.end());
    if (files_.size() < 100) fail("fixture tree too small", root_);
  }
  const std::string& root() const { return root_; }

  void apply(const uint8_t* data, size_t size) {
    size_t i = 0;
    while (i + 4 <= size) {
      const size_t idx = (data[i] | (data[i + 1] << 8)) % files_.size();
      const size_t len = data[i + 2] | (data[i + 3] << 8);
      i += 4;
      const std::string p = root_ + "/" + files_[idx];
      if (!saved_.count(p)) saved_[p] = slurp(p);
      if (len == 0xFFFF) {
        ::unlink(p.c_str());
        continue;
      }
      const size_t n = std::min(len, size - i);
      put(p, std::string(reinterpret_cast<const char*>(data) + i, n));
      i += n;
    }
  }

  void restore() {
    for (const auto& [p, orig] : saved_) {
      if (orig) put(p, *orig);
      else ::unlink(p.c_str());
    }
    saved_.clear();
  }

 private:
  void walk(const std::string& rel) {
    const std::string abs = rel.empty() ? root_ : root_ + "/" + rel;
    for (const auto& name : list_dir(abs)) {
      const std::string r = rel.empty() ? name : rel + "/" + name;
      struct stat st {};
      if (::lstat((root_ + "/" + r).c_str(), &st) != 0 || S_ISLNK(st.st_mode)) continue;
      if (S_ISDIR(st.st_mode)) {
        if (r == "devices/system") continue;
        walk(r);
      } else if (S_ISREG(st.st_mode)) {
        files_.push_back(r);
      }
    }
  }
  static std::optional<std::string> slurp(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    if (!f) return std::nullopt;
    std::ostringstream o;
    o << f.rdbuf();
    return o.str();
  }
  static void put(const std::string& p, const std::string& data) {
    std::ofstream f(p, std::ios::binary | std::ios::trunc);
    f << data;
  }

  std::string root_;
  std::vector<std::string> files_;
  std::map<std::string, std::optional<std::string>> saved_;
};

}  // namespace mi355x::fuzz
