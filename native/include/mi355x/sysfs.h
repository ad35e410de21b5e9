// Root-injectable sysfs reader.
//
// Every path the framework reads is resolved against a caller-supplied sysfs
// root (default "/sys") so the whole discovery stack runs against captured or
// generated fixture trees. The reference hard-codes "/sys" in its discovery
// (internal/pkg/amdgpu/amdgpu.go:449-455,521), which is why it could never be
// fixture-tested; this header is the fix for that.
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

namespace mi355x {

// "key value" pairs of one kfd/sysfs properties file, parsed in a single pass.
// First occurrence of a key wins. Values are kept as raw strings; typed access
// goes through the helpers below so 64-bit unsigned ids (hive_id, unique_id)
// survive intact.
using KeyValues = std::unordered_map<std::string, std::string>;

std::string path_join(const std::string& a, const std::string& b);
std::string trim(const std::string& s);
std::string to_lower(std::string s);
std::string basename(const std::string& p);

std::optional<std::string> read_file(const std::string& path);
std::optional<std::string> read_trimmed(const std::string& path);
std::optional<std::string> read_link(const std::string& path);
bool path_exists(const std::string& path);
bool is_dir(const std::string& path);

// Directory entries (names only, no "." / ".."), sorted lexicographically.
std::vector<std::string> list_dir(const std::string& path);
// Entries whose name starts with `prefix`.
std::vector<std::string> list_dir_prefix(const std::string& path, const std::string& prefix);

// Parse a "key value" per-line file. Returns nullopt if unreadable.
std::optional<KeyValues> parse_kv_file(const std::string& path);

// Integer parsing that accepts decimal and 0x-hex; returns fallback on error.
int64_t parse_i64(const std::string& s, int64_t fallback);
uint64_t parse_u64(const std::string& s, uint64_t fallback);
bool is_all_digits(const std::string& s);

int64_t kv_i64(const KeyValues& kv, const char* key, int64_t fallback);
uint64_t kv_u64(const KeyValues& kv, const char* key, uint64_t fallback);
std::string kv_str(const KeyValues& kv, const char* key, const std::string& fallback = "");

}  // namespace mi355x
