#pragma once
// Value parsing as Go's flag package does it (both daemons and their glog
// flags), so a command line the reference's binaries accept is accepted here
// with the same value, and one they refuse is refused:
//   bool flags   strconv.ParseBool   ("1 t T TRUE true True 0 f F FALSE false False"; "" is an error)
//   int flags    strconv.ParseInt(s, 0, bits): sign, 0x / 0o / 0b / leading-0 octal
//                prefixes, '_' between digits (Go literal syntax), range-checked
//   float flags  strconv.ParseFloat(s, 64)
#include <cstdint>
#include <string>

namespace mi355x::goflag {

bool parse_bool(const std::string& s, bool* out);
// strconv.ParseInt(s, base, bits): base 0 (Go's int flags) or 10 (glog's
// Level); bits 32 for an int32-backed value, 64 for Go's int on amd64
bool parse_int(const std::string& s, int base, int bits, int64_t* out);
// an int flag stored in a C++ int: Go's range (int64) and ours must both hold
bool parse_int_flag(const std::string& s, int* out);
bool parse_float(const std::string& s, double* out);

}  // namespace mi355x::goflag
