// glog for the native daemons: the flag set and output rules of
// github.com/golang/glog, which the reference binaries link
// (vendor/github.com/golang/glog/glog_flags.go:388-397, glog_file.go), so a
// DaemonSet's `-logtostderr=false -log_dir=/var/log/amdgpu -v=5` keeps working
// when it switches to the native binaries:
//
//   -logtostderr          everything to stderr, no files (this project's default,
//                         as the reference images pass -logtostderr=true)
//   -logtostderr=false    one file per severity under -log_dir (default $TMPDIR
//                         or /tmp) named <program>.<host>.<user>.log.<SEV>.
//                         <yyyymmdd-hhmmss>.<pid>, created on first use with
//                         glog's header, plus a <program>.<SEV> symlink; a
//                         record goes to its severity's file and every lower one
//   -stderrthreshold=S    with files: records at or above S are copied to stderr
//   -alsologtostderr      with files: every record is copied to stderr
//   -v=N / -vmodule=p=N   VLOG(n) enabled globally / per source file (glob on the
//                         file's base name without extension, or on the path
//                         when the pattern contains '/')
//   -log_link=DIR         also a <program>.<SEV> symlink in DIR to each log file
//                         (glog_file.go:45,133-137)
//   -logbuflevel=N        accepted (glog_file.go:46); records are never buffered:
//                         each is written and flushed as it is logged
//   -log_backtrace_at=f:N a record logged from file f, line N carries a stack trace
//   -log_format=json      one JSON object per record instead of the glog line:
//                         {"ts", "level", "src", "msg"} plus the record's fields,
//                         as the Python CLIs' JsonFormatter (utils/log.py) writes
//
// Thread-safe; line format "Lmmdd hh:mm:ss.uuuuuu tid file:line] msg".
#pragma once

#include <string>
#include <utility>
#include <vector>

namespace mi355x::glog {

enum Severity { kInfo = 0, kWarning = 1, kError = 2, kFatal = 3 };

struct Options {
  int v = 0;
  bool logtostderr = true;
  bool alsologtostderr = false;
  int stderrthreshold = kError;
  std::string log_dir;
  std::string vmodule;
  std::string log_backtrace_at;
  std::string program;  // file name prefix (default: basename of argv[0])
  bool json = false;    // -log_format=json
  std::string log_link; // -log_link
  int logbuflevel = 0;  // -logbuflevel (accepted, see above)
  bool discard = false; // not a flag: drop every record (fuzz targets, embedders)
};

using Fields = std::vector<std::pair<std::string, std::string>>;

// One command-line flag: true if `name` is a glog flag (then *err may be set
// for a bad value). `has_value` = "-name=value" form; boolean flags accept
// a bare "-name".
bool parse_flag(const std::string& name, const std::string& value, bool has_value, Options* o, std::string* err);
bool is_bool_flag(const std::string& name);
// true for every flag parse_flag handles (defined-flag check before a value is consumed)
bool is_flag(const std::string& name);

// Applies the options ("" or an error, e.g. a malformed -vmodule).
std::string init(const Options& o);

void log(Severity sev, const char* file, int line, const char* fmt, ...) __attribute__((format(printf, 4, 5)));
// A record with structured fields: "msg k=v ..." in glog format, extra keys in JSON
// (utils/log.py info_fields).
void log_fields(Severity sev, const char* file, int line, const std::string& msg, const Fields& fields);
bool vlog_is_on(int level, const char* file);
// path of the current file of `sev` ("" before the first record / with -logtostderr)
std::string file_path(Severity sev);

}  // namespace mi355x::glog

#define MI_LOG(sev, ...) ::mi355x::glog::log(::mi355x::glog::sev, __FILE__, __LINE__, __VA_ARGS__)
#define MI_LOG_FIELDS(sev, msg, ...) \
  ::mi355x::glog::log_fields(::mi355x::glog::sev, __FILE__, __LINE__, msg, ::mi355x::glog::Fields __VA_ARGS__)
#define MI_VLOG(level, ...)                                      \
  do {                                                           \
    if (::mi355x::glog::vlog_is_on(level, __FILE__)) MI_LOG(kInfo, __VA_ARGS__); \
  } while (0)
