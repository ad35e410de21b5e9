// glog output rules for the native daemons (see mi355x/glog.h).
#include "mi355x/glog.h"

#include "../kube/json.h"
#include "mi355x/goflag.h"

#include <execinfo.h>
#include <fnmatch.h>
#include <pwd.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

namespace mi355x::glog {
namespace {

const char kSevChar[] = "IWEF";
const char* kSevName[] = {"INFO", "WARNING", "ERROR", "FATAL"};

struct State {
  std::mutex mu;
  Options opt;
  std::vector<std::pair<std::string, int>> vmodule;
  std::string bt_file;
  int bt_line = -1;
  FILE* files[4] = {nullptr, nullptr, nullptr, nullptr};
  std::string paths[4];
};

State& state() {
  static State* s = new State();  // never destroyed: loggable from atexit / other threads
  return *s;
}

std::string base_no_ext(const char* file) {
  const char* b = std::strrchr(file, '/');
  std::string s = b ? b + 1 : file;
  const size_t dot = s.rfind('.');
  return dot == std::string::npos ? s : s.substr(0, dot);
}

std::string stem(const char* file) {
  std::string s = file;
  const size_t slash = s.rfind('/');
  const size_t dot = s.rfind('.');
  return dot != std::string::npos && (slash == std::string::npos || dot > slash) ? s.substr(0, dot) : s;
}

std::string program_name(const Options& o) {
  if (!o.program.empty()) return o.program;
  char buf[4096];
  const ssize_t n = ::readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return "mi355x";
  buf[n] = 0;
  const char* b = std::strrchr(buf, '/');
  return b ? b + 1 : buf;
}

FILE* open_file(State& s, int sev, const tm& lt) {
  const Options& o = s.opt;
  std::string dir = o.log_dir;
  if (dir.empty()) {
    const char* t = std::getenv("TMPDIR");
    dir = t && *t ? t : "/tmp";
  }
  ::mkdir(dir.c_str(), 0755);
  char host[256] = "unknownhost";
  ::gethostname(host, sizeof(host) - 1);
  if (char* dot = std::strchr(host, '.')) *dot = 0;
  std::string user = "unknownuser";
  if (const passwd* pw = ::getpwuid(::getuid())) user = pw->pw_name;
  char stamp[32];
  std::strftime(stamp, sizeof(stamp), "%Y%m%d-%H%M%S", &lt);
  const std::string prog = program_name(o);
  const std::string name =
      prog + "." + host + "." + user + ".log." + kSevName[sev] + "." + stamp + "." + std::to_string(::getpid());
  const std::string path = dir + "/" + name;
  FILE* f = std::fopen(path.c_str(), "a");
  if (!f) return nullptr;
  char created[32];
  std::strftime(created, sizeof(created), "%Y/%m/%d %H:%M:%S", &lt);
  std::fprintf(f,
               "Log file created at: %s\nRunning on machine: %s\nBinary: %s (MI355X-native, C++)\n"
               "Log line format: [IWEF]mmdd hh:mm:ss.uuuuuu threadid file:line] msg\n",
               created, host, prog.c_str());
  const std::string link = dir + "/" + prog + "." + kSevName[sev];
  ::unlink(link.c_str());
  if (::symlink(name.c_str(), link.c_str()) != 0) {
  }
  if (!o.log_link.empty()) {  // glog_file.go:133-137: a link to the full path
    const std::string l2 = o.log_link + "/" + prog + "." + kSevName[sev];
    ::unlink(l2.c_str());
    if (::symlink(path.c_str(), l2.c_str()) != 0) {
    }
  }
  s.paths[sev] = path;
  return f;
}

}  // namespace

bool is_bool_flag(const std::string& name) { return name == "logtostderr" || name == "alsologtostderr"; }

bool is_flag(const std::string& name) {
  static const char* kNames[] = {"logtostderr", "alsologtostderr", "v", "stderrthreshold", "log_dir", "log_link",
                                 "logbuflevel", "vmodule", "log_backtrace_at", "log_format"};
  for (const char* n : kNames)
    if (name == n) return true;
  return false;
}

bool parse_flag(const std::string& name, const std::string& value, bool has_value, Options* o, std::string* err) {
  auto as_bool = [&](bool* out) {
    if (!has_value) *out = true;
    else if (!goflag::parse_bool(value, out)) *err = "invalid boolean value \"" + value + "\" for -" + name;
  };
  if (name == "logtostderr") return as_bool(&o->logtostderr), true;
  if (name == "alsologtostderr") return as_bool(&o->alsologtostderr), true;
  if (name == "v") {  // glog's Level.Set: strconv.Atoi (64-bit), stored as int32 (glog_flags.go:115-130)
    int64_t v = 0;
    if (goflag::parse_int(value, 10, 64, &v))
      o->v = static_cast<int32_t>(static_cast<uint32_t>(static_cast<uint64_t>(v)));
    else
      *err = "invalid value \"" + value + "\" for flag -v";
    return true;
  }
  if (name == "stderrthreshold") {
    // glog's severityFlag.Set (glog_flags.go:341-356): a severity name in any
    // case, else strconv.Atoi; the number becomes a logsink.Severity (int8) and
    // must be INFO..FATAL
    std::string u;
    for (char c : value) u.push_back(static_cast<char>(std::toupper(static_cast<unsigned char>(c))));
    for (int i = 0; i < 4; ++i)
      if (u == kSevName[i]) return o->stderrthreshold = i, true;
    int64_t v = 0;
    if (!goflag::parse_int(value, 10, 64, &v)) {
      *err = "invalid value \"" + value + "\" for flag -stderrthreshold";
      return true;
    }
    const int sev = static_cast<int8_t>(static_cast<uint8_t>(static_cast<uint64_t>(v)));
    if (sev < 0 || sev > 3)
      *err = "invalid value \"" + value + "\" for flag -stderrthreshold: Severity " + std::to_string(v) +
             " out of range (min 0, max 3).";
    else
      o->stderrthreshold = sev;
    return true;
  }
  if (name == "log_dir") return o->log_dir = value, true;
  if (name == "log_link") return o->log_link = value, true;
  if (name == "logbuflevel") {  // an int flag
    if (!goflag::parse_int_flag(value, &o->logbuflevel)) *err = "invalid value \"" + value + "\" for flag -logbuflevel";
    return true;
  }
  if (name == "vmodule") return o->vmodule = value, true;
  if (name == "log_backtrace_at") return o->log_backtrace_at = value, true;
  if (name == "log_format") {
    if (value == "json") o->json = true;
    else if (value == "glog" || value.empty()) o->json = false;
    else *err = "invalid value \"" + value + "\" for flag -log_format (glog | json)";
    return true;
  }
  return false;
}

std::string init(const Options& o) {
  std::vector<std::pair<std::string, int>> vm;
  size_t pos = 0;
  while (pos <= o.vmodule.size() && !o.vmodule.empty()) {
    size_t comma = o.vmodule.find(',', pos);
    if (comma == std::string::npos) comma = o.vmodule.size();
    const std::string part = o.vmodule.substr(pos, comma - pos);
    pos = comma + 1;
    if (part.empty()) continue;
    const size_t eq = part.rfind('=');
    char* end = nullptr;
    if (eq == std::string::npos || eq == 0 || eq + 1 >= part.size())
      return "invalid -vmodule entry \"" + part + "\" (want pattern=N)";
    const long lvl = std::strtol(part.c_str() + eq + 1, &end, 10);
    if (*end) return "invalid -vmodule entry \"" + part + "\" (want pattern=N)";
    vm.emplace_back(part.substr(0, eq), static_cast<int>(lvl));
  }
  std::string bt_file;
  int bt_line = -1;
  if (!o.log_backtrace_at.empty()) {
    const size_t c = o.log_backtrace_at.rfind(':');
    char* end = nullptr;
    if (c == std::string::npos) return "invalid -log_backtrace_at \"" + o.log_backtrace_at + "\" (want file:N)";
    bt_line = static_cast<int>(std::strtol(o.log_backtrace_at.c_str() + c + 1, &end, 10));
    if (*end || bt_line <= 0) return "invalid -log_backtrace_at \"" + o.log_backtrace_at + "\" (want file:N)";
    bt_file = o.log_backtrace_at.substr(0, c);
  }
  State& s = state();
  std::lock_guard<std::mutex> lk(s.mu);
  for (int i = 0; i < 4; ++i) {
    if (s.files[i]) std::fclose(s.files[i]);
    s.files[i] = nullptr;
    s.paths[i].clear();
  }
  s.opt = o;
  s.vmodule = std::move(vm);
  s.bt_file = bt_file;
  s.bt_line = bt_line;
  return "";
}

bool vlog_is_on(int level, const char* file) {
  State& s = state();
  if (s.opt.v >= level) return true;
  if (s.vmodule.empty()) return false;
  const std::string base = base_no_ext(file), st = stem(file);
  for (const auto& [pat, lvl] : s.vmodule) {
    const bool has_slash = pat.find('/') != std::string::npos;
    const bool hit = has_slash ? (fnmatch(pat.c_str(), st.c_str(), 0) == 0 ||
                                  fnmatch(("*/" + pat).c_str(), st.c_str(), 0) == 0)
                               : fnmatch(pat.c_str(), base.c_str(), 0) == 0;
    if (hit) return lvl >= level;
  }
  return false;
}

std::string file_path(Severity sev) {
  State& s = state();
  std::lock_guard<std::mutex> lk(s.mu);
  return s.paths[sev];
}

namespace {

const char* kJsonLevel[4] = {"INFO", "WARNING", "ERROR", "CRITICAL"};  // Python logging level names

void emit(Severity sev, const char* file, int line, const std::string& msg, const Fields& fields) {
  timespec ts{};
  clock_gettime(CLOCK_REALTIME, &ts);
  tm lt{};
  localtime_r(&ts.tv_sec, &lt);
  const char* base = std::strrchr(file, '/');
  base = base ? base + 1 : file;
  State& s = state();
  std::lock_guard<std::mutex> lk(s.mu);
  const Options& o = s.opt;
  if (o.discard) return;
  std::string rec;
  if (o.json) {
    char t[48];
    std::snprintf(t, sizeof(t), "%lld.%06ld", static_cast<long long>(ts.tv_sec), ts.tv_nsec / 1000);
    rec = std::string("{\"ts\": ") + t + ", \"level\": \"" + kJsonLevel[sev] + "\", \"src\": " +
          json::quote(std::string(base) + ":" + std::to_string(line)) + ", \"msg\": " + json::quote(msg);
    for (const auto& [k, v] : fields) rec += ", " + json::quote(k) + ": " + json::quote(v);
  } else {
    char head[128];
    std::snprintf(head, sizeof(head), "%c%02d%02d %02d:%02d:%02d.%06ld %7ld %s:%d] ", kSevChar[sev], lt.tm_mon + 1,
                  lt.tm_mday, lt.tm_hour, lt.tm_min, lt.tm_sec, ts.tv_nsec / 1000,
                  static_cast<long>(::syscall(SYS_gettid)), base, line);
    rec = head + msg;
    for (const auto& [k, v] : fields) rec += " " + k + "=" + v;
  }
  std::string trace;
  if (s.bt_line == line && s.bt_file == base) {
    void* frames[64];
    const int n = ::backtrace(frames, 64);
    if (char** syms = ::backtrace_symbols(frames, n)) {
      for (int i = 2; i < n; ++i) trace += std::string("    ") + syms[i] + "\n";
      std::free(syms);
    }
  }
  if (o.json) {
    if (!trace.empty()) rec += ", \"exc\": " + json::quote(trace);
    rec += "}\n";
  } else {
    rec += "\n" + trace;
  }
  if (o.logtostderr || o.alsologtostderr || sev >= o.stderrthreshold) {
    std::fputs(rec.c_str(), stderr);
    std::fflush(stderr);
  }
  if (!o.logtostderr) {
    for (int i = sev; i >= 0; --i) {  // this severity's file and every lower one
      if (!s.files[i]) s.files[i] = open_file(s, i, lt);
      if (s.files[i]) {
        std::fputs(rec.c_str(), s.files[i]);
        std::fflush(s.files[i]);
      }
    }
  }
}

}  // namespace

void log(Severity sev, const char* file, int line, const char* fmt, ...) {
  char msg[2048];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  emit(sev, file, line, msg, {});
}

void log_fields(Severity sev, const char* file, int line, const std::string& msg, const Fields& fields) {
  emit(sev, file, line, msg, fields);
}

}  // namespace mi355x::glog
