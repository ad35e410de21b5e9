// Chrome-trace spans (mi355x/trace.h).
#include "mi355x/trace.h"

#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>

#include "../kube/json.h"

namespace mi355x::trace {

namespace {

std::string fmt_us(uint64_t ns) {  // microseconds with ns precision, as Python's ns / 1e3
  char b[48];
  std::snprintf(b, sizeof(b), "%llu.%03llu", static_cast<unsigned long long>(ns / 1000),
                static_cast<unsigned long long>(ns % 1000));
  return b;
}

std::string args_json(const Args& args) {
  std::string o = "{";
  for (size_t i = 0; i < args.size(); ++i)
    o += (i ? ", " : "") + json::quote(args[i].first) + ": " + json::quote(args[i].second);
  return o + "}";
}

long tid16() { return static_cast<long>(::syscall(SYS_gettid)) & 0xFFFF; }

}  // namespace

uint64_t now_ns() {
  timespec ts{};
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
}

void Tracer::configure(const std::string& path, size_t max_events) {
  std::lock_guard<std::mutex> lk(mu_);
  path_ = path;
  max_ = max_events ? max_events : 1;
  enabled_ = !path.empty();
}

void Tracer::push(std::string ev) {
  std::lock_guard<std::mutex> lk(mu_);
  events_.push_back(std::move(ev));
  while (events_.size() > max_) events_.pop_front();
}

void Tracer::complete(const std::string& name, const std::string& cat, uint64_t t0_ns, uint64_t dur_ns,
                      const Args& args) {
  if (!enabled_) return;
  push("{\"name\": " + json::quote(name) + ", \"cat\": " + json::quote(cat) + ", \"ph\": \"X\", \"ts\": " +
       fmt_us(t0_ns) + ", \"dur\": " + fmt_us(dur_ns) + ", \"pid\": " + std::to_string(::getpid()) +
       ", \"tid\": " + std::to_string(tid16()) + ", \"args\": " + args_json(args) + "}");
}

void Tracer::instant(const std::string& name, const std::string& cat, const Args& args) {
  if (!enabled_) return;
  push("{\"name\": " + json::quote(name) + ", \"cat\": " + json::quote(cat) + ", \"ph\": \"i\", \"s\": \"p\", \"ts\": " +
       fmt_us(now_ns()) + ", \"pid\": " + std::to_string(::getpid()) + ", \"tid\": " + std::to_string(tid16()) +
       ", \"args\": " + args_json(args) + "}");
}

size_t Tracer::size() const {
  std::lock_guard<std::mutex> lk(mu_);
  return events_.size();
}

std::string Tracer::flush() {
  std::string body, path;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!enabled_ || path_.empty()) return "";
    path = path_;
    body = "{\"traceEvents\": [";
    bool first = true;
    for (const auto& e : events_) {
      body += (first ? "" : ", ") + e;
      first = false;
    }
    body += "], \"displayTimeUnit\": \"ms\"}";
  }
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "w");
  if (!f) return tmp + ": " + std::strerror(errno);
  const bool ok = std::fwrite(body.data(), 1, body.size(), f) == body.size();
  if (std::fclose(f) != 0 || !ok) return tmp + ": write failed";
  if (std::rename(tmp.c_str(), path.c_str()) != 0) return path + ": " + std::strerror(errno);
  return "";
}

Tracer& global() {
  static Tracer t;
  return t;
}

Span::Span(const char* name, const char* cat, Args args) : name_(name), cat_(cat), args_(std::move(args)) {
  on_ = global().enabled();
  if (on_) t0_ = now_ns();
}

Span::~Span() {
  if (on_) global().complete(name_, cat_, t0_, now_ns() - t0_, args_);
}

}  // namespace mi355x::trace
