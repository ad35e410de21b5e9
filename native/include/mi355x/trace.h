// Chrome-trace (chrome://tracing / Perfetto) spans for the native daemon
// (-trace_file): the same events as the Python CLI's tracer
// (rocm_k8s_device_plugin_amd/utils/trace.py). Spans cover the admission path
// (RPC -> allocator) and the health path (sweep -> probe request / process ->
// throughput check), so a slow Allocate or a stuck probe shows on one timeline.
// Events go into a bounded ring and are written as {"traceEvents": [...]} on
// flush (shutdown); timestamps are CLOCK_MONOTONIC microseconds.
#pragma once

#include <atomic>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace mi355x::trace {

using Args = std::vector<std::pair<std::string, std::string>>;

class Tracer {
 public:
  void configure(const std::string& path, size_t max_events = 200000);
  bool enabled() const { return enabled_.load(std::memory_order_relaxed); }
  // a span recorded elsewhere (the gRPC server's RPC events): monotonic ns
  void complete(const std::string& name, const std::string& cat, uint64_t t0_ns, uint64_t dur_ns, const Args& args);
  void instant(const std::string& name, const std::string& cat, const Args& args);
  size_t size() const;
  std::string flush();  // "" or the write error

 private:
  void push(std::string ev);
  std::atomic<bool> enabled_{false};
  std::string path_;
  size_t max_ = 200000;
  mutable std::mutex mu_;
  std::deque<std::string> events_;  // serialised event objects
};

Tracer& global();
uint64_t now_ns();  // CLOCK_MONOTONIC

// RAII span on the global tracer (no cost when tracing is off)
class Span {
 public:
  Span(const char* name, const char* cat, Args args = {});
  ~Span();
  Span(const Span&) = delete;
  Span& operator=(const Span&) = delete;

 private:
  const char* name_;
  const char* cat_;
  Args args_;
  uint64_t t0_ = 0;
  bool on_ = false;
};

}  // namespace mi355x::trace
