// Prometheus metrics for the native daemon: counters, gauges and latency
// histograms with labels, rendered in the text exposition format (0.0.4), and a
// small HTTP/1.0 endpoint for GET /metrics, /healthz and /readyz.
//
// Same names, labels, buckets and text layout as the Python registry
// (rocm_k8s_device_plugin_amd/utils/metrics.py), so dashboards and the alert
// rules in example/monitoring/ work with either entrypoint. The reference
// exposes no metrics (its labeller turns controller-runtime's server off,
// cmd/k8s-node-labeller/main.go:529-532).
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace mi355x::metrics {

using Labels = std::vector<std::pair<std::string, std::string>>;

class Registry {
 public:
  void inc(const std::string& name, const Labels& labels = {}, double v = 1.0, const std::string& help = "");
  void set(const std::string& name, double v, const Labels& labels = {}, const std::string& help = "");
  // one observation in milliseconds (rendered in seconds, as the Python registry does)
  void observe_ms(const std::string& name, double ms, const Labels& labels = {}, const std::string& help = "");
  double value(const std::string& name, const Labels& labels = {}) const;  // counter or gauge, 0 if absent
  uint64_t count(const std::string& name, const Labels& labels = {}) const;  // histogram observations
  std::string render() const;
  void clear();

  static const std::vector<double>& buckets_ms();

 private:
  using Key = std::pair<std::string, Labels>;  // labels sorted by name
  struct Hist {
    std::vector<uint64_t> counts;
    double sum_ms = 0;
    uint64_t n = 0;
  };
  static Key key(const std::string& name, Labels labels);
  mutable std::mutex mu_;
  std::map<Key, double> counters_, gauges_;
  std::map<Key, Hist> hist_;
  void note_help(const std::string& name, const std::string& help);  // caller holds mu_
  std::map<std::string, std::string> help_;
};

Registry& global();

// GET /metrics (render), /healthz and /readyz ("ok", or 503 with the reason
// a check gives), anything else 404; one thread, connections answered one at a
// time with a 5 s read deadline.
class HttpEndpoint {
 public:
  // "" = healthy / ready; anything else is the 503 body. Called on the
  // endpoint's thread, so a check reads only atomics. Unset: always "ok".
  using Check = std::function<std::string()>;
  explicit HttpEndpoint(Registry& reg = global()) : reg_(reg) {}
  ~HttpEndpoint() { stop(); }
  HttpEndpoint(const HttpEndpoint&) = delete;
  HttpEndpoint& operator=(const HttpEndpoint&) = delete;
  // set before start()
  void set_checks(Check healthz, Check readyz) {
    healthz_ = std::move(healthz);
    readyz_ = std::move(readyz);
  }
  // "" on success; port 0 picks a free port (see port())
  std::string start(const std::string& host, int port);
  void stop();
  int port() const { return port_; }
  uint64_t requests() const { return requests_.load(); }

 private:
  void loop();
  Registry& reg_;
  int fd_ = -1, port_ = 0;
  int stop_[2] = {-1, -1};
  std::thread thread_;
  std::atomic<uint64_t> requests_{0};
  Check healthz_, readyz_;
};

}  // namespace mi355x::metrics
