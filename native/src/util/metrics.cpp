// Prometheus registry and /metrics endpoint (mi355x/metrics.h).
#include "mi355x/metrics.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>

namespace mi355x::metrics {

namespace {

// Python's repr() of a float: integral values as "N.0", else the shortest
// representation that round-trips (so both registries render alike).
std::string py_float(double v) {
  if (std::isnan(v)) return "nan";
  if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
  char b[64];
  if (v == std::floor(v) && std::fabs(v) < 1e16) {
    std::snprintf(b, sizeof(b), "%.1f", v);
    return b;
  }
  for (int p = 1; p <= 17; ++p) {
    std::snprintf(b, sizeof(b), "%.*g", p, v);
    if (std::strtod(b, nullptr) == v) break;
  }
  return b;
}

std::string g_fmt(double v) {  // Python's f"{v:g}"
  char b[64];
  std::snprintf(b, sizeof(b), "%g", v);
  return b;
}

std::string escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '\\' || c == '"') o += '\\', o += c;
    else if (c == '\n') o += "\\n";
    else o += c;
  }
  return o;
}

std::string lbl(const std::vector<std::pair<std::string, std::string>>& labels, const char* extra_k = nullptr,
                const std::string& extra_v = "") {
  if (labels.empty() && !extra_k) return "";
  std::string o = "{";
  bool first = true;
  for (const auto& [k, v] : labels) {
    o += (first ? "" : ",") + k + "=\"" + escape(v) + "\"";
    first = false;
  }
  if (extra_k) o += std::string(first ? "" : ",") + extra_k + "=\"" + extra_v + "\"";
  return o + "}";
}

}  // namespace

const std::vector<double>& Registry::buckets_ms() {
  static const std::vector<double> b = {0.05, 0.1, 0.25, 0.5,  1,    2.5,  5,    10,   25,
                                        50,   100, 250,  500,  1000, 2500, 5000, 10000};
  return b;
}

Registry::Key Registry::key(const std::string& name, Labels labels) {
  std::sort(labels.begin(), labels.end());
  return {name, std::move(labels)};
}

// the first non-empty HELP text a family gets is kept (a call site without one adds none)
void Registry::note_help(const std::string& name, const std::string& help) {
  auto [it, fresh] = help_.emplace(name, help);
  if (!fresh && it->second.empty() && !help.empty()) it->second = help;
}

void Registry::inc(const std::string& name, const Labels& labels, double v, const std::string& help) {
  std::lock_guard<std::mutex> lk(mu_);
  counters_[key(name, labels)] += v;
  note_help(name, help);
}

void Registry::set(const std::string& name, double v, const Labels& labels, const std::string& help) {
  std::lock_guard<std::mutex> lk(mu_);
  gauges_[key(name, labels)] = v;
  note_help(name, help);
}

void Registry::observe_ms(const std::string& name, double ms, const Labels& labels, const std::string& help) {
  const auto& b = buckets_ms();
  const size_t i = static_cast<size_t>(std::lower_bound(b.begin(), b.end(), ms) - b.begin());  // bisect_left
  std::lock_guard<std::mutex> lk(mu_);
  Hist& h = hist_[key(name, labels)];
  if (h.counts.empty()) h.counts.assign(b.size() + 1, 0);
  h.counts[i]++;
  h.sum_ms += ms;
  h.n++;
  note_help(name, help);
}

double Registry::value(const std::string& name, const Labels& labels) const {
  std::lock_guard<std::mutex> lk(mu_);
  const Key k = key(name, labels);
  if (auto it = counters_.find(k); it != counters_.end()) return it->second;
  if (auto it = gauges_.find(k); it != gauges_.end()) return it->second;
  return 0;
}

uint64_t Registry::count(const std::string& name, const Labels& labels) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = hist_.find(key(name, labels));
  return it == hist_.end() ? 0 : it->second.n;
}

void Registry::clear() {
  std::lock_guard<std::mutex> lk(mu_);
  counters_.clear();
  gauges_.clear();
  hist_.clear();
  help_.clear();
}

std::string Registry::render() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::string out;
  std::set<std::string> done;
  auto head = [&](const std::string& name, const char* type) {
    if (!done.insert(name).second) return;
    auto h = help_.find(name);
    out += "# HELP " + name + " " + (h == help_.end() ? "" : h->second) + "\n# TYPE " + name + " " + type + "\n";
  };
  for (const auto& [k, v] : counters_) {
    head(k.first, "counter");
    out += k.first + lbl(k.second) + " " + py_float(v) + "\n";
  }
  for (const auto& [k, v] : gauges_) {
    head(k.first, "gauge");
    out += k.first + lbl(k.second) + " " + py_float(v) + "\n";
  }
  const auto& b = buckets_ms();
  for (const auto& [k, h] : hist_) {
    head(k.first, "histogram");
    uint64_t cum = 0;
    for (size_t i = 0; i <= b.size(); ++i) {
      cum += h.counts[i];
      const std::string le = i == b.size() ? "+Inf" : g_fmt(b[i] / 1000);
      out += k.first + "_bucket" + lbl(k.second, "le", le) + " " + std::to_string(cum) + "\n";
    }
    out += k.first + "_sum" + lbl(k.second) + " " + g_fmt(h.sum_ms / 1000) + "\n";
    out += k.first + "_count" + lbl(k.second) + " " + std::to_string(h.n) + "\n";
  }
  return out;
}

Registry& global() {
  static Registry r;
  return r;
}

// ---- HTTP endpoint -------------------------------------------------------------
std::string HttpEndpoint::start(const std::string& host, int port) {
  if (fd_ >= 0) return "already started";
  fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd_ < 0) return std::string("socket: ") + std::strerror(errno);
  const int one = 1;
  ::setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (::inet_pton(AF_INET, host.empty() ? "0.0.0.0" : host.c_str(), &a.sin_addr) != 1) {
    ::close(fd_);
    fd_ = -1;
    return "bad metrics address " + host;
  }
  if (::bind(fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(fd_, 16) != 0) {
    const std::string e = std::strerror(errno);
    ::close(fd_);
    fd_ = -1;
    return "metrics port " + std::to_string(port) + ": " + e;
  }
  socklen_t len = sizeof(a);
  ::getsockname(fd_, reinterpret_cast<sockaddr*>(&a), &len);
  port_ = ntohs(a.sin_port);
  if (::pipe2(stop_, O_CLOEXEC | O_NONBLOCK) != 0) {
    ::close(fd_);
    fd_ = -1;
    return "pipe failed";
  }
  thread_ = std::thread([this] { loop(); });
  return "";
}

void HttpEndpoint::stop() {
  if (thread_.joinable()) {
    const char b = 1;
    if (::write(stop_[1], &b, 1) < 0) {
    }
    thread_.join();
  }
  for (int* f : {&fd_, &stop_[0], &stop_[1]})
    if (*f >= 0) ::close(*f), *f = -1;
}

void HttpEndpoint::loop() {
  using Clock = std::chrono::steady_clock;
  for (;;) {
    pollfd p[2] = {{fd_, POLLIN, 0}, {stop_[0], POLLIN, 0}};
    if (::poll(p, 2, -1) < 0) {
      if (errno == EINTR) continue;
      return;
    }
    if (p[1].revents) return;
    if (!(p[0].revents & POLLIN)) continue;
    const int c = ::accept4(fd_, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK);
    if (c < 0) {
      // out of fds (EMFILE/ENFILE) leaves the connection queued and the listener
      // readable: back off instead of spinning on it
      if (errno != EAGAIN && errno != EINTR && errno != ECONNABORTED) {
        pollfd q{stop_[0], POLLIN, 0};
        ::poll(&q, 1, 100);
      }
      continue;
    }
    // the request head, within 5 s
    std::string req;
    const auto deadline = Clock::now() + std::chrono::seconds(5);
    bool stopping = false;
    while (req.find("\r\n\r\n") == std::string::npos && req.find("\n\n") == std::string::npos && req.size() < 16384) {
      const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
      if (left <= 0) break;
      pollfd q[2] = {{c, POLLIN, 0}, {stop_[0], POLLIN, 0}};
      if (::poll(q, 2, static_cast<int>(left)) < 0) {
        if (errno == EINTR) continue;
        break;
      }
      if (q[1].revents) {
        stopping = true;
        break;
      }
      char buf[2048];
      const ssize_t n = ::read(c, buf, sizeof(buf));
      if (n < 0 && (errno == EAGAIN || errno == EINTR)) continue;
      if (n <= 0) break;
      req.append(buf, static_cast<size_t>(n));
    }
    if (stopping) {
      ::close(c);
      return;
    }
    std::string path = "/";
    if (const size_t sp = req.find(' '); sp != std::string::npos) {
      const size_t e = req.find_first_of(" \r\n", sp + 1);
      path = req.substr(sp + 1, e == std::string::npos ? std::string::npos : e - sp - 1);
    }
    std::string body, status;
    auto probe = [&](const Check& check) {
      const std::string why = check ? check() : std::string();
      if (why.empty()) body = "ok\n", status = "200 OK";
      else body = why + "\n", status = "503 Service Unavailable";
    };
    if (path.rfind("/metrics", 0) == 0) body = reg_.render(), status = "200 OK";
    else if (path.rfind("/healthz", 0) == 0) probe(healthz_);
    else if (path.rfind("/readyz", 0) == 0) probe(readyz_);
    else body = "not found\n", status = "404 Not Found";
    requests_++;
    std::string resp = "HTTP/1.0 " + status + "\r\nContent-Type: text/plain; version=0.0.4\r\nContent-Length: " +
                       std::to_string(body.size()) + "\r\n\r\n" + body;
    size_t off = 0;
    const auto wdeadline = Clock::now() + std::chrono::seconds(5);
    while (off < resp.size() && Clock::now() < wdeadline) {
      const ssize_t n = ::send(c, resp.data() + off, resp.size() - off, MSG_NOSIGNAL);
      if (n > 0) {
        off += static_cast<size_t>(n);
      } else if (n < 0 && (errno == EAGAIN || errno == EINTR)) {
        pollfd q{c, POLLOUT, 0};
        ::poll(&q, 1, 100);
      } else {
        break;
      }
    }
    // Lingering close: a client whose request was not read to the end (a head
    // cut at 16 KiB, a body) would otherwise get a RST, which can destroy the
    // response in flight. Half-close, then drain until it closes (200 ms at most).
    ::shutdown(c, SHUT_WR);
    const auto ldeadline = Clock::now() + std::chrono::milliseconds(200);
    char sink[4096];
    while (Clock::now() < ldeadline) {
      pollfd q{c, POLLIN, 0};
      if (::poll(&q, 1, 50) < 0 && errno != EINTR) break;
      const ssize_t n = ::read(c, sink, sizeof(sink));
      if (n == 0 || (n < 0 && errno != EAGAIN && errno != EINTR)) break;
    }
    ::close(c);
  }
}

}  // namespace mi355x::metrics
