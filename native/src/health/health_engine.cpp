// Native per-device health engine (see mi355x/health_engine.h). The policy is
// the Python monitor's (rocm_k8s_device_plugin_amd/health/monitor.py,
// liveness.py), re-expressed for a daemon without an interpreter: probe
// children are posix_spawn()ed with pipes, every wait is a poll() bounded by
// a deadline and an abort fd.
#include "mi355x/health_engine.h"

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../kube/json.h"
#include "mi355x/dp_service.h"
#include "mi355x/glog.h"
#include "mi355x/metrics.h"
#include "mi355x/trace.h"
#include "mi355x/grpc_server.h"
#include "mi355x/smi_query.h"
#include "mi355x/sysfs.h"

extern char** environ;

namespace mi355x::health {
namespace {

using Clock = std::chrono::steady_clock;

double mono_s() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }

uint32_t make_nonce(int ordinal) {
  const uint64_t t = static_cast<uint64_t>(Clock::now().time_since_epoch().count());
  return static_cast<uint32_t>((t ^ (static_cast<uint64_t>(ordinal) * 0x9E3779B1ull)) & 0xFFFFFFFFull);
}

const char* kVisibilityVars[] = {"ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                 "GPU_DEVICE_ORDINAL"};

// ---- JSON accessors ----------------------------------------------------------
double jnum(const json::Value* v, const char* key, double fallback) {
  const json::Value* x = v ? v->get(key) : nullptr;
  if (!x) return fallback;
  if (x->kind == json::Value::Number) return std::strtod(x->s.c_str(), nullptr);
  if (x->kind == json::Value::Bool) return x->b ? 1 : 0;
  return fallback;
}
bool jbool(const json::Value* v, const char* key) {
  const json::Value* x = v ? v->get(key) : nullptr;
  if (!x) return false;
  if (x->kind == json::Value::Bool) return x->b;
  if (x->kind == json::Value::Number) return std::strtod(x->s.c_str(), nullptr) != 0;
  return false;
}
std::string jstr(const json::Value* v, const char* key) {
  const json::Value* x = v ? v->get(key) : nullptr;
  return x && x->kind == json::Value::String ? x->s : "";
}

// ---- child processes ---------------------------------------------------------
struct Child {
  pid_t pid = -1;
  int in = -1;   // its stdin (write end), -1 when not piped
  int out = -1;  // its stdout (read end)
  std::string buf;
  bool eof = false;
};

std::vector<std::string> child_env(const ProberConfig& cfg, const std::string& visible) {
  std::vector<std::string> env;
  for (char** e = environ; e && *e; ++e) {
    const std::string kv = *e;
    bool drop = false;
    for (const char* v : kVisibilityVars)
      if (kv.compare(0, std::strlen(v) + 1, std::string(v) + "=") == 0) drop = true;
    for (const auto& [k, val] : cfg.extra_env)
      if (kv.compare(0, k.size() + 1, k + "=") == 0) drop = true;
    if (!drop) env.push_back(kv);
  }
  for (const auto& [k, v] : cfg.extra_env) env.push_back(k + "=" + v);
  if (!visible.empty()) env.push_back("ROCR_VISIBLE_DEVICES=" + visible);
  return env;
}

// posix_spawn in a new session with stdout piped (and stdin when `with_stdin`)
bool spawn_child(const std::vector<std::string>& argv, const std::vector<std::string>& env, bool with_stdin, Child* c,
                 std::string* err) {
  int out_p[2], in_p[2] = {-1, -1};
  if (::pipe2(out_p, O_CLOEXEC) != 0) return *err = std::string("pipe: ") + std::strerror(errno), false;
  if (with_stdin && ::pipe2(in_p, O_CLOEXEC) != 0) {
    ::close(out_p[0]);
    ::close(out_p[1]);
    return *err = std::string("pipe: ") + std::strerror(errno), false;
  }
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, out_p[1], 1);
  if (with_stdin) posix_spawn_file_actions_adddup2(&fa, in_p[0], 0);
  else posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  posix_spawn_file_actions_addopen(&fa, 2, "/dev/null", O_WRONLY, 0);
  posix_spawnattr_t at;
  posix_spawnattr_init(&at);
  posix_spawnattr_setflags(&at, POSIX_SPAWN_SETSID | POSIX_SPAWN_SETSIGMASK | POSIX_SPAWN_SETSIGDEF);
  sigset_t none, all;
  sigemptyset(&none);
  sigfillset(&all);
  posix_spawnattr_setsigmask(&at, &none);
  posix_spawnattr_setsigdefault(&at, &all);
  std::vector<char*> av, ev;
  for (const auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
  av.push_back(nullptr);
  for (const auto& e : env) ev.push_back(const_cast<char*>(e.c_str()));
  ev.push_back(nullptr);
  pid_t pid = -1;
  const int rc = ::posix_spawnp(&pid, av[0], &fa, &at, av.data(), ev.data());
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&at);
  ::close(out_p[1]);
  if (with_stdin) ::close(in_p[0]);
  if (rc != 0) {
    ::close(out_p[0]);
    if (with_stdin) ::close(in_p[1]);
    return *err = "spawn " + argv[0] + ": " + std::strerror(rc), false;
  }
  ::fcntl(out_p[0], F_SETFL, O_NONBLOCK);
  c->pid = pid;
  c->out = out_p[0];
  c->in = with_stdin ? in_p[1] : -1;
  return true;
}

void kill_child(Child* c) {
  if (c->pid > 0) {
    ::kill(-c->pid, SIGKILL);
    ::kill(c->pid, SIGKILL);
    int st = 0;
    while (::waitpid(c->pid, &st, 0) < 0 && errno == EINTR) {
    }
  }
  if (c->in >= 0) ::close(c->in);
  if (c->out >= 0) ::close(c->out);
  c->pid = c->in = c->out = -1;
}

// drains what is readable; false on EOF
bool drain(Child* c) {
  char b[8192];
  while (true) {
    const ssize_t n = ::read(c->out, b, sizeof(b));
    if (n > 0) {
      c->buf.append(b, static_cast<size_t>(n));
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return true;
    c->eof = true;
    return false;
  }
}

enum class Got { kLine, kTimeout, kEof, kAbort };

// next '\n'-terminated line of c's stdout within `deadline`
Got read_line(Child* c, double deadline, int abort_fd, std::string* line) {
  while (true) {
    const size_t nl = c->buf.find('\n');
    if (nl != std::string::npos) {
      *line = c->buf.substr(0, nl);
      c->buf.erase(0, nl + 1);
      return Got::kLine;
    }
    if (c->eof) return Got::kEof;
    const double left = deadline - mono_s();
    if (left <= 0) return Got::kTimeout;
    pollfd p[2] = {{c->out, POLLIN, 0}, {abort_fd, POLLIN, 0}};
    const int r = ::poll(p, abort_fd >= 0 ? 2 : 1, static_cast<int>(left * 1000) + 1);
    if (r < 0 && errno != EINTR) return Got::kEof;
    if (abort_fd >= 0 && (p[1].revents & POLLIN)) return Got::kAbort;
    if (r > 0) drain(c);
  }
}

bool write_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t n = ::write(fd, s.data() + off, s.size() - off);
    if (n > 0) {
      off += static_cast<size_t>(n);
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    return false;
  }
  return true;
}

ProbeOutcome judge(bool doc_ok, const json::Value* d, uint32_t nonce, double ms, int rc = 0) {
  ProbeOutcome o;
  o.latency_ms = ms;
  if (d) {
    o.kfd_node_id = static_cast<int>(jnum(d, "kfd_node_id", -1));
    o.pci_bus_id = jstr(d, "pci_bus_id");
    for (const char* k : {"cu_count", "hbm_read_gbps", "hbm_write_gbps", "hbm_bad_words", "mfma_tflops",
                          "clock_mhz_median", "total_us"})
      if (const json::Value* v = d->get(k); v && v->kind == json::Value::Number) o.detail[k] = std::strtod(v->s.c_str(), nullptr);
    if (const json::Value* x = d->get("xcd_clock_mhz"); x && x->kind == json::Value::Array)
      for (const auto& c : x->arr)
        if (c.kind == json::Value::Number) o.xcd_clock_mhz.push_back(std::strtod(c.s.c_str(), nullptr));
  }
  if (rc != 0 || !doc_ok || !jbool(d, "ok")) {
    o.reason = jstr(d, "error");
    if (o.reason.empty()) o.reason = "probe exit " + std::to_string(rc);
    return o;
  }
  const json::Value* n = d->get("nonce");
  const uint32_t got = n && n->kind == json::Value::Number ? static_cast<uint32_t>(std::strtoull(n->s.c_str(), nullptr, 10))
                                                           : 0;
  if (!n || got != nonce) {
    o.reason = "stale probe result (nonce " + (n ? n->s : std::string("missing")) + " != " + std::to_string(nonce) + ")";
    return o;
  }
  o.ok = true;
  return o;
}

std::string join_ints(const std::vector<int>& v, const char* sep) {
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) s += (i ? sep : "") + std::to_string(v[i]);
  return s;
}

}  // namespace

// =============================================================== LivenessProber
struct LivenessProber::Server {
  Child c;
  bool alive() {
    if (c.pid <= 0) return false;
    int st = 0;
    const pid_t r = ::waitpid(c.pid, &st, WNOHANG);
    if (r == c.pid) {
      c.pid = -1;
      return false;
    }
    return true;
  }
};

LivenessProber::LivenessProber(ProberConfig cfg) : cfg_(std::move(cfg)) {}
LivenessProber::~LivenessProber() { close(); }

bool LivenessProber::server_running() const { return server_ && server_->c.pid > 0; }

void LivenessProber::close() {
  pending_nonce_.clear();  // a new server starts without outstanding dispatches
  if (server_) {
    if (server_->c.in >= 0) write_all(server_->c.in, "quit\n");
    kill_child(&server_->c);
    server_.reset();
  }
  server_visible_.reset();
  own_kfd_.clear();
}

void LivenessProber::set_visible(std::optional<std::vector<int>> ordinals) {
  if (ordinals) {
    std::sort(ordinals->begin(), ordinals->end());
    ordinals->erase(std::unique(ordinals->begin(), ordinals->end()), ordinals->end());
  }
  visible_ = std::move(ordinals);
}

std::set<std::string> LivenessProber::own_kfd_entries(const std::set<int64_t>& gpu_ids) {
  if (!server_ || !server_->alive()) return {};
  if (own_kfd_.size() > 1) {  // another GPU process started with the server: keep what still exists
    std::set<std::string> still;
    for (const auto& e : list_dir(cfg_.kfd_proc_dir))
      if (own_kfd_.count(e)) still.insert(e);
    own_kfd_ = still;
  }
  if (own_kfd_.size() == 1) return own_kfd_;
  if (own_kfd_.size() > 1 && cfg_.keep_queues && !gpu_ids.empty()) {
    // the kept-queue server holds a queue on every GPU it probed; a pod's process only on the pod's
    std::vector<std::string> match;
    for (const auto& e : own_kfd_) {
      std::set<int64_t> have;
      const std::string qdir = path_join(path_join(cfg_.kfd_proc_dir, e), "queues");
      for (const auto& q : list_dir(qdir))
        if (auto g = read_trimmed(path_join(path_join(qdir, q), "gpuid"))) have.insert(parse_i64(*g, 0));
      if (std::includes(have.begin(), have.end(), gpu_ids.begin(), gpu_ids.end())) match.push_back(e);
    }
    if (match.size() == 1) own_kfd_ = {match[0]};
    if (own_kfd_.size() == 1) return own_kfd_;
  }
  return {};
}

ProbeOutcome LivenessProber::probe_ordinal(int ordinal, const std::string& kind) {
  return spawn_all({ordinal}, kind)[ordinal];
}

std::map<int, ProbeOutcome> LivenessProber::spawn_all(const std::vector<int>& ords, const std::string& kind) {
  std::map<int, ProbeOutcome> out;
  const size_t par = static_cast<size_t>(std::max(1, cfg_.max_parallel));
  for (size_t start = 0; start < ords.size(); start += par) {
    struct Job {
      int ordinal;
      uint32_t nonce;
      Child c;
      double t0;
      bool done = false;
      int rc = -1;
      bool timed_out = false;
    };
    std::vector<Job> jobs;
    for (size_t i = start; i < std::min(ords.size(), start + par); ++i) {
      Job j;
      j.ordinal = ords[i];
      j.nonce = make_nonce(j.ordinal);
      char tmo[32];
      std::snprintf(tmo, sizeof(tmo), "%.2f", std::max(0.5, cfg_.timeout_s - 0.5));
      std::vector<std::string> argv = cfg_.argv_prefix;
      for (const std::string& a : {cfg_.exe, std::string("--devices"), std::string("0"), std::string("--iters"),
                                   std::to_string(cfg_.iters), std::string("--nonce"), std::to_string(j.nonce),
                                   std::string("--timeout"), std::string(tmo)})
        argv.push_back(a);
      if (kind == "sweep") argv.push_back("--sweep");
      if (kind == "perf")
        for (const std::string& a : {std::string("--perf"), std::string("--perf-mib"), std::to_string(cfg_.perf_mib),
                                     std::string("--perf-iters"), std::to_string(cfg_.perf_iters)})
          argv.push_back(a);
      std::string err;
      j.t0 = mono_s();
      if (!spawn_child(argv, child_env(cfg_, std::to_string(j.ordinal)), false, &j.c, &err)) {
        ProbeOutcome o;
        o.reason = "spawn failed: " + err;
        out[j.ordinal] = o;
        continue;
      }
      jobs.push_back(std::move(j));
    }
    const double deadline = mono_s() + cfg_.timeout_s;
    bool aborted = false;
    while (true) {
      std::vector<pollfd> pf;
      std::vector<size_t> idx;
      for (size_t i = 0; i < jobs.size(); ++i)
        if (!jobs[i].c.eof) {
          pf.push_back({jobs[i].c.out, POLLIN, 0});
          idx.push_back(i);
        }
      if (pf.empty()) break;
      const double left = deadline - mono_s();
      if (left <= 0) break;
      if (abort_fd_ >= 0) pf.push_back({abort_fd_, POLLIN, 0});
      const int r = ::poll(pf.data(), pf.size(), static_cast<int>(left * 1000) + 1);
      if (r < 0 && errno != EINTR) break;
      if (abort_fd_ >= 0 && (pf.back().revents & POLLIN)) {
        aborted = true;
        break;
      }
      for (size_t k = 0; k < idx.size(); ++k)
        if (pf[k].revents) drain(&jobs[idx[k]].c);
    }
    for (auto& j : jobs) {
      const double ms = (mono_s() - j.t0) * 1e3;
      if (trace::global().enabled()) {
        const uint64_t dur = static_cast<uint64_t>(ms * 1e6);
        trace::global().complete("liveness.probe", "health", trace::now_ns() - dur, dur,
                                 {{"ordinal", std::to_string(j.ordinal)}, {"kind", kind}});
      }
      if (!j.c.eof) {  // deadline (or shutdown): the dispatch did not complete
        kill_child(&j.c);
        ProbeOutcome o;
        char why[64];
        std::snprintf(why, sizeof(why), "deadline exceeded (%.1fs)", cfg_.timeout_s);
        o.reason = aborted ? "probe interrupted (shutdown)" : why;
        o.latency_ms = ms;
        o.pending = kind == "probe" && !aborted;  // inconclusive on a busy GPU
        out[j.ordinal] = o;
        continue;
      }
      int st = 0;
      while (::waitpid(j.c.pid, &st, 0) < 0 && errno == EINTR) {
      }
      j.c.pid = -1;
      const int rc = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
      ::close(j.c.out);
      j.c.out = -1;
      // the last line is the JSON document
      std::string text = j.c.buf;
      while (!text.empty() && (text.back() == '\n' || text.back() == '\r')) text.pop_back();
      const size_t nl = text.rfind('\n');
      const std::string last = nl == std::string::npos ? text : text.substr(nl + 1);
      std::string perr;
      auto doc = json::parse(last, &perr);
      if (!doc) {
        ProbeOutcome o;
        o.reason = "unparseable probe output (rc=" + std::to_string(rc) + "): " + last.substr(0, 200);
        o.latency_ms = ms;
        out[j.ordinal] = o;
        continue;
      }
      const json::Value* devs = doc->get("devices");
      const json::Value* d = devs && devs->kind == json::Value::Array && !devs->arr.empty() ? &devs->arr[0] : nullptr;
      json::Value errdoc = json::Value::object();
      if (!d) {
        errdoc.set("error", json::Value::string(jstr(&*doc, "error")));
        d = &errdoc;
      }
      out[j.ordinal] = judge(jbool(&*doc, "ok"), d, j.nonce, ms, rc);
    }
  }
  return out;
}

std::map<int, ProbeOutcome> LivenessProber::probe_server(const std::vector<int>& uniq, const std::string& kind,
                                                         std::string* err) {
  trace::Span span("liveness.request", "health", {{"ordinals", std::to_string(uniq.size())}, {"kind", kind}});
  const double t0 = mono_s();
  std::optional<std::vector<int>> visible = visible_;
  if (visible) {
    std::set<int> u(visible->begin(), visible->end());
    bool grow = false;
    for (int o : uniq) grow |= u.insert(o).second;
    if (grow) visible = std::vector<int>(u.begin(), u.end());
  }
  if (server_ && server_->alive() && visible != server_visible_) close();  // the GPUs it may touch changed
  if (!server_ || !server_->alive()) {
    if (server_) close();
    std::vector<std::string> argv = cfg_.argv_prefix;
    argv.push_back(cfg_.exe);
    argv.push_back("--serve");
    if (cfg_.keep_queues) argv.push_back("--keep");
    std::set<std::string> before;
    for (const auto& e : list_dir(cfg_.kfd_proc_dir)) before.insert(e);
    auto srv = std::make_unique<Server>();
    if (!spawn_child(argv, child_env(cfg_, visible ? join_ints(*visible, ",") : ""), true, &srv->c, err)) return {};
    std::string hello;
    const Got g = read_line(&srv->c, mono_s() + cfg_.timeout_s, abort_fd_, &hello);
    auto doc = g == Got::kLine ? json::parse(hello) : std::nullopt;
    if (!doc || !jbool(&*doc, "serve") || !jbool(&*doc, "ok")) {
      kill_child(&srv->c);
      *err = g == Got::kTimeout ? "probe server did not start within the deadline"
                                : "probe server failed to start: " + hello.substr(0, 200);
      return {};
    }
    server_ = std::move(srv);
    server_visible_ = visible;
    own_kfd_.clear();
    for (const auto& e : list_dir(cfg_.kfd_proc_dir))
      if (!before.count(e)) own_kfd_.insert(e);
    server_starts++;
  }
  // the server numbers the GPUs it sees: with a visibility list, their positions
  std::map<int, int> local, host;
  for (int o : uniq) {
    int l = o;
    if (server_visible_) l = static_cast<int>(std::find(server_visible_->begin(), server_visible_->end(), o) -
                                              server_visible_->begin());
    local[o] = l;
    host[l] = o;
  }
  std::map<int, uint32_t> nonces;
  for (int o : uniq) nonces[o] = make_nonce(o);
  const double inner = cfg_.timeout_s - std::min(0.5, 0.25 * cfg_.timeout_s);
  char head[96];
  if (kind == "perf")
    std::snprintf(head, sizeof(head), "perf %d %.2f %d", cfg_.perf_iters, inner, cfg_.perf_mib);
  else
    std::snprintf(head, sizeof(head), "%s %d %.2f", kind.c_str(), cfg_.iters, inner);
  std::string line = head;
  for (int o : uniq) line += " " + std::to_string(local[o]) + ":" + std::to_string(nonces[o]);
  if (!write_all(server_->c.in, line + "\n")) {
    *err = "probe server gone (write failed)";
    return {};
  }
  std::string reply;
  const Got g = read_line(&server_->c, mono_s() + cfg_.timeout_s, abort_fd_, &reply);
  if (g != Got::kLine) {
    *err = g == Got::kTimeout ? "probe server missed its deadline"
           : g == Got::kAbort ? "interrupted"
                              : "probe server exited";
    return {};
  }
  std::string perr;
  auto doc = json::parse(reply, &perr);
  if (!doc) {
    *err = "unparseable probe server output: " + reply.substr(0, 200);
    return {};
  }
  const double ms = (mono_s() - t0) * 1e3;
  std::map<int, const json::Value*> by_ord;
  if (const json::Value* devs = doc->get("devices"); devs && devs->kind == json::Value::Array)
    for (const auto& d : devs->arr) {
      const int l = static_cast<int>(jnum(&d, "ordinal", -1));
      if (host.count(l)) by_ord[host[l]] = &d;
    }
  std::map<int, ProbeOutcome> out;
  for (int o : uniq) {
    auto it = by_ord.find(o);
    if (it == by_ord.end()) {
      ProbeOutcome r;
      r.reason = "device missing from probe server reply";
      r.latency_ms = ms;
      out[o] = r;
      continue;
    }
    const json::Value* d = it->second;
    if (kind != "probe") {  // sweeps run on their own queue: the kept slot is untouched
      out[o] = judge(jbool(d, "ok"), d, nonces[o], ms);
      continue;
    }
    // a late verdict answers the dispatch (and nonce) of the probe that left it pending
    const bool late = jbool(d, "late");
    uint32_t expect = nonces[o];
    if (late) {
      auto pn = pending_nonce_.find(o);
      if (pn != pending_nonce_.end()) {
        expect = pn->second;
        pending_nonce_.erase(pn);
      }
    }
    ProbeOutcome r = judge(jbool(d, "ok"), d, expect, ms);
    if (!r.ok && jnum(d, "pending_s", 0) > 0) {
      r.pending = true;
      pending_nonce_.emplace(o, nonces[o]);
    } else if (!r.ok && jnum(d, "hip_error", 0) == -1 && !cfg_.keep_queues) {
      r.pending = true;  // timed out without a kept slot: no late verdict will follow
    } else if (!late) {
      pending_nonce_.erase(o);
    }
    out[o] = r;
  }
  if (!cfg_.keep_queues)
    for (const auto& [o, d] : by_ord)
      if (jnum(d, "hip_error", 0) == -1 || jnum(d, "hsa_error", 0) == -1) {
        close();  // a timed-out dispatch's queue can never be freed by the server: restart it
        break;
      }
  return out;
}

std::map<int, ProbeOutcome> LivenessProber::probe(const std::vector<int>& ordinals, const std::set<int>& busy,
                                                  const std::string& kind) {
  std::vector<int> uniq(ordinals);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  if (uniq.empty()) return {};
  const bool use_server = cfg_.persistent && backoff_ == 0;
  backoff_ = std::max(0, backoff_ - 1);
  if (use_server) {
    std::string err;
    auto res = probe_server(uniq, kind, &err);
    if (err.empty()) {
      std::vector<int> failed;
      for (int o : uniq)
        if (!res[o].ok && !(res[o].pending && busy.count(o))) failed.push_back(o);
      if (!failed.empty()) {
        // the server's runtime lives across sweeps: a failure only counts if a fresh process confirms it
        auto fresh = spawn_all(failed, kind);
        bool stale = false;
        std::vector<int> healed;
        for (int o : failed) {
          ProbeOutcome& f = fresh[o];
          if (f.ok) {
            stale = true;
            healed.push_back(o);
            res[o] = f;
          } else {
            f.reason += " (server: " + res[o].reason + ")";
            res[o] = f;
          }
        }
        if (stale) {
          server_restarts++;
          MI_LOG(kWarning, "probe server failed ordinals %s that a fresh process found healthy; restarting it",
                 join_ints(healed, ",").c_str());
          close();
        }
      }
      sweeps++;
      return res;
    }
    if (err == "interrupted") {  // shutdown: no fresh processes now
      std::map<int, ProbeOutcome> out;
      for (int o : uniq) out[o].reason = "probe interrupted (shutdown)";
      return out;
    }
    // a wedged device stalls the whole server: drop it and isolate per device
    MI_LOG(kWarning, "probe server failed (%s); re-probing each device in its own process", err.c_str());
    fallbacks++;
    backoff_ = 4;
    close();
  }
  auto res = spawn_all(uniq, kind);
  sweeps++;
  return res;
}

// =============================================================== helpers
// GPUStateResponse{GPUState=1: GPUState{ID=1, UUID=2, Health=3, AssociatedWorkload=4, Device=5}}
// (internal/pkg/exporter/metricssvc/metricssvc.pb.go:95-110,284-291), decoded
// strictly as protobuf does: a malformed message is an error, not a partial map
std::map<std::string, bool> parse_exporter_states(const std::string& body, std::string* error) {
  std::map<std::string, bool> out;
  const bool ok = rpc::pb::scan(
      body.data(), body.size(),
      [&](int f, const char* p, size_t n) {
        if (f != 1) return true;
        std::string health, device;
        const bool inner = rpc::pb::scan(
            p, n,
            [&](int g, const char* q, size_t m) {
              if (g == 3) health.assign(q, m);
              else if (g == 5) device.assign(q, m);
              return true;
            },
            nullptr);
        if (inner && !device.empty()) out[device] = to_lower(trim(health)) == "healthy";
        return inner;
      },
      nullptr);
  if (!ok) {
    if (error) *error = "malformed GPUStateResponse from the metrics exporter";
    return {};
  }
  return out;
}

std::map<std::string, bool> exporter_list(const std::string& socket, double timeout_s, int abort_fd,
                                          std::string* error) {
  std::map<std::string, bool> out;
  if (socket.empty() || !path_exists(socket)) return out;
  rpc::GrpcClient c;
  c.set_abort_fd(abort_fd);
  const std::string cerr = c.connect(socket, timeout_s);
  if (!cerr.empty()) {
    if (error) *error = cerr;
    return out;
  }
  const rpc::Reply rep = c.unary("/metricssvc.MetricsService/List", "", timeout_s);
  if (rep.status != 0) {
    if (error) *error = rep.message;
    return out;
  }
  return parse_exporter_states(rep.body, error);
}

std::map<std::string, int> hip_ordinals(const std::vector<GpuDevice>& devices, const KfdTopology& topo,
                                        const std::string& dev_root) {
  std::map<int, int> pos;  // kfd node id -> ordinal
  const bool check = is_dir(path_join(dev_root, "dri"));
  int n = 0;
  for (const KfdNode* node : topo.gpu_nodes()) {
    const int minor = node->drm_render_minor();
    if (minor <= 0) continue;
    if (check && ::access(path_join(dev_root, "dri/renderD" + std::to_string(minor)).c_str(), R_OK | W_OK) != 0)
      continue;
    pos[node->id] = n++;
  }
  std::map<std::string, int> out;
  for (const auto& d : devices)
    if (auto it = pos.find(d.node_id); it != pos.end()) out[d.id] = it->second;
  return out;
}

// =============================================================== Engine
Engine::Engine(std::vector<GpuDevice> devices, const KfdTopology& topo, Config cfg)
    : devices_(std::move(devices)), topo_(topo), cfg_(std::move(cfg)) {
  for (size_t i = 0; i < devices_.size(); ++i) {
    by_id_[devices_[i].id] = i;
    track_[devices_[i].id] = Track{};
    snapshot_[devices_[i].id] = Verdict{};
    std::string b = devices_[i].bdf;
    for (auto& c : b) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    gpu_by_bdf_.emplace(b, !devices_[i].unique_id.empty() ? devices_[i].unique_id : "bdf:" + devices_[i].bdf);
  }
  if (cfg_.liveness) {
    if (cfg_.prober.kfd_proc_dir.empty() || cfg_.prober.kfd_proc_dir == "/sys/class/kfd/kfd/proc")
      cfg_.prober.kfd_proc_dir = path_join(cfg_.sysfs_root, "class/kfd/kfd/proc");
    prober_ = std::make_unique<LivenessProber>(cfg_.prober);
  }
}

Engine::~Engine() { close(); }

void Engine::set_abort_fd(int fd) {
  abort_fd_ = fd;
  if (prober_) prober_->set_abort_fd(fd);
}

void Engine::close() {
  if (prober_) prober_->close();
  if (events_) events_->stop();
  events_.reset();
  events_started_ = false;
  if (smi_held_) smi_unhold();
  smi_held_ = false;
}

std::map<std::string, Verdict> Engine::snapshot() const {
  std::lock_guard<std::mutex> lk(mu_);
  return snapshot_;
}

uint64_t Engine::version() const {
  std::lock_guard<std::mutex> lk(mu_);
  return version_;
}

const GpuDevice* Engine::dev(const std::string& id) const {
  auto it = by_id_.find(id);
  return it == by_id_.end() ? nullptr : &devices_[it->second];
}

const std::map<std::string, int>& Engine::ordinals() {
  if (!ordinals_) ordinals_ = hip_ordinals(devices_, topo_, cfg_.dev_root);
  return *ordinals_;
}

int64_t Engine::gpu_id(const std::string& id) const {
  const GpuDevice* d = dev(id);
  const KfdNode* n = d && d->node_id >= 0 ? topo_.node(d->node_id) : nullptr;
  return n ? n->gpu_id : 0;
}

std::map<std::string, std::string> Engine::kfd_verdicts() const {
  std::map<std::string, std::string> out;
  const std::string nodes = path_join(cfg_.sysfs_root, "class/kfd/kfd/topology/nodes");
  const bool have = is_dir(nodes);
  for (const auto& d : devices_) {
    if (!have) {
      out[d.id] = "kfd topology unavailable";
      continue;
    }
    if (d.node_id < 0) continue;  // no kfd data (cgroup-denied): not evidence of a fault
    const auto kv = parse_kv_file(path_join(nodes, std::to_string(d.node_id) + "/properties"));
    if (!kv) {
      out[d.id] = "kfd node " + std::to_string(d.node_id) + " missing";
      continue;
    }
    const int64_t cores = kv_i64(*kv, "cpu_cores_count", 0), gfx = kv_i64(*kv, "gfx_target_version", 0);
    if (!(cores == 0 && gfx > 0)) out[d.id] = "kfd node " + std::to_string(d.node_id) + " not a live GPU";
  }
  return out;
}

std::map<std::string, bool> Engine::exporter_health() const {
  if (exporter_source) return exporter_source();
  std::string err;
  auto m = exporter_list(cfg_.exporter_socket, cfg_.exporter_timeout_s, abort_fd_, &err);
  if (!err.empty()) MI_LOG(kError, "Error getting health info svc : %s", err.c_str());
  return m;
}

std::map<std::string, int> Engine::gfx_activity() {
  if (activity_source) return activity_source();
  std::map<std::string, int> out;
  if (!smi_available()) return out;
  if (!smi_held_) smi_held_ = smi_hold();
  const SmiSnapshot snap = smi_snapshot();
  if (!snap.ok) return out;
  for (const auto& g : snap.gpus)
    if (g.gfx_activity >= 0) out[g.bdf] = g.gfx_activity;
  return out;
}

bool Engine::kfd_load(const std::set<std::string>& exclude, std::map<int64_t, std::pair<int, int>>* out) const {
  out->clear();
  const std::string root = path_join(cfg_.sysfs_root, "class/kfd/kfd/proc");
  if (!is_dir(root)) return path_exists(root) ? false : true;  // no list at all: no process has queues
  if (::access(root.c_str(), R_OK | X_OK) != 0) return false;
  std::map<int64_t, std::pair<int, int>> load;
  for (const auto& pid : list_dir(root)) {
    if (exclude.count(pid)) continue;
    const std::string qdir = path_join(path_join(root, pid), "queues");
    if (!is_dir(qdir)) continue;  // exited meanwhile
    if (::access(qdir.c_str(), R_OK | X_OK) != 0) return false;
    std::map<int64_t, int> mine;
    for (const auto& q : list_dir(qdir)) {
      auto g = read_trimmed(path_join(path_join(qdir, q), "gpuid"));
      if (!g) continue;
      const int64_t gid = parse_i64(*g, 0);
      if (gid) mine[gid]++;
    }
    for (const auto& [gid, nq] : mine) {
      load[gid].first += 1;
      load[gid].second += nq;
    }
  }
  *out = std::move(load);
  return true;
}

bool Engine::identity_matches(const GpuDevice& d, const ProbeOutcome& o) const {
  int dom = -1, loc = -1;
  unsigned D = 0, B = 0, Dv = 0, F = 0;
  if (!o.pci_bus_id.empty() && std::sscanf(o.pci_bus_id.c_str(), "%x:%x:%x.%x", &D, &B, &Dv, &F) == 4) {
    dom = static_cast<int>(D);
    loc = static_cast<int>((B << 8) | (Dv << 3) | F);
  }
  if (o.kfd_node_id < 0 && loc < 0) return true;  // the reply names no agent
  // the PCI location (partition index in the function bits) is exact; the
  // agent's node id is the thunk's, renumbered under a device cgroup
  if (loc >= 0 && d.location_id) return dom == d.domain && loc == d.location_id;
  if (o.kfd_node_id >= 0 && d.node_id >= 0) return o.kfd_node_id == d.node_id;
  return true;
}

std::map<std::string, ProbeOutcome> Engine::verify_identity(const std::map<std::string, int>& ords,
                                                            const std::map<std::string, ProbeOutcome>& outcomes) {
  bool bad = false;
  for (const auto& [id, o] : outcomes)
    if (const GpuDevice* d = dev(id); d && !identity_matches(*d, o)) bad = true;
  if (!bad) return outcomes;
  // re-key by identity: every reply names its agent's PCI location
  std::map<std::pair<int, int>, std::pair<int, const ProbeOutcome*>> by_loc;
  std::map<int, std::pair<int, const ProbeOutcome*>> by_node;
  for (const auto& [id, o] : outcomes) {
    unsigned D = 0, B = 0, Dv = 0, F = 0;
    if (!o.pci_bus_id.empty() && std::sscanf(o.pci_bus_id.c_str(), "%x:%x:%x.%x", &D, &B, &Dv, &F) == 4)
      by_loc[{static_cast<int>(D), static_cast<int>((B << 8) | (Dv << 3) | F)}] = {ords.at(id), &o};
    else if (o.kfd_node_id >= 0)
      by_node[o.kfd_node_id] = {ords.at(id), &o};
  }
  std::map<std::string, ProbeOutcome> fixed;
  std::map<std::string, int> new_ords;
  for (const auto& [id, ord] : ords) {
    const GpuDevice* d = dev(id);
    if (!d) continue;
    const std::pair<int, const ProbeOutcome*>* hit = nullptr;
    if (d->location_id)
      if (auto it = by_loc.find({d->domain, d->location_id}); it != by_loc.end()) hit = &it->second;
    if (!hit && d->node_id >= 0)
      if (auto it = by_node.find(d->node_id); it != by_node.end()) hit = &it->second;
    if (hit && identity_matches(*d, *hit->second)) {
      new_ords[id] = hit->first;
      fixed[id] = *hit->second;
      if (hit->first != ord)
        MI_LOG(kError, "probe identity: device %s is ordinal %d, not %d (verdict re-keyed)", id.c_str(), hit->first,
               ord);
    }
  }
  std::string lost;
  for (const auto& [id, ord] : ords)
    if (!new_ords.count(id)) lost += (lost.empty() ? "" : ",") + id;
  if (!lost.empty()) MI_LOG(kError, "probe identity: no probed agent matches %s; they lose their ordinal", lost.c_str());
  std::map<std::string, int> merged;
  for (const auto& [id, o] : ordinals())
    if (!ords.count(id)) merged[id] = o;
  for (const auto& [id, o] : new_ords) merged[id] = o;
  ordinals_ = merged;
  identity_remaps_++;
  metrics::global().inc("mi355x_dp_probe_identity_mismatch_total", {}, 1.0,
                        "sweeps whose probe replies came from other devices than the positional ordinal map");
  return fixed;
}

bool Engine::sweep() {
  trace::Span span("health.sweep", "health", {{"devices", std::to_string(devices_.size())}});
  const double t0 = mono_s();
  std::map<std::string, std::vector<std::string>> reasons;
  for (const auto& d : devices_) reasons[d.id];
  for (const auto& [id, r] : kfd_verdicts()) reasons[id].push_back(r);

  if (!cfg_.exporter_socket.empty() || exporter_source) {
    const auto hmap = exporter_health();
    for (const auto& d : devices_)
      if (auto it = hmap.find(d.bdf); it != hmap.end() && !it->second)
        reasons[d.id].push_back("exporter reports " + d.bdf + " unhealthy");
  }

  if (cfg_.liveness && prober_) {
    std::map<std::string, int> ords;
    for (const auto& [id, o] : ordinals())
      if (reasons.count(id)) ords[id] = o;
    // busy GPUs: other processes' queues (the probe server's own excluded)
    std::set<int64_t> probed_gids;
    for (const auto& [id, o] : ords) probed_gids.insert(gpu_id(id));
    probed_gids.erase(0);
    const std::set<std::string> own = prober_->own_kfd_entries(probed_gids);
    const bool unresolved = own.empty() && prober_->server_running() && cfg_.prober.keep_queues;
    std::set<std::string> busy_devs;
    const bool known = kfd_load(own, &load_);
    if (!known) {
      load_.clear();
      for (const auto& [id, o] : ords) busy_devs.insert(id);
    } else {
      for (const auto& [id, o] : ords)
        if (int64_t g = gpu_id(id); g && load_.count(g)) busy_devs.insert(id);
    }
    const bool now_known = known && !unresolved;
    if (now_known != busy_known_)
      glog::log(now_known ? glog::kInfo : glog::kWarning, __FILE__, __LINE__, "%s",
                now_known ? "busy-GPU state readable again"
                          : "busy-GPU state unknown: every GPU counts as busy, pending probes get the short grace");
    busy_known_ = now_known;
    metrics::global().set("mi355x_dp_busy_state_known", now_known ? 1.0 : 0.0, {},
                          "1 if busy GPUs can be told from idle ones (kfd process list readable)");
    // crowded GPUs: the probe server steps off them
    std::set<std::string> crowded;
    if (cfg_.crowded_procs > 0) {
      for (const auto& [id, o] : ords) {
        const GpuDevice* d = dev(id);
        const KfdNode* node = d && d->node_id >= 0 ? topo_.node(d->node_id) : nullptr;
        const auto ld = load_.count(gpu_id(id)) ? load_.at(gpu_id(id)) : std::make_pair(0, 0);
        const int64_t cp = node ? node->prop("num_cp_queues", 0) : 0;
        const bool is_crowded = ld.first >= cfg_.crowded_procs || (cp > 0 && ld.second + 2 > cp);
        if (is_crowded) {
          if (!crowded_.count(id))
            MI_LOG(kInfo, "GPU of %s is crowded (%d other processes, %d queues): the probe server steps off it",
                   id.c_str(), ld.first, ld.second);
          crowded_[id] = 0;
        } else if (crowded_.count(id) && ++crowded_[id] >= cfg_.crowded_release_sweeps) {
          crowded_.erase(id);
          MI_LOG(kInfo, "GPU of %s is no longer crowded: probing it again", id.c_str());
        }
        if (crowded_.count(id)) crowded.insert(id);
      }
    } else {
      crowded_.clear();
    }
    std::map<std::string, int> probe_ords;
    for (const auto& [id, o] : ords)
      if (!crowded.count(id)) probe_ords[id] = o;
    if (!crowded.empty()) {
      std::vector<int> vis;
      for (const auto& [id, o] : probe_ords) vis.push_back(o);
      prober_->set_visible(vis);
      if (probe_ords.empty() && prober_->server_running()) prober_->close();  // hold nothing on any GPU
    } else {
      prober_->set_visible(std::nullopt);
    }
    // idle GPUs (no other process's queues) for the full-chip sweep and the
    // throughput check; none while busy state is unknown (both hold every CU)
    std::set<std::string> idle;
    if (known)
      for (const auto& [id, o] : probe_ords)
        if (int64_t g = gpu_id(id); g && !load_.count(g)) idle.insert(id);
    std::map<std::string, ProbeOutcome> outcomes;
    if (!probe_ords.empty()) {
      const bool chip = cfg_.chip_sweep_every > 0 && sweeps_ % static_cast<uint64_t>(cfg_.chip_sweep_every) == 0;
      if (chip && !known) MI_LOG(kWarning, "full-chip sweep skipped: busy-GPU state unknown");
      std::map<std::string, ProbeOutcome> raw;
      auto run = [&](const std::map<std::string, int>& sel, const char* kind) {
        std::vector<int> uniq;
        std::set<int> busy_ords;
        for (const auto& [id, o] : sel) {
          uniq.push_back(o);
          if (busy_devs.count(id)) busy_ords.insert(o);
        }
        const auto by_ord = prober_->probe(uniq, busy_ords, kind);
        for (const auto& [id, o] : sel)
          if (auto it = by_ord.find(o); it != by_ord.end()) raw[id] = it->second;
      };
      std::map<std::string, int> swept, rest;
      for (const auto& [id, o] : probe_ords) (chip && idle.count(id) ? swept : rest)[id] = o;
      if (!swept.empty()) {
        run(swept, "sweep");
        chip_sweeps_++;
        metrics::global().inc("mi355x_dp_chip_sweeps_total", {}, 1.0,
                              "full-chip sweeps run (every CU of every XCD on the idle GPUs)");
      }
      if (!rest.empty()) run(rest, "probe");
      outcomes = verify_identity(probe_ords, raw);
    }
    if (!crowded.empty()) {
      const auto act = gfx_activity();
      for (const auto& id : crowded) {
        const GpuDevice* d = dev(id);
        auto a = d ? act.find(d->bdf) : act.end();
        if (a != act.end() && a->second == 0) {
          outcomes[id] = prober_->probe_ordinal(ords[id]);  // crowded but idle: probe from a fresh process
        } else {
          crowded_skips_++;
          metrics::global().inc("mi355x_dp_liveness_crowded_skips_total", {{"device", id}}, 1.0,
                                "probes skipped on GPUs crowded with tenant processes");
        }
      }
    }
    ords.clear();
    for (const auto& [id, o] : ordinals())
      if (reasons.count(id)) ords[id] = o;
    const double now = mono_s();
    const double grace = busy_known_ ? cfg_.busy_grace_s : std::min(cfg_.busy_grace_s, cfg_.unknown_busy_grace_s);
    std::set<std::string> idle_wedged;
    std::vector<std::string> waiting;
    for (const auto& [id, o] : outcomes)
      if (o.pending && busy_devs.count(id)) waiting.push_back(id);
    if (!waiting.empty() && cfg_.corroborate) {
      const auto act = gfx_activity();
      for (const auto& id : waiting) {
        const GpuDevice* d = dev(id);
        auto a = d ? act.find(d->bdf) : act.end();
        Track& tr = track_[id];
        tr.idle_pending = a != act.end() && a->second == 0 ? tr.idle_pending + 1 : 0;
        if (tr.idle_pending >= cfg_.idle_sweeps) idle_wedged.insert(id);
      }
    }
    for (const auto& [id, o] : outcomes) {
      Track& tr = track_[id];
      metrics::global().set("mi355x_dp_liveness_probe_ms", o.latency_ms, {{"device", id}},
                            "last liveness probe round trip");
      if (!o.pending) tr.idle_pending = 0;
      if (o.ok) {
        tr.fails = 0;
        tr.oks++;
        tr.pending_since = -1;
        if (!tr.live && tr.oks >= cfg_.recover_threshold) tr.live = true;
      } else if (o.pending && busy_devs.count(id) && !idle_wedged.count(id) &&
                 now - (tr.pending_since >= 0 ? tr.pending_since : now) < grace) {
        if (tr.pending_since < 0) tr.pending_since = now;  // queued behind a tenant: inconclusive
        metrics::global().inc("mi355x_dp_liveness_inconclusive_total", {{"device", id}}, 1.0,
                              "probes queued behind a busy GPU");
      } else {
        tr.oks = 0;
        tr.fails++;
        tr.last_reason = o.reason;
        if (idle_wedged.count(id)) {
          tr.last_reason += " while the GPU reports 0% GFX activity (" + std::to_string(tr.idle_pending) +
                            " sweeps): no tenant kernel is running";
          metrics::global().inc("mi355x_dp_liveness_idle_pending_total", {{"device", id}}, 1.0,
                                "pending probes on an idle GFX engine");
        }
        if (!o.pending) tr.pending_since = -1;
        if (tr.live && tr.fails >= cfg_.fail_threshold) tr.live = false;
      }
      if (!tr.live) reasons[id].push_back("liveness probe: " + tr.last_reason);
    }
    for (auto& [id, rs] : reasons)
      if (!ords.count(id)) rs.push_back("no HIP device for this ID (render node inaccessible?)");
    if (cfg_.perf_check_every > 0 && sweeps_ % static_cast<uint64_t>(cfg_.perf_check_every) == 0) {
      std::map<std::string, int> cand;
      for (const auto& [id, o] : probe_ords)
        if (idle.count(id) && track_[id].live && ords.count(id)) cand[id] = o;
      if (!cand.empty()) perf_check(cand);
    }
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto& [id, pv] : perf_)
      if (reasons.count(id) && (pv.first == "failed" || (pv.first == "degraded" && cfg_.perf_action == "unhealthy")))
        reasons[id].push_back(pv.second);
  }

  if (cfg_.smi_ecc && smi_available()) {
    if (!smi_held_) smi_held_ = smi_hold();
    const SmiSnapshot snap = smi_snapshot();
    if (snap.ok) {
      std::map<std::string, const SmiGpu*> by_bdf;
      for (const auto& g : snap.gpus)
        if (g.ecc_ok) by_bdf[g.bdf] = &g;
      for (const auto& d : devices_) {
        auto it = by_bdf.find(d.bdf);
        if (it == by_bdf.end()) continue;
        const uint64_t cur = it->second->ecc_uncorrectable;
        auto prev = ecc_.find(d.id);
        if (prev != ecc_.end() && cur > prev->second)
          reasons[d.id].push_back("uncorrectable ECC errors rose " + std::to_string(prev->second) + "->" +
                                  std::to_string(cur));
        ecc_[d.id] = cur;
      }
    }
  }

  if (cfg_.smi_events) {
    if (!events_started_) {
      events_started_ = true;
      events_ = std::make_unique<SmiEventWatcher>();
      // vmfault 1, thermal_throttle 2, gpu_pre_reset 3, gpu_post_reset 4, queue_eviction 9
      const uint64_t mask = (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3) | (1ull << 8);
      const std::string err = events_->start(mask);
      if (!err.empty()) MI_LOG(kWarning, "amd-smi event notification unavailable: %s", err.c_str());
    }
    if (events_ && events_->running()) {
      for (const auto& ev : events_->poll(0)) {
        metrics::global().inc("mi355x_dp_gpu_events_total", {{"bdf", ev.bdf}, {"event", ev.name}}, 1.0,
                              "amd-smi GPU events");
        if (ev.name == "gpu_pre_reset") {
          resetting_[ev.bdf] = ev.message;
          MI_LOG(kWarning, "GPU %s: reset starting (%s)", ev.bdf.c_str(), ev.message.c_str());
        } else if (ev.name == "gpu_post_reset") {
          resetting_.erase(ev.bdf);
          MI_LOG(kWarning, "GPU %s: reset finished", ev.bdf.c_str());
        } else {
          MI_LOG(kInfo, "GPU %s: %s %s", ev.bdf.c_str(), ev.name.c_str(), ev.message.c_str());
        }
      }
    }
    for (const auto& d : devices_)
      if (resetting_.count(d.bdf))
        reasons[d.id].push_back("GPU reset in progress (amd-smi gpu_pre_reset, no post_reset yet)");
  }

  if (cfg_.smi_xgmi) fabric_check();

  std::map<std::string, Verdict> next;
  for (auto& [id, rs] : reasons) next[id] = Verdict{rs.empty(), rs};
  bool changed = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto& [id, v] : next) {
      auto old = snapshot_.find(id);
      if (old == snapshot_.end() || old->second.healthy != v.healthy) {
        changed = true;
        std::string why;
        for (const auto& r : v.reasons) why += (why.empty() ? "" : "; ") + r;
        MI_LOG(kWarning, "device %s: %s -> %s %s", id.c_str(),
               old == snapshot_.end() ? "?" : (old->second.healthy ? "Healthy" : "Unhealthy"),
               v.healthy ? "Healthy" : "Unhealthy", why.c_str());
      }
    }
    if (changed) version_++;
    snapshot_ = std::move(next);
    for (const auto& [id, v] : snapshot_)
      metrics::global().set("mi355x_dp_device_healthy", v.healthy ? 1.0 : 0.0, {{"device", id}},
                            "1 if the device is advertised Healthy");
  }
  sweeps_++;
  last_sweep_ms_ = (mono_s() - t0) * 1e3;
  return changed;
}

// ---- xGMI link state (health/fabric.py FabricWatcher) ----------------------------
namespace {
constexpr int kLinkUp = 1;
constexpr int kLinkTypeXgmi = 2;

std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

// the JSON shape of core().smi_xgmi_links()
SmiXgmiSnapshot xgmi_from_json(const std::string& text) {
  SmiXgmiSnapshot snap;
  std::string err;
  auto doc = json::parse(text, &err);
  if (!doc || doc->kind != json::Value::Object) {
    snap.error = "xgmi snapshot: " + (err.empty() ? std::string("not an object") : err);
    return snap;
  }
  auto flag = [](const json::Value* v) { return v && v->kind == json::Value::Bool && v->b; };
  auto num = [](const json::Value* v, long long dflt) {
    return v && v->kind == json::Value::Number ? std::strtoll(v->s.c_str(), nullptr, 10) : dflt;
  };
  snap.ok = flag(doc->get("ok"));
  snap.error = doc->str("error");
  if (const json::Value* gpus = doc->get("gpus"); gpus && gpus->kind == json::Value::Array)
    for (const auto& g : gpus->arr) {
      SmiXgmiLinks l;
      l.bdf = g.str("bdf");
      l.status_ok = flag(g.get("status_ok"));
      if (const json::Value* st = g.get("status"); st && st->kind == json::Value::Array)
        for (const auto& x : st->arr) l.status.push_back(static_cast<int>(num(&x, -1)));
      l.metrics_ok = flag(g.get("metrics_ok"));
      if (const json::Value* ps = g.get("peers"); ps && ps->kind == json::Value::Array)
        for (const auto& p : ps->arr) {
          SmiLinkPeer q;
          q.peer_bdf = p.str("peer_bdf");
          q.link_type = static_cast<int>(num(p.get("link_type"), -1));
          q.bit_rate_gbps = static_cast<uint32_t>(num(p.get("bit_rate_gbps"), 1));
          l.peers.push_back(q);
        }
      snap.gpus.push_back(std::move(l));
    }
  return snap;
}
}  // namespace

SmiXgmiSnapshot Engine::read_xgmi() {
  if (xgmi_source) return xgmi_source();
  if (!cfg_.xgmi_file.empty()) {
    auto text = read_file(cfg_.xgmi_file);
    if (!text) {
      SmiXgmiSnapshot s;
      s.error = "xgmi snapshot " + cfg_.xgmi_file + " unreadable";
      return s;
    }
    return xgmi_from_json(*text);
  }
  return smi_xgmi_links();
}

void Engine::fabric_check() {
  const SmiXgmiSnapshot snap = read_xgmi();
  if (!snap.ok) {
    if (snap.error != xgmi_error_) MI_LOG(kWarning, "xGMI link state unavailable: %s", snap.error.c_str());
    xgmi_error_ = snap.error;
    return;
  }
  xgmi_error_.clear();
  xgmi_readings_++;
  std::set<std::pair<std::string, std::string>> degraded;
  std::map<std::string, int> down;
  auto pair = [](const std::string& a, const std::string& b) { return a <= b ? std::make_pair(a, b) : std::make_pair(b, a); };
  for (const auto& g : snap.gpus) {
    const std::string bdf = lower(g.bdf);
    auto me_it = gpu_by_bdf_.find(bdf);
    if (me_it == gpu_by_bdf_.end()) continue;  // a GPU this plugin does not advertise
    const std::string& me = me_it->second;
    int up = -1;
    if (g.status_ok) up = static_cast<int>(std::count(g.status.begin(), g.status.end(), kLinkUp));
    std::set<std::string> live;
    if (g.metrics_ok)
      for (const auto& p : g.peers) {
        const std::string pb = lower(p.peer_bdf);
        if (p.link_type == kLinkTypeXgmi && gpu_by_bdf_.count(pb) && p.bit_rate_gbps > 0) live.insert(pb);
      }
    auto base = xgmi_base_.find(bdf);
    if (base == xgmi_base_.end()) {
      xgmi_base_[bdf] = {up, live};
      continue;
    }
    std::vector<std::string> lost_peers;
    for (const auto& pb : base->second.second)
      if (!live.count(pb)) lost_peers.push_back(pb);
    const int lost_links = base->second.first >= 0 && up >= 0 ? base->second.first - up : 0;
    if (!lost_peers.empty()) {
      for (const auto& pb : lost_peers) degraded.insert(pair(me, gpu_by_bdf_.at(pb)));
    } else if (lost_links > 0) {
      // no peer can be named: every xGMI pair of this GPU
      std::set<std::string> peers = base->second.second;
      if (peers.empty())
        for (const auto& [b, k] : gpu_by_bdf_)
          if (b != bdf) peers.insert(b);
      for (const auto& pb : peers) {
        auto o = gpu_by_bdf_.find(pb);
        if (o != gpu_by_bdf_.end() && o->second != me) degraded.insert(pair(me, o->second));
      }
    }
    if (lost_links > 0 || !lost_peers.empty())
      down[bdf] = std::max(lost_links, static_cast<int>(lost_peers.size()));
  }
  int total = 0;
  for (const auto& [b, n] : down) total += n;
  std::lock_guard<std::mutex> lk(mu_);
  links_down_ = down;
  if (degraded == degraded_) return;
  for (const auto& p : degraded)
    if (!degraded_.count(p))
      MI_LOG(kWarning, "xGMI link between GPUs %s and %s is down: multi-GPU placement avoids the pair",
             p.first.c_str(), p.second.c_str());
  for (const auto& p : degraded_)
    if (!degraded.count(p))
      MI_LOG(kWarning, "xGMI link between GPUs %s and %s is back up", p.first.c_str(), p.second.c_str());
  degraded_ = std::move(degraded);
  fabric_version_++;
  metrics::global().set("mi355x_dp_xgmi_links_down", total, {}, "xGMI links down vs the first reading");
}

std::vector<std::pair<std::string, std::string>> Engine::degraded_links() const {
  std::lock_guard<std::mutex> lk(mu_);
  return {degraded_.begin(), degraded_.end()};
}

uint64_t Engine::fabric_version() const {
  std::lock_guard<std::mutex> lk(mu_);
  return fabric_version_;
}

std::map<std::string, int> Engine::links_down() const {
  std::lock_guard<std::mutex> lk(mu_);
  return links_down_;
}

// ---- throughput check (health/monitor.py _perf_check) ----------------------------
std::vector<std::string> Engine::perf_problems(const ProbeOutcome& o) const {
  auto get = [&](const char* k) {
    auto it = o.detail.find(k);
    return it == o.detail.end() ? 0.0 : it->second;
  };
  const double cus = get("cu_count");
  const double share = cus > 0 ? std::min(1.0, cus / 256.0) : 1.0;  // a CPX partition has 1/8 of the CUs
  std::vector<std::string> out;
  struct Floor {
    const char* key;
    double floor;
    const char* what;
    const char* unit;
  };
  for (const Floor& f : {Floor{"hbm_read_gbps", cfg_.perf_min_hbm_read_gbps, "HBM read", "GB/s"},
                         Floor{"hbm_write_gbps", cfg_.perf_min_hbm_write_gbps, "HBM write", "GB/s"},
                         Floor{"mfma_tflops", cfg_.perf_min_mfma_tflops, "bf16 MFMA", "TFLOP/s"}}) {
    const double v = get(f.key);
    if (f.floor > 0 && v < f.floor * share) {
      char b[128];
      std::snprintf(b, sizeof(b), "%s %.0f %s < %.0f", f.what, v, f.unit, f.floor * share);
      out.push_back(b);
    }
  }
  std::vector<double> clocks;
  for (double c : o.xcd_clock_mhz)
    if (c > 0) clocks.push_back(c);
  if (clocks.size() >= 2 && cfg_.perf_min_xcd_clock_ratio > 0) {
    std::vector<double> sorted = clocks;
    std::sort(sorted.begin(), sorted.end());
    const double med = sorted[sorted.size() / 2];
    const size_t i = static_cast<size_t>(std::min_element(clocks.begin(), clocks.end()) - clocks.begin());
    if (clocks[i] < cfg_.perf_min_xcd_clock_ratio * med) {
      char b[128];
      std::snprintf(b, sizeof(b), "XCD %zu at %.0f MHz vs median %.0f MHz under MFMA load", i, clocks[i], med);
      out.push_back(b);
    }
  }
  return out;
}

void Engine::perf_check(const std::map<std::string, int>& ords) {
  trace::Span span("health.perf_check", "health", {{"devices", std::to_string(ords.size())}});
  std::vector<int> uniq;
  for (const auto& [id, o] : ords) uniq.push_back(o);
  const auto by_ord = prober_->probe(uniq, {}, "perf");
  perf_checks_++;
  auto& m = metrics::global();
  m.inc("mi355x_dp_perf_checks_total", {}, 1.0, "throughput checks run (HBM pattern + MFMA + clocks)");
  static const std::map<std::string, double> kState = {{"ok", 0.0}, {"degraded", 1.0}, {"failed", 2.0}};
  for (const auto& [id, ord] : ords) {
    auto it = by_ord.find(ord);
    if (it == by_ord.end()) continue;
    const ProbeOutcome& o = it->second;
    std::string state = "ok", why;
    if (!o.ok) {
      state = "failed";
      why = "throughput check: " + o.reason;
    } else if (const auto probs = perf_problems(o); !probs.empty()) {
      state = "degraded";
      why = "throughput check: ";
      for (size_t i = 0; i < probs.size(); ++i) why += (i ? "; " : "") + probs[i];
    }
    std::string prev = "ok";
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (auto p = perf_.find(id); p != perf_.end()) prev = p->second.first;
      perf_[id] = {state, why};
      perf_last_[id] = o;
    }
    if (state != prev)
      glog::log(state == "ok" ? glog::kInfo : glog::kWarning, __FILE__, __LINE__, "device %s: throughput check %s -> %s %s",
                id.c_str(), prev.c_str(), state.c_str(), why.c_str());
    auto get = [&](const char* k) {
      auto d = o.detail.find(k);
      return d == o.detail.end() ? 0.0 : d->second;
    };
    if (o.ok)
      MI_VLOG(2, "device %s: throughput HBM write %.0f / read %.0f GB/s, bf16 MFMA %.0f TFLOP/s at %.0f MHz", id.c_str(),
              get("hbm_write_gbps"), get("hbm_read_gbps"), get("mfma_tflops"), get("clock_mhz_median"));
    const metrics::Labels dev = {{"device", id}};
    m.set("mi355x_dp_perf_state", kState.at(state), dev,
          "last throughput check: 0 ok, 1 degraded (rates under the floors), 2 failed");
    if (o.ok) {
      m.set("mi355x_dp_perf_hbm_read_gbps", get("hbm_read_gbps"), dev, "last throughput check: HBM read bandwidth");
      m.set("mi355x_dp_perf_hbm_write_gbps", get("hbm_write_gbps"), dev, "last throughput check: HBM write bandwidth");
      m.set("mi355x_dp_perf_mfma_tflops", get("mfma_tflops"), dev,
            "last throughput check: sustained dense bf16 MFMA rate");
      m.set("mi355x_dp_perf_clock_mhz", get("clock_mhz_median"), dev,
            "last throughput check: median workgroup shader clock under MFMA load");
      for (size_t x = 0; x < o.xcd_clock_mhz.size(); ++x)
        m.set("mi355x_dp_perf_xcd_clock_mhz", o.xcd_clock_mhz[x], {{"device", id}, {"xcd", std::to_string(x)}},
              "last throughput check: median shader clock per XCD");
    }
  }
}

std::map<std::string, ProbeOutcome> Engine::perf_last() const {
  std::lock_guard<std::mutex> lk(mu_);
  return perf_last_;
}

uint64_t Engine::xgmi_readings() const { return xgmi_readings_; }
std::string Engine::xgmi_error() const { return xgmi_error_; }

std::map<std::string, std::pair<std::string, std::string>> Engine::perf_verdicts() const {
  std::lock_guard<std::mutex> lk(mu_);
  return perf_;
}

}  // namespace mi355x::health
