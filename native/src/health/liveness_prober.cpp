// The liveness probe processes (LivenessProber in mi355x/health_engine.h;
// health/liveness.py for the Python policy): a persistent
// `mi355x-liveness-probe --serve` child, or a process per device, started with
// posix_spawn() and pipes; every wait is a poll() bounded by a deadline and an
// abort fd. Replies are nonce-checked here and identity-checked by the Engine.
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
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>

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

using Got = LivenessProber::Got;

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
// The running --serve child. Replies are routed by request id: whichever
// caller is waiting reads the pipe for everyone (reading), files each line
// under its id and wakes the others. The pipe fds live as long as the object,
// so a reader never polls a descriptor another thread closed.
struct LivenessProber::Server {
  Child c;
  std::mutex mu;
  std::condition_variable cv;
  bool reading = false;  // a caller is reading c.out (c.buf and c.eof are its own meanwhile)
  bool dead = false;     // EOF, write failure or shut down
  bool aborted = false;  // the abort fd became readable (shutdown)
  bool reaped = false;
  bool concurrent = false;  // the hello line: tagged requests are answered as they complete
  std::map<uint64_t, std::string> replies;
  std::set<uint64_t> waiting;
  std::deque<uint64_t> order;  // waiting ids in send order (a reply without an id answers the oldest)
  std::optional<std::vector<int>> visible;
  std::set<std::string> own_kfd;

  ~Server() {
    stop();
    if (c.in >= 0) ::close(c.in);
    if (c.out >= 0) ::close(c.out);
  }
  bool alive() {
    std::lock_guard<std::mutex> lk(mu);
    if (dead || c.pid <= 0) return false;
    int st = 0;
    if (::waitpid(c.pid, &st, WNOHANG) == c.pid) {
      reaped = true;
      dead = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
  // "quit", SIGKILL to its session, reaped; the waiters see EOF
  void stop() {
    pid_t pid;
    {
      std::lock_guard<std::mutex> lk(mu);
      if (!dead && c.in >= 0) write_all(c.in, "quit\n");
      dead = true;
      pid = reaped ? -1 : c.pid;
      reaped = true;
      cv.notify_all();
    }
    if (pid > 0) {
      ::kill(-pid, SIGKILL);
      ::kill(pid, SIGKILL);
      int st = 0;
      while (::waitpid(pid, &st, 0) < 0 && errno == EINTR) {
      }
    }
  }
  // a reply line -> the waiting caller it answers (under mu)
  void file(const std::string& line) {
    uint64_t id = 0;
    bool tagged = false;
    if (line.compare(0, 6, "{\"id\":") == 0) {
      char* end = nullptr;
      id = std::strtoull(line.c_str() + 6, &end, 10);
      tagged = end != line.c_str() + 6;
    }
    if (!tagged) {
      if (order.empty()) return;
      id = order.front();
    }
    if (waiting.count(id)) replies[id] = line;
  }
};

LivenessProber::LivenessProber(ProberConfig cfg) : cfg_(std::move(cfg)) {}
LivenessProber::~LivenessProber() { close(); }

bool LivenessProber::server_running() const {
  std::shared_ptr<Server> s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    s = server_;
  }
  if (!s) return false;
  std::lock_guard<std::mutex> lk(s->mu);
  return s->c.pid > 0 && !s->dead;
}

int LivenessProber::server_pid() const {
  std::shared_ptr<Server> s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    s = server_;
  }
  if (!s) return -1;
  std::lock_guard<std::mutex> lk(s->mu);
  return s->dead ? -1 : static_cast<int>(s->c.pid);
}

double LivenessProber::inner_timeout() const { return cfg_.timeout_s - std::min(0.5, 0.25 * cfg_.timeout_s); }

void LivenessProber::close() {
  std::shared_ptr<Server> old;
  {
    std::lock_guard<std::mutex> lk(mu_);
    old.swap(server_);
    issued_.clear();  // a new server starts without outstanding dispatches
    restart_wanted_ = false;
  }
  if (old) old->stop();  // outside mu_: the GPU process' teardown can take a while
}

void LivenessProber::set_visible(std::optional<std::vector<int>> ordinals) {
  if (ordinals) {
    std::sort(ordinals->begin(), ordinals->end());
    ordinals->erase(std::unique(ordinals->begin(), ordinals->end()), ordinals->end());
  }
  std::lock_guard<std::mutex> lk(mu_);
  visible_ = std::move(ordinals);
}

std::set<std::string> LivenessProber::own_kfd_entries(const std::set<int64_t>& gpu_ids) {
  std::shared_ptr<Server> s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    s = server_;
  }
  if (!s || !s->alive()) return {};
  std::lock_guard<std::mutex> lk(s->mu);
  if (s->own_kfd.size() > 1) {  // another GPU process started with the server: keep what still exists
    std::set<std::string> still;
    for (const auto& e : list_dir(cfg_.kfd_proc_dir))
      if (s->own_kfd.count(e)) still.insert(e);
    s->own_kfd = still;
  }
  if (s->own_kfd.size() == 1) return s->own_kfd;
  if (s->own_kfd.size() > 1 && cfg_.keep_queues && !gpu_ids.empty()) {
    // the kept-queue server holds a queue on every GPU it probed; a pod's process only on the pod's
    std::vector<std::string> match;
    for (const auto& e : s->own_kfd) {
      std::set<int64_t> have;
      const std::string qdir = path_join(path_join(cfg_.kfd_proc_dir, e), "queues");
      for (const auto& q : list_dir(qdir))
        if (auto g = read_trimmed(path_join(path_join(qdir, q), "gpuid"))) have.insert(parse_i64(*g, 0));
      if (std::includes(have.begin(), have.end(), gpu_ids.begin(), gpu_ids.end())) match.push_back(e);
    }
    if (match.size() == 1) s->own_kfd = {match[0]};
    if (s->own_kfd.size() == 1) return s->own_kfd;
  }
  return {};
}

ProbeOutcome LivenessProber::probe_ordinal(int ordinal, const std::string& kind) {
  return spawn_all({ordinal}, kind, cfg_.timeout_s)[ordinal];
}

std::map<int, ProbeOutcome> LivenessProber::spawn_all(const std::vector<int>& ords, const std::string& kind,
                                                      double timeout_s) {
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
      std::snprintf(tmo, sizeof(tmo), "%.2f", std::max(0.5, timeout_s - 0.5));
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
    const double deadline = mono_s() + timeout_s;
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
        std::snprintf(why, sizeof(why), "deadline exceeded (%.1fs)", timeout_s);
        o.reason = aborted ? "probe interrupted (shutdown)" : why;
        o.latency_ms = ms;
        o.pending = kind == "probe" && !aborted;  // inconclusive on a busy GPU
        o.interrupted = aborted;
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

// The server for the sweep's next request: started (or restarted, when the
// GPUs it may touch changed or a check asked for it) here and only here.
std::shared_ptr<LivenessProber::Server> LivenessProber::ensure_server(const std::vector<int>& uniq,
                                                                      std::string* err) {
  std::optional<std::vector<int>> visible;
  std::shared_ptr<Server> stale;
  {
    std::lock_guard<std::mutex> lk(mu_);
    visible = visible_;
    if (visible) {
      std::set<int> u(visible->begin(), visible->end());
      bool grow = false;
      for (int o : uniq) grow |= u.insert(o).second;
      if (grow) visible = std::vector<int>(u.begin(), u.end());
    }
    if (server_ && !restart_wanted_ && server_->visible == visible && server_->alive()) return server_;
    if (restart_wanted_ && server_) {
      server_restarts++;
      MI_LOG(kWarning, "probe server failed a device that a fresh process found healthy (PreStartContainer check); "
                       "restarting it");
    }
    restart_wanted_ = false;
    stale.swap(server_);
    issued_.clear();
  }
  if (stale) stale->stop();
  std::vector<std::string> argv = cfg_.argv_prefix;
  argv.push_back(cfg_.exe);
  argv.push_back("--serve");
  if (cfg_.keep_queues) argv.push_back("--keep");
  std::set<std::string> before;
  for (const auto& e : list_dir(cfg_.kfd_proc_dir)) before.insert(e);
  auto srv = std::make_shared<Server>();
  if (!spawn_child(argv, child_env(cfg_, visible ? join_ints(*visible, ",") : ""), true, &srv->c, err)) return nullptr;
  std::string hello;
  const Got g = read_line(&srv->c, mono_s() + cfg_.timeout_s, abort_fd_, &hello);
  auto doc = g == Got::kLine ? json::parse(hello) : std::nullopt;
  if (!doc || !jbool(&*doc, "serve") || !jbool(&*doc, "ok")) {
    srv->stop();
    // shutdown interrupted the start: "interrupted", so probe() reports interrupted
    // outcomes instead of falling back to fresh GPU processes while the daemon stops
    *err = g == Got::kAbort     ? "interrupted"
           : g == Got::kTimeout ? "probe server did not start within the deadline"
                                : "probe server failed to start: " + hello.substr(0, 200);
    return nullptr;
  }
  // informational: a server built on the HIP runtime answers tagged requests in
  // order, so a check there waits its turn (within its own budget)
  srv->concurrent = jbool(&*doc, "concurrent");
  srv->visible = visible;
  for (const auto& e : list_dir(cfg_.kfd_proc_dir))
    if (!before.count(e)) srv->own_kfd.insert(e);
  std::lock_guard<std::mutex> lk(mu_);
  server_ = srv;
  issued_.clear();
  server_starts++;
  return srv;
}

// Sends "@<id> <body>" and waits for the reply with that id until `deadline`.
LivenessProber::Got LivenessProber::transact(const std::shared_ptr<Server>& s, const std::string& body,
                                             double deadline, std::string* reply) {
  const uint64_t id = next_id_++;
  std::unique_lock<std::mutex> lk(s->mu);
  if (s->dead) return Got::kEof;
  if (!write_all(s->c.in, "@" + std::to_string(id) + " " + body + "\n")) {
    s->dead = true;
    s->cv.notify_all();
    return Got::kEof;
  }
  s->waiting.insert(id);
  s->order.push_back(id);
  Got result;
  while (true) {
    if (auto it = s->replies.find(id); it != s->replies.end()) {
      *reply = std::move(it->second);
      s->replies.erase(it);
      result = Got::kLine;
      break;
    }
    if (s->aborted) {
      result = Got::kAbort;
      break;
    }
    if (s->dead) {
      result = Got::kEof;
      break;
    }
    if (mono_s() >= deadline) {
      result = Got::kTimeout;
      break;
    }
    if (!s->reading) {
      s->reading = true;
      lk.unlock();
      std::string line;
      const Got g = read_line(&s->c, deadline, abort_fd_, &line);
      lk.lock();
      s->reading = false;
      if (g == Got::kLine) s->file(line);
      else if (g == Got::kEof) s->dead = true;
      else if (g == Got::kAbort) s->aborted = true;
      s->cv.notify_all();
      continue;
    }
    // a bounded wait on the system clock: libstdc++ implements it with
    // pthread_cond_timedwait (steady-clock waits use pthread_cond_clockwait,
    // which GCC 11's ThreadSanitizer does not intercept); the loop re-checks
    // the steady deadline, so a clock step costs at most one 50 ms slice
    const double left = std::min(0.05, std::max(0.0, deadline - mono_s()));
    s->cv.wait_until(lk, std::chrono::system_clock::now() +
                             std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                 std::chrono::duration<double>(left)));
  }
  s->waiting.erase(id);  // a reply that comes later is dropped
  s->order.erase(std::remove(s->order.begin(), s->order.end(), id), s->order.end());
  return result;
}

std::map<int, ProbeOutcome> LivenessProber::request(const std::shared_ptr<Server>& s, const std::vector<int>& uniq,
                                                    const std::string& kind, const std::map<int, double>& deadlines,
                                                    double wait_until, std::string* err) {
  const double t0 = mono_s();
  // the server numbers the GPUs it sees: with a visibility list, their positions
  std::map<int, int> local, host;
  for (int o : uniq) {
    int l = o;
    if (s->visible) l = static_cast<int>(std::find(s->visible->begin(), s->visible->end(), o) - s->visible->begin());
    local[o] = l;
    host[l] = o;
  }
  std::map<int, uint32_t> nonces;
  for (int o : uniq) nonces[o] = make_nonce(o);
  double top = 0;
  for (const auto& [o, d] : deadlines) top = std::max(top, d);
  char head[96];
  if (kind == "perf")
    std::snprintf(head, sizeof(head), "perf %d %.3f %d", cfg_.perf_iters, top, cfg_.perf_mib);
  else
    std::snprintf(head, sizeof(head), "%s %d %.3f", kind.c_str(), cfg_.iters, top);
  std::string line = head;
  for (int o : uniq) {
    char tok[64];
    std::snprintf(tok, sizeof(tok), " %d:%u:%.3f", local[o], nonces[o], deadlines.at(o));
    line += tok;
  }
  std::string reply;
  const Got g = transact(s, line, wait_until, &reply);
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
  std::lock_guard<std::mutex> lk(mu_);  // issued_
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
    const bool timed_out = jnum(d, "hip_error", 0) == -1 || jnum(d, "hsa_error", 0) == -1;
    if (kind != "probe") {  // sweeps run on their own queue: the kept slot is untouched
      out[o] = judge(jbool(d, "ok"), d, nonces[o], ms);
      out[o].queue_lost = timed_out && !cfg_.keep_queues;
      continue;
    }
    // a late verdict answers the dispatch (and nonce) of an earlier request that left it pending
    auto& mine = issued_[o];
    const bool late = jbool(d, "late");
    uint32_t expect = nonces[o];
    if (late) {
      const json::Value* n = d->get("nonce");
      const uint32_t got = n && n->kind == json::Value::Number
                               ? static_cast<uint32_t>(std::strtoull(n->s.c_str(), nullptr, 10)) : 0;
      if (auto f = std::find(mine.begin(), mine.end(), got); f != mine.end()) {
        expect = got;
        mine.erase(f);
      }
    }
    ProbeOutcome r = judge(jbool(d, "ok"), d, expect, ms);
    r.queue_lost = timed_out && !cfg_.keep_queues;
    if (!r.ok && jnum(d, "pending_s", 0) > 0) {
      r.pending = true;
      mine.push_back(nonces[o]);  // may be the dispatch still queued on the kept slot
      if (mine.size() > 8) mine.erase(mine.begin());
    } else if (!r.ok && jnum(d, "hip_error", 0) == -1 && !cfg_.keep_queues) {
      r.pending = true;  // timed out without a kept slot: no late verdict will follow
    } else if (!late) {
      mine.clear();  // the slot had nothing outstanding
    }
    out[o] = r;
  }
  return out;
}

std::map<int, ProbeOutcome> LivenessProber::probe_server(const std::vector<int>& uniq, const std::set<int>& busy,
                                                         const std::string& kind, std::string* err) {
  trace::Span span("liveness.request", "health", {{"ordinals", std::to_string(uniq.size())}, {"kind", kind}});
  std::shared_ptr<Server> srv = ensure_server(uniq, err);
  if (!srv) return {};
  const double inner = inner_timeout();
  std::map<int, double> deadlines;
  for (int o : uniq)  // a dispatch queued behind a tenant's kernel stays on the kept queue for the next request
    deadlines[o] = kind == "probe" && cfg_.keep_queues && busy.count(o) ? std::min(inner, cfg_.busy_deadline_s) : inner;
  double top = 0;
  for (const auto& [o, d] : deadlines) top = std::max(top, d);
  // the reply is due at the longest device deadline; the margin covers the
  // server's own bookkeeping (the full timeout when every device gets it)
  const double wait = mono_s() + std::min(cfg_.timeout_s, top + (cfg_.timeout_s - inner));
  auto out = request(srv, uniq, kind, deadlines, wait, err);
  if (!err->empty()) return {};
  for (const auto& [o, r] : out)
    if (r.queue_lost) {
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
  bool use_server;
  {
    std::lock_guard<std::mutex> lk(mu_);
    use_server = cfg_.persistent && backoff_ == 0;
    backoff_ = std::max(0, backoff_ - 1);
  }
  if (use_server) {
    std::string err;
    auto res = probe_server(uniq, busy, kind, &err);
    if (err.empty()) {
      std::vector<int> failed;
      for (int o : uniq)
        if (!res[o].ok && !(res[o].pending && busy.count(o))) failed.push_back(o);
      if (!failed.empty()) {
        // the server's runtime lives across sweeps: a failure only counts if a fresh process confirms it
        auto fresh = spawn_all(failed, kind, cfg_.timeout_s);
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
      for (int o : uniq) {
        out[o].reason = "probe interrupted (shutdown)";
        out[o].interrupted = true;
      }
      return out;
    }
    // a wedged device stalls the whole server: drop it and isolate per device
    MI_LOG(kWarning, "probe server failed (%s); re-probing each device in its own process", err.c_str());
    fallbacks++;
    {
      std::lock_guard<std::mutex> lk(mu_);
      backoff_ = 4;
    }
    close();
  }
  auto res = spawn_all(uniq, kind, cfg_.timeout_s);
  sweeps++;
  return res;
}

std::map<int, ProbeOutcome> LivenessProber::check(const std::vector<int>& ordinals,
                                                  const std::function<std::set<int>()>& busy_of, double budget_s) {
  trace::Span span("liveness.check", "health", {{"ordinals", std::to_string(ordinals.size())}});
  const double t0 = mono_s(), end = t0 + budget_s;
  std::vector<int> uniq(ordinals);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  checks++;
  std::map<int, ProbeOutcome> out;
  if (uniq.empty()) return out;
  auto inconclusive = [&](int o, const std::string& why) {
    ProbeOutcome r;
    r.pending = true;
    r.reason = why;
    r.latency_ms = (mono_s() - t0) * 1e3;
    out[o] = r;
    check_inconclusive++;
  };
  // which GPUs other processes use: read (a kfd process-list scan) only when a
  // probe did not pass at once, i.e. never on the common path
  std::optional<std::set<int>> busy_memo;
  auto busy = [&]() -> const std::set<int>& {
    if (!busy_memo) busy_memo = busy_of ? busy_of() : std::set<int>{};
    return *busy_memo;
  };
  std::shared_ptr<Server> srv;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (cfg_.persistent && backoff_ == 0 && server_ && !restart_wanted_) {
      bool covers = true;
      if (server_->visible)
        for (int o : uniq)
          covers = covers && std::count(server_->visible->begin(), server_->visible->end(), o);
      if (covers) srv = server_;
    }
  }
  bool interrupted = false;
  auto ask = [&](const std::vector<int>& ords, double deadline) {
    std::map<int, double> dl;
    for (int o : ords) dl[o] = deadline;
    std::string err;
    auto got = request(srv, ords, "probe", dl, std::min(end, mono_s() + deadline + 0.25), &err);
    if (!err.empty()) {
      interrupted = err == "interrupted";
      if (!interrupted) MI_LOG(kWarning, "PreStartContainer check: probe server: %s", err.c_str());
      return std::map<int, ProbeOutcome>{};
    }
    for (const auto& [o, r] : got)
      if (r.queue_lost) {
        std::lock_guard<std::mutex> lk(mu_);
        restart_wanted_ = true;  // its timed-out queue cannot be freed: the next sweep restarts it
      }
    return got;
  };
  std::map<int, ProbeOutcome> got;  // the server's last verdict per ordinal
  std::vector<int> confirm;
  if (srv && srv->alive()) {
    const double inner = inner_timeout();
    // 1: every GPU with the busy deadline. An idle GPU answers in microseconds;
    // a dispatch queued behind a tenant's kernel stays on the kept queue.
    got = ask(uniq, std::min(inner, cfg_.busy_deadline_s));
    std::vector<int> idle_pending;
    for (int o : uniq) {
      if (interrupted) break;
      auto it = got.find(o);
      if (it != got.end() && it->second.ok) {
        out[o] = it->second;
      } else if (it != got.end() && !it->second.pending) {
        confirm.push_back(o);  // a definite failure (a wrong tile, an error): busy or not
      } else if (busy().count(o)) {
        inconclusive(o, it != got.end() ? it->second.reason : "no probe server answer on a busy GPU");
      } else if (it != got.end()) {
        idle_pending.push_back(o);
      } else {
        confirm.push_back(o);
      }
    }
    // 2: pending where no other process runs: wait for that same dispatch up
    // to 40% of the budget in all (the rest is for a fresh process' confirmation)
    const double idle_dl = std::min(inner, std::max(0.2, 0.4 * budget_s)) - (mono_s() - t0);
    if (!interrupted && !idle_pending.empty()) {
      auto again = ask(idle_pending, std::max(0.01, idle_dl));
      for (int o : idle_pending) {
        if (auto it = again.find(o); it != again.end()) got[o] = it->second;
        if (got.count(o) && got[o].ok) out[o] = got[o];
        else confirm.push_back(o);
      }
    }
  } else {
    for (int o : uniq) {
      if (busy().count(o)) inconclusive(o, "no probe server answer on a busy GPU");
      else confirm.push_back(o);
    }
  }
  if (interrupted) {
    for (int o : uniq) {
      out[o] = ProbeOutcome{};
      out[o].reason = "probe interrupted (shutdown)";
      out[o].interrupted = true;
    }
    return out;
  }
  if (confirm.empty()) return out;
  const double left = end - mono_s();
  if (left < 1.0) {  // a fresh GPU process needs its runtime start-up: not within what is left
    for (int o : confirm)
      inconclusive(o, "check budget spent" + (got.count(o) ? " (server: " + got[o].reason + ")" : std::string()));
    return out;
  }
  check_fresh += static_cast<int>(confirm.size());
  auto fresh = spawn_all(confirm, "probe", std::min(cfg_.timeout_s, left));
  for (int o : confirm) {
    ProbeOutcome f = fresh[o];
    const bool server_failed = got.count(o) && !got[o].ok;
    if (f.ok) {
      if (server_failed) {
        std::lock_guard<std::mutex> lk(mu_);
        restart_wanted_ = true;  // a stale server runtime: the next sweep restarts it
      }
    } else if (!f.interrupted) {
      // a fresh process that got nothing back: on a GPU no other process uses
      // that is a fault; on a busy one it may wait behind the tenant's kernels
      if (f.pending && !busy().count(o)) f.pending = false;
      if (f.pending) check_inconclusive++;
      if (server_failed) f.reason += " (server: " + got[o].reason + ")";
    }
    out[o] = f;
  }
  return out;
}

}  // namespace mi355x::health
