// mi355x-node-labeller: the node labeller as one native process.
//
// The reference ships its labeller as a compiled binary
// (cmd/k8s-node-labeller/main.go). This is the same job built from the
// framework's C++ core, with no interpreter in the process:
//
//   flags        one boolean per label kind (-vram, -cu-count, ... main.go:507-528),
//                -driver_type, node name from -node_name / $DS_NODE_NAME /
//                /labeller/hostname; -resync, -watch, -topology_watch, -dry_run,
//                -sysfs_root, -dev_root as in the Python CLI; glog flags accepted
//   labels       the 13 generators of main.go:123-385 plus the opt-in
//                gfx-target / xgmi-hive-count / xgmi-links-down, over the kfd
//                topology, sysfs, libdrm and amd-smi; container -> VF -> PF
//                (main.go:389-505); values sanitised to the Kubernetes rules.
//                Output is identical to rocm_k8s_device_plugin_amd/labeller/labels.py
//                (tests/test_native_labeller.py compares them on every fixture mode)
//   apiserver    in-cluster service account (token re-read when kubelet rotates
//                it), HTTPS with the cluster CA; GET the Node, JSON merge-PATCH
//                of metadata.labels; GET + PUT (409 retry) when RBAC has no
//                "patch" (controller.go:23-58 does the Update)
//   watch        ?watch=1&fieldSelector=metadata.name=<node>: a node re-created
//                or a label stripped is relabelled at once (the reference
//                reconciles on Create events, main.go:551-577); 410 re-lists;
//                reconnects with backoff; labels re-asserted every -resync.
//                -resync 0 is the reference's controller: label at start and
//                again only when the Node object is re-created (an ADDED event),
//                never exiting; -once applies once and exits (a Job)
//   topology     kfd generation_id + partition modes polled every
//                -topology_watch s: a partition switch relabels at once
//   config       -kubeconfig, else in-cluster unless $KUBECONFIG is set, else
//                $KUBECONFIG / $HOME/.kube/config (controller-runtime's order,
//                config.go:116-156): token, tokenFile or client-certificate auth
//   logging      glog's flags and output rules (mi355x/glog.h)
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <functional>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "../kube/http.h"
#include "../kube/json.h"
#include "../kube/kubeconfig.h"
#include "../kube/labels.h"
#include "mi355x/glog.h"
#include "mi355x/goflag.h"
#include "mi355x/drm_query.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/metrics.h"
#include "mi355x/pci_scan.h"
#include "mi355x/smi_query.h"
#include "mi355x/sysfs.h"
#include "mi355x/versions.h"

namespace {

using namespace mi355x;
using Labels = std::map<std::string, std::string>;
using labeller::prefix_of;
const std::vector<std::string>& kKinds = labeller::label_kinds();

struct Flags {
  std::map<std::string, bool> enabled;
  std::string driver_type;
  std::string node_name;
  std::string kubeconfig;
  double resync_s = 300.0;
  bool watch = true;
  double topology_watch_s = 5.0;
  bool dry_run = false;
  bool once = false;
  std::string sysfs_root = "/sys";
  std::string dev_root = "/dev";
  std::string sa_dir = "/var/run/secrets/kubernetes.io/serviceaccount";
  std::string apiserver;  // overrides KUBERNETES_SERVICE_HOST/PORT (tests, host-network debugging)
  std::string token_file;
  std::string ca_file;
  double watch_backoff_max_s = 30.0;
  int watch_timeout_s = 300;
  int metrics_port = 0;  // /metrics, /healthz, /readyz (0 = off; the reference serves none)
  glog::Options log;
};

constexpr const char* kTitle = "AMD GPU Node Labeller for Kubernetes (MI355X-native, native daemon)";


// the version banner, then the flags (main.go flag.Usage)
void print_usage(FILE* out, const char* argv0, const std::string& sysfs_root) {
  for (const auto& line : versions::banner(kTitle, argv0, sysfs_root)) std::fprintf(out, "%s\n", line.c_str());
  std::fprintf(out, "usage: %s [-<label kind> ...] [-driver_type container|vf-passthrough|pf-passthrough] "
               "[-node_name NAME] [-kubeconfig PATH] [-resync S] [-once] [-watch=false] [-topology_watch S] "
               "[-dry_run] [-metrics_port N] [-sysfs_root DIR] [-dev_root DIR] [-v N] [-logtostderr] [-alsologtostderr] "
               "[-stderrthreshold SEV] [-log_dir DIR] [-vmodule P=N] [-log_backtrace_at FILE:N]\nlabel kinds:",
               argv0);
  for (const auto& k : kKinds) std::fprintf(out, " -%s", k.c_str());
  std::fprintf(out, "\n");
}

// Go flag syntax: -name=value, -name value, --name; booleans only take =value;
// parsing stops at the first non-flag argument or after "--". *syntax: the
// flag package itself would have refused the line (exit 2 with the usage);
// otherwise the error is the labeller's own validation (exit 1).
bool parse_flags(int argc, char** argv, Flags* f, std::string* err, bool* syntax) {
  for (const auto& k : kKinds) f->enabled[k] = false;
  if (const char* n = std::getenv("DS_NODE_NAME")) f->node_name = n;
  static const std::set<std::string> kBool = {"watch", "dry_run", "once"};
  static const std::set<std::string> kValued = {"driver_type", "node_name", "kubeconfig", "resync", "topology_watch",
                                                "watch_backoff_max", "watch_timeout", "sysfs_root", "dev_root",
                                                "sa_dir", "apiserver", "token_file", "ca_file", "metrics_port"};
  *syntax = false;
  auto bad = [&](std::string msg) {
    *err = std::move(msg);
    *syntax = true;
    return false;
  };
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--") break;                            // terminator, consumed
    if (a.size() < 2 || a[0] != '-') break;          // first non-flag argument: parsing stops
    a = a.substr(a[1] == '-' ? 2 : 1);
    if (a.empty() || a[0] == '-' || a[0] == '=') return bad("bad flag syntax: " + std::string(argv[i]));
    std::string name = a, value;
    bool has_value = false;
    const size_t eq = a.find('=');
    if (eq != std::string::npos) {
      name = a.substr(0, eq);
      value = a.substr(eq + 1);
      has_value = true;
    }
    if (name == "h" || name == "help") {
      print_usage(stdout, argv[0], f->sysfs_root);
      std::exit(0);
    }
    const bool is_kind = f->enabled.count(name) > 0;
    if (!is_kind && !kBool.count(name) && !kValued.count(name) && !glog::is_flag(name))
      return bad("flag provided but not defined: -" + name);
    if (glog::is_bool_flag(name)) {
      glog::parse_flag(name, value, has_value, &f->log, err);
      if (!err->empty()) return bad(*err);
      continue;
    }
    if (is_kind || kBool.count(name)) {
      bool v = true;
      if (has_value && !goflag::parse_bool(value, &v)) return bad("invalid boolean value \"" + value + "\" for -" + name);
      if (is_kind) f->enabled[name] = v;
      if (name == "watch") f->watch = v;
      if (name == "dry_run") f->dry_run = v;
      if (name == "once") f->once = v;
      continue;
    }
    if (!has_value) {
      if (i + 1 >= argc) return bad("flag needs an argument: -" + name);
      value = argv[++i];
    }
    if (glog::parse_flag(name, value, true, &f->log, err)) {
      if (!err->empty()) return bad(*err);
    } else if (name == "driver_type") {
      f->driver_type = value;
    } else if (name == "node_name") {
      f->node_name = value;
    } else if (name == "kubeconfig") {
      f->kubeconfig = value;
    } else if (name == "resync") {
      if (!goflag::parse_float(value, &f->resync_s)) return bad("invalid value \"" + value + "\" for flag -resync");
    } else if (name == "topology_watch") {
      if (!goflag::parse_float(value, &f->topology_watch_s))
        return bad("invalid value \"" + value + "\" for flag -topology_watch");
    } else if (name == "watch_backoff_max") {
      if (!goflag::parse_float(value, &f->watch_backoff_max_s))
        return bad("invalid value \"" + value + "\" for flag -watch_backoff_max");
    } else if (name == "watch_timeout") {
      int v = 0;
      if (!goflag::parse_int_flag(value, &v)) return bad("invalid value \"" + value + "\" for flag -watch_timeout");
      f->watch_timeout_s = std::max(1, v);
    } else if (name == "metrics_port") {
      int v = 0;
      if (!goflag::parse_int_flag(value, &v) || v < 0 || v > 65535)
        return bad("invalid value \"" + value + "\" for flag -metrics_port");
      f->metrics_port = v;
    } else if (name == "sysfs_root") {
      f->sysfs_root = value;
    } else if (name == "dev_root") {
      f->dev_root = value;
    } else if (name == "sa_dir") {
      f->sa_dir = value;
    } else if (name == "apiserver") {
      f->apiserver = value;
    } else if (name == "token_file") {
      f->token_file = value;
    } else if (name == "ca_file") {
      f->ca_file = value;
    }
  }
  if (!f->driver_type.empty() && f->driver_type != "container" && f->driver_type != "vf-passthrough" &&
      f->driver_type != "pf-passthrough")
    return *err = "invalid driver_type " + f->driver_type, false;
  return true;
}

// the generators, key / value validation and mode selection live in
// src/kube/labels.cpp (shared with the fuzz target)
labeller::LabelOptions label_options(const Flags& f) {
  labeller::LabelOptions o;
  o.enabled = f.enabled;
  o.driver_type = f.driver_type;
  o.sysfs_root = f.sysfs_root;
  o.dev_root = f.dev_root;
  return o;
}

// ---- removal sets (main.go:50-83) and the merge patch -------------------------
std::vector<std::string> all_label_keys() {
  std::vector<std::string> keys;
  for (const auto& k : kKinds) keys.push_back(prefix_of(k, false));
  keys.push_back("amd.com/compute-partitioning-supported");
  keys.push_back("amd.com/memory-partitioning-supported");
  keys.push_back("amd.com/compute-memory-partition");
  return keys;
}

Labels remove_old_node_labels(Labels l) {
  for (const auto& k : all_label_keys()) l.erase(k);
  for (const auto& kind : kKinds) {
    const std::string k = prefix_of(kind, true);
    auto it = l.find(k);
    if (it != l.end()) {
      l.erase(k + "." + it->second);
      l.erase(it);
    }
    // orphaned beta counters <key>.<value> go too
    for (auto j = l.lower_bound(k + "."); j != l.end() && j->first.compare(0, k.size() + 1, k + ".") == 0;)
      j = l.erase(j);
  }
  return l;
}

// key -> value, or nullopt = delete
std::map<std::string, std::optional<std::string>> label_patch(const Labels& current, const Labels& desired) {
  Labels target = remove_old_node_labels(current);
  for (const auto& [k, v] : desired) target[k] = v;
  std::map<std::string, std::optional<std::string>> patch;
  for (const auto& [k, v] : current)
    if (!target.count(k)) patch[k] = std::nullopt;
  for (const auto& [k, v] : target) {
    auto it = current.find(k);
    if (it == current.end() || it->second != v) patch[k] = v;
  }
  return patch;
}

// ---- apiserver client -------------------------------------------------------
class Kube {
 public:
  http::Config cfg;
  std::string token_file;
  std::string token;
  int wake_fd = -1;

  // current bearer token: re-read when the file changes (kubelet rotates projected tokens)
  const std::string& bearer(bool force = false) {
    if (!token_file.empty()) {
      struct stat st {};
      if (::stat(token_file.c_str(), &st) == 0) {
        const long long mt = static_cast<long long>(st.st_mtim.tv_sec) * 1000000000LL + st.st_mtim.tv_nsec;
        if (force || mt != mtime_) {
          if (auto t = read_trimmed(token_file); t && !t->empty()) {
            token = *t;
            mtime_ = mt;
          }
        }
      }
    }
    return token;
  }

  http::Headers headers(const std::string& content_type = "") {
    http::Headers h = {{"Accept", "application/json"}, {"User-Agent", "mi355x-node-labeller-native"}};
    if (!content_type.empty()) h.emplace_back("Content-Type", content_type);
    const std::string& t = bearer();
    if (!t.empty()) h.emplace_back("Authorization", "Bearer " + t);
    return h;
  }

  http::Response call(const std::string& method, const std::string& path, const std::string& body = "",
                      const std::string& content_type = "") {
    const std::string before = bearer();
    http::Response r = http::request(cfg, method, path, headers(content_type), body, wake_fd);
    if (r.status == 401 && !token_file.empty() && bearer(true) != before)
      r = http::request(cfg, method, path, headers(content_type), body, wake_fd);  // rotated token: once
    return r;
  }

 private:
  long long mtime_ = -1;
};

std::string describe(const http::Response& r) {
  if (r.status == 0) return r.error;
  return "HTTP " + std::to_string(r.status) + ": " + r.body.substr(0, 300);
}

std::string path_escape(const std::string& s) {
  std::string out;
  for (const char ch : s) {
    const auto c = static_cast<unsigned char>(ch);
    if (std::isalnum(c) || c == '-' || c == '.' || c == '_' || c == '~') {
      out.push_back(ch);
    } else {
      char b[4];
      std::snprintf(b, sizeof(b), "%%%02X", c);
      out += b;
    }
  }
  return out;
}

struct Stats {
  int passes = 0, patches = 0, updates = 0, errors = 0;
  int watch_events = 0, watch_kicks = 0, watch_errors = 0, watch_restarts = 0, topology_changes = 0;
};

class Labeller {
 public:
  Labeller(const Flags& f, Kube* k) : f_(f), k_(k) {}

  bool reconcile() {
    ++st.passes;
    desired_ = labeller::generate_labels(label_options(f_));
    have_desired_ = true;
    const std::string path = "/api/v1/nodes/" + path_escape(f_.node_name);
    http::Response r = k_->call("GET", path);
    if (r.status != 200) return fail("reconcile of node " + f_.node_name + " failed: " + describe(r));
    auto node = json::parse(r.body);
    if (!node) return fail("reconcile of node " + f_.node_name + " failed: unparseable Node");
    const auto patch = label_patch(json::node_labels(*node), desired_);
    if (patch.empty()) return true;
    json::Value labels = json::Value::object();
    for (const auto& [k, v] : patch) labels.set(k, v ? json::Value::string(*v) : json::Value{});
    json::Value md = json::Value::object();
    md.set("labels", labels);
    json::Value body = json::Value::object();
    body.set("metadata", md);
    r = k_->call("PATCH", path, json::serialize(body), "application/merge-patch+json");
    if (r.status == 403) {
      // the upstream ClusterRole grants "update" but not "patch": GET + Update (controller.go:23-58)
      if (!update_with_retry(path)) return false;
    } else if (r.status != 200) {
      return fail("reconcile of node " + f_.node_name + " failed: " + describe(r));
    }
    ++st.patches;
    MI_LOG_FIELDS(kInfo, "node labels updated", ({{"node", f_.node_name}, {"changed", std::to_string(patch.size())}}));
    return true;
  }

  bool needs_reconcile(const json::Value& node) const {
    return !have_desired_ || !label_patch(json::node_labels(node), desired_).empty();
  }

  Stats st;

 private:
  bool fail(const std::string& msg) {
    ++st.errors;
    MI_LOG(kError, "%s", msg.c_str());
    return false;
  }

  bool update_with_retry(const std::string& path) {
    for (int attempt = 0; attempt < 5; ++attempt) {
      http::Response r = k_->call("GET", path);
      if (r.status != 200) return fail("update of node " + f_.node_name + " failed: " + describe(r));
      auto node = json::parse(r.body);
      if (!node || node->kind != json::Value::Object) return fail("update: unparseable Node");
      Labels l = remove_old_node_labels(json::node_labels(*node));
      for (const auto& [k, v] : desired_) l[k] = v;
      json::Value* md = node->get("metadata");
      if (!md) md = &node->set("metadata", json::Value::object());
      json::Value labels = json::Value::object();
      for (const auto& [k, v] : l) labels.set(k, json::Value::string(v));
      md->set("labels", labels);
      r = k_->call("PUT", path, json::serialize(*node), "application/json");
      if (r.status == 200) {
        ++st.updates;
        return true;
      }
      if (r.status != 409 || attempt == 4) return fail("update of node " + f_.node_name + " failed: " + describe(r));
    }
    return false;
  }

  const Flags& f_;
  Kube* k_;
  Labels desired_;
  bool have_desired_ = false;
};

std::string node_name_from(const Flags& f) {
  if (!f.node_name.empty()) return f.node_name;
  return read_trimmed("/labeller/hostname").value_or("");
}

void print_json(const Labels& l) {
  if (l.empty()) {
    std::printf("{}\n");
    return;
  }
  std::printf("{\n");
  size_t i = 0;
  for (const auto& [k, v] : l)
    std::printf(" %s: %s%s\n", json::quote(k).c_str(), json::quote(v).c_str(), ++i < l.size() ? "," : "");
  std::printf("}\n");
}

volatile sig_atomic_t g_stop = 0;
int g_sig_pipe[2] = {-1, -1};

void on_signal(int) {
  g_stop = 1;
  const char b = 1;
  if (g_sig_pipe[1] >= 0 && ::write(g_sig_pipe[1], &b, 1) < 0) {
  }
}

using clk = std::chrono::steady_clock;

int ms_until(clk::time_point t) {
  const auto d = std::chrono::duration_cast<std::chrono::milliseconds>(t - clk::now()).count();
  return static_cast<int>(std::max<long long>(0, std::min<long long>(d, 3600 * 1000)));
}

clk::time_point after_s(double s) {
  return clk::now() + std::chrono::microseconds(static_cast<long long>(s * 1e6));
}

// The apiserver client as controller-runtime's GetConfigOrDie sets it up:
// -kubeconfig, else in-cluster unless $KUBECONFIG is set, else $KUBECONFIG (the
// list's files merged) / $HOME/.kube/config; in-cluster: the service account's token and CA.
bool configure_kube(const Flags& f, Kube* kube) {
  std::string err;
  const char* svc_host = std::getenv("KUBERNETES_SERVICE_HOST");
  const bool in_cluster = (svc_host && *svc_host) || !f.apiserver.empty();
  const std::vector<std::string> kc_paths =
      !f.kubeconfig.empty() ? std::vector<std::string>{f.kubeconfig} : kube::default_kubeconfig_paths(in_cluster);
  if (!kc_paths.empty()) {
    auto kc = kube::load_kubeconfig_files(kc_paths, &err);
    std::string kc_path;
    for (const auto& p : kc_paths) kc_path += (kc_path.empty() ? "" : ":") + p;
    if (!kc) {
      MI_LOG(kError, "unable to set up kubernetes client: %s", err.c_str());
      return false;
    }
    kube->cfg = kc->http;
    kube->token = kc->token;
    kube->token_file = kc->token_file;
    MI_LOG(kInfo, "kubeconfig %s: server %s", kc_path.c_str(), kube->cfg.server.c_str());
    return true;
  }
  if (!f.apiserver.empty()) {
    kube->cfg.server = f.apiserver;
  } else {
    const char* host = std::getenv("KUBERNETES_SERVICE_HOST");
    const char* port = std::getenv("KUBERNETES_SERVICE_PORT");
    if (!host || !*host) {
      MI_LOG(kError, "unable to set up kubernetes client: not running in a cluster (KUBERNETES_SERVICE_HOST unset)");
      return false;
    }
    std::string h = host;
    if (h.find(':') != std::string::npos && h[0] != '[') h = "[" + h + "]";
    kube->cfg.server = "https://" + h + ":" + (port && *port ? port : "443");
  }
  kube->token_file = !f.token_file.empty() ? f.token_file : path_join(f.sa_dir, "token");
  kube->cfg.ca_file = !f.ca_file.empty() ? f.ca_file
                      : path_exists(path_join(f.sa_dir, "ca.crt")) ? path_join(f.sa_dir, "ca.crt")
                                                                    : "";
  if (kube->bearer().empty() && f.apiserver.empty()) {
    MI_LOG(kError, "unable to set up kubernetes client: service-account token %s is unreadable or empty",
           kube->token_file.c_str());
    return false;
  }
  return true;
}

// The watch of this node's object (?watch=1&fieldSelector=metadata.name=<node>):
// an ADDED event (and, unless -resync 0, a MODIFIED one whose labels differ
// from the desired set) asks for a reconcile; 410 re-lists; a failed or
// short-lived stream is reopened with exponential backoff, a stream the server
// ended after its timeout at once.
class NodeWatch {
 public:
  enum Event { kIdle, kKick, kStop };

  NodeWatch(const Flags& f, Kube* kube, Labeller* lab, bool created_only, int wake_fd)
      : f_(f), kube_(kube), lab_(lab), created_only_(created_only), wake_fd_(wake_fd), cfg_(kube->cfg) {
    cfg_.timeout_s = f.watch_timeout_s + 30.0;
  }

  // Waits up to wait_ms for the next watch event (or only for a signal while
  // no stream is open), opening the stream first when it is due.
  Event wait(int wait_ms) {
    if (f_.watch && !open_ && clk::now() >= retry_) {
      open();
      if (g_stop) return kStop;
    }
    if (!open_) {
      if (f_.watch) wait_ms = std::min(wait_ms, ms_until(retry_));
      pollfd p{wake_fd_, POLLIN, 0};
      ::poll(&p, 1, wait_ms);
      return kIdle;
    }
    std::string line;
    const int rc = stream_.next_line(&line, wait_ms, wake_fd_);
    if (rc == -2) return kIdle;  // timer due
    if (rc == -3 || g_stop) return kStop;
    if (rc == 1) return on_line(line);
    ended(rc);
    return kIdle;
  }

 private:
  void open() {
    std::string q = "/api/v1/nodes?watch=1&fieldSelector=" + path_escape("metadata.name=" + f_.node_name) +
                    "&timeoutSeconds=" + std::to_string(f_.watch_timeout_s) + "&allowWatchBookmarks=true";
    if (!rv_.empty()) q += "&resourceVersion=" + path_escape(rv_);
    int status = 0;
    std::string ebody;
    const std::string e = stream_.open(cfg_, q, kube_->headers(), &status, &ebody,
                                       static_cast<int>(kube_->cfg.timeout_s * 1000), wake_fd_);
    if (g_stop) return;
    if (!e.empty() || status != 200) {
      if (status == 410) rv_.clear();
      if (status == 401) kube_->bearer(true);
      ++lab_->st.watch_errors;
      MI_LOG(kWarning, "watch of node %s failed (%s); retrying in %.1fs", f_.node_name.c_str(),
             e.empty() ? ("HTTP " + std::to_string(status) + ": " + ebody.substr(0, 200)).c_str() : e.c_str(),
             backoff_);
      stream_.close();
      back_off();
      return;
    }
    open_ = true;
    opened_ = clk::now();
    ++lab_->st.watch_restarts;
  }

  Event on_line(const std::string& line) {
    if (line.find_first_not_of(" \t\r") == std::string::npos) return kIdle;
    ++lab_->st.watch_events;
    auto ev = json::parse(line);
    if (!ev) return kIdle;
    const std::string type = ev->str("type");
    const json::Value* obj = ev->get("object");
    if (type == "ERROR") {
      const bool gone = obj && obj->str("code") == "410";  // resourceVersion too old: re-list
      if (gone) rv_.clear();
      stream_.close();
      open_ = false;
      back_off();
      return gone ? kKick : kIdle;
    }
    if (!obj) return kIdle;
    const json::Value* md = obj->get("metadata");
    if (md && !md->str("resourceVersion").empty()) rv_ = md->str("resourceVersion");
    if ((type == "ADDED" || (type == "MODIFIED" && !created_only_)) && lab_->needs_reconcile(*obj)) {
      ++lab_->st.watch_kicks;
      return kKick;
    }
    return kIdle;
  }

  // the stream ended (server timeout, rc 0) or broke
  void ended(int rc) {
    stream_.close();
    open_ = false;
    const bool lived = clk::now() - opened_ >= std::chrono::seconds(1);
    if (rc == 0 && lived) {
      backoff_ = 0.2;
      retry_ = clk::now();
      return;
    }
    if (rc != 0) {
      ++lab_->st.watch_errors;
      MI_LOG(kWarning, "watch of node %s broke; retrying in %.1fs", f_.node_name.c_str(), backoff_);
    }
    back_off();  // a server that ends every stream at once is not hammered
  }

  void back_off() {
    retry_ = after_s(backoff_);
    backoff_ = std::min(backoff_ * 2, f_.watch_backoff_max_s);
  }

  const Flags& f_;
  Kube* kube_;
  Labeller* lab_;
  const bool created_only_;
  const int wake_fd_;
  http::Config cfg_;  // the apiserver's, with a timeout past the watch's own
  http::Stream stream_;
  bool open_ = false;
  clk::time_point opened_ = clk::now();
  clk::time_point retry_ = clk::now();
  double backoff_ = 0.2;
  std::string rv_;
};

// -metrics_port: /healthz is 200 while the controller loop runs (it wakes at
// least every kLoopWakeS; one reconcile against a hung apiserver can take
// ~180 s of 15 s call timeouts, so a loop that has not run for kLoopStallS is
// stuck past every timeout) and /readyz while the last reconcile succeeded.
// The checks run on the endpoint's thread and read only these atomics.
constexpr double kLoopWakeS = 15, kLoopStallS = 300;
std::atomic<int64_t> g_loop_tick_ns{0};
std::atomic<bool> g_reconciled{false};

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now().time_since_epoch()).count();
}

std::string labeller_healthz() {
  const double age = (now_ns() - g_loop_tick_ns.load()) * 1e-9;
  if (age <= kLoopStallS) return "";
  char b[128];
  std::snprintf(b, sizeof(b), "controller loop stalled: last ran %.0f s ago", age);
  return b;
}

std::string labeller_readyz() { return g_reconciled.load() ? "" : "node labels not reconciled yet (see the log)"; }

// The controller loop: reconcile at start, every -resync s, on watch events
// and on a partition switch (a kfd fingerprint that held one -topology_watch
// interval: a switch passes through half states).
int run(const Flags& f, Labeller& lab, Kube& kube) {
  // -resync 0: the reference's controller (main.go:553-586): label at start,
  // then only when the Node object is (re-)created; no periodic re-assert
  const bool created_only = f.resync_s <= 0;
  const double resync_s = created_only ? 3600.0 * 24 * 365 : f.resync_s;
  g_loop_tick_ns = now_ns();
  metrics::HttpEndpoint endpoint;
  if (f.metrics_port > 0) {
    endpoint.set_checks(labeller_healthz, labeller_readyz);
    if (const std::string e = endpoint.start("0.0.0.0", f.metrics_port); !e.empty()) {
      MI_LOG(kError, "cannot serve /metrics: %s", e.c_str());
      return 1;
    }
    MI_LOG(kInfo, "serving /metrics, /healthz, /readyz on :%d", endpoint.port());
  }
  auto& m = metrics::global();
  NodeWatch watch(f, &kube, &lab, created_only, g_sig_pipe[0]);
  bool kick = true;
  auto next_resync = clk::now();
  const bool topo_watch = f.topology_watch_s > 0;
  auto next_topo = after_s(f.topology_watch_s);
  std::string topo_last = topo_watch ? topology_signature(f.sysfs_root) : "", topo_seen = topo_last;
  while (!g_stop) {
    if (kick || clk::now() >= next_resync) {
      kick = false;
      const int patches = lab.st.patches;
      const bool ok = lab.reconcile();
      g_reconciled = ok;
      m.inc("mi355x_labeller_reconciles_total", {{"result", ok ? "ok" : "error"}}, 1.0,
            "node label reconciles: ok (labels match, or patched) or error");
      if (lab.st.patches > patches)
        m.inc("mi355x_labeller_patches_total", {}, 1.0, "node label patches (or GET + update) the apiserver accepted");
      next_resync = after_s(ok ? resync_s : 5.0);
    }
    g_loop_tick_ns = now_ns();
    if (topo_watch && clk::now() >= next_topo) {
      next_topo = after_s(f.topology_watch_s);
      const std::string cur = topology_signature(f.sysfs_root);
      if (cur != topo_last && cur == topo_seen) {
        topo_last = cur;
        ++lab.st.topology_changes;
        m.inc("mi355x_labeller_topology_changes_total", {}, 1.0, "GPU partition switches that triggered a relabel");
        MI_LOG(kInfo, "GPU topology changed (partition switch?): relabelling node %s", f.node_name.c_str());
        kick = true;
      }
      topo_seen = cur;
      if (kick) continue;
    }
    int wait_ms = std::min(ms_until(next_resync), static_cast<int>(kLoopWakeS * 1000));
    if (topo_watch) wait_ms = std::min(wait_ms, ms_until(next_topo));
    const NodeWatch::Event ev = watch.wait(wait_ms);
    if (ev == NodeWatch::kStop) break;
    if (ev == NodeWatch::kKick) kick = true;
  }
  MI_LOG(kInfo, "Received signal, shutting down. passes=%d patches=%d updates=%d errors=%d watch_events=%d "
                "watch_kicks=%d watch_errors=%d watch_restarts=%d topology_changes=%d",
         lab.st.passes, lab.st.patches, lab.st.updates, lab.st.errors, lab.st.watch_events, lab.st.watch_kicks,
         lab.st.watch_errors, lab.st.watch_restarts, lab.st.topology_changes);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Flags f;
  std::string err;
  bool syntax = false;
  if (!parse_flags(argc, argv, &f, &err, &syntax)) {
    if (syntax) {  // the flag package's failure: the error, then the usage, exit 2
      std::fprintf(stderr, "%s\n", err.c_str());
      print_usage(stderr, argv[0], f.sysfs_root);
      return 2;
    }
    glog::init(f.log);
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  if (f.log.program.empty()) f.log.program = "k8s-node-labeller";
  err = glog::init(f.log);
  if (!err.empty()) {
    glog::init(glog::Options());
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  if (f.dry_run) {
    print_json(labeller::generate_labels(label_options(f)));
    return 0;
  }
  for (const auto& line : versions::banner(kTitle, argv[0], f.sysfs_root)) MI_LOG(kInfo, "%s", line.c_str());
  f.node_name = node_name_from(f);
  if (f.node_name.empty()) {
    MI_LOG(kError, "node name unknown: set DS_NODE_NAME or -node_name (or mount /labeller/hostname)");
    return 1;
  }
  Kube kube;
  if (!configure_kube(f, &kube)) return 1;

  if (::pipe(g_sig_pipe) != 0) return 1;
  ::fcntl(g_sig_pipe[0], F_SETFL, O_NONBLOCK);
  ::fcntl(g_sig_pipe[1], F_SETFL, O_NONBLOCK);
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);
  kube.wake_fd = g_sig_pipe[0];

  Labeller lab(f, &kube);
  if (f.once) {  // apply once and exit (a Job)
    while (!g_stop) {
      if (lab.reconcile()) return 0;
      pollfd p{g_sig_pipe[0], POLLIN, 0};
      ::poll(&p, 1, 5000);
    }
    return 0;
  }
  return run(f, lab, kube);
}
