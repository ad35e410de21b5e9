// kubeconfig loading for the native node labeller (see kubeconfig.h).
#include "kubeconfig.h"

#include "yaml.h"

#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "mi355x/sysfs.h"

namespace mi355x::kube {
namespace {

std::string b64decode(const std::string& in, bool* ok) {
  static const std::string tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  uint32_t acc = 0;
  int bits = 0;
  *ok = true;
  for (char c : in) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ') continue;
    const size_t v = tbl.find(c);
    if (v == std::string::npos) {
      *ok = false;
      return "";
    }
    acc = (acc << 6) | static_cast<uint32_t>(v);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back(static_cast<char>((acc >> bits) & 0xFF));
    }
  }
  return out;
}

const json::Value* named(const json::Value* list, const std::string& name, const char* inner) {
  if (!list || list->kind != json::Value::Array) return nullptr;
  const json::Value* first = nullptr;
  for (const auto& e : list->arr) {
    const json::Value* body = e.get(inner);
    if (!first) first = body;
    if (e.str("name") == name) return body;
  }
  return name.empty() ? first : nullptr;
}

// the file paths an entry names, made absolute against the file's directory (as
// clientcmd resolves them before it merges files)
void resolve_paths(json::Value* doc, const std::string& base) {
  static const std::pair<const char*, std::vector<const char*>> kFields[] = {
      {"clusters", {"certificate-authority"}},
      {"users", {"client-certificate", "client-key", "tokenFile"}}};
  for (const auto& [list, fields] : kFields) {
    json::Value* l = doc->get(list);
    if (!l || l->kind != json::Value::Array) continue;
    for (auto& e : l->arr) {
      json::Value* body = e.get(std::string(list) == "clusters" ? "cluster" : "user");
      if (!body || body->kind != json::Value::Object) continue;
      for (const char* f : fields) {
        json::Value* v = body->get(f);
        if (v && v->kind == json::Value::String && !v->s.empty() && v->s[0] != '/') v->s = base + "/" + v->s;
      }
    }
  }
}

}  // namespace

std::optional<KubeConfig> load_kubeconfig(const std::string& path, std::string* error) {
  return load_kubeconfig_files({path}, error);
}

std::optional<KubeConfig> load_kubeconfig_files(const std::vector<std::string>& paths, std::string* error) {
  // clientcmd's merge of a $KUBECONFIG list: the first file that sets current-context
  // wins it, and a cluster / context / user comes from the first file that names it
  json::Value merged = json::Value::object();
  std::string path;  // for messages: the files, ':'-joined
  for (const auto& p : paths) {
    path += (path.empty() ? "" : ":") + p;
    auto text = read_file(p);
    if (!text) {
      *error = "kubeconfig " + p + ": unreadable";
      return std::nullopt;
    }
    std::string perr;
    auto doc = yaml::parse(*text, &perr);
    if (!doc || doc->kind != json::Value::Object) {
      *error = "kubeconfig " + p + ": " + (perr.empty() ? "not a mapping" : perr);
      return std::nullopt;
    }
    resolve_paths(&*doc, p.find('/') == std::string::npos ? "." : p.substr(0, p.rfind('/')));
    if (merged.str("current-context").empty() && !doc->str("current-context").empty())
      merged.set("current-context", json::Value::string(doc->str("current-context")));
    for (const char* list : {"clusters", "contexts", "users"}) {
      const json::Value* l = doc->get(list);
      if (!l || l->kind != json::Value::Array) continue;
      json::Value* into = merged.get(list);
      if (!into) {
        json::Value arr;
        arr.kind = json::Value::Array;
        into = &merged.set(list, std::move(arr));
      }
      for (const auto& e : l->arr) {
        bool seen = false;
        for (const auto& have : into->arr) seen = seen || have.str("name") == e.str("name");
        if (!seen) into->arr.push_back(e);
      }
    }
  }
  const json::Value* doc = &merged;
  // a name that is set must be found (as client-go validates it); an unset one takes the first entry
  const std::string ctx_name = doc->str("current-context");
  const json::Value* ctx = named(doc->get("contexts"), ctx_name, "context");
  if (!ctx && !ctx_name.empty()) {
    *error = "kubeconfig " + path + ": context \"" + ctx_name + "\" not found";
    return std::nullopt;
  }
  const std::string cluster_name = ctx ? ctx->str("cluster") : "", user_name = ctx ? ctx->str("user") : "";
  const json::Value* cluster = named(doc->get("clusters"), cluster_name, "cluster");
  const json::Value* user = named(doc->get("users"), user_name, "user");
  if ((!cluster && !cluster_name.empty()) || (!user && !user_name.empty())) {
    *error = "kubeconfig " + path + ": " + (!cluster && !cluster_name.empty() ? "cluster \"" + cluster_name
                                                                                : "user \"" + user_name) +
             "\" of context \"" + ctx_name + "\" not found";
    return std::nullopt;
  }
  if (!cluster || cluster->str("server").empty()) {
    *error = "kubeconfig " + path + ": no cluster server for context \"" + ctx_name + "\"";
    return std::nullopt;
  }
  auto data = [&](const json::Value* v, const char* key, std::string* out) {
    const std::string enc = v ? v->str(key) : "";
    if (enc.empty()) return true;
    bool ok = false;
    *out = b64decode(enc, &ok);
    if (!ok) *error = std::string("kubeconfig ") + path + ": " + key + " is not base64";
    return ok;
  };
  KubeConfig kc;
  std::string server = cluster->str("server");
  while (!server.empty() && server.back() == '/') server.pop_back();
  kc.http.server = server;
  kc.http.ca_file = cluster->str("certificate-authority");
  if (!data(cluster, "certificate-authority-data", &kc.http.ca_pem)) return std::nullopt;
  kc.http.tls_server_name = cluster->str("tls-server-name");
  kc.http.proxy_url = cluster->str("proxy-url");
  if (const json::Value* ins = cluster->get("insecure-skip-tls-verify"))
    kc.http.insecure = ins->kind == json::Value::Bool ? ins->b : ins->s == "true";
  if (user) {
    kc.token = user->str("token");
    if (kc.token.empty()) kc.token_file = user->str("tokenFile");
    kc.http.cert_file = user->str("client-certificate");
    kc.http.key_file = user->str("client-key");
    if (!data(user, "client-certificate-data", &kc.http.cert_pem)) return std::nullopt;
    if (!data(user, "client-key-data", &kc.http.key_pem)) return std::nullopt;
  }
  if (kc.http.insecure && (!kc.http.ca_file.empty() || !kc.http.ca_pem.empty())) {
    // as client-go's transport refuses it (vendor/k8s.io/client-go/transport/transport.go:81-83)
    *error = "kubeconfig " + path + ": specifying a root certificates file with the insecure flag is not allowed";
    return std::nullopt;
  }
  if (user && kc.token.empty() && kc.token_file.empty() && kc.http.cert_file.empty() && kc.http.cert_pem.empty()) {
    // credentials this labeller cannot produce: refused rather than sent unauthenticated
    for (const char* plugin : {"exec", "auth-provider", "username"})
      if (user->get(plugin)) {
        *error = "kubeconfig " + path + ": user \"" + user_name + "\" authenticates with " + plugin +
                 ", which the labeller does not support; give it a token, tokenFile or client certificate";
        return std::nullopt;
      }
  }
  if (!kc.token_file.empty()) {
    auto t = read_trimmed(kc.token_file);
    if (!t || t->empty()) {
      *error = "kubeconfig tokenFile " + kc.token_file + " is unreadable or empty";
      return std::nullopt;
    }
  }
  return kc;
}

std::vector<std::string> default_kubeconfig_paths(bool in_cluster_available) {
  const char* env = std::getenv("KUBECONFIG");
  if (!env || !*env) {
    if (in_cluster_available) return {};
    const char* home = std::getenv("HOME");
    const std::string p = std::string(home && *home ? home : "") + "/.kube/config";
    if (home && *home && path_exists(p)) return {p};
    return {};
  }
  std::vector<std::string> out;
  const std::string list = env;
  size_t pos = 0;
  while (pos <= list.size()) {
    size_t c = list.find(':', pos);
    if (c == std::string::npos) c = list.size();
    const std::string p = list.substr(pos, c - pos);
    bool dup = false;
    for (const auto& q : out) dup = dup || q == p;
    if (!p.empty() && !dup && path_exists(p)) out.push_back(p);  // missing entries are skipped
    pos = c + 1;
  }
  return out;
}

}  // namespace mi355x::kube
