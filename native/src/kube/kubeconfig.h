// kubeconfig for the native node labeller: the reference labeller takes
// -kubeconfig through controller-runtime (vendor/sigs.k8s.io/controller-runtime/
// pkg/client/config/config.go:32-58,116-156): the flag, else in-cluster when
// $KUBECONFIG is unset, else $KUBECONFIG (a ':'-separated list, merged) /
// $HOME/.kube/config.
//
// The file is YAML (or JSON). Only what a client needs is read: the current
// context's cluster (server, certificate-authority[-data], tls-server-name,
// insecure-skip-tls-verify) and user (token, tokenFile,
// client-certificate[-data], client-key[-data]); relative paths resolve
// against the file's directory, as clientcmd does.
#pragma once

#include <optional>
#include <string>
#include <vector>

#include "http.h"
#include "json.h"

namespace mi355x::kube {

struct KubeConfig {
  http::Config http;       // server, CA, client certificate, insecure
  std::string token;       // static bearer token
  std::string token_file;  // re-read when it changes
};

std::optional<KubeConfig> load_kubeconfig(const std::string& path, std::string* error);
// several files merged as clientcmd merges a $KUBECONFIG list: the first file
// that sets current-context wins it, and each cluster / context / user comes
// from the first file that names it (its relative paths against that file)
std::optional<KubeConfig> load_kubeconfig_files(const std::vector<std::string>& paths, std::string* error);

// controller-runtime's order after the flag: in-cluster unless $KUBECONFIG is
// set, then the existing entries of $KUBECONFIG or $HOME/.kube/config.
// Empty when none applies (callers then use the in-cluster config).
std::vector<std::string> default_kubeconfig_paths(bool in_cluster_available);

}  // namespace mi355x::kube
