// mi355x-liveness-probe: run the gfx950 MFMA liveness kernel on GPU agents
// and print one JSON document.
//
//   mi355x-liveness-probe [--devices all|0,2,..] [--nonce N] [--iters N] [--identify] [--timeout S]
//
// Built twice from this file: `mi355x-liveness-probe` launches through ROCr
// directly (MI355X_PROBE_HSA; links only libhsa-runtime64, one AQL dispatch),
// `mi355x-liveness-probe-hip` through the HIP runtime.
//
// Exit status: 0 all probed devices live, 1 at least one failed, 2 usage or
// HIP runtime unavailable. The parent (the plugin's health loop, or the
// benchmark's fake container runtime) enforces the deadline by killing us.
#include <sys/resource.h>
#include <time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mi355x/liveness_probe.h"

namespace {

double cpu_ms() {
  rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  return (ru.ru_utime.tv_sec + ru.ru_stime.tv_sec) * 1e3 + (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec) / 1e3;
}

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + ts.tv_nsec;
}

std::string json_escape(const char* s) {
  std::string o;
  for (; *s; ++s) {
    char c = *s;
    if (c == '"' || c == '\\') {
      o += '\\';
      o += c;
    } else if (static_cast<unsigned char>(c) < 0x20) {
      char b[8];
      std::snprintf(b, sizeof(b), "\\u%04x", c);
      o += b;
    } else {
      o += c;
    }
  }
  return o;
}

void print_device(const mi355x_probe_result& r, bool last) {
  std::printf(
      "{\"ordinal\":%d,\"ok\":%s,\"hip_error\":%d,\"mismatches\":%d,\"nonce\":%u,\"xcc_id\":%u,"
      "\"hw_id\":%u,\"iters\":%d,\"dispatches\":%d,\"kfd_node_id\":%d,\"runtime\":\"%s\","
      "\"kernel_us\":%.3f,\"setup_us\":%.3f,\"total_us\":%.3f,"
      "\"phase_us\":{\"code_object\":%.1f,\"queue\":%.1f,\"buffers\":%.1f,\"dispatch_wait\":%.1f},"
      "\"pci_bus_id\":\"%s\","
      "\"arch\":\"%s\",\"name\":\"%s\",\"uuid\":\"%s\",\"pci_domain\":%d,\"pci_bus\":%d,"
      "\"pci_device\":%d,\"cu_count\":%d,\"total_mem\":%llu,\"error\":\"%s\"}%s",
      r.ordinal, r.ok ? "true" : "false", r.hip_error, r.mismatches, r.nonce, r.xcc_id, r.hw_id, r.iters,
      r.dispatches, r.kfd_node_id, r.runtime, r.kernel_us, r.setup_us, r.total_us, r.phase_us[0], r.phase_us[1],
      r.phase_us[2], r.phase_us[3], json_escape(r.pci_bus_id).c_str(), json_escape(r.arch).c_str(),
      json_escape(r.name).c_str(), json_escape(r.uuid).c_str(), r.pci_domain, r.pci_bus, r.pci_device,
      r.cu_count, static_cast<unsigned long long>(r.total_mem), json_escape(r.error).c_str(), last ? "" : ",");
}

#ifdef MI355X_PROBE_HSA
int device_count() { return mi355x_hsa_probe_init(); }
int probe(int o, uint32_t nonce, int iters, double timeout_s, mi355x_probe_result* r) {
  return mi355x_hsa_probe_device(o, nonce, iters, timeout_s, r);
}
int identify_dev(int o, mi355x_probe_result* r) { return mi355x_hsa_probe_identify(o, r); }
void init_phases(double out[3]) { mi355x_hsa_init_phases(out); }
#else
void init_phases(double out[3]) { out[0] = out[1] = out[2] = 0; }
int device_count() { return mi355x_probe_device_count(); }
int probe(int o, uint32_t nonce, int iters, double, mi355x_probe_result* r) {
  return mi355x_probe_device(o, nonce, iters, r);
}
int identify_dev(int o, mi355x_probe_result* r) { return mi355x_probe_identify(o, r); }
#endif

}  // namespace

int main(int argc, char** argv) {
  const uint64_t t_start = mono_ns();
  std::string devices = "all";
  uint32_t nonce = static_cast<uint32_t>(t_start ^ (t_start >> 32));
  int iters = 4;
  double timeout_s = 5.0;
  bool identify = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", what);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--devices") {
      devices = next("--devices");
    } else if (a == "--nonce") {
      nonce = static_cast<uint32_t>(std::strtoul(next("--nonce"), nullptr, 0));
    } else if (a == "--iters") {
      iters = std::atoi(next("--iters"));
    } else if (a == "--timeout") {
      timeout_s = std::atof(next("--timeout"));
    } else if (a == "--identify") {
      identify = true;
    } else if (a == "-h" || a == "--help") {
      std::printf("usage: %s [--devices all|0,1,..] [--nonce N] [--iters N] [--identify] [--timeout S]\n",
                  argv[0]);
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }

  const int n = device_count();
  const uint64_t t_runtime = mono_ns();  // HIP runtime + ROCr initialised
  const double cpu_runtime = cpu_ms();
  double iph[3];
  init_phases(iph);
  if (n < 0) {
    std::printf("{\"ok\":false,\"hip_device_count\":0,\"error\":\"GPU runtime init failed (%d)\",\"devices\":[],"
                "\"t_start_ns\":%llu,\"t_ready_ns\":0}\n",
                -n, static_cast<unsigned long long>(t_start));
    return 2;
  }
  std::vector<int> ords;
  if (devices == "all") {
    for (int i = 0; i < n; ++i) ords.push_back(i);
  } else {
    size_t pos = 0;
    while (pos <= devices.size()) {
      size_t c = devices.find(',', pos);
      if (c == std::string::npos) c = devices.size();
      std::string tok = devices.substr(pos, c - pos);
      if (!tok.empty()) ords.push_back(std::atoi(tok.c_str()));
      pos = c + 1;
    }
  }

  std::vector<mi355x_probe_result> results(ords.size());
  bool all_ok = !ords.empty();
  for (size_t i = 0; i < ords.size(); ++i) {
    if (ords[i] < 0 || ords[i] >= n) {
      std::memset(&results[i], 0, sizeof(results[i]));
      results[i].ordinal = ords[i];
      std::snprintf(results[i].error, sizeof(results[i].error), "no such HIP device (count=%d)", n);
      all_ok = false;
      continue;
    }
    int rc = identify ? identify_dev(ords[i], &results[i])
                      : probe(ords[i], nonce + static_cast<uint32_t>(i), iters, timeout_s, &results[i]);
    if (identify && rc == 0) results[i].ok = 1;
    if (rc != 0) all_ok = false;
  }
  const uint64_t t_ready = mono_ns();
  const double cpu_ready = cpu_ms();
  std::printf("{\"ok\":%s,\"hip_device_count\":%d,\"identify\":%s,\"t_start_ns\":%llu,\"t_runtime_ns\":%llu,"
              "\"t_ready_ns\":%llu,\"cpu_ms_runtime\":%.2f,\"cpu_ms_ready\":%.2f,"
              "\"init_us\":{\"hsa_init\":%.1f,\"agents\":%.1f,\"pools\":%.1f},\"devices\":[",
              all_ok ? "true" : "false", n, identify ? "true" : "false", static_cast<unsigned long long>(t_start),
              static_cast<unsigned long long>(t_runtime), static_cast<unsigned long long>(t_ready), cpu_runtime,
              cpu_ready, iph[0], iph[1], iph[2]);
  for (size_t i = 0; i < results.size(); ++i) print_device(results[i], i + 1 == results.size());
  std::printf("]}\n");
  std::fflush(stdout);
  return all_ok ? 0 : 1;
}
