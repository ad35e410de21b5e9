// mi355x-device-plugin: the kubelet device plugin as one native process — the
// primary entrypoint of this framework (docs/architecture.md).
//
// The reference ships its plugin as a single compiled binary
// (cmd/k8s-device-plugin/main.go). This is the same thing built from the
// framework's C++ core, with no interpreter in the process:
//
//   flags          -pulse, -driver_type, -resource_naming_strategy (main.go:50-75),
//                  glog's flags, and this build's health / allocation /
//                  observability flags (daemon/flags.h)
//   banner         "<argv0> version <git describe>" and the libraries this build
//                  uses, in -h and as the first log lines (main.go:37-48,77-79;
//                  mi355x/versions.h)
//   discovery      container driver over the kfd topology, VF / PF passthrough
//                  over the IOMMU groups; without -driver_type: container -> VF
//                  -> PF (main.go:85-115) (daemon/resources.h)
//   per resource   the native gRPC server on <kubelet_dir>/amd.com_<resource>
//                  with the DevicePlugin service; registration with kubelet and
//                  the transport watchdog (daemon/registration.h)
//   health         every -pulse on a worker thread (daemon/health_controller.h)
//   control loop   daemon/daemon.h
//   signals        SIGTERM / SIGINT / SIGQUIT stop the servers, the probe server
//                  and the workers, and remove the sockets; a probe in flight
//                  (also the first sweep, before registration) ends at once
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <string>

#include "daemon.h"
#include "flags.h"
#include "mi355x/glog.h"
#include "mi355x/trace.h"
#include "mi355x/versions.h"

namespace {

constexpr const char* kTitle = "AMD GPU device plugin for Kubernetes (MI355X-native, native daemon)";

volatile sig_atomic_t g_stop = 0;
int g_sig_pipe[2] = {-1, -1};
volatile sig_atomic_t g_daemon_stop_fd = -1;  // the daemon's stop pipe: aborts in-flight probes and peer calls

void on_signal(int) {
  g_stop = 1;
  const char b = 1;
  if (g_sig_pipe[1] >= 0 && ::write(g_sig_pipe[1], &b, 1) < 0) {
  }
  if (g_daemon_stop_fd >= 0 && ::write(g_daemon_stop_fd, &b, 1) < 0) {
  }
}

}  // namespace

int main(int argc, char** argv) {
  using namespace mi355x;
  daemon::Flags f;
  std::string err;
  bool help = false, syntax = false;
  if (!daemon::parse_flags(argc, argv, &f, &err, &help, &syntax)) {
    if (syntax) {  // the flag package's failure: the error, then flag.Usage (main.go:43-49), exit 2
      std::fprintf(stderr, "%s\n", err.c_str());
      for (const auto& line : versions::banner(kTitle, argv[0], f.sysfs_root)) std::fprintf(stderr, "%s\n", line.c_str());
      std::fprintf(stderr, "%s", daemon::usage(argv[0]).c_str());
      return 2;
    }
    glog::init(f.log);
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  if (help) {  // flag.Usage (main.go:43-49): the version banner, then the flags
    for (const auto& line : versions::banner(kTitle, argv[0], f.sysfs_root)) std::printf("%s\n", line.c_str());
    std::printf("%s", daemon::usage(argv[0]).c_str());
    return 0;
  }
  if (f.log.program.empty()) f.log.program = "k8s-device-plugin";
  err = glog::init(f.log);
  if (!err.empty()) {
    glog::Options o;
    glog::init(o);
    MI_LOG(kError, "%s", err.c_str());
    return 1;
  }
  for (const auto& line : versions::banner(kTitle, argv[0], f.sysfs_root)) MI_LOG(kInfo, "%s", line.c_str());
  trace::global().configure(f.trace_file);
  if (::pipe2(g_sig_pipe, O_CLOEXEC | O_NONBLOCK) != 0) return 1;
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGQUIT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);

  daemon::Daemon d(f);
  g_daemon_stop_fd = d.stop_fd();
  // declared after `d`, so destroyed first: the handler never writes to the pipe `d` closes
  struct ForgetStopFd {
    ~ForgetStopFd() { g_daemon_stop_fd = -1; }
  } forget_stop_fd;
  if (g_stop) return 0;     // a signal before the daemon existed
  const int rc = d.init();
  if (rc >= 0) return rc;
  return d.run(g_sig_pipe[0], &g_stop);
}
