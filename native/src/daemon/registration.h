// One resource's registration with kubelet and its transport watchdog, as
// pure state: the daemon feeds it the clock, the server's counters and the
// Register outcomes, and it says when to register and when to give up. No
// threads, no sockets (native/tests/test_core.cpp drives it directly).
//
// Registration (vendored dpm/plugin.go:127-162, with the retry schedule of
// manager.go:205-219 replaced by a backoff): a Register goes out as soon as
// the server is up and kubelet.sock exists, on a worker thread; a failure is
// retried after 100 ms, doubling to 3 s. Generations make late answers
// harmless:
//   * server_gen  - bumped on every (re)start of the resource's server; an
//                   answer for an earlier server is ignored outright (a newer
//                   Register may already be in flight);
//   * kubelet_gen - bumped on every kubelet (re)start (kubelet.sock replaced or
//                   removed); an answer from the previous kubelet ends the
//                   in-flight state but registers nothing.
//
// Transport watchdog. kubelet dials back and opens ListAndWatch right after
// Register (in kubelet's Register handler: connectClient -> Connect ->
// GetDevicePluginOptions, then `go runClient` -> ListAndWatch, possibly before
// the Register reply reaches us). The baseline of the server's counters is
// therefore taken when the Register is *sent* (begin()), not when its answer
// arrives, so a stream kubelet opened meanwhile counts. Until that first
// ListAndWatch the watchdog is armed and trips (the daemon exits 3 and the
// DaemonSet restarts it, instead of staying registered and invisible) when
//   * no ListAndWatch opened within watchdog_s of the Register answer, or
//   * a protocol error ended a connection that had made a DevicePlugin call
//     (kubelet's; ServerStats::caller_protocol_errors).
// A stray client on the plugin socket (curl, a socket health check, a bad
// preface) never trips it: its connection made no call, and the server closes
// it with GOAWAY as grpc-go does (vendor/google.golang.org/grpc/
// server.go:984-998). Once ListAndWatch has been seen the watchdog is
// disarmed for good (until the next registration).
//
// Lost streams. kubelet ends ListAndWatch when it drops a plugin (its
// runClient -> disconnectClient marks the devices unhealthy and forgets the
// endpoint after a grace period). If every stream of a registered resource has
// been closed for reregister_s while kubelet.sock stayed the same, the
// resource registers again (the reference waits for a kubelet restart).
#pragma once

#include <chrono>
#include <cstdint>
#include <string>

#include "mi355x/grpc_server.h"

namespace mi355x::daemon {

using Clock = std::chrono::steady_clock;

struct RegistrationPolicy {
  double watchdog_s = 10.0;   // 0 = no watchdog
  double reregister_s = 2.0;  // 0 = never re-register on lost streams
  int retry_initial_ms = 100;
  int retry_max_ms = 3000;
};

class Registration {
 public:
  enum class Outcome { kStale, kRegistered, kFailed };

  explicit Registration(RegistrationPolicy p = {}) : p_(p) {}

  // the resource's server (re)started (`server_gen` names it): register now
  void server_started(uint64_t server_gen, Clock::time_point now);
  // the server stopped (shutdown, kubelet gone, resource removed)
  void server_stopped();
  // kubelet must read new options: register again (same server)
  void force(Clock::time_point now);

  // should a Register be sent now? (the server is up and kubelet.sock exists)
  bool due(Clock::time_point now) const;
  // a Register is about to be sent for kubelet generation `kubelet_gen`;
  // `st` = the server's counters right now (the watchdog baseline)
  void begin(uint64_t kubelet_gen, const rpc::ServerStats& st);
  // a Register answered: for `server_gen`, sent under `req_kubelet_gen`;
  // `kubelet_gen_now` is the current kubelet generation
  Outcome complete(uint64_t server_gen, uint64_t req_kubelet_gen, uint64_t kubelet_gen_now, bool ok,
                   Clock::time_point now);

  // every loop turn: "" or why the watchdog tripped; may schedule a new
  // Register (lost streams: reregistering() turns true)
  std::string observe(const rpc::ServerStats& st, Clock::time_point now);

  // the next time observe()/due() may change their answer (poll timeout)
  Clock::time_point next_event(Clock::time_point now) const;

  bool serving() const { return serving_; }
  bool registered() const { return registered_; }
  bool inflight() const { return inflight_; }
  bool list_seen() const { return list_seen_; }
  bool armed() const { return serving_ && (inflight_ || registered_) && !list_seen_ && p_.watchdog_s > 0; }
  uint64_t server_gen() const { return server_gen_; }
  uint64_t registrations() const { return registrations_; }
  uint64_t reregistrations() const { return reregistrations_; }  // after lost streams
  int retry_ms() const { return retry_ms_; }

 private:
  RegistrationPolicy p_;
  bool serving_ = false;
  bool registered_ = false;
  bool inflight_ = false;
  bool list_seen_ = false;
  uint64_t server_gen_ = 0;
  uint64_t req_kubelet_gen_ = 0;
  Clock::time_point next_register_{};
  Clock::time_point registered_at_{};
  int retry_ms_ = 100;
  // watchdog baseline, taken at begin()
  uint64_t base_streams_ = 0;
  uint64_t base_caller_errors_ = 0;
  bool lost_ = false;
  Clock::time_point lost_since_{};
  uint64_t registrations_ = 0;
  uint64_t reregistrations_ = 0;
};

}  // namespace mi355x::daemon
