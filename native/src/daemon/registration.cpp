#include "registration.h"

#include <algorithm>
#include <cstdio>

namespace mi355x::daemon {
namespace {

Clock::duration secs(double s) {
  return std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(s));
}

}  // namespace

void Registration::server_started(uint64_t server_gen, Clock::time_point now) {
  serving_ = true;
  server_gen_ = server_gen;
  registered_ = false;
  inflight_ = false;  // a Register for the previous server completes as stale
  list_seen_ = false;
  lost_ = false;
  retry_ms_ = p_.retry_initial_ms;
  next_register_ = now;
}

void Registration::server_stopped() {
  serving_ = false;
  registered_ = false;
  list_seen_ = false;
  lost_ = false;
}

void Registration::force(Clock::time_point now) {
  if (!serving_) return;
  registered_ = false;
  list_seen_ = false;
  lost_ = false;
  next_register_ = now;
}

bool Registration::due(Clock::time_point now) const {
  return serving_ && !registered_ && !inflight_ && now >= next_register_;
}

void Registration::begin(uint64_t kubelet_gen, const rpc::ServerStats& st) {
  inflight_ = true;
  req_kubelet_gen_ = kubelet_gen;
  base_streams_ = st.streams_opened;
  base_caller_errors_ = st.caller_protocol_errors;
  list_seen_ = false;
}

Registration::Outcome Registration::complete(uint64_t server_gen, uint64_t req_kubelet_gen, uint64_t kubelet_gen_now,
                                             bool ok, Clock::time_point now) {
  if (server_gen != server_gen_) return Outcome::kStale;  // an earlier server's answer
  inflight_ = false;
  if (req_kubelet_gen != kubelet_gen_now || !serving_) return Outcome::kStale;  // a previous kubelet's answer
  if (!ok) {
    next_register_ = now + std::chrono::milliseconds(retry_ms_);
    retry_ms_ = std::min(2 * retry_ms_, p_.retry_max_ms);
    return Outcome::kFailed;
  }
  registered_ = true;
  registered_at_ = now;
  retry_ms_ = p_.retry_initial_ms;
  lost_ = false;
  registrations_++;
  return Outcome::kRegistered;
}

std::string Registration::observe(const rpc::ServerStats& st, Clock::time_point now) {
  if (!serving_ || (!registered_ && !inflight_)) return "";
  if (st.streams_opened > base_streams_) list_seen_ = true;
  if (!list_seen_ && p_.watchdog_s > 0) {
    if (st.caller_protocol_errors > base_caller_errors_) {
      return std::to_string(st.caller_protocol_errors - base_caller_errors_) +
             " HTTP/2 protocol error(s) on kubelet's connection before its ListAndWatch";
    }
    if (registered_ && now - registered_at_ > secs(p_.watchdog_s)) {
      char b[96];
      std::snprintf(b, sizeof(b), "no ListAndWatch stream within %gs of Register", p_.watchdog_s);
      return b;
    }
  }
  // kubelet ended every stream of a registered resource: it dropped the plugin
  if (registered_ && list_seen_ && p_.reregister_s > 0) {
    if (st.streams_open > 0) {
      lost_ = false;
    } else if (!lost_) {
      lost_ = true;
      lost_since_ = now;
    } else if (now - lost_since_ >= secs(p_.reregister_s)) {
      registered_ = false;
      list_seen_ = false;
      lost_ = false;
      next_register_ = now;
      reregistrations_++;
    }
  }
  return "";
}

Clock::time_point Registration::next_event(Clock::time_point now) const {
  Clock::time_point t = now + std::chrono::hours(1);
  if (!serving_) return t;
  if (!registered_ && !inflight_) t = std::min(t, next_register_);
  if (armed()) t = std::min(t, now + std::chrono::milliseconds(250));
  if (registered_ && list_seen_ && p_.reregister_s > 0)
    t = std::min(t, lost_ ? lost_since_ + secs(p_.reregister_s) : now + std::chrono::milliseconds(1000));
  return std::max(t, now);
}

}  // namespace mi355x::daemon
