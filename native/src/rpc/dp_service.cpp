// v1beta1.DevicePlugin service on the native gRPC server (see mi355x/dp_service.h).
#include "mi355x/dp_service.h"

#include <sys/eventfd.h>
#include <unistd.h>

#include <chrono>

namespace mi355x::rpc {

namespace pb {

void put_varint(std::string* out, uint64_t v) {
  while (v >= 0x80) {
    out->push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  out->push_back(static_cast<char>(v));
}

void put_tag(std::string* out, int field, int wire) { put_varint(out, (static_cast<uint64_t>(field) << 3) | wire); }

void put_bytes(std::string* out, int field, const std::string& v) {
  put_tag(out, field, 2);
  put_varint(out, v.size());
  out->append(v);
}

void put_bool(std::string* out, int field, bool v) {
  if (!v) return;  // proto3 default is omitted
  put_tag(out, field, 0);
  out->push_back(1);
}

namespace {
bool get_varint(const char*& p, const char* end, uint64_t* v) {
  uint64_t x = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (p >= end) return false;
    const uint8_t b = static_cast<uint8_t>(*p++);
    x |= static_cast<uint64_t>(b & 0x7F) << shift;
    if (!(b & 0x80)) {
      *v = x;
      return true;
    }
  }
  return false;
}
}  // namespace

bool scan(const char* p, size_t n, const std::function<bool(int, const char*, size_t)>& on_bytes,
          const std::function<bool(int, uint64_t)>& on_varint) {
  const char* end = p + n;
  while (p < end) {
    uint64_t key = 0;
    if (!get_varint(p, end, &key)) return false;
    const int field = static_cast<int>(key >> 3);
    const int wire = static_cast<int>(key & 7);
    if (field <= 0) return false;
    switch (wire) {
      case 0: {
        uint64_t v = 0;
        if (!get_varint(p, end, &v)) return false;
        if (on_varint && !on_varint(field, v)) return false;
        break;
      }
      case 1:
        if (end - p < 8) return false;
        p += 8;
        break;
      case 2: {
        uint64_t len = 0;
        if (!get_varint(p, end, &len) || len > static_cast<uint64_t>(end - p)) return false;
        if (on_bytes && !on_bytes(field, p, static_cast<size_t>(len))) return false;
        p += len;
        break;
      }
      case 5:
        if (end - p < 4) return false;
        p += 4;
        break;
      default:
        return false;
    }
  }
  return true;
}

}  // namespace pb

namespace {

uint64_t mono_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
          .count());
}

constexpr size_t kMaxEvents = 4096;

}  // namespace

const char* DevicePluginService::path(const char* method) {
  static const std::unordered_map<std::string, std::string> paths = [] {
    std::unordered_map<std::string, std::string> m;
    for (const char* x : {"GetDevicePluginOptions", "ListAndWatch", "GetPreferredAllocation", "Allocate",
                          "PreStartContainer"})
      m[x] = std::string("/v1beta1.DevicePlugin/") + x;
    return m;
  }();
  auto it = paths.find(method);
  return it == paths.end() ? "" : it->second.c_str();
}

DevicePluginService::DevicePluginService() { evfd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC); }

DevicePluginService::~DevicePluginService() {
  detach();
  if (evfd_ >= 0) ::close(evfd_);
}

void DevicePluginService::detach() {
  std::shared_ptr<Sink> s;  // outlives the lock on its mutex below
  {
    std::lock_guard<std::mutex> lk(mu_);
    s.swap(sink_);
  }
  if (!s) return;
  std::lock_guard<std::mutex> sk(s->mu);  // waits out an answer being delivered
  s->srv = nullptr;
}

void DevicePluginService::set_prestart_gate(PreStartGate g) {
  std::lock_guard<std::mutex> lk(mu_);
  gate_ = g ? std::make_shared<const PreStartGate>(std::move(g)) : nullptr;
}

std::optional<Reply> DevicePluginService::prestart(uint64_t call_id, const std::string& req) {
  RpcEvent ev;
  ev.rpc = "PreStartContainer";
  ev.t0_ns = mono_ns();
  std::shared_ptr<const PreStartGate> gate;
  std::shared_ptr<Sink> sink;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (native_) gate = gate_;
    sink = sink_;
  }
  auto now = [&](Reply r) {
    ev.dur_ns = mono_ns() - ev.t0_ns;
    ev.status = r.status;
    ev.message = r.message;
    record(std::move(ev));
    return r;
  };
  if (!gate || !sink) return now(Reply{kOk, "", ""});  // the reference's no-op: the request is not even read
  std::vector<std::string> ids;
  const bool ok = pb::scan(
      req.data(), req.size(),
      [&](int f, const char* p, size_t n) {
        if (f == 1) ids.emplace_back(p, n);
        return true;
      },
      nullptr);
  if (!ok) return now(Reply{kInternal, "malformed PreStartContainerRequest", ""});
  ev.ids = ids;
  if (ids.empty()) return now(Reply{kOk, "", ""});
  (*gate)(std::move(ids), [this, sink, call_id, ev](Reply r) mutable {
    std::lock_guard<std::mutex> lk(sink->mu);
    if (!sink->srv) return;  // detached: the call was answered UNAVAILABLE at stop (this service may be gone)
    ev.dur_ns = mono_ns() - ev.t0_ns;
    ev.status = r.status;
    ev.message = r.message;
    record(std::move(ev));
    sink->srv->complete(call_id, std::move(r));
  });
  return std::nullopt;
}

void DevicePluginService::set_fallback(Fallback f) {
  std::lock_guard<std::mutex> lk(mu_);
  fallback_ = f ? std::make_shared<const Fallback>(std::move(f)) : nullptr;
}

void DevicePluginService::set_options(std::optional<std::string> bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  options_ = bytes ? std::make_shared<const std::string>(std::move(*bytes)) : nullptr;
}

void DevicePluginService::set_allocator(std::shared_ptr<const HiveAllocator> a) {
  std::lock_guard<std::mutex> lk(mu_);
  alloc_ = std::move(a);
}

void DevicePluginService::set_allocate_template(std::optional<AllocateTemplate> t) {
  std::lock_guard<std::mutex> lk(mu_);
  tmpl_ = t ? std::make_shared<const AllocateTemplate>(std::move(*t)) : nullptr;
}

void DevicePluginService::set_device_list(std::optional<std::string> bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  list_ = bytes ? std::make_shared<const std::string>(std::move(*bytes)) : nullptr;
}

void DevicePluginService::set_native_enabled(bool on) {
  std::lock_guard<std::mutex> lk(mu_);
  native_ = on;
}

std::vector<RpcEvent> DevicePluginService::drain_events() {
  uint64_t v;
  while (evfd_ >= 0 && ::read(evfd_, &v, sizeof(v)) > 0) {
  }
  std::lock_guard<std::mutex> lk(ev_mu_);
  std::vector<RpcEvent> out;
  out.swap(events_);
  return out;
}

void DevicePluginService::record(RpcEvent ev) {
  {
    std::lock_guard<std::mutex> lk(ev_mu_);
    if (events_.size() >= kMaxEvents) events_.erase(events_.begin(), events_.begin() + kMaxEvents / 2);
    events_.push_back(std::move(ev));
  }
  // the consumer is woken once the response is on the wire (after_io below), so
  // its wakeup never competes with the reply the caller is waiting for
  notify_pending_.store(true, std::memory_order_release);
}

void DevicePluginService::notify() {
  if (!notify_pending_.exchange(false, std::memory_order_acq_rel)) return;
  const uint64_t one = 1;
  ssize_t r = ::write(evfd_, &one, sizeof(one));
  (void)r;
}

Reply DevicePluginService::fallback(const char* method, const std::string& req, RpcEvent* ev) {
  std::shared_ptr<const Fallback> f;
  {
    std::lock_guard<std::mutex> lk(mu_);
    f = fallback_;
  }
  ev->native = false;
  if (!f) return Reply{kUnimplemented, std::string("no handler for ") + method, ""};
  return (*f)(method, req);
}

Reply DevicePluginService::preferred(const std::string& req, RpcEvent* ev) {
  std::shared_ptr<const HiveAllocator> alloc;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (native_) alloc = alloc_;
  }
  if (!alloc) return fallback("GetPreferredAllocation", req, ev);
  std::string body;
  std::string error;
  const bool ok = pb::scan(
      req.data(), req.size(),
      [&](int field, const char* p, size_t n) {
        if (field != 1) return true;
        std::vector<std::string> avail, must;
        int64_t size = 0;
        if (!pb::scan(
                p, n,
                [&](int f, const char* q, size_t m) {
                  if (f == 1) avail.emplace_back(q, m);
                  else if (f == 2) must.emplace_back(q, m);
                  return true;
                },
                [&](int f, uint64_t v) {
                  if (f == 3) size = static_cast<int32_t>(static_cast<uint32_t>(v));
                  return true;
                }))
          return false;
        const auto t0 = std::chrono::steady_clock::now();
        ev->alloc_t0_ns = mono_ns();
        AllocResult r = alloc->allocate(avail, must, static_cast<int>(size));
        ev->alloc_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        ev->candidates = static_cast<int>(r.candidates);
        ev->short_circuit = r.short_circuit;
        ev->weight = r.weight;
        if (!r.error.empty()) {
          error = r.error;
          return false;
        }
        std::string cr;
        for (auto& id : r.ids) {
          pb::put_bytes(&cr, 1, id);
          ev->ids.push_back(id);
        }
        pb::put_bytes(&body, 1, cr);
        return true;
      },
      nullptr);
  if (!error.empty()) return Reply{kUnknown, "unable to get preferred allocation list. Error:" + error, ""};
  if (!ok) return Reply{kInternal, "malformed PreferredAllocationRequest", ""};
  return Reply{kOk, "", std::move(body)};
}

Reply DevicePluginService::allocate(const std::string& req, RpcEvent* ev) {
  std::shared_ptr<const AllocateTemplate> t;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (native_) t = tmpl_;
  }
  if (!t) return fallback("Allocate", req, ev);
  std::string body;
  std::string error;
  const bool ok = pb::scan(
      req.data(), req.size(),
      [&](int field, const char* p, size_t n) {
        if (field != 1) return true;
        std::string car = t->container_prefix;
        std::string ann, env;
        bool any = false;
        std::vector<std::string> ids;
        const bool scanned = pb::scan(
            p, n,
            [&](int f, const char* q, size_t m) {
              if (f != 1) return true;
              std::string id(q, m);
              auto it = t->per_device.find(id);
              if (it == t->per_device.end()) {
                error = "unknown device ID '" + id + "' for resource " + t->resource;
                return false;
              }
              car += it->second;
              if (!t->annotation_key.empty()) {
                auto a = t->annotation_names.find(id);
                if (any) ann += ",";
                ann += a == t->annotation_names.end() ? id : a->second;
              }
              if (!t->env_key.empty()) {
                auto e = t->env_values.find(id);
                if (e != t->env_values.end() && !e->second.empty()) {
                  if (!env.empty()) env += ",";
                  env += e->second;
                }
              }
              any = true;
              if (t->container_extra) ids.push_back(id);
              ev->ids.push_back(std::move(id));
              return true;
            },
            nullptr);
        if (!scanned) return false;
        if (any && t->container_extra) car += t->container_extra(ids);
        if (any) car += t->container_nonempty;
        if (any && !t->annotation_key.empty()) {
          std::string entry;
          pb::put_bytes(&entry, 1, t->annotation_key);
          pb::put_bytes(&entry, 2, ann);
          pb::put_bytes(&car, 4, entry);
        }
        if (any && !t->env_key.empty()) {
          std::string entry;
          pb::put_bytes(&entry, 1, t->env_key);
          pb::put_bytes(&entry, 2, env);
          pb::put_bytes(&car, 1, entry);
        }
        pb::put_bytes(&body, 1, car);
        return true;
      },
      nullptr);
  if (!error.empty()) return Reply{kInvalidArgument, error, ""};
  if (!ok) return Reply{kInternal, "malformed AllocateRequest", ""};
  return Reply{kOk, "", std::move(body)};
}

void DevicePluginService::attach(GrpcServer& srv) {
  detach();
  {
    std::lock_guard<std::mutex> lk(mu_);
    sink_ = std::make_shared<Sink>();
    sink_->srv = &srv;
  }
  srv.set_after_io([this] { notify(); });
  auto wrap = [this](const char* method, std::function<Reply(const std::string&, RpcEvent*)> fn) {
    return [this, method, fn](const std::string& req) {
      RpcEvent ev;
      ev.rpc = method;
      ev.t0_ns = mono_ns();
      Reply r = fn(req, &ev);
      ev.dur_ns = mono_ns() - ev.t0_ns;
      ev.status = r.status;
      ev.message = r.message;
      record(std::move(ev));
      return r;
    };
  };
  srv.add_unary(path("GetDevicePluginOptions"),
                wrap("GetDevicePluginOptions", [this](const std::string& req, RpcEvent* ev) {
                  std::shared_ptr<const std::string> o;
                  {
                    std::lock_guard<std::mutex> lk(mu_);
                    if (native_) o = options_;
                  }
                  return o ? Reply{kOk, "", *o} : fallback("GetDevicePluginOptions", req, ev);
                }));
  srv.add_unary(path("GetPreferredAllocation"),
                wrap("GetPreferredAllocation",
                     [this](const std::string& req, RpcEvent* ev) { return preferred(req, ev); }));
  srv.add_unary(path("Allocate"),
                wrap("Allocate", [this](const std::string& req, RpcEvent* ev) { return allocate(req, ev); }));
  srv.add_unary_deferrable(path("PreStartContainer"),
                           [this](uint64_t call_id, const std::string& req) { return prestart(call_id, req); });
  srv.add_server_stream(path("ListAndWatch"), [this](uint64_t, const std::string& req) {
    RpcEvent ev;
    ev.rpc = "ListAndWatch";
    ev.t0_ns = mono_ns();
    std::shared_ptr<const std::string> l;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (native_) l = list_;
    }
    Reply r = l ? Reply{kOk, "", *l} : fallback("ListAndWatch", req, &ev);
    ev.dur_ns = mono_ns() - ev.t0_ns;
    ev.status = r.status;
    ev.message = r.message;
    record(std::move(ev));
    return r;
  });
}

}  // namespace mi355x::rpc
