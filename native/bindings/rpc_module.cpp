// pybind11 bindings of the native device-plugin gRPC server (part of _native).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../src/rpc/hpack.h"
#include "mi355x/dp_service.h"
#include "mi355x/grpc_server.h"

namespace py = pybind11;
using namespace mi355x;
using namespace mi355x::rpc;

namespace {

// One kubelet-facing endpoint: the HTTP/2 server plus the DevicePlugin service.
struct PyDevicePluginServer {
  GrpcServer server;
  DevicePluginService svc;
  bool attached = false;
  bool has_fallback = false;

  ~PyDevicePluginServer() {
    // the I/O thread may be waiting for the GIL inside a fallback
    py::gil_scoped_release nogil;
    server.stop(0.0);
  }
};

}  // namespace

void bind_rpc(py::module_& m) {
  py::class_<PyDevicePluginServer>(m, "DevicePluginServer")
      .def(py::init<>())
      .def(
          "set_fallback",
          [](PyDevicePluginServer& s, py::function fn) {
            if (s.server.running()) throw std::runtime_error("set_fallback before start()");
            py::object keep = fn;
            s.svc.set_fallback([keep](const std::string& method, const std::string& req) -> Reply {
              py::gil_scoped_acquire gil;
              try {
                py::tuple t = keep(method, py::bytes(req)).cast<py::tuple>();
                Reply r;
                r.status = t[0].cast<int>();
                r.message = t[1].cast<std::string>();
                r.body = t[2].cast<std::string>();
                return r;
              } catch (py::error_already_set& e) {
                return Reply{kUnknown, e.what(), ""};
              } catch (const std::exception& e) {
                return Reply{kUnknown, e.what(), ""};
              }
            });
            s.has_fallback = true;
          },
          py::arg("fn"),
          "fn(method: str, request: bytes) -> (status: int, message: str, body: bytes), called on the server "
          "thread (with the GIL) for whatever has no native state")
      .def(
          "start",
          [](PyDevicePluginServer& s, const std::string& path) {
            if (!s.attached) {
              s.svc.attach(s.server);
              s.attached = true;
            }
            py::gil_scoped_release nogil;
            return s.server.start(path);
          },
          py::arg("unix_path"), "bind and serve; returns '' or an error")
      .def(
          "stop",
          [](PyDevicePluginServer& s, double grace_s) {
            py::gil_scoped_release nogil;
            s.server.stop(grace_s);
          },
          py::arg("grace_s") = 0.5)
      .def_property_readonly("running", [](const PyDevicePluginServer& s) { return s.server.running(); })
      .def("set_options", [](PyDevicePluginServer& s, std::optional<std::string> b) { s.svc.set_options(b); })
      .def(
          "set_allocator",
          [](PyDevicePluginServer& s, std::shared_ptr<HiveAllocator> a) { s.svc.set_allocator(std::move(a)); },
          py::arg("allocator").none(true))
      .def(
          "set_allocate_template",
          [](PyDevicePluginServer& s, const std::string& resource, const std::string& prefix,
             const std::unordered_map<std::string, std::string>& per_device, const std::string& annotation_key,
             const std::unordered_map<std::string, std::string>& annotation_names,
             const std::string& container_nonempty) {
            AllocateTemplate t;
            t.resource = resource;
            t.container_prefix = prefix;
            t.per_device = per_device;
            t.container_nonempty = container_nonempty;
            t.annotation_key = annotation_key;
            t.annotation_names = annotation_names;
            s.svc.set_allocate_template(std::move(t));
          },
          py::arg("resource"), py::arg("container_prefix"), py::arg("per_device"), py::arg("annotation_key") = "",
          py::arg("annotation_names") = std::unordered_map<std::string, std::string>(),
          py::arg("container_nonempty") = "")
      .def("clear_allocate_template", [](PyDevicePluginServer& s) { s.svc.set_allocate_template(std::nullopt); })
      .def("set_device_list", [](PyDevicePluginServer& s, std::optional<std::string> b) { s.svc.set_device_list(b); })
      .def("set_native_enabled", [](PyDevicePluginServer& s, bool on) { s.svc.set_native_enabled(on); })
      .def(
          "publish_list",
          [](PyDevicePluginServer& s, const std::string& b) {
            s.svc.set_device_list(b);
            return s.server.broadcast(DevicePluginService::path("ListAndWatch"), b);
          },
          "set the ListAndWatch list and send it on every open stream; returns the number of streams")
      .def("open_streams",
           [](const PyDevicePluginServer& s) {
             return s.server.open_streams(DevicePluginService::path("ListAndWatch"));
           })
      .def_property_readonly("event_fd", [](const PyDevicePluginServer& s) { return s.svc.event_fd(); })
      .def("drain_events",
           [](PyDevicePluginServer& s) {
             std::vector<RpcEvent> evs = s.svc.drain_events();
             py::list out;
             for (auto& e : evs) {
               py::dict d;
               d["rpc"] = e.rpc;
               d["status"] = e.status;
               d["message"] = e.message;
               d["t0_ns"] = e.t0_ns;
               d["dur_ns"] = e.dur_ns;
               d["native"] = e.native;
               d["candidates"] = e.candidates;
               d["short_circuit"] = e.short_circuit;
               d["weight"] = e.weight;
               d["alloc_us"] = e.alloc_us;
               d["alloc_t0_ns"] = e.alloc_t0_ns;
               d["ids"] = e.ids;
               out.append(d);
             }
             return out;
           })
      .def("stats", [](const PyDevicePluginServer& s) {
        ServerStats st = s.server.stats();
        py::dict d;
        d["connections"] = st.connections;
        d["calls"] = st.calls;
        d["streams_open"] = st.streams_open;
        d["streams_opened"] = st.streams_opened;
        d["protocol_errors"] = st.protocol_errors;
        d["caller_protocol_errors"] = st.caller_protocol_errors;
        d["bytes_in"] = st.bytes_in;
        d["bytes_out"] = st.bytes_out;
        return d;
      });

  py::class_<GrpcClient>(m, "GrpcClient")
      .def(py::init<>())
      .def(
          "connect",
          [](GrpcClient& c, const std::string& path, double timeout_s) {
            py::gil_scoped_release nogil;
            return c.connect(path, timeout_s);
          },
          py::arg("unix_path"), py::arg("timeout_s") = 10.0)
      .def(
          "unary",
          [](GrpcClient& c, const std::string& path, const std::string& req, double timeout_s) {
            Reply r;
            {
              py::gil_scoped_release nogil;
              r = c.unary(path, req, timeout_s);
            }
            return py::make_tuple(r.status, r.message, py::bytes(r.body));
          },
          py::arg("path"), py::arg("request"), py::arg("timeout_s") = 10.0,
          "-> (grpc status, message, response bytes); status -1 = transport error")
      .def("close", &GrpcClient::close)
      .def("set_abort_fd", &GrpcClient::set_abort_fd, py::arg("fd"),
           "a readable fd ends any wait at once (status -1, 'interrupted'); -1 = none")
      .def_property_readonly("going_away", &GrpcClient::going_away)
      .def_property_readonly("connected", &GrpcClient::connected);

  // HPACK primitives, exposed for the interop / conformance tests
  m.def("hpack_huffman_decode", [](const std::string& b) -> py::object {
    std::string out;
    if (!huffman_decode(reinterpret_cast<const uint8_t*>(b.data()), b.size(), &out)) return py::none();
    return py::bytes(out);
  });
  m.def("hpack_huffman_encode", [](const std::string& s) {
    std::string out;
    huffman_encode(s, &out);
    return py::bytes(out);
  });
  m.def("hpack_decode_block", [](const std::string& block) -> py::object {
    HpackDecoder dec;
    HeaderList hl;
    if (!dec.decode(reinterpret_cast<const uint8_t*>(block.data()), block.size(), &hl)) return py::none();
    py::list out;
    for (auto& [k, v] : hl) out.append(py::make_tuple(py::bytes(k), py::bytes(v)));
    return out;
  });
}
