// pybind11 bindings for the in-process liveness probe (_hip): the HIP launch
// path and the HSA-direct path over the same gfx950 kernel. Importing it loads
// the GPU runtimes, so the control plane never imports it — only GPU tests and
// smoke() do. The plugin itself runs the probe executable in a child process.
#include <pybind11/pybind11.h>

#include "mi355x/liveness_probe.h"

namespace py = pybind11;

namespace {

py::dict to_dict(const mi355x_probe_result& r) {
  py::dict d;
  d["ordinal"] = r.ordinal;
  d["ok"] = static_cast<bool>(r.ok);
  d["hip_error"] = r.hip_error;
  d["mismatches"] = r.mismatches;
  d["nonce"] = r.nonce;
  d["xcc_id"] = r.xcc_id;
  d["hw_id"] = r.hw_id;
  d["iters"] = r.iters;
  d["dispatches"] = r.dispatches;
  d["kfd_node_id"] = r.kfd_node_id;
  d["runtime"] = std::string(r.runtime);
  d["setup_us"] = r.setup_us;
  d["kernel_us"] = r.kernel_us;
  d["total_us"] = r.total_us;
  py::dict ph;
  ph["code_object"] = r.phase_us[0];
  ph["queue"] = r.phase_us[1];
  ph["buffers"] = r.phase_us[2];
  ph["dispatch_wait"] = r.phase_us[3];
  d["phase_us"] = ph;
  d["pci_bus_id"] = std::string(r.pci_bus_id);
  d["arch"] = std::string(r.arch);
  d["name"] = std::string(r.name);
  d["uuid"] = std::string(r.uuid);
  d["pci_domain"] = r.pci_domain;
  d["pci_bus"] = r.pci_bus;
  d["pci_device"] = r.pci_device;
  d["cu_count"] = r.cu_count;
  d["total_mem"] = r.total_mem;
  d["error"] = std::string(r.error);
  return d;
}

}  // namespace

PYBIND11_MODULE(_hip, m) {
  m.doc() = "gfx950 MFMA liveness probe (in-process)";
  m.def("device_count", [] {
    int n;
    {
      py::gil_scoped_release nogil;
      n = mi355x_probe_device_count();
    }
    return n;
  });
  m.def(
      "probe",
      [](int ordinal, uint32_t nonce, int iters) {
        // The first launch on a device in this process includes the HIP
        // runtime's lazy code-object load (hundreds of us); its event time is
        // reported as first_launch_us. kernel_us is the event-timed launch of a
        // second, warm probe (fresh nonce, verified too).
        static bool warm[64] = {false};
        const bool first = ordinal >= 0 && ordinal < 64 && !warm[ordinal];
        mi355x_probe_result cold{}, r{};
        {
          py::gil_scoped_release nogil;
          if (first) {
            mi355x_probe_device(ordinal, nonce ^ 0xA5A5A5A5u, iters, &cold);
            if (cold.ok) warm[ordinal] = true;
          }
          mi355x_probe_device(ordinal, nonce, iters, &r);
        }
        py::dict d = to_dict(r);
        d["first_launch"] = first;
        d["first_launch_us"] = first ? cold.kernel_us : 0.0;
        if (first && !cold.ok) {  // a cold failure is a failure
          d["ok"] = false;
          d["error"] = std::string("first launch: ") + cold.error;
        }
        return d;
      },
      py::arg("ordinal") = 0, py::arg("nonce") = 12345u, py::arg("iters") = 4);
  m.def(
      "identify",
      [](int ordinal) {
        mi355x_probe_result r;
        {
          py::gil_scoped_release nogil;
          mi355x_probe_identify(ordinal, &r);
        }
        return to_dict(r);
      },
      py::arg("ordinal") = 0);
  // HSA-direct path (same code object, one AQL dispatch, no HIP runtime involvement)
  m.def("hsa_device_count", [] {
    int n;
    {
      py::gil_scoped_release nogil;
      n = mi355x_hsa_probe_init();
    }
    return n;
  });
  m.def(
      "hsa_probe",
      [](int ordinal, uint32_t nonce, int iters, double timeout_s) {
        mi355x_probe_result r;
        {
          py::gil_scoped_release nogil;
          mi355x_hsa_probe_device(ordinal, nonce, iters, timeout_s, &r);
        }
        return to_dict(r);
      },
      py::arg("ordinal") = 0, py::arg("nonce") = 12345u, py::arg("iters") = 4, py::arg("timeout_s") = 5.0);
  m.def(
      "hsa_identify",
      [](int ordinal) {
        mi355x_probe_result r;
        {
          py::gil_scoped_release nogil;
          mi355x_hsa_probe_identify(ordinal, &r);
        }
        return to_dict(r);
      },
      py::arg("ordinal") = 0);
}
