// -dry_run: the node report (what kubelet would be told), the Python CLI's
// cli/device_plugin.py dry_run_report, as one JSON document on stdout.
#pragma once

#include <string>
#include <vector>

#include "flags.h"
#include "resources.h"
#include "mi355x/health_engine.h"

namespace mi355x::daemon {

// xGMI fabric of an allocated set (parallel/fabric.py Fabric.report): whether it
// is one hive, and the ring all-reduce bound its links imply (GB/s)
struct FabricReport {
  bool one_hive = false;
  bool has_bound = false;
  double bound_gbs = 0;
};
FabricReport fabric_report(const std::vector<const GpuDevice*>& devs, const KfdTopology& topo);

std::string dry_run_report(const Flags& f, bool impl_ok, Driver driver, const std::vector<Resource>& resources,
                           const KfdTopology& topo, const std::vector<std::string>& warnings,
                           const health::Engine* engine);

}  // namespace mi355x::daemon
