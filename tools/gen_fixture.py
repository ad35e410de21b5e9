#!/usr/bin/env python3
"""Write a synthetic MI355X node (sysfs + /dev trees) for manual runs:

  python tools/gen_fixture.py /tmp/node --mode cpx --nps nps1 --gpus 8 --hive-size 8
  ./scripts/k8s-device-plugin -sysfs_root /tmp/node/sys -dev_root /tmp/node/dev -kubelet_dir /tmp/dp
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rocm_k8s_device_plugin_amd.testing.fixtures import FixtureSpec, make_mi355x_node  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("root")
    ap.add_argument("--mode", default="spx", choices=["spx", "dpx", "qpx", "cpx"])
    ap.add_argument("--nps", default="nps1", choices=["nps1", "nps2"])
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--numa", type=int, default=2)
    ap.add_argument("--hive-size", type=int, default=8)
    ap.add_argument("--driver", default="container", choices=["container", "vf", "pf"])
    ap.add_argument("--vfs-per-gpu", type=int, default=1)
    a = ap.parse_args()
    info = make_mi355x_node(a.root, FixtureSpec(num_gpus=a.gpus, compute_partition=a.mode, memory_partition=a.nps,
                                                numa_nodes=a.numa, hive_size=a.hive_size, mode=a.driver,
                                                vfs_per_gpu=a.vfs_per_gpu))
    print(json.dumps({"sysfs": str(info.sysfs), "dev": str(info.dev), "devices": info.device_ids}, indent=1))


if __name__ == "__main__":
    main()
