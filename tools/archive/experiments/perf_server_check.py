"""Throughput-check replies of the probe server vs the one-shot CLI on the same
GPU (debugging implausible rates from the kept-queue server)."""
import json
import subprocess
import sys

sys.path.insert(0, ".")
from rocm_k8s_device_plugin_amd.ops.native import probe_executable  # noqa: E402

exe = str(probe_executable("hsa"))
keys = ("ok", "hbm_write_gbps", "hbm_read_gbps", "mfma_tflops", "clock_mhz_median", "fill_us", "check_us",
        "check2_us", "mfma_us", "total_us", "error")


def show(tag, doc):
    d = (doc.get("devices") or [{}])[0]
    print(tag, json.dumps({k: d.get(k) for k in keys}), flush=True)


cli = subprocess.run([exe, "--perf", "--perf-mib", "1024", "--devices", "0", "--timeout", "30"],
                     capture_output=True, text=True, timeout=120)
show("cli", json.loads(cli.stdout.strip().splitlines()[-1]))
for argv, reqs in ((["--serve", "--keep"], ["perf 65536 9.5 1024 0:11", "perf 65536 9.5 1024 0:12"]),
                   (["--serve", "--keep"], ["probe 4 9.5 0:21", "sweep 4 9.5 0:22", "perf 65536 9.5 1024 0:23"]),
                   (["--serve"], ["perf 65536 9.5 1024 0:31", "perf 65536 9.5 1024 0:32"])):
    p = subprocess.Popen([exe, *argv], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    hello = p.stdout.readline()
    for r in reqs:
        p.stdin.write(r + "\n")
        p.stdin.flush()
        show(" ".join(argv) + " | " + r.split()[0], json.loads(p.stdout.readline()))
    p.stdin.write("quit\n")
    p.stdin.flush()
    p.wait(timeout=30)
