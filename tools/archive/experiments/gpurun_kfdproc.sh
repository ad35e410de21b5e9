#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ls /sys/class/kfd/kfd/proc | head -50 | tr '\n' ' '; echo
echo "count: $(ls /sys/class/kfd/kfd/proc | wc -l)"
timeout -k 5 60 python - <<'PY'
import os, subprocess, time, json
exe = "rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe"
p = subprocess.Popen([exe, "--serve"], stdin=subprocess.PIPE, stdout=subprocess.PIPE)
print("hello", p.stdout.readline()[:80])
print("child pid", p.pid, "my pid", os.getpid())
print("in kfd proc:", os.path.exists(f"/sys/class/kfd/kfd/proc/{p.pid}"), sorted(os.listdir("/sys/class/kfd/kfd/proc"))[:40])
p.stdin.write(b"quit\n"); p.stdin.flush(); p.wait()
t0 = time.monotonic()
for i in range(100):
    ex = os.path.exists(f"/sys/class/kfd/kfd/proc/{p.pid}")
    if not ex: break
    time.sleep(0.01)
print("gone after ms", (time.monotonic()-t0)*1e3, "exists", ex)
for f in os.listdir("/sys/class/kfd/kfd/proc")[:2]:
    print(f, os.listdir(f"/sys/class/kfd/kfd/proc/{f}"))
PY
