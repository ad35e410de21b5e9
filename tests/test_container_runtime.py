"""Fake CRI runtime helpers used by bench.py (CPU)."""
import threading
import time

from rocm_k8s_device_plugin_amd.container_runtime import kfd_processes, wait_kfd_released


def test_wait_kfd_released_tracks_procfs(tmp_path):
    proc = tmp_path / "proc"
    proc.mkdir()
    for pid in ("100", "200", "300"):
        (proc / pid).mkdir()
    assert kfd_processes(str(proc)) == {"100", "200", "300"}
    assert kfd_processes(str(tmp_path / "missing")) == set()

    def teardown():
        time.sleep(0.05)
        (proc / "200").rmdir()
        time.sleep(0.05)
        (proc / "300").rmdir()

    th = threading.Thread(target=teardown)
    th.start()
    waited = wait_kfd_released({"200", "300"}, timeout_s=5.0, proc_dir=str(proc))
    th.join()
    assert 80 <= waited < 2000
    assert kfd_processes(str(proc)) == {"100"}     # unrelated processes are not waited for
    assert wait_kfd_released(set(), proc_dir=str(proc)) < 5
    # a process that never goes away costs at most the timeout
    assert 90 <= wait_kfd_released({"100"}, timeout_s=0.1, proc_dir=str(proc)) < 1000


def test_mount_redirects():
    from rocm_k8s_device_plugin_amd.container_runtime import mount_redirects
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    ms = [pb.Mount(container_path="/sys/devices/system/node", host_path="/var/lib/x/node", read_only=True),
          pb.Mount(container_path="/sys/devices/system/node", host_path="/sys/devices/system/node")]
    assert mount_redirects(ms) == "/sys/devices/system/node=/var/lib/x/node"
    assert mount_redirects([("/a", "/b"), ("/c", "/d")]) == "/a=/b;/c=/d"
    assert mount_redirects([]) == ""
