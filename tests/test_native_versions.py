"""Version banner of both native binaries (C18 / reference main.go:37-48,77-79).

The reference prints "AMD GPU device plugin for Kubernetes", "<argv0> version
<gitDescribe>" and its library versions in -h and logs them at start-up; the
describe string is stamped at build time (Dockerfile:21). Here the build
stamps MI355X_GIT_DESCRIBE (rocm_k8s_device_plugin_amd/_build.py git_describe,
or the Dockerfiles' GIT_DESCRIBE argument).
"""
import os
import re
import subprocess

import pytest

from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

BIN = os.path.join(str(PKG_DIR), "bin")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TITLES = {"mi355x-device-plugin": "AMD GPU device plugin for Kubernetes (MI355X-native, native daemon)",
          "mi355x-node-labeller": "AMD GPU Node Labeller for Kubernetes (MI355X-native, native daemon)"}


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _stamped():
    cache = os.path.join(REPO, "build", "native", "CMakeCache.txt")
    if not os.path.exists(cache):
        return None
    m = re.search(r"^MI355X_GIT_DESCRIBE:STRING=(.*)$", open(cache).read(), re.M)
    return m.group(1) if m else None


def _check_banner(lines, exe):
    from rocm_k8s_device_plugin_amd import _build
    assert lines[0] == TITLES[os.path.basename(exe)]
    m = re.fullmatch(re.escape(exe) + r" version (\S+) \(native sources ([0-9a-f]{12})\)", lines[1])
    assert m, lines[1]
    assert m.group(2) == _build._source_digest()[:12]
    # HEAD's describe (<package>/VERSION, kept current without a relink), else the compiled-in one
    version = os.path.join(os.path.dirname(BIN), "VERSION")
    if os.path.exists(version):
        assert "describe=" + m.group(1) in open(version).read().split()
    elif _stamped():
        assert m.group(1) == _stamped()
    assert re.fullmatch(r"rocm: \S+, amdgpu: \S+, libdrm_amdgpu: \S+, amd-smi: \S+, numa_source: sysfs", lines[2]), lines[2]


@pytest.mark.parametrize("name", sorted(TITLES))
def test_help_starts_with_the_version_banner(name):
    exe = os.path.join(BIN, name)
    p = subprocess.run([exe, "-h"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0
    lines = p.stdout.splitlines()
    _check_banner(lines, exe)
    assert lines[3].startswith("usage: " + exe)


def test_device_plugin_logs_the_banner_first(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    exe = os.path.join(BIN, "mi355x-device-plugin")
    p = subprocess.run([exe, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket",
                        "", "-kubelet_dir", str(tmp_path / "dp")], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    msgs = [l.split("] ", 1)[1] for l in p.stderr.splitlines()[:3]]
    _check_banner(msgs, exe)
    # the amdgpu field is the module version under -sysfs_root
    ver = (fi.sysfs / "module" / "amdgpu" / "version").read_text().strip()
    assert f"amdgpu: {ver}," in msgs[2]


def test_labeller_logs_the_banner_first(tmp_path):
    exe = os.path.join(BIN, "mi355x-node-labeller")
    env = {k: v for k, v in os.environ.items() if k not in ("DS_NODE_NAME", "KUBERNETES_SERVICE_HOST")}
    p = subprocess.run([exe, "-sysfs_root", str(tmp_path)], capture_output=True, text=True, timeout=30, env=env,
                       cwd=str(tmp_path))
    assert p.returncode == 1
    msgs = [l.split("] ", 1)[1] for l in p.stderr.splitlines()[:3]]
    _check_banner(msgs, exe)
