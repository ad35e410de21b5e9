"""Build provenance of the native binaries: the banner
names the native sources' digest it was compiled from and the current commit,
without relinking when only HEAD moves.

Reference: the version banner "<argv0> version <gitDescribe>" stamped at build
time (cmd/k8s-device-plugin/main.go:37-48, Dockerfile:21).
"""
import os
import re
import shutil
import subprocess

from rocm_k8s_device_plugin_amd import _build
from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR

EXE = os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")


def _banner(exe):
    out = subprocess.run([exe, "-h"], capture_output=True, text=True, timeout=20)
    m = re.search(r" version (\S+) \(native sources ([0-9a-f]+)\)", out.stdout + out.stderr)
    assert m, out.stdout + out.stderr
    return m.group(1), m.group(2)


def test_banner_names_the_source_digest_and_current_describe():
    _build.ensure_built(hip=False)
    describe, digest = _banner(EXE)
    assert digest == _build._source_digest()[:12]
    want = _build.git_describe()
    if want:                                     # a git checkout: the describe of HEAD, as the tree is now
        assert describe == want, (describe, want)


def test_version_file_is_used_only_for_its_own_digest(tmp_path):
    """A copy of the daemon with a VERSION file beside its bin/ directory: the
    describe there is reported when the digest is the binary's own, and
    ignored (the compiled-in describe wins) when it names other sources."""
    _build.ensure_built(hip=False)
    (tmp_path / "bin").mkdir()
    exe = str(tmp_path / "bin" / "mi355x-device-plugin")
    shutil.copy(EXE, exe)
    _, digest = _banner(exe)
    (tmp_path / "VERSION").write_text(f"describe=v9.9.9-0-gabcdef1\ndigest={digest}\n")
    assert _banner(exe) == ("v9.9.9-0-gabcdef1", digest)
    (tmp_path / "VERSION").write_text("describe=v0.0.1-0-g0000000\ndigest=000000000000\n")
    compiled, _ = _banner(exe)
    assert compiled != "v0.0.1-0-g0000000"


def test_stamp_version_follows_head(tmp_path, monkeypatch):
    """stamp_version() writes HEAD's describe (here $GIT_DESCRIBE) with the digest, atomically."""
    monkeypatch.setattr(_build, "VERSION_FILE", tmp_path / "VERSION")
    monkeypatch.setenv("GIT_DESCRIBE", "r6-test-0-g1234567")
    _build.stamp_version("deadbeefcafe0123")
    assert (tmp_path / "VERSION").read_text() == "describe=r6-test-0-g1234567\ndigest=deadbeefcafe\n"
