"""glog flag semantics of the logger (utils/log.py): -logtostderr / -log_dir
files per severity with glog's names and symlinks, -stderrthreshold,
-alsologtostderr, -vmodule, -log_backtrace_at (reference:
vendor/github.com/golang/glog/glog_flags.go:388-397, glog_file.go)."""
import glob
import json
import os
import subprocess
import sys

import pytest

from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.utils import log

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _restore_logging():
    yield
    log.setup(0)


def _emit():
    lg = log.get("t")
    lg.info("info-line")
    lg.warning("warning-line")
    lg.error("error-line")


def test_log_dir_files_per_severity(tmp_path, capsys):
    log.setup(0, logtostderr=False, log_dir=str(tmp_path), program="k8s-device-plugin")
    _emit()
    files = {os.path.basename(p) for p in glob.glob(str(tmp_path / "*"))}
    for sev in ("INFO", "WARNING", "ERROR"):
        link = tmp_path / f"k8s-device-plugin.{sev}"
        assert link.is_symlink(), files
        target = os.readlink(link)
        assert target.startswith("k8s-device-plugin.") and f".log.{sev}." in target
        assert target.rsplit(".", 1)[1] == str(os.getpid())
    info = (tmp_path / "k8s-device-plugin.INFO").read_text()
    assert info.startswith("Log file created at:") and "Log line format: [IWEF]mmdd" in info
    assert all(x in info for x in ("info-line", "warning-line", "error-line"))
    warn = (tmp_path / "k8s-device-plugin.WARNING").read_text()
    assert "info-line" not in warn and "warning-line" in warn and "error-line" in warn
    err = (tmp_path / "k8s-device-plugin.ERROR").read_text()
    assert "warning-line" not in err and "error-line" in err
    assert not (tmp_path / "k8s-device-plugin.FATAL").exists()   # created on first use only
    stderr = capsys.readouterr().err
    assert "error-line" in stderr and "warning-line" not in stderr   # -stderrthreshold=ERROR


def test_log_link_and_logbuflevel(tmp_path, capsys):
    """glog_file.go:44-46,133-137: -log_link adds a <prog>.<SEV> link to the full
    path in another directory; -logbuflevel is accepted (records are never buffered)."""
    from rocm_k8s_device_plugin_amd.utils import flags as F
    p = F.GoFlagParser(prog="k8s-device-plugin")
    F.add_glog_flags(p)
    ns = p.parse_args(["-logtostderr=false", f"-log_dir={tmp_path / 'logs'}", f"-log_link={tmp_path}",
                       "-logbuflevel=-1"])
    assert ns.logbuflevel == -1
    log.setup_from_flags(ns, "k8s-device-plugin")
    _emit()
    target = os.readlink(tmp_path / "logs" / "k8s-device-plugin.INFO")
    assert os.readlink(tmp_path / "k8s-device-plugin.INFO") == str(tmp_path / "logs" / target)
    assert "info-line" in (tmp_path / "k8s-device-plugin.INFO").read_text()
    log.setup(0)


def test_alsologtostderr_and_threshold(tmp_path, capsys):
    log.setup(0, logtostderr=False, alsologtostderr=True, log_dir=str(tmp_path), program="p")
    _emit()
    assert "info-line" in capsys.readouterr().err
    log.setup(0, logtostderr=False, stderr_threshold="WARNING", log_dir=str(tmp_path / "b"), program="p")
    _emit()
    err = capsys.readouterr().err
    assert "warning-line" in err and "info-line" not in err


def test_logtostderr_writes_no_files(tmp_path, capsys):
    log.setup(0, logtostderr=True, log_dir=str(tmp_path), program="p")
    _emit()
    assert os.listdir(tmp_path) == []
    assert "info-line" in capsys.readouterr().err


def test_vmodule_per_file_verbosity():
    log.setup(0, vmodule="test_logging=3,labels=9")
    assert log.V(3) and not log.V(4)
    log.setup(0, vmodule="other=5")
    assert not log.V(1)
    log.setup(2)
    assert log.V(2) and not log.V(3)
    with pytest.raises(ValueError):
        log.setup(0, vmodule="nolevel")


def test_log_backtrace_at(tmp_path, capsys):
    line = sys._getframe().f_lineno + 2
    log.setup(0, log_backtrace_at=f"test_logging.py:{line}")
    log.get("t").info("with-stack")
    log.get("t").info("without-stack")
    err = capsys.readouterr().err
    first, second = err.split("without-stack")[0], err.split("without-stack")[1]
    assert "with-stack" in first and "test_log_backtrace_at" in first
    assert "test_log_backtrace_at" not in second


def test_device_plugin_cli_writes_log_files(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    env = dict(os.environ, PYTHONPATH=REPO)
    p = subprocess.run([sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin", "-dry_run",
                        "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket", "",
                        "-kubelet_dir", str(tmp_path / "dp"), "-logtostderr=false", f"-log_dir={tmp_path / 'logs'}",
                        "-vmodule=servicer=2"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    json.loads(p.stdout)
    info = (tmp_path / "logs" / "k8s-device-plugin.INFO").read_text()
    assert "Found 8 AMDGPUs" in info or "AMD GPU device plugin" in info, info[:2000]
    assert "I" in p.stderr or p.stderr == ""            # INFO lines stay out of stderr (threshold ERROR)
    assert "Found 8 AMDGPUs" not in p.stderr
    bad = subprocess.run([sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin", "-dry_run",
                          "-vmodule=broken"], capture_output=True, text=True, timeout=120, env=env)
    assert bad.returncode == 1 and "vmodule" in bad.stderr


@pytest.mark.parametrize("cli,flags", [
    ("device_plugin", ("-pulse", "-driver_type", "-resource_naming_strategy", "-kubelet_dir", "-log_dir",
                       "-liveness_corroborate", "-allocator_search")),
    ("node_labeller", ("-vram", "-log_dir", "-vmodule", "-dry_run")),
])
def test_cli_help_renders(cli, flags):
    """-h must render every help string (argparse %-formats them) and name the
    reference's flags (cmd/k8s-device-plugin/main.go:53-55)."""
    p = subprocess.run([sys.executable, "-m", f"rocm_k8s_device_plugin_amd.cli.{cli}", "-h"], capture_output=True,
                       text=True, timeout=120, env=dict(os.environ, PYTHONPATH=REPO))
    assert p.returncode == 0, p.stderr[-1500:]
    for f in flags:
        assert f in p.stdout, f
