"""Drop-in packaging checks: DaemonSet manifests, Helm values, images, examples."""
import json
import os
import re
from pathlib import Path

import pytest
import yaml

REPO = Path(__file__).resolve().parent.parent


def _docs(name):
    return [d for d in yaml.safe_load_all((REPO / name).read_text()) if d]


def _ds(doc):
    return doc["spec"]["template"]["spec"]


def test_device_plugin_manifests():
    for name, cname in [("k8s-ds-amdgpu-dp.yaml", "amdgpu-dp-cntr"),
                        ("k8s-ds-amdgpu-dp-health.yaml", "amdgpu-dp-cntr-health")]:
        (ds,) = _docs(name)
        assert ds["kind"] == "DaemonSet" and ds["metadata"]["name"] == "amdgpu-device-plugin-daemonset"
        assert ds["metadata"]["namespace"] == "kube-system"
        assert ds["spec"]["selector"]["matchLabels"] == {"name": "amdgpu-dp-ds"}
        spec = _ds(ds)
        assert spec["priorityClassName"] == "system-node-critical"
        assert {"key": "CriticalAddonsOnly", "operator": "Exists"} in spec["tolerations"]
        c = spec["containers"][0]
        assert c["name"] == cname
        mounts = {m["mountPath"] for m in c["volumeMounts"]}
        assert {"/var/lib/kubelet/device-plugins", "/sys"} <= mounts
    (health,) = _docs("k8s-ds-amdgpu-dp-health.yaml")
    c = _ds(health)["containers"][0]
    assert c["command"] == ["./k8s-device-plugin"]
    assert "-pulse=2" in c["args"] and "-liveness=true" in c["args"] and "-smi_xgmi=true" in c["args"]
    assert c["resources"]["requests"]["memory"] == "3Gi"
    assert "/dev" in {m["mountPath"] for m in c["volumeMounts"]}
    # the health DaemonSet restarts a wedged daemon and gates rollouts on registration
    assert "-metrics_port=9400" in c["args"] and c["ports"] == [{"name": "metrics", "containerPort": 9400}]
    assert c["livenessProbe"]["httpGet"] == {"path": "/healthz", "port": "metrics"}
    assert c["readinessProbe"]["httpGet"] == {"path": "/readyz", "port": "metrics"}
    assert c["startupProbe"]["httpGet"] == c["livenessProbe"]["httpGet"]
    plain = _ds(_docs("k8s-ds-amdgpu-dp.yaml")[0])["containers"][0]
    assert "livenessProbe" not in plain                # the plain manifest stays as upstream


def test_labeller_manifest():
    docs = {d["kind"]: d for d in _docs("k8s-ds-amdgpu-labeller.yaml")}
    assert docs["ClusterRole"]["metadata"]["name"] == "cr-node-labeller"
    verbs = set(docs["ClusterRole"]["rules"][0]["verbs"])
    assert {"get", "list", "watch", "update", "patch"} <= verbs
    assert docs["ServiceAccount"]["metadata"]["name"] == "node-labeller-sa"
    ds = docs["DaemonSet"]
    assert ds["metadata"]["name"] == "amdgpu-labeller-daemonset"
    c = _ds(ds)["containers"][0]
    assert c["command"] == ["./k8s-node-labeller"]
    assert c["args"] == ["-vram", "-cu-count", "-simd-count", "-device-id", "-family"]
    assert c["env"][0]["name"] == "DS_NODE_NAME"
    # every labeller arg is a flag of the native labeller the image runs (and of the label oracle)
    import subprocess
    exe = REPO / "rocm_k8s_device_plugin_amd" / "bin" / "mi355x-node-labeller"
    p = subprocess.run([str(exe), "-dry_run", *c["args"]], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-1000:]
    from rocm_k8s_device_plugin_amd.cli.node_labeller import build_parser
    build_parser().parse_args(c["args"])


def _keys(d, prefix=""):
    out = set()
    for k, v in d.items():
        out.add(prefix + k)
        if isinstance(v, dict):
            out |= _keys(v, prefix + k + ".")
    return out


def test_helm_values_superset_of_upstream(ref_testdata):
    ours = yaml.safe_load((REPO / "helm/amd-gpu/values.yaml").read_text())
    ref = yaml.safe_load((ref_testdata.parent / "helm/amd-gpu/values.yaml").read_text())
    missing = _keys(ref) - _keys(ours)
    assert not missing, missing
    chart = yaml.safe_load((REPO / "helm/amd-gpu/Chart.yaml").read_text())
    assert chart["name"] == "amd-gpu"


def test_helm_object_names():
    t = (REPO / "helm/amd-gpu/templates")
    assert "{{ .Chart.Name }}-device-plugin-daemonset" in (t / "deviceplugin-daemonset.yaml").read_text()
    assert "{{ .Chart.Name }}-labeller-daemonset" in (t / "labeller.yaml").read_text()
    assert "cr-{{ .Chart.Name }}-node-labeller" in (t / "rbac.yaml").read_text()
    assert "{{ .Chart.Name }}-node-labeller-sa" in (t / "serviceaccount.yaml").read_text()
    # Helm template braces balance (cheap syntax sanity without a helm binary)
    for f in t.iterdir():
        s = f.read_text()
        assert s.count("{{") == s.count("}}"), f
        opens = len(re.findall(r"\{\{-?\s*(if|with|range|define)\b", s))
        ends = len(re.findall(r"\{\{-?\s*end\s*-?\}\}", s))
        assert opens == ends, f


def test_images_entrypoints():
    for f, exe in [("Dockerfile", "k8s-device-plugin"), ("labeller.Dockerfile", "k8s-node-labeller"),
                   ("ubi-dp.Dockerfile", "k8s-device-plugin"), ("ubi-labeller.Dockerfile", "k8s-node-labeller")]:
        s = (REPO / f).read_text()
        assert f"CMD [\"./{exe}\"" in s, f
        assert "WORKDIR /root" in s
    assert "-pulse=30" in (REPO / "ubi-dp.Dockerfile").read_text()
    for exe in ("k8s-device-plugin", "k8s-node-labeller"):
        p = REPO / "scripts" / exe
        assert os.access(p, os.X_OK)


def test_examples_parse_and_request_gpus():
    n = 0
    for f in (REPO / "example").rglob("*.yaml"):
        for d in yaml.safe_load_all(f.read_text()):
            n += 1
            assert "kind" in d
    assert n >= 7
    pod = _docs("example/pod/alexnet-gpu.yaml")[0]
    assert pod["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == 1


def test_cpx_example_requests_a_resource_the_plugin_advertises(tmp_path):
    """example/pod/cpx-partitions.yaml: its resource and node selector are what
    the plugin (mixed naming) and the labeller produce on an MI355X CPX / NPS1 node."""
    from rocm_k8s_device_plugin_amd import constants as C
    from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
    from rocm_k8s_device_plugin_amd.labeller import labels as L
    from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    pod = _docs("example/pod/cpx-partitions.yaml")[0]
    (res, n), = pod["spec"]["containers"][0]["resources"]["limits"].items()
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx")
    names = ContainerImpl("mixed", str(fi.sysfs), HealthConfig(exporter_socket=None)).resource_names()
    assert res == f"amd.com/{names[0]}" and names == ["cpx_nps1"] and n == 2
    labels = L.generate_labels({k: k == "compute-memory-partition" for k in C.SUPPORTED_LABELS + L.EXTRA_LABELS}, "",
                               str(fi.sysfs), str(fi.dev))
    assert pod["spec"]["nodeSelector"].items() <= labels.items()


@pytest.mark.parametrize("tool", sorted(p.name for p in (REPO / "tools").glob("*.py")))
def test_every_tool_parses_its_arguments(tool):
    """Each maintained measurement tool starts (its --help runs without a GPU)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, str(REPO / "tools" / tool), "--help"], capture_output=True, text=True,
                       timeout=120, cwd=REPO)
    assert r.returncode == 0 and "usage" in r.stdout.lower(), r.stderr[-1500:]


def _workflow_commands():
    """(workflow, step name, argv) for every command line of every run: step."""
    import shlex
    root = REPO / ".github" / "workflows"
    for f in sorted(root.iterdir()):
        doc = yaml.safe_load(f.read_text())
        for job in doc["jobs"].values():
            for step in job["steps"]:
                for line in step.get("run", "").splitlines():
                    for part in line.split("&&"):
                        if part.strip():
                            yield f.name, step.get("name", ""), shlex.split(part)


def test_ci_workflows_parse_and_run_real_entry_points():
    docs = {f.name: yaml.safe_load(f.read_text()) for f in (REPO / ".github" / "workflows").iterdir()}
    assert set(docs) == {"ci.yaml", "helm-chart-release.yaml"}
    steps = " ".join(s.get("run", "") for j in docs["ci.yaml"]["jobs"].values() for s in j["steps"])
    for cmd in ("rocm_k8s_device_plugin_amd._build", '-m "not gpu"', "-m gpu", "bench.py"):
        assert cmd in steps
    assert "--sanitize address,undefined" in steps and "--sanitize thread" in steps
    assert docs["helm-chart-release.yaml"]["jobs"]["release"]["steps"][-1]["with"]["charts_dir"] == "helm"


def test_ci_command_lines_pass_the_real_argument_parsers():
    """Every workflow command goes through the argparse parser of the entry
    point it calls (a wrong flag fails here, not on the CI runner). pytest
    lines run pytest's own option parsing and collection; unknown commands
    fail so new steps must be added to this check."""
    import importlib.util
    import subprocess
    import sys
    from rocm_k8s_device_plugin_amd import _build
    spec = importlib.util.spec_from_file_location("bench_under_test", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    checked = 0
    for wf, name, argv in _workflow_commands():
        where = f"{wf}: {name}: {' '.join(argv)}"
        if argv[0] in ("git", "helm"):
            continue
        if argv[0] == "make":            # a Makefile target, with VAR=value overrides only
            targets = re.findall(r"^([A-Za-z0-9_-]+):", (REPO / "Makefile").read_text(), re.M)
            assert all(a in targets or re.fullmatch(r"[A-Z_]+=\S*", a) for a in argv[1:]), where
            checked += 1
            continue
        if argv[0] == "docker":          # docker run of an image the Makefile builds
            from test_image_layout import image_map
            assert argv[1] == "run" and any(a in image_map() for a in argv), where
            continue
        assert argv[0] in ("python3", "python"), where
        if argv[1:4] == ["-m", "pip", "install"]:
            continue
        try:
            if argv[1:3] == ["-m", "rocm_k8s_device_plugin_amd._build"]:
                _build.make_parser().parse_args(argv[3:])
            elif argv[1] == "bench.py":
                bench.make_parser().parse_args(argv[2:])
            elif argv[1] == "tools/analyze_native.py":
                aspec = importlib.util.spec_from_file_location("analyze_native", REPO / "tools" / "analyze_native.py")
                anm = importlib.util.module_from_spec(aspec)
                aspec.loader.exec_module(anm)
                anm.make_parser().parse_args(argv[2:])
            elif argv[1] == "tools/native_coverage.py":
                cspec = importlib.util.spec_from_file_location("native_coverage", REPO / "tools" / "native_coverage.py")
                cvm = importlib.util.module_from_spec(cspec)
                cspec.loader.exec_module(cvm)
                cvm.make_parser().parse_args(argv[2:])
                assert all((REPO / t).exists() for t in cvm.TESTS), where
            elif argv[1] == "tools/fuzz_native.py":
                fspec = importlib.util.spec_from_file_location("fuzz_native", REPO / "tools" / "fuzz_native.py")
                fzm = importlib.util.module_from_spec(fspec)
                fspec.loader.exec_module(fzm)
                fzm.make_parser().parse_args(argv[2:])
            elif argv[1:3] == ["-m", "pytest"]:
                r = subprocess.run([sys.executable, "-m", "pytest", *argv[3:], "--collect-only", "-q",
                                    "-p", "no:cacheprovider"], cwd=REPO, capture_output=True, text=True, timeout=300)
                assert r.returncode == 0, f"{where}\n{r.stdout[-2000:]}{r.stderr[-2000:]}"
            else:
                raise AssertionError(f"unchecked workflow command: {where}")
        except SystemExit as e:   # argparse error
            raise AssertionError(f"argument error in {where}") from e
        checked += 1
    assert checked >= 7


def test_ci_check_catches_a_bad_flag():
    from rocm_k8s_device_plugin_amd import _build
    with pytest.raises(SystemExit):
        _build.make_parser().parse_args(["--no-hip", "--sanitize", "--ctest"])   # the round-1 CI bug


def test_build_stamp_follows_content_not_mtime(tmp_path, monkeypatch):
    """A copied tree (gpurun snapshot, image layer) gets new mtimes: that must not
    trigger a rebuild on a box without the build directory; an edit must."""
    import os
    from rocm_k8s_device_plugin_amd import _build
    src = tmp_path / "native"
    (src / "src").mkdir(parents=True)
    f = src / "src" / "a.cpp"
    f.write_text("int a;\n")
    out = tmp_path / "out.so"
    out.write_text("")
    monkeypatch.setattr(_build, "NATIVE_DIR", src)
    monkeypatch.setattr(_build, "STAMP", tmp_path / "stamp")
    assert not _build._up_to_date([out])
    _build.STAMP.write_text(f"hip=True\ndigest={_build._source_digest()}\n")
    assert _build._up_to_date([out])
    os.utime(f, (1e10, 1e10))                      # touched, same content
    assert _build._up_to_date([out])
    (src / "tools").mkdir()
    (src / "tools" / "adhoc_measurement.cpp").write_text("int m;\n")   # compiled on the box, not by CMake
    assert _build._up_to_date([out])
    f.write_text("int a = 1;\n")                   # edited
    assert not _build._up_to_date([out])
    assert not _build._up_to_date([tmp_path / "missing.so"])


def test_docs_tooling_matches_the_tree(tmp_path):
    """docs/conf.py runs without Sphinx installed, every _toc entry is a page,
    every page is in the _toc, and readthedocs/dependabot point at real paths."""
    import runpy
    conf = runpy.run_path(str(REPO / "docs" / "conf.py"))
    assert conf["project"] and conf["version"] == yaml.safe_load((REPO / "helm/amd-gpu/Chart.yaml").read_text())[
        "appVersion"]
    toc = yaml.safe_load((REPO / "docs/sphinx/_toc.yml.in").read_text())
    files = [toc["root"]] + [e["file"] for s in toc["subtrees"] for e in s["entries"]]
    for f in files:
        assert (REPO / "docs" / f"{f}.md").exists(), f
    pages = {p.stem for p in (REPO / "docs").glob("*.md")}
    assert pages == set(files), pages ^ set(files)
    rtd = yaml.safe_load((REPO / ".readthedocs.yaml").read_text())
    assert (REPO / rtd["sphinx"]["configuration"]).exists()
    assert all((REPO / r["requirements"]).exists() for r in rtd["python"]["install"])
    dep = yaml.safe_load((REPO / ".github/dependabot.yml").read_text())
    for u in dep["updates"]:
        assert (REPO / u["directory"].lstrip("/")).is_dir()


def test_alert_rules_use_exported_metrics():
    """example/monitoring/prometheusrule.yaml names only metrics the plugin exports."""
    import re
    rules = yaml.safe_load((REPO / "example/monitoring/prometheusrule.yaml").read_text())
    exprs = [r["expr"] for g in rules["spec"]["groups"] for r in g["rules"]]
    used = {m for e in exprs for m in re.findall(r"mi355x_dp_[a-z_]+", e)}
    src = "\n".join(p.read_text() for p in (REPO / "rocm_k8s_device_plugin_amd").rglob("*.py"))
    assert used and all(f'"{m}"' in src for m in used), sorted(m for m in used if f'"{m}"' not in src)


def test_helm_runs_the_native_binaries():
    """Every chart value runs on the native daemon / labeller: ./k8s-device-plugin
    and ./k8s-node-labeller, which the images link to the native binaries
    (tests/test_image_layout.py runs each rendered command from the image)."""
    t = (REPO / "helm/amd-gpu/templates/deviceplugin-daemonset.yaml").read_text()
    assert 'command: ["./k8s-device-plugin"]' in t and "$native" not in t and "else if" not in t
    for flag in ("-liveness=true", "-smi_ecc=true", "-smi_events=true", "-liveness_keep_queues", "-metrics_port",
                 "-device_list_strategy", "-cdi_spec_dir", "-smi_xgmi",
                 "-liveness_chip_sweep_every", "-perf_check_every", "-perf_action"):
        assert flag in t
    values = yaml.safe_load((REPO / "helm/amd-gpu/values.yaml").read_text())
    assert "native" not in values["dp"] and "native" not in values["lbl"]
    lt = (REPO / "helm/amd-gpu/templates/labeller.yaml").read_text()
    assert 'command: ["./k8s-node-labeller"]' in lt and "lbl.native" not in lt
    for df in ("Dockerfile", "ubi-dp.Dockerfile"):
        assert "ln -s /opt/mi355x/bin/mi355x-device-plugin /root/k8s-device-plugin" in (REPO / df).read_text(), df
    for df in ("labeller.Dockerfile", "ubi-labeller.Dockerfile"):
        assert "ln -s /opt/mi355x/bin/mi355x-node-labeller /root/k8s-node-labeller" in (REPO / df).read_text(), df


def test_launchers_run_the_native_binaries(tmp_path):
    """scripts/k8s-device-plugin and scripts/k8s-node-labeller (a source
    checkout's ./k8s-*) exec the native binaries; the labeller's labels equal
    the Python labeller's (the test oracle)."""
    import subprocess
    import sys
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    launcher = str(REPO / "scripts/k8s-device-plugin")
    p = subprocess.run([launcher, "-h"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and "mi355x-device-plugin version" in p.stdout and "-liveness_probe" in p.stdout
    fi = make_mi355x_node(tmp_path / "n")
    base = [launcher, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket", "",
            "-kubelet_dir", str(tmp_path / "dp")]
    p = subprocess.run(base, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and json.loads(p.stdout)["resources"], p.stderr[-2000:]
    assert "native daemon" in p.stderr
    p = subprocess.run(base + ["-grpc_server", "aio"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "flag provided but not defined: -grpc_server" in p.stderr   # Go's flag package
    lbl = str(REPO / "scripts/k8s-node-labeller")
    args = ["-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-vram", "-device-id"]
    nat = subprocess.run([lbl, "-node_name", "n", *args], capture_output=True, text=True, timeout=60)
    py = subprocess.run([sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.node_labeller", *args],
                        capture_output=True, text=True, timeout=120, cwd=str(REPO))
    assert nat.returncode == 0 and py.returncode == 0, (nat.stderr[-1000:], py.stderr[-1000:])
    assert json.loads(nat.stdout) == json.loads(py.stdout)
    h = subprocess.run([lbl, "-h"], capture_output=True, text=True, timeout=60)
    lines = h.stdout.splitlines()   # the native binary answered: its version banner, then the usage
    assert lines[0].startswith("AMD GPU Node Labeller") and "mi355x-node-labeller version " in lines[1]
    assert lines[3].startswith("usage: ")



def test_installed_console_scripts_run_the_native_daemons():
    """pyproject's console scripts point at cli/launch.py, which execs the native
    binaries: no installable command runs the Python oracle plugin or labeller."""
    import re
    import subprocess
    import sys
    text = (REPO / "pyproject.toml").read_text()
    scripts = dict(re.findall(r'^(k8s-[a-z-]+) = "([^"]+)"', text, re.M))
    assert scripts == {"k8s-device-plugin": "rocm_k8s_device_plugin_amd.cli.launch:device_plugin",
                       "k8s-node-labeller": "rocm_k8s_device_plugin_amd.cli.launch:node_labeller"}, scripts
    for name, target in scripts.items():
        mod, fn = target.split(":")
        # what the generated console script does: import the module, call the function
        code = f"import sys; sys.argv[0] = {name!r}; from {mod} import {fn}; sys.exit({fn}())"
        p = subprocess.run([sys.executable, "-c", code, "-h"], capture_output=True, text=True, timeout=60,
                           cwd=str(REPO))
        assert p.returncode == 0, p.stderr[-1000:]
        banner = "mi355x-device-plugin version" if name == "k8s-device-plugin" else "version"
        assert f"{name} version" in p.stdout or banner in p.stdout, p.stdout[:500]
        assert "native daemon" in p.stdout.splitlines()[0], p.stdout[:300]
