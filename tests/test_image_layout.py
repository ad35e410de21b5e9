"""Every deploy path runs from the image it names.

The reference builds the image its manifests and chart use (/root/reference/
Dockerfile:14-33 -> k8s-ds-amdgpu-dp.yaml, helm/amd-gpu/values.yaml:7-11).
Here, without a container runtime:

1. the image each manifest / rendered chart names must be one the Makefile
   builds (IMAGE_REPO:VERSION -> Dockerfile, :labeller-VERSION ->
   labeller.Dockerfile; VERSION = the chart's appVersion);
2. that Dockerfile's runtime stage (COPY / ln -s / WORKDIR / ENV / CMD) is
   replayed into a temporary root, with the build stage's outputs taken from
   this tree's in-tree build;
3. the container's command (or the image CMD) and args run from that root,
   in the working directory the pod spec or the image sets, with -dry_run
   against the synthetic MI355X node: the process must exit 0 and report the
   node's resources (device plugin) or labels (labeller). A flag the binary
   does not know, or a command the image does not have, fails here.

The chart is rendered by testing/helm_lite.py (no helm binary in this image)
for its default values and for every value that changes the command line.
"""
import glob
import json
import os
import re
import shlex
import shutil
import subprocess

import pytest
import yaml

from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.testing.helm_lite import rendered_objects

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHART = os.path.join(REPO, "helm", "amd-gpu")
MANIFESTS = ["k8s-ds-amdgpu-dp.yaml", "k8s-ds-amdgpu-dp-health.yaml", "k8s-ds-amdgpu-labeller.yaml"]


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=None)


# ------------------------------------------------------------------ Makefile: image -> Dockerfile
def image_map():
    mk = open(os.path.join(REPO, "Makefile")).read()
    repo = re.search(r"^IMAGE_REPO \?= (\S+)$", mk, re.M).group(1)
    version = yaml.safe_load(open(os.path.join(CHART, "Chart.yaml")))["appVersion"]
    out = {}
    for df, tag in re.findall(r"-f (\S+) -t \$\(IMAGE_REPO\):(\S+)", mk):
        out[f"{repo}:{tag.replace('$(VERSION)', version)}"] = df
    return out


# ------------------------------------------------------------------ Dockerfile runtime stage
def runtime_stage(dockerfile):
    text = open(os.path.join(REPO, dockerfile)).read().replace("\\\n", " ")
    lines = [l.strip() for l in text.splitlines() if l.strip() and not l.strip().startswith("#")]
    stages, cur = [], None
    for l in lines:
        op, _, rest = l.partition(" ")
        if op.upper() == "FROM":
            cur = []
            stages.append(cur)
        elif cur is not None:
            cur.append((op.upper(), rest.strip()))
    return stages[-1]


def replay(dockerfile, root):
    """The runtime stage's file system under `root`: {"workdir", "env", "cmd", "runs"}."""
    st = {"workdir": "/", "env": {}, "cmd": None, "runs": []}
    for op, rest in runtime_stage(dockerfile):
        if op == "WORKDIR":
            st["workdir"] = rest
            os.makedirs(root + rest, exist_ok=True)
        elif op == "COPY":
            args = shlex.split(rest)
            frm = None
            if args[0].startswith("--from="):
                frm, args = args[0][len("--from="):], args[1:]
            srcs, dst = args[:-1], args[-1]
            for src in srcs:
                if frm is not None:
                    if not src.startswith("/src/"):
                        continue         # system libraries of the build stage (the host has its own)
                    paths = glob.glob(os.path.join(REPO, src[len("/src/"):]))
                else:
                    paths = glob.glob(os.path.join(REPO, src))
                assert paths or frm is None or "*" in src, f"{dockerfile}: COPY {src}: nothing built there"
                for p in paths:
                    target = root + dst + (os.path.basename(p) if dst.endswith("/") else "")
                    os.makedirs(os.path.dirname(target), exist_ok=True)
                    if os.path.isdir(p):
                        shutil.copytree(p, target, symlinks=True, dirs_exist_ok=True)
                    else:
                        shutil.copy2(p, target)
        elif op == "RUN":
            st["runs"].append(rest)
            for part in rest.split("&&"):
                words = shlex.split(part)
                if words[:2] == ["ln", "-s"]:
                    target, link = words[2], words[3]
                    os.makedirs(os.path.dirname(root + link), exist_ok=True)
                    os.symlink(root + target, root + link)
        elif op == "ENV":
            for kv in shlex.split(rest):
                k, _, v = kv.partition("=")
                st["env"][k] = v
        elif op == "CMD":
            st["cmd"] = json.loads(rest)
    return st


# ------------------------------------------------------------------ running a container spec
def containers(objs):
    for o in objs:
        if o.get("kind") == "DaemonSet":
            for c in o["spec"]["template"]["spec"]["containers"]:
                yield o["metadata"]["name"], c


def container_argv(c, tmp_path):
    """Container spec `c` as it starts from its image's replayed root: (argv with the image's executable, cwd,
    env, image kind)."""
    images = image_map()
    assert c["image"] in images, f"{c['image']} is not an image this build makes ({sorted(images)})"
    df = images[c["image"]]
    root = str(tmp_path / "root")
    shutil.rmtree(root, ignore_errors=True)
    os.makedirs(root)
    st = replay(df, root)
    argv = list(c.get("command") or st["cmd"][:1]) + list(c.get("args") if "args" in c or "command" in c
                                                         else st["cmd"][1:])
    cwd = root + (c.get("workingDir") or st["workdir"])
    exe = argv[0] if argv[0].startswith("/") else os.path.normpath(os.path.join(cwd, argv[0]))
    if argv[0].startswith("/"):
        exe = root + argv[0]
    assert os.access(exe, os.X_OK), f"{df}: {argv[0]} does not exist in the image (from {cwd})"
    env = {k: v for k, v in os.environ.items() if not k.startswith("MI355X_")}
    env.update({k: (root + v if v.startswith("/opt/mi355x") else v) for k, v in st["env"].items()})
    return [exe] + argv[1:], cwd, env, "labeller" if "labeller" in df else "device-plugin"


def run_container(c, tmp_path, fi):
    """Run container spec `c` from its image's replayed root; (returncode, stdout, stderr, kind)."""
    argv, cwd, env, kind = container_argv(c, tmp_path)
    extra = (["-dry_run", "-node_name", "node-0", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)]
             if kind == "labeller" else
             ["-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-kubelet_dir", str(tmp_path / "dp"),
              "-exporter_socket", "", "-cdi_spec_dir", str(tmp_path / "cdi"), "-liveness_timeout", "5"])
    p = subprocess.run(argv + extra, cwd=cwd, env=env, capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout, p.stderr, kind


def check_ok(c, tmp_path, fi):
    rc, out, err, kind = run_container(c, tmp_path, fi)
    assert rc == 0, (c.get("command"), c.get("args"), err[-2000:])
    doc = json.loads(out)
    if kind == "labeller":
        assert doc and all(k.startswith(("amd.com/", "beta.amd.com/")) for k in doc), doc
    else:
        devs = [d for r in doc["resources"].values() for d in r["devices"]]
        assert doc["implementation"] == "container" and len(devs) == 8, doc
    return doc


@pytest.fixture(scope="module")
def node(tmp_path_factory):
    return make_mi355x_node(tmp_path_factory.mktemp("node"))


# ------------------------------------------------------------------ the tests
def test_every_image_named_is_built_here():
    images = image_map()
    assert set(images.values()) == {"Dockerfile", "labeller.Dockerfile", "ubi-dp.Dockerfile", "ubi-labeller.Dockerfile"}
    named = set()
    for m in MANIFESTS:
        named |= {c["image"] for _, c in containers(yaml.safe_load_all(open(os.path.join(REPO, m))))}
    named |= {c["image"] for _, c in containers(rendered_objects(CHART, {"labeller": {"enabled": True}}))}
    assert named and named <= set(images), named - set(images)
    assert not any("rocm/k8s-device-plugin" in i for i in named)      # never the upstream image


@pytest.mark.parametrize("df", ["Dockerfile", "labeller.Dockerfile", "ubi-dp.Dockerfile", "ubi-labeller.Dockerfile"])
def test_runtime_stage_has_no_interpreter(df, tmp_path):
    """The images run the native binaries only: no Python, grpcio or protobuf."""
    st = replay(df, str(tmp_path))
    runs = " ".join(st["runs"])
    assert not re.search(r"python|pip|grpcio|protobuf", runs), runs
    bins = os.listdir(tmp_path / "opt" / "mi355x" / "bin")
    want = {"mi355x-node-labeller"} if "labeller" in df else {"mi355x-device-plugin", "mi355x-liveness-probe"}
    assert set(bins) == want
    assert st["cmd"][0] == ("./k8s-node-labeller" if "labeller" in df else "./k8s-device-plugin")


@pytest.mark.parametrize("manifest", MANIFESTS)
def test_manifest_containers_run_from_their_image(manifest, tmp_path, node):
    cs = list(containers(yaml.safe_load_all(open(os.path.join(REPO, manifest)))))
    assert cs
    for _, c in cs:
        check_ok(c, tmp_path, node)


CHART_VALUES = {
    "defaults": {"labeller": {"enabled": True}},
    "health": {"dp": {"pulse": 2, "liveness": {"enabled": True, "chipSweepEvery": 3, "perfCheckEvery": 5,
                                                 "perfAction": "unhealthy"},
                      "smi": {"ecc": True, "events": True, "xgmi": True}}},
    "cdi-metrics": {"dp": {"cdi": {"enabled": True, "strategy": "device-specs,cdi-cri"}, "metricsPort": 9400}},
    "mixed-args": {"dp": {"args": ["-resource_naming_strategy=mixed", "-allocator_search=extended"]},
                   "labeller": {"enabled": True}, "lbl": {"args": ["-vram", "-compute-memory-partition"], "resync": 0}},
}


@pytest.mark.parametrize("name", sorted(CHART_VALUES))
def test_chart_containers_run_from_their_image(name, tmp_path, node):
    cs = list(containers(rendered_objects(CHART, CHART_VALUES[name])))
    assert len(cs) == (2 if CHART_VALUES[name].get("labeller", {}).get("enabled") else 1)
    for _, c in cs:
        doc = check_ok(c, tmp_path, node)
        if name == "cdi-metrics" and "resources" in doc:
            assert doc["device_list_strategy"] == ["device-specs", "cdi-cri"]
            assert (tmp_path / "cdi").is_dir() and os.listdir(tmp_path / "cdi")


def test_chart_probes_reach_the_running_binaries(tmp_path, node):
    """With dp.metricsPort / lbl.metricsPort, the rendered containers run from their images (not a dry run) and
    the paths and ports of the rendered liveness and readiness probes answer 200 once the daemon is registered
    with kubelet and the labeller has labelled its node: the probes point at what the binaries serve."""
    import asyncio
    import socket
    import time
    import urllib.error
    import urllib.request

    from rocm_k8s_device_plugin_amd.testing.fake_apiserver import FakeApiServer
    from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet

    def free_port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]

    def status(port, path):
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
                return r.status
        except urllib.error.HTTPError as e:
            return e.code
        except OSError:
            return 0

    def probes_ok(c):
        port = next(p["containerPort"] for p in c["ports"] if p["name"] == c["livenessProbe"]["httpGet"]["port"])
        paths = [c[k]["httpGet"]["path"] for k in ("livenessProbe", "readinessProbe")]
        deadline = time.monotonic() + 30
        while time.monotonic() < deadline:
            if all(status(port, path) == 200 for path in paths):
                return True
            time.sleep(0.1)
        return {path: status(port, path) for path in paths}

    cs = dict((kind, c) for kind, c in (
        ("labeller" if "labeller" in o["metadata"]["name"] else "dp", o["spec"]["template"]["spec"]["containers"][0])
        for o in rendered_objects(CHART, {"dp": {"metricsPort": free_port()}, "labeller": {"enabled": True},
                                          "lbl": {"metricsPort": free_port()}})
        if o.get("kind") == "DaemonSet"))
    # the device plugin: a kubelet to register with
    kdir = tmp_path / "dp"
    kdir.mkdir()
    argv, cwd, env, kind = container_argv(cs["dp"], tmp_path / "dp-image")
    assert kind == "device-plugin"

    async def dp():
        k = FakeKubelet(str(kdir))
        await k.start()
        p = subprocess.Popen(argv + ["-sysfs_root", str(node.sysfs), "-dev_root", str(node.dev), "-kubelet_dir",
                                     str(kdir), "-exporter_socket", ""], cwd=cwd, env=env,
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        try:
            await k.wait_for_resource("amd.com/gpu", 8, timeout=30)
            return await asyncio.to_thread(probes_ok, cs["dp"])
        finally:
            p.terminate()
            p.communicate(timeout=20)
            await k.stop()

    assert asyncio.run(asyncio.wait_for(dp(), 90)) is True
    # the labeller: an apiserver with its node
    srv = FakeApiServer(token="tok").start()
    tok = tmp_path / "token"
    tok.write_text("tok\n")
    argv, cwd, env, kind = container_argv(cs["labeller"], tmp_path / "lbl-image")
    assert kind == "labeller"
    p = None
    try:
        srv.add_node("node-0")
        p = subprocess.Popen(argv + ["-node_name", "node-0", "-apiserver", srv.url, "-token_file", str(tok),
                                     "-sysfs_root", str(node.sysfs), "-dev_root", str(node.dev)],
                             cwd=cwd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        assert probes_ok(cs["labeller"]) is True
        assert srv.labels("node-0")
    finally:
        if p is not None:
            p.terminate()
            p.communicate(timeout=20)
        srv.stop()


def test_a_wrong_flag_or_command_fails(tmp_path, node):
    c = dict(next(containers(yaml.safe_load_all(open(os.path.join(REPO, "k8s-ds-amdgpu-dp-health.yaml")))))[1])
    bad = dict(c, args=list(c["args"]) + ["-liveness_sweep_evry=3"])
    rc, _, err, _ = run_container(bad, tmp_path, node)
    assert rc == 2 and "flag provided but not defined: -liveness_sweep_evry" in err   # Go's flag package: exit 2
    with pytest.raises(AssertionError, match="does not exist in the image"):
        run_container(dict(c, command=["./k8s-device-plugin-py"]), tmp_path, node)
    with pytest.raises(AssertionError, match="is not an image this build makes"):
        run_container(dict(c, image="docker.io/rocm/k8s-device-plugin:1.31.0.2"), tmp_path, node)


# ------------------------------------------------------------------ shared libraries of the runtime stage
# sonames each runtime base image ships itself (its C/C++ runtime; zlib for the package manager)
BASE_LIBS = {
    "ubuntu:22.04": {"libc.so.6", "libm.so.6", "libdl.so.2", "libpthread.so.0", "librt.so.1",
                     "ld-linux-x86-64.so.2", "libgcc_s.so.1", "libstdc++.so.6", "libz.so.1"},
    "registry.access.redhat.com/ubi9/ubi-minimal:latest": {"libc.so.6", "libm.so.6", "libdl.so.2", "libpthread.so.0",
                                                           "librt.so.1", "ld-linux-x86-64.so.2", "libgcc_s.so.1",
                                                           "libz.so.1"},
}
# distro package -> sonames it installs (Ubuntu 22.04 / UBI 9 names)
PACKAGE_LIBS = {
    "libdrm2": {"libdrm.so.2"}, "libdrm-amdgpu1": {"libdrm_amdgpu.so.1"}, "libelf1": {"libelf.so.1"},
    "libnuma1": {"libnuma.so.1"}, "libssl3": {"libssl.so.3", "libcrypto.so.3"}, "libstdc++6": {"libstdc++.so.6"},
    "libdrm": {"libdrm.so.2", "libdrm_amdgpu.so.1"}, "elfutils-libelf": {"libelf.so.1"},
    "numactl-libs": {"libnuma.so.1"}, "zlib": {"libz.so.1"}, "libstdc++": {"libstdc++.so.6"},
    "openssl-libs": {"libssl.so.3", "libcrypto.so.3"},
}
# what copied third-party libraries dlopen() at run time, beyond their DT_NEEDED (from
# their strings; librocprofiler-register's names of other ROCm libraries are ones it looks
# for among those already loaded, not load targets)
THIRD_PARTY_DLOPEN = {"libamd_smi": {"libdrm_amdgpu.so.1"}}
_SONAME = re.compile(rb"(lib[A-Za-z0-9_+-]+\.so(?:\.[0-9]+)*)")


def _stem(soname):
    return soname.split(".so", 1)[0]


def _elf_needed(path):
    out = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    return set(re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out))


def stage_libraries(dockerfile, drop=None):
    """(provided sonames, required {(binary or library, soname or dlopen stem)}) of the runtime
    stage; `drop`: one COPY source to leave out (what removing that line would do)."""
    text = open(os.path.join(REPO, dockerfile)).read().replace("\\\n", " ")
    base = [l.split()[1] for l in text.splitlines() if l.strip().upper().startswith("FROM ")][-1]
    provided = set(BASE_LIBS[base])
    binaries, libs = [], []
    for op, rest in runtime_stage(dockerfile):
        if op == "RUN":
            for part in rest.split("&&"):
                w = shlex.split(part)
                if "install" in w and w[0] in ("apt-get", "microdnf", "dnf"):
                    for pkg in (x for x in w[w.index("install") + 1:] if not x.startswith("-")):
                        assert pkg in PACKAGE_LIBS, f"{dockerfile}: package {pkg} is not in PACKAGE_LIBS"
                        provided |= PACKAGE_LIBS[pkg]
        elif op == "COPY" and rest.startswith("--from="):
            for src in shlex.split(rest)[1:-1]:
                if src == drop:
                    continue
                if src.startswith("/src/"):
                    binaries += glob.glob(os.path.join(REPO, src[len("/src/"):]))
                else:                       # the build stage's ROCm libraries: this host's copy
                    found = glob.glob(src)
                    assert found, f"{dockerfile}: COPY {src}: no such library here"
                    provided |= {os.path.basename(p) for p in found}
                    libs += [p for p in found if not os.path.islink(p)]
    required = set()
    for b in binaries:
        required |= {(os.path.basename(b), s) for s in _elf_needed(b)}
        # our own dlopen() targets: any of a library's names will do (so.1, .so, /opt/rocm/lib/...)
        required |= {(os.path.basename(b), "dlopen:" + _stem(m.decode()))
                     for m in _SONAME.findall(open(b, "rb").read())}
    for lib in libs:
        name = os.path.basename(lib)
        required |= {(name, s) for s in _elf_needed(lib)}
        required |= {(name, "dlopen:" + _stem(s)) for s in THIRD_PARTY_DLOPEN.get(_stem(name), ())}
    return provided, required


def missing_libraries(dockerfile, drop=None):
    provided, required = stage_libraries(dockerfile, drop)
    stems = {_stem(s) for s in provided}
    return sorted((who, need) for who, need in required
                  if not (need[len("dlopen:"):] in stems if need.startswith("dlopen:") else need in provided))


@pytest.mark.parametrize("df", ["Dockerfile", "labeller.Dockerfile", "ubi-dp.Dockerfile", "ubi-labeller.Dockerfile"])
def test_runtime_stage_provides_every_library_its_binaries_load(df):
    """Every DT_NEEDED and dlopen() target of the copied binaries, and of the ROCm
    libraries copied for them, is in the stage: the base image, a package it
    installs or a library it copies (on the library path: LD_LIBRARY_PATH)."""
    assert missing_libraries(df) == []
    st = runtime_stage(df)
    copied_dirs = {shlex.split(rest)[-1].rstrip("/") for op, rest in st
                   if op == "COPY" and rest.startswith("--from=") and ".so" in rest}
    env = dict(kv.partition("=")[::2] for op, rest in st if op == "ENV" for kv in shlex.split(rest))
    assert copied_dirs <= set(env.get("LD_LIBRARY_PATH", "").split(":")), (copied_dirs, env)
    assert not re.search(r"^FROM\s+rocm/", open(os.path.join(REPO, df)).read().split(" AS build")[-1], re.M), \
        "the runtime stage is not a ROCm development image"


@pytest.mark.parametrize("df", ["Dockerfile", "labeller.Dockerfile", "ubi-dp.Dockerfile", "ubi-labeller.Dockerfile"])
def test_the_library_check_fails_without_any_one_copied_library(df):
    """Dropping any one library COPY source leaves something unresolved."""
    srcs = [s for op, rest in runtime_stage(df) if op == "COPY" and rest.startswith("--from=")
            for s in shlex.split(rest)[1:-1] if not s.startswith("/src/")]
    assert srcs
    for s in srcs:
        assert missing_libraries(df, drop=s), f"{df}: removing {s} went unnoticed"


# newest symbol versions the base image's C / C++ runtime provides (jammy: glibc 2.35,
# libstdc++6 from GCC 12); UBI images copy libraries built on EL9, not this host's
BASE_SYMBOL_VERSIONS = {"ubuntu:22.04": {"GLIBC": (2, 35), "GLIBCXX": (3, 4, 30)}}


@pytest.mark.parametrize("df", ["Dockerfile", "labeller.Dockerfile"])
def test_runtime_stage_c_runtime_is_new_enough(df):
    """Every copied binary and library links symbol versions the base image's
    glibc and libstdc++ have (a binary built against a newer runtime would fail
    to start on the slim base with 'version GLIBCXX_... not found')."""
    text = open(os.path.join(REPO, df)).read().replace("\\\n", " ")
    base = [l.split()[1] for l in text.splitlines() if l.strip().upper().startswith("FROM ")][-1]
    have = BASE_SYMBOL_VERSIONS[base]
    files = []
    for op, rest in runtime_stage(df):
        if op == "COPY" and rest.startswith("--from="):
            for src in shlex.split(rest)[1:-1]:
                files += glob.glob(os.path.join(REPO, src[len("/src/"):]) if src.startswith("/src/") else src)
    files = [f for f in files if not os.path.islink(f)]
    assert files
    for f in files:
        out = subprocess.run(["readelf", "-V", f], capture_output=True, text=True, check=True).stdout
        for lib, ver in re.findall(r"Name: (GLIBCXX|GLIBC)_([0-9.]+)", out):
            need = tuple(int(x) for x in ver.split("."))
            assert need <= have[lib], f"{df}: {os.path.basename(f)} needs {lib}_{ver}, {base} has {have[lib]}"
