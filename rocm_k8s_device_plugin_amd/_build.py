"""Build driver for the native core (CMake + Ninja, in-tree outputs).

Outputs land inside the package so they travel with the repo snapshot:

* ``_native*.so``                 host core (kfd/sysfs, allocator, PCI, drm, amd-smi)
* ``_hip*.so``                    in-process gfx950 liveness probe
* ``bin/mi355x-liveness-probe``   HSA-direct probe executable (health loop, bench "container")
* ``bin/mi355x-liveness-probe-hip`` the same probe through the HIP runtime
* ``kernels/liveness_gfx950.hsaco``

``ensure_built()`` is cheap when everything is up to date (one ninja no-op).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
NATIVE_DIR = REPO_DIR / "native"
BUILD_DIR = REPO_DIR / "build" / "native"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

NATIVE_SO = PKG_DIR / f"_native{EXT_SUFFIX}"
HIP_SO = PKG_DIR / f"_hip{EXT_SUFFIX}"
PROBE_EXE = PKG_DIR / "bin" / "mi355x-liveness-probe"
PROBE_EXE_HIP = PKG_DIR / "bin" / "mi355x-liveness-probe-hip"
MOUNTEMU_EXE = PKG_DIR / "bin" / "mi355x-probe-mountemu"
HIP_DEVEMU_EXE = PKG_DIR / "bin" / "mi355x-probe-hip-devemu"
HSACO = PKG_DIR / "kernels" / "liveness_gfx950.hsaco"


def hipcc_available() -> bool:
    return shutil.which("hipcc") is not None or Path("/opt/rocm/bin/hipcc").exists()


STAMP = REPO_DIR / "build" / ".native.stamp"
_checked: set = set()


# native/tools/ holds measurement programs compiled ad hoc on the GPU box; only
# these two are part of the CMake build (the container-entrypoint emulation)
_CMAKE_TOOLS = {"probe_emu.cpp", "path_interpose.h"}


def _source_digest() -> str:
    """Content hash of every native source the CMake build uses (paths + bytes)."""
    import hashlib
    h = hashlib.sha1()
    for p in sorted(NATIVE_DIR.rglob("*")):
        if p.parent.name == "tools" and p.parent.parent == NATIVE_DIR and p.name not in _CMAKE_TOOLS:
            continue
        if p.is_file() and p.suffix in {".cpp", ".h", ".hip", ".txt"}:
            h.update(str(p.relative_to(NATIVE_DIR)).encode())
            h.update(p.read_bytes())
    return h.hexdigest()


def _up_to_date(targets, hip: bool = False) -> bool:
    # Compare the sources' content hash with the one recorded after the last
    # successful build, not mtimes: a copy of the tree (the gpurun snapshot, a
    # container image layer) changes mtimes without changing what was built.
    # A host-only build (hip=False) stamps the same digest without building the
    # GPU targets: it does not count as up to date for a HIP build.
    if not all(t.exists() for t in targets):
        return False
    if not STAMP.exists():
        return False
    words = STAMP.read_text().split()
    if hip and "hip=True" not in words:
        return False
    return f"digest={_source_digest()}" in words


VERSION_FILE = PKG_DIR / "VERSION"


def stamp_version(digest: str | None = None) -> None:
    """<package>/VERSION: this tree's `git describe` next to the native
    sources' digest. The binaries' banner reads it when the digest is their
    own (native/src/util/versions.cpp), so a commit that changes no native
    source still names itself, without relinking binaries a running suite may
    be executing. Rewritten only when its content changes."""
    digest = (digest or _source_digest())[:12]
    describe = git_describe()
    if not describe:
        return
    text = f"describe={describe}\ndigest={digest}\n"
    try:
        if VERSION_FILE.exists() and VERSION_FILE.read_text() == text:
            return
        tmp = VERSION_FILE.with_suffix(".tmp")
        tmp.write_text(text)
        tmp.replace(VERSION_FILE)
    except OSError:
        pass


def git_describe() -> str:
    """The version the native binaries report: $GIT_DESCRIBE (image builds),
    else ``git describe --always --long --dirty`` of this tree (the reference's
    Dockerfile:21), else "" (no git metadata, e.g. a copied tree: keep what the
    last build stamped)."""
    env = os.environ.get("GIT_DESCRIBE", "").strip()
    if env:
        return env
    try:
        r = subprocess.run(["git", "-C", str(REPO_DIR), "describe", "--always", "--long", "--dirty"],
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, timeout=10)
    except (OSError, subprocess.TimeoutExpired):
        return ""
    return r.stdout.strip() if r.returncode == 0 else ""


def variant_dir(sanitize: str = "", coverage: bool = False) -> Path:
    """The build tree of a variant: the package build, a sanitizer build or the gcov build."""
    if coverage:
        return REPO_DIR / "build" / "native-coverage"
    return BUILD_DIR if not sanitize else REPO_DIR / "build" / f"native-{sanitize.replace(',', '-')}"


def build(hip: bool | None = None, sanitize: str = "", build_dir: Path | None = None,
          jobs: int | None = None, quiet: bool = True, coverage: bool = False) -> None:
    """Configure + build. ``hip=None`` builds the HIP probe when hipcc exists.
    ``sanitize`` / ``coverage``: a host-only variant in its own tree, with its
    binaries under ``<tree>/pkg`` (the package outputs stay untouched)."""
    import fcntl
    if hip is None:
        hip = hipcc_available()
    bdir = build_dir or variant_dir(sanitize, coverage)
    bdir.mkdir(parents=True, exist_ok=True)
    # one build per tree at a time, across processes (pytest workers, ranks)
    with open(bdir.parent / f".{bdir.name}.build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            _build_tree(bdir, hip, sanitize, coverage, build_dir, jobs, quiet)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_tree(bdir: Path, hip: bool, sanitize: str, coverage: bool, build_dir, jobs, quiet: bool) -> None:
    variant = bool(sanitize) or coverage
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    cfg = [
        "cmake", "-S", str(NATIVE_DIR), "-B", str(bdir), *gen,
        f"-DPython3_EXECUTABLE={sys.executable}",
        f"-DMI355X_BUILD_HIP={'ON' if hip else 'OFF'}",
        f"-DMI355X_SANITIZE={sanitize}",
        f"-DMI355X_COVERAGE={'ON' if coverage else 'OFF'}",
        "-DCMAKE_BUILD_TYPE=Release",
    ]
    describe = git_describe()
    if describe:
        cfg.append(f"-DMI355X_GIT_DESCRIBE={describe}")
    digest12 = _source_digest()[:12]
    cfg.append(f"-DMI355X_SOURCE_DIGEST={digest12}")
    if variant:
        # sanitizer / coverage builds keep the package outputs untouched
        cfg.append(f"-DMI355X_PKG_DIR={bdir / 'pkg'}")
    out = subprocess.DEVNULL if quiet else None
    if not (bdir / "CMakeCache.txt").exists() or variant:
        subprocess.run(cfg, check=True, stdout=out)
    else:
        # re-run configure only if the HIP option flipped, or for a new version
        # stamp when something is rebuilt anyway (sources changed since the last
        # build) or one is given explicitly ($GIT_DESCRIBE): a commit alone must
        # not relink the binaries under a running test suite
        cache = (bdir / "CMakeCache.txt").read_text()
        want = f"MI355X_BUILD_HIP:BOOL={'ON' if hip else 'OFF'}"
        restamp = bool(describe) and f"MI355X_GIT_DESCRIBE:STRING={describe}\n" not in cache and (
            bool(os.environ.get("GIT_DESCRIBE")) or not STAMP.exists()
            or f"digest={_source_digest()}" not in STAMP.read_text().split())
        # the digest changes only with the sources, when the binaries are rebuilt anyway
        stale_digest = f"MI355X_SOURCE_DIGEST:STRING={digest12}\n" not in cache
        if want not in cache or restamp or stale_digest:
            subprocess.run(cfg, check=True, stdout=out)
    j = jobs or min(8, os.cpu_count() or 4)
    res = subprocess.run(["cmake", "--build", str(bdir), "-j", str(j)], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout)
        raise RuntimeError("native build failed")
    if not variant and build_dir is None:
        STAMP.parent.mkdir(parents=True, exist_ok=True)
        STAMP.write_text(f"hip={hip}\ndigest={_source_digest()}\n")
        stamp_version()
    if not quiet:
        sys.stdout.write(res.stdout)


def ensure_built(hip: bool | None = None) -> None:
    """Build if any output is missing or older than the native sources.

    Serialised across processes with a lock file, so ranks or pytest workers
    that start together do not run two builds into the same tree.
    """
    import fcntl

    if hip is None:
        hip = hipcc_available()
    if hip in _checked:
        return
    targets = [NATIVE_SO] + ([HIP_SO, PROBE_EXE, PROBE_EXE_HIP, MOUNTEMU_EXE, HIP_DEVEMU_EXE, HSACO] if hip else [])
    if not _up_to_date(targets, hip):
        BUILD_DIR.mkdir(parents=True, exist_ok=True)
        with open(BUILD_DIR.parent / ".build.lock", "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                if not _up_to_date(targets, hip):
                    try:
                        build(hip=hip)
                    except (RuntimeError, OSError, subprocess.CalledProcessError) as e:
                        # a tree shipped with its outputs (e.g. to a GPU box without
                        # the build directory) keeps working on what was built; the
                        # warning names the sources that no longer match them
                        if not all(t.exists() for t in targets):
                            raise
                        import warnings
                        warnings.warn(f"native sources changed since the last build and the rebuild failed "
                                      f"({e}); using the existing build outputs")
            finally:
                fcntl.flock(lk, fcntl.LOCK_UN)
    elif STAMP.exists():
        stamp_version()  # HEAD may have moved since the build
    _checked.add(hip)


def run_ctest(sanitize: str = "", coverage: bool = False) -> subprocess.CompletedProcess:
    bdir = variant_dir(sanitize, coverage)
    build(hip=False if (sanitize or coverage) else None, sanitize=sanitize, coverage=coverage)
    env = dict(os.environ)
    if "thread" in sanitize:
        env.setdefault("TSAN_OPTIONS", "halt_on_error=1")
    return subprocess.run(["ctest", "--test-dir", str(bdir), "--output-on-failure"],
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)


def make_parser():
    import argparse
    ap = argparse.ArgumentParser(prog="python -m rocm_k8s_device_plugin_amd._build",
                                 description="build the native core")
    ap.add_argument("--no-hip", action="store_true")
    ap.add_argument("--sanitize", default="",
                    help="comma-separated -fsanitize= list for a ctest-only build, e.g. address,undefined or thread")
    ap.add_argument("--ctest", action="store_true")
    return ap


def main(argv=None) -> int:
    a = make_parser().parse_args(argv)
    if a.ctest:
        r = run_ctest(a.sanitize)
        print(r.stdout)
        return r.returncode
    build(hip=False if a.no_hip else None, sanitize=a.sanitize, quiet=False)
    return 0


if __name__ == "__main__":
    sys.exit(main())
