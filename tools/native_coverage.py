#!/usr/bin/env python3
"""Line coverage of the native host code by the CPU test suite (gcov).

Builds the gcov variant of the native tree (``build/native-coverage``, host
code only, ``-O0 --coverage``), runs the C++ unit tests (ctest) and the test
files that drive the two native binaries with ``MI355X_NATIVE_DAEMON_EXE`` /
``MI355X_NATIVE_LABELLER_EXE`` pointing at the instrumented builds, then asks
gcov for every source's executed lines. Prints a per-file / per-directory
table and writes the JSON summary (``--json-out``).

The suite's in-process extension is the instrumented one too
(``MI355X_NATIVE_CORE_SO``), so the Python tests that drive the native engine,
allocator and parsers through the bindings count. GPU-only paths (the HSA /
HIP probes, amd-smi and libdrm queries) do not run on the CPU.

    python tools/native_coverage.py --json-out profiles/r4/native_coverage_cpu.json
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

# the test files whose native processes honour MI355X_NATIVE_{DAEMON,LABELLER}_EXE
# (and the files that import their EXE); the default run is the whole CPU suite
TESTS = ["tests/test_native_daemon.py", "tests/test_native_health.py", "tests/test_native_labeller.py",
         "tests/test_native_config_logging.py", "tests/test_native_stress.py", "tests/test_go_interop.py",
         "tests/test_native_cdi.py", "tests/test_native_reload.py", "tests/test_native_views.py",
         "tests/test_native_metrics.py", "tests/test_native_dryrun.py", "tests/test_native_perf.py",
         "tests/test_native_fabric.py", "tests/test_prestart_gate.py", "tests/test_kfd_denied.py",
         "tests/test_provenance.py"]

_LINES = re.compile(r"Lines executed:\s*([\d.]+)% of (\d+)")


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--json-out", default="", help="write the summary here")
    ap.add_argument("--workers", type=int, default=0,
                    help="pytest-xdist workers (default serial: the -O0 build is slow and the stress tests are throughput-bound)")
    ap.add_argument("--tests", nargs="*", default=["tests/"],
                    help="what pytest runs against the instrumented builds (default: the whole CPU suite)")
    ap.add_argument("--native-only", action="store_true", help="only the test files that drive the two binaries")
    ap.add_argument("--no-build", action="store_true", help="reuse the existing coverage build")
    ap.add_argument("--merge", default="",
                    help="a GCOV_PREFIX tree from a GPU-box run of the same build (GCOV_PREFIX_STRIP=3: "
                         "<dir>/native-coverage/...), merged into this run's counts before the report")
    ap.add_argument("--stage", default="",
                    help="copy the instrumented _native, daemon and labeller here for a GPU-box run, then exit")
    return ap


def gcov_file(gcda: Path) -> tuple[str, int, int] | None:
    """(source path relative to the repo, lines executed, executable lines) of one object's .gcda."""
    r = subprocess.run(["gcov", "-n", "-o", str(gcda.parent), str(gcda)], capture_output=True, text=True,
                       cwd=str(gcda.parent))
    cur = None
    for line in r.stdout.splitlines():
        if line.startswith("File '"):
            cur = line[6:-1]
        m = _LINES.search(line)
        if m and cur:
            path = Path(cur)
            if not path.is_absolute():
                path = (gcda.parent / path).resolve()
            try:
                rel = path.resolve().relative_to(REPO)
            except ValueError:
                cur = None
                continue
            if str(rel).startswith("native/src/") and rel.name == gcda.name.replace(".gcda", ""):
                total = int(m.group(2))
                return str(rel), round(float(m.group(1)) * total / 100.0), total
            cur = None
    return None


def main(argv=None) -> int:
    a = make_parser().parse_args(argv)
    from rocm_k8s_device_plugin_amd import _build
    bdir = _build.variant_dir(coverage=True)
    if not a.no_build:
        _build.build(hip=False, coverage=True)
    if a.stage:
        import shutil
        dst = Path(a.stage)
        dst.mkdir(parents=True, exist_ok=True)
        for f in [*(bdir / "pkg").glob("_native*.so"), bdir / "pkg" / "bin" / "mi355x-device-plugin",
                  bdir / "pkg" / "bin" / "mi355x-node-labeller"]:
            shutil.copy2(f, dst / f.name)
        print(f"staged in {dst}; on the box: MI355X_NATIVE_CORE_SO / MI355X_NATIVE_DAEMON_EXE / "
              f"MI355X_NATIVE_LABELLER_EXE pointing there, GCOV_PREFIX=<dir> GCOV_PREFIX_STRIP=3")
        return 0
    for g in bdir.rglob("*.gcda"):
        g.unlink()
    if a.no_build:  # the build as it is: a rebuild would restamp versions.cpp and orphan a box run's counts
        ct = subprocess.run(["ctest", "--test-dir", str(bdir), "--output-on-failure"], stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True)
    else:
        ct = _build.run_ctest(coverage=True)
    if ct.returncode != 0:
        sys.stderr.write(ct.stdout[-3000:])
        return 1
    so = next((bdir / "pkg").glob("_native*.so"), None)
    env = dict(os.environ, MI355X_NATIVE_DAEMON_EXE=str(bdir / "pkg" / "bin" / "mi355x-device-plugin"),
               MI355X_NATIVE_LABELLER_EXE=str(bdir / "pkg" / "bin" / "mi355x-node-labeller"))
    if so is not None:
        env["MI355X_NATIVE_CORE_SO"] = str(so)   # the suite's in-process native core, instrumented too
    tests = TESTS if a.native_only else a.tests
    cmd = [sys.executable, "-m", "pytest", *tests, "-q", "-m", "not gpu", "-p", "no:cacheprovider"]
    if a.workers > 0:
        cmd += ["-n", str(a.workers)]
    t = subprocess.run(cmd, cwd=str(REPO), env=env, capture_output=True, text=True)
    tail = (t.stdout.strip().splitlines() or [""])[-1]
    print(f"pytest: {tail}")
    for line in t.stdout.splitlines():
        if line.startswith(("FAILED", "ERROR")):
            print(line)
    if a.merge:
        # counts from the GPU box (same build, relocated by GCOV_PREFIX) added to this run's
        import shutil
        import tempfile
        box = Path(a.merge) / bdir.name
        with tempfile.TemporaryDirectory() as out:
            r = subprocess.run(["gcov-tool", "merge", "-o", out, str(box), str(bdir)], capture_output=True, text=True)
            if r.returncode != 0:
                sys.stderr.write(r.stderr[-2000:])
                return 1
            for g in Path(out).rglob("*.gcda"):
                shutil.copy2(g, bdir / g.relative_to(out))
        print(f"merged {sum(1 for _ in box.rglob('*.gcda'))} profiles from {box}")
    files = {}
    for gcda in sorted(bdir.rglob("*.gcda")):
        got = gcov_file(gcda)
        if not got:
            continue
        rel, hit, total = got
        h0, t0 = files.get(rel, (0, 0))
        # a source built into two targets reports its lines twice: keep the better-covered object
        files[rel] = max((h0, t0), (hit, total), key=lambda x: (x[0], -x[1]))
    by_dir: dict[str, list[int]] = {}
    for rel, (hit, total) in files.items():
        d = str(Path(rel).parent)
        s = by_dir.setdefault(d, [0, 0])
        s[0] += hit
        s[1] += total
    hit_all = sum(h for h, _ in files.values())
    tot_all = sum(t for _, t in files.values())
    for rel, (hit, total) in sorted(files.items()):
        print(f"{100.0 * hit / total if total else 0:6.1f}%  {hit:5d}/{total:<5d}  {rel}")
    print(f"{100.0 * hit_all / tot_all if tot_all else 0:6.1f}%  {hit_all:5d}/{tot_all:<5d}  total")
    if a.json_out:
        doc = {"what": "gcov line coverage of the native host code: ctest (test_core) plus the CPU tests, with the "
                       "instrumented mi355x-device-plugin, mi355x-node-labeller and _native extension "
                       "(tools/native_coverage.py)",
               "tests": tests, "pytest": tail, "ctest_ok": ct.returncode == 0,
               "merged_gpu_run": a.merge or None,
               "total": {"lines": tot_all, "executed": hit_all,
                         "pct": round(100.0 * hit_all / tot_all, 1) if tot_all else None},
               "by_dir": {d: {"lines": s[1], "executed": s[0], "pct": round(100.0 * s[0] / s[1], 1) if s[1] else None}
                          for d, s in sorted(by_dir.items())},
               "files": {rel: {"lines": t_, "executed": h, "pct": round(100.0 * h / t_, 1) if t_ else None}
                         for rel, (h, t_) in sorted(files.items())}}
        Path(a.json_out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.json_out).write_text(json.dumps(doc, indent=1) + "\n")
    return 0 if t.returncode == 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
