#!/usr/bin/env python3
"""clang static analyzer over every native source (native/src, native/fuzz).

Runs ``clang++ --analyze`` with the default checkers on each translation unit
and fails on any warning not in the reviewed list below. CPU only.

    python tools/analyze_native.py            # prints findings, exit 1 if any is new
"""
from __future__ import annotations

import argparse
import re
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
NATIVE = REPO / "native"
CLANG = Path("/opt/rocm/lib/llvm/bin/clang++")

# reviewed false positives: (file, checker) -> why
REVIEWED = {
    ("native/src/topology/sysfs.cpp", "unix.Stream"):
        "read_file's fread loop: the analyzer models the read after EOF; fread at EOF returns 0 and ends the loop",
    ("native/src/health/probe_main.cpp", "unix.BlockInCriticalSection"):
        "serve_worker: the checker counts one std::unique_lock acquisition as three nested critical sections "
        "(unique_lock::lock, mutex::lock, __gthread_mutex_lock) and the scope's unlock as one, so answer() "
        "after the scoped lock looks locked; the worker holds no lock while it answers",
}

_WARN = re.compile(r"^(?P<file>[^:]+):(?P<line>\d+):\d+: warning: (?P<msg>.*) \[(?P<checker>[\w.]+)\]$")


def clang() -> str | None:
    return str(CLANG) if CLANG.exists() else shutil.which("clang++")


def sources() -> list[Path]:
    return sorted(p for d in (NATIVE / "src", NATIVE / "fuzz") for p in d.rglob("*.cpp"))


HSACO = REPO / "rocm_k8s_device_plugin_amd" / "kernels" / "liveness_gfx950.hsaco"


def analyze(cc: str, src: Path) -> list[dict]:
    extra = []
    if src.name == "hsa_probe.cpp":  # embeds the built code object (.incbin); the build passes its path
        if not HSACO.exists():
            return []
        extra = [f'-DMI355X_HSACO_PATH="{HSACO}"', f"-I{NATIVE / 'src' / 'health'}"]
    p = subprocess.run([cc, "--analyze", "-Xanalyzer", "-analyzer-output=text", "-std=c++17",
                        f"-I{NATIVE / 'include'}", f"-I{NATIVE / 'src'}", "-isystem", "/opt/rocm/include", *extra,
                        str(src), "-o", "/dev/null"], capture_output=True, text=True, timeout=600)
    out = []
    for line in p.stderr.splitlines():
        m = _WARN.match(line.strip())
        if m:
            f = str(Path(m["file"]).resolve().relative_to(REPO)) if m["file"].startswith("/") else m["file"]
            out.append({"file": f, "line": int(m["line"]), "checker": m["checker"], "msg": m["msg"]})
    if p.returncode != 0 and not out:
        out.append({"file": str(src.relative_to(REPO)), "line": 0, "checker": "compile", "msg": p.stderr[-500:]})
    return out


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--jobs", type=int, default=6)
    return ap


def main(argv=None) -> int:
    a = make_parser().parse_args(argv)
    cc = clang()
    if not cc:
        print("clang++ not available", file=sys.stderr)
        return 2
    srcs = sources()
    with ThreadPoolExecutor(max_workers=max(1, a.jobs)) as ex:
        found = [w for ws in ex.map(lambda s: analyze(cc, s), srcs) for w in ws]
    uniq = {(w["file"], w["line"], w["checker"]): w for w in found}
    new = [w for w in uniq.values() if (w["file"], w["checker"]) not in REVIEWED]
    for w in sorted(uniq.values(), key=lambda w: (w["file"], w["line"])):
        tag = "reviewed" if (w["file"], w["checker"]) in REVIEWED else "NEW"
        print(f"{tag}: {w['file']}:{w['line']}: {w['msg']} [{w['checker']}]")
    print(f"{len(srcs)} translation units, {len(uniq)} findings, {len(new)} new")
    return 1 if new else 0


if __name__ == "__main__":
    sys.exit(main())
