#!/usr/bin/env python3
"""Coverage-guided fuzzing of the native daemons' input parsers (native/fuzz/).

Builds the libFuzzer targets with clang twice: the core instrumented for
coverage with ASan (fuzzing), and with ASan + UBSan (replaying every input the
fuzzing kept). Generates the MI355X sysfs fixture trees and a seed
corpus per target from the repo's own encoders (the grpc-go frame and HPACK
emulation in testing/gopeer.py, the kubelet protobuf messages, fixture Nodes
and kubeconfigs), runs every target for a time budget and writes a JSON
summary (executions, coverage, corpus, findings).

    python tools/fuzz_native.py --seconds 600 --json profiles/archive/r3/fuzz_native.json
    python tools/fuzz_native.py --targets h2_server,dp_rpc --seconds 60

A finding leaves its reproducer in <work>/artifacts/<target>/; re-run it with
``build/native-fuzz/fuzz_<target> <file>``. CPU only: nothing here touches a GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Dict, List, Optional

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
NATIVE = REPO / "native"
BUILD = REPO / "build" / "native-fuzz"            # coverage + ASan
BUILD_REPLAY = REPO / "build" / "native-fuzz-replay"  # ASan + full UBSan, runs the corpus once
BUILD_TSAN = REPO / "build" / "native-fuzz-tsan"      # TSan, runs the corpus of the threaded targets once
TARGETS = ("hpack", "json", "yaml", "sysfs", "labels", "exporter", "h2_server", "h2_client", "dp_rpc",
           "http_client")
# targets whose code under test runs on more than one thread (the server's I/O thread, the HTTP peer thread)
TSAN_TARGETS = ("h2_server", "dp_rpc", "h2_client", "http_client")
CLANG = Path("/opt/rocm/lib/llvm/bin/clang++")


def clang() -> Optional[str]:
    if CLANG.exists():
        return str(CLANG)
    return shutil.which("clang++")


def available() -> bool:
    """clang with the libFuzzer runtime, cmake, OpenSSL headers."""
    cc = clang()
    if not cc or not shutil.which("cmake"):
        return False
    with tempfile.TemporaryDirectory() as d:
        src = Path(d) / "t.cpp"
        src.write_text('#include <cstdint>\n#include <cstddef>\n'
                       'extern "C" int LLVMFuzzerTestOneInput(const uint8_t*, size_t) { return 0; }\n')
        r = subprocess.run([cc, "-fsanitize=fuzzer,address", str(src), "-o", str(Path(d) / "t")],
                           capture_output=True)
        return r.returncode == 0


def build(jobs: int = 8) -> None:
    """Configure and build the three fuzz trees; serialised across processes (pytest
    workers that start together must not run two builds into one tree)."""
    import fcntl
    BUILD.parent.mkdir(parents=True, exist_ok=True)
    with open(BUILD.parent / ".fuzz-build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            _build_locked(jobs)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(jobs: int) -> None:
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    for mode, bdir in (("fuzz", BUILD), ("replay", BUILD_REPLAY), ("tsan", BUILD_TSAN)):
        bdir.mkdir(parents=True, exist_ok=True)
        cache = bdir / "CMakeCache.txt"
        if not cache.exists() or f"MI355X_FUZZ:STRING={mode}" not in cache.read_text():
            subprocess.run(["cmake", "-S", str(NATIVE), "-B", str(bdir), *gen, f"-DCMAKE_CXX_COMPILER={clang()}",
                            f"-DMI355X_FUZZ={mode}", "-DMI355X_BUILD_HIP=OFF",
                            f"-DPython3_EXECUTABLE={sys.executable}"], check=True, stdout=subprocess.DEVNULL)
        only = [x for t in TSAN_TARGETS for x in ("--target", f"fuzz_{t}")] if mode == "tsan" else []
        r = subprocess.run(["cmake", "--build", str(bdir), "-j", str(jobs), *only], capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout[-6000:] + r.stderr[-3000:])
            raise RuntimeError(f"fuzz build ({mode}) failed")


# ---------------------------------------------------------------------- seeds
def _h2_request_session(path: str, body: bytes) -> bytes:
    """A grpc-go client's connection after the preface: SETTINGS, connection
    WINDOW_UPDATE, HEADERS (x/net HPACK), DATA, a BDP ping."""
    from rocm_k8s_device_plugin_amd.testing import gopeer as g
    enc = g.GoHpackEncoder()
    fields = [(":method", "POST"), (":scheme", "http"), (":path", path), (":authority", "localhost"),
              ("content-type", "application/grpc"), ("user-agent", g.GRPC_GO_USER_AGENT), ("te", "trailers"),
              ("grpc-timeout", g.encode_duration(10.0))]
    out = g.frame(4, 0, 0, g.settings_payload([(2, 0), (4, 4 << 20), (6, 16 << 20)]))
    out += g.frame(8, 0, 0, (1 << 20).to_bytes(4, "big"))
    out += g.frame(1, 4, 1, enc.encode(fields))
    out += g.frame(0, 1, 1, g.grpc_message(body))
    out += g.frame(6, 0, 0, g.BDP_PING)
    return out


def _h2_response(body: bytes, split: bool = False) -> bytes:
    """A grpc-go server's side of one unary call: SETTINGS, SETTINGS ACK,
    response HEADERS (optionally split by CONTINUATION), DATA, trailers."""
    from rocm_k8s_device_plugin_amd.testing import gopeer as g
    enc = g.GoHpackEncoder()
    head = enc.encode([(":status", "200"), ("content-type", "application/grpc")])
    out = g.frame(4, 0, 0, g.settings_payload([(5, 16384), (6, 16 << 20)])) + g.frame(4, 1, 0)
    if split and len(head) > 1:
        out += g.frame(1, 0, 1, head[:1]) + g.frame(9, 4, 1, head[1:])
    else:
        out += g.frame(1, 4, 1, head)
    out += g.frame(0, 0, 1, g.grpc_message(body))
    out += g.frame(1, 5, 1, enc.encode([("grpc-status", "0"), ("grpc-message", "")]))
    return out


def make_fixtures(work: Path) -> Dict[str, str]:
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    cpx = make_mi355x_node(work / "cpx", compute_partition="cpx")
    dpx = make_mi355x_node(work / "dpx", compute_partition="dpx")
    return {"MI355X_FUZZ_SYSFS": str(cpx.sysfs), "MI355X_FUZZ_SYSFS_MUT": str(dpx.sysfs)}


def make_seeds(work: Path, env: Dict[str, str]) -> Dict[str, Path]:
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    from rocm_k8s_device_plugin_amd.testing import gopeer as g
    from rocm_k8s_device_plugin_amd.topology import discover
    ids = [d.id for d in discover(env["MI355X_FUZZ_SYSFS"]).devices]
    seeds: Dict[str, List[bytes]] = {t: [] for t in TARGETS}

    enc = g.GoHpackEncoder()
    req = [(":method", "POST"), (":scheme", "http"), (":path", "/v1beta1.DevicePlugin/Allocate"),
           (":authority", "localhost"), ("content-type", "application/grpc"), ("te", "trailers")]
    seeds["hpack"] += [enc.encode(req), enc.encode(req) + b"\xff\x00" + enc.encode(req),
                       g.huffman_encode(b"application/grpc"), bytes([0x3f, 0xe1, 0x1f]) + enc.encode(req)]

    node = {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": "n", "resourceVersion": "7", "labels": {"amd.com/gpu.family": "AI", "k": "é"},
                         "annotations": {"a": "line\nbreak \"q\" \\"}},
            "status": {"capacity": {"amd.com/gpu": "8", "cpu": "256"}, "allocatable": {"memory": 1.5e12}}}
    seeds["json"] += [json.dumps(node).encode(), json.dumps({"type": "MODIFIED", "object": node}).encode(),
                      b'[1, -2.5e-3, true, null, "\\ud83d\\ude00", {}]']
    kubeconfig = (b"apiVersion: v1\nkind: Config\ncurrent-context: c\nclusters:\n- name: k\n  cluster:\n"
                  b"    server: https://10.0.0.1:6443\n    certificate-authority-data: QUJD\ncontexts:\n"
                  b"- name: c\n  context: {cluster: k, user: u}\nusers:\n- name: u\n  user:\n"
                  b"    token: \"abc\"  # inline comment\n    tokenFile: ./t\n")
    config = (b"# plugin config\npulse: 10\nliveness: true\nresource_naming_strategy: mixed\n"
              b"allocator_search: auto\nexporter_socket: ''\nmessage: |\n  literal\n  block\nfolded: >\n"
              b"  a\n  b\nlist: [1, 2, \"three\"]\nnested:\n  - a: 1\n    b: [x, y]\n")
    anchors = (b"base: &b {x: p, y: q}\nl: &l\n- a\n- *b\nd:\n  <<: [*b, {z: r}]\n  y: s\n"
               b"e: !!str &t |\n  text\nf: [&q k, *q, {&k2 m: *t}]\n&key g: *l\n")
    seeds["yaml"] += [kubeconfig, config, json.dumps(node).encode(), anchors]

    seeds["sysfs"] += [b"", bytes([0, 0, 5, 0]) + b"bad\n\n", bytes([7, 0, 0xFF, 0xFF]),
                       bytes([40, 0, 12, 0]) + b"node_to 999\n"]
    from rocm_k8s_device_plugin_amd.proto import metricssvc as ms
    states = ms.GPUStateResponse()
    for i, bdf in enumerate(sorted({d.id[:12] for d in discover(env["MI355X_FUZZ_SYSFS"]).devices})):
        states.GPUState.add(ID=str(i), UUID=f"u{i}", Health="healthy" if i % 3 else "Unhealthy", Device=bdf,
                            AssociatedWorkload=["pod-a"])
    seeds["exporter"] += [states.SerializeToString(), b"", b"\x0a\x02\x2a\x00"]
    seeds["labels"] += seeds["sysfs"] + [bytes([0x60, 0, 20, 0]) + b"AMD Instinct (x) /?\n"]

    gpa = pb.PreferredAllocationRequest(container_requests=[pb.ContainerPreferredAllocationRequest(
        available_deviceIDs=ids[:16], must_include_deviceIDs=ids[:1], allocation_size=4)]).SerializeToString()
    gpa_all = pb.PreferredAllocationRequest(container_requests=[pb.ContainerPreferredAllocationRequest(
        available_deviceIDs=ids, allocation_size=24)]).SerializeToString()
    alloc = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=ids[:3]),
                                                   pb.ContainerAllocateRequest(devices_ids=[])]).SerializeToString()
    seeds["dp_rpc"] += [b"\x00" + gpa, b"\x00" + gpa_all, b"\x01" + alloc, b"\x02", b"\x03", b"\x04"]

    seeds["h2_server"] += [_h2_request_session("/v1beta1.DevicePlugin/GetPreferredAllocation", gpa),
                           _h2_request_session("/v1beta1.DevicePlugin/Allocate", alloc),
                           _h2_request_session("/v1beta1.DevicePlugin/ListAndWatch", b"")
                           + g.frame(3, 0, 1, (8).to_bytes(4, "big"))]

    reg_ok = b""
    seeds["h2_client"] += [_h2_response(reg_ok), _h2_response(b"\x0a\x02ok", split=True),
                           g.frame(4, 0, 0) + g.frame(7, 0, 0, (0).to_bytes(4, "big") + (11).to_bytes(4, "big")
                                                      + b"too_many_pings")]

    ev = json.dumps({"type": "ADDED", "object": node}).encode() + b"\n"
    chunked = b"".join(b"%x\r\n%s\r\n" % (len(x), x) for x in (ev[:20], ev[20:], ev)) + b"0\r\n\r\n"
    seeds["http_client"] += [b"\x00HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\n{}",
                             b"\x01HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + chunked,
                             b"\x01HTTP/1.1 410 Gone\r\nContent-Type: application/json\r\n\r\n{\"kind\":\"Status\"}",
                             b"\x00HTTP/1.1 200 OK\r\n\r\n" + json.dumps(node).encode()]
    dirs = {}
    for t, items in seeds.items():
        d = work / "seeds" / t
        d.mkdir(parents=True, exist_ok=True)
        for i, b in enumerate(items):
            (d / f"seed{i:02d}").write_bytes(b)
        dirs[t] = d
    return dirs


# ---------------------------------------------------------------------- runs
_STAT = re.compile(r"^stat::(\w+):\s+(\d+)", re.M)
_COV = re.compile(r"#(\d+)\s+(?:INITED|NEW|REDUCE|pulse|DONE)\s+cov: (\d+) ft: (\d+) corp: (\d+)")


def _replay(build: Path, t: str, name: str, work: Path, dirs, env: Dict[str, str], timeout_s: float):
    """Every input in `dirs` once through `build`'s fuzz_<t>: (rc, inputs run, reproducers, stderr)."""
    art = work / "artifacts" / f"{t}-{name}"
    art.mkdir(parents=True, exist_ok=True)
    p = subprocess.run([str(build / f"fuzz_{t}"), "-runs=0", "-timeout=60", "-rss_limit_mb=4096",
                        f"-artifact_prefix={art}/", *map(str, dirs)],
                       env=env, capture_output=True, text=True, errors="replace", timeout=timeout_s)
    (work / f"{t}-{name}.log").write_text(p.stderr)
    m = re.search(r"#(\d+)\s+(?:INITED|DONE)", p.stderr)
    return p.returncode, int(m.group(1)) if m else 0, sorted(f"{name}/{x.name}" for x in art.iterdir()), p.stderr


def run_target(t: str, seconds: float, work: Path, seeds: Path, env: Dict[str, str], runs: int = 0) -> dict:
    """Fuzz `t` for `seconds` (coverage + ASan), then replay everything it kept
    under ASan + UBSan, and for the threaded targets under TSan. ``runs`` > 0:
    stop after that many executions instead, with `seconds` only as a cap (a
    fixed amount of work however loaded the machine is)."""
    corpus = work / "corpus" / t
    art = work / "artifacts" / t
    corpus.mkdir(parents=True, exist_ok=True)
    art.mkdir(parents=True, exist_ok=True)
    # sockets live here: keep the path well under the 108-byte sun_path limit
    scratch = Path(tempfile.mkdtemp(prefix=f"mf-{t}-", dir="/tmp"))
    try:
        e = dict(os.environ, **env, MI355X_FUZZ_TMP=str(scratch))
        if t in ("sysfs", "labels"):  # a private copy per run: the target rewrites files in place
            mut = work / f"sysfs-mut-{t}"
            shutil.rmtree(mut, ignore_errors=True)
            shutil.copytree(env["MI355X_FUZZ_SYSFS_MUT"], mut, symlinks=True)
            e["MI355X_FUZZ_SYSFS_MUT"] = str(mut)
        argv = [str(BUILD / f"fuzz_{t}"), f"-max_total_time={int(max(1, seconds))}", "-timeout=25",
                "-rss_limit_mb=4096", "-print_final_stats=1", "-max_len=65536", f"-artifact_prefix={art}/",
                str(corpus), str(seeds)] + ([f"-runs={runs}"] if runs > 0 else [])
        t0 = time.monotonic()
        p = subprocess.run(argv, env=e, capture_output=True, text=True, errors="replace", timeout=seconds + 300)
        wall = time.monotonic() - t0
        log = p.stderr
        (work / f"{t}.log").write_text(log)
        stats = {k: int(v) for k, v in _STAT.findall(log)}
        cov = _COV.findall(log)
        findings = sorted(x.name for x in art.iterdir())
        rrc, replayed, rfind, rerr = _replay(BUILD_REPLAY, t, "replay", work, (corpus, seeds), e, seconds + 600)
        findings += rfind
        if rrc != 0:
            log += "\n--- replay (ASan + UBSan) ---\n" + rerr
        trc = None
        if t in TSAN_TARGETS:
            trc, _, tfind, terr = _replay(BUILD_TSAN, t, "tsan", work, (corpus, seeds),
                                          dict(e, TSAN_OPTIONS="halt_on_error=1"), seconds + 1200)
            findings += tfind
            if trc != 0:
                log += "\n--- replay (TSan) ---\n" + terr
    finally:
        shutil.rmtree(scratch, ignore_errors=True)
    ok = p.returncode == 0 and rrc == 0 and not trc
    return {"target": t, "rc": p.returncode, "seconds": round(wall, 1),
            "execs": stats.get("number_of_executed_units", 0),
            "execs_per_s": stats.get("average_exec_per_sec", 0),
            "peak_rss_mb": stats.get("peak_rss_mb", 0),
            "coverage_edges": int(cov[-1][1]) if cov else None, "features": int(cov[-1][2]) if cov else None,
            "corpus": len(list(corpus.iterdir())), "seeds": len(list(seeds.iterdir())),
            "replayed_full_ubsan": replayed, "replay_rc": rrc, "tsan_replay_rc": trc,
            "findings": findings, "error_tail": "" if ok else "\n".join(log.splitlines()[-40:])}


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--targets", default=",".join(TARGETS))
    ap.add_argument("--seconds", type=float, default=30.0, help="per target")
    ap.add_argument("--parallel", type=int, default=4)
    ap.add_argument("--work", default="", help="corpora / artifacts / logs (default: a temp dir)")
    ap.add_argument("--json", default="", help="write the summary here")
    ap.add_argument("--build-only", action="store_true")
    return ap


def main(argv=None) -> int:
    a = make_parser().parse_args(argv)
    if not available():
        print("clang with libFuzzer is not available", file=sys.stderr)
        return 2
    build()
    if a.build_only:
        return 0
    work = Path(a.work) if a.work else Path(tempfile.mkdtemp(prefix="mi355x-fuzz-"))
    work.mkdir(parents=True, exist_ok=True)
    env = make_fixtures(work / "fixtures")
    seeds = make_seeds(work, env)
    targets = [t for t in a.targets.split(",") if t]
    for t in targets:
        if t not in TARGETS:
            raise SystemExit(f"unknown target {t}")
    with ThreadPoolExecutor(max_workers=max(1, a.parallel)) as ex:
        rows = list(ex.map(lambda t: run_target(t, a.seconds, work, seeds[t], env), targets))
    summary = {"tool": "tools/fuzz_native.py", "engine": "libFuzzer", "sanitizers": "fuzzing: ASan (+ leak check); replay of every corpus input: ASan + UBSan (all but null); "
               "threaded targets' corpora once more under TSan",
               "seconds_per_target": a.seconds, "work": str(work), "targets": rows,
               "total_execs": sum(r["execs"] for r in rows),
               "findings": sum(len(r["findings"]) for r in rows)}
    text = json.dumps(summary, indent=1)
    print(text)
    if a.json:
        Path(a.json).write_text(text + "\n")
    return 0 if all(r["rc"] == 0 and r["replay_rc"] == 0 and not r["tsan_replay_rc"] and not r["findings"]
                    for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
