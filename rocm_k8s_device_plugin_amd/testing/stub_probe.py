#!/usr/bin/env python3
"""Fault-injection stand-in for ``mi355x-liveness-probe`` (CPU tests).

Speaks the same CLI and JSON contract, one-shot and ``--serve``. Behaviour
per ROCr ordinal comes from the JSON file named by $MI355X_STUB_PROBE_CONTROL
(re-read on every request), e.g.
``{"0": "ok", "3": "fail", "5": "hang", "6": "stale", "7": "garbage"}``
(missing ordinals are "ok"; "serve": "broken" makes --serve fail to start,
"serve": "slow_start" delays its hello by "serve_start_s" seconds;
"server_fail" fails only inside --serve: a stale server runtime; "slow" is a
dispatch that completes "slow_s" seconds after it was submitted: in --serve a
request whose deadline comes first is answered pending and a later one collects
the late verdict; "pending" keeps the dispatch queued and, like the real server,
answers only when the device's deadline has passed).
--serve speaks the real server's protocol: "@<id>"-tagged requests answered
concurrently with their id, per-device deadlines ("<ordinal>:<nonce>:<s>"),
requests on one device serialised on its slot.
Exercises the real LivenessProber code path: process spawn, server protocol,
deadline kill, fallback to per-device isolation, output parsing, nonce check,
hysteresis. Each start appends a line to $MI355X_STUB_PROBE_LOG if set.
Throughput-check replies ("perf" requests / --perf) follow the control file's
"perf" map, e.g. ``{"perf": {"3": "slow_xcd", "4": "corrupt"}}``.
"""
import json
import os
import sys
import time


def _control():
    path = os.environ.get("MI355X_STUB_PROBE_CONTROL")
    if path and os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return {}


def _identity(ordinal):
    """Agent identity per host ordinal from $MI355X_STUB_PROBE_IDENTITY (JSON
    {ordinal: {"kfd_node_id": N, "pci_bus_id": "dddd:bb:dd.f"}}); unknown otherwise."""
    raw = os.environ.get("MI355X_STUB_PROBE_IDENTITY")
    ident = json.loads(raw).get(str(ordinal), {}) if raw else {}
    return {"kfd_node_id": int(ident.get("kfd_node_id", -1)), "pci_bus_id": ident.get("pci_bus_id", "")}


def _device(ordinal_reported, mode, nonce, host_ordinal=None):
    ok = mode == "ok"
    return {**_identity(ordinal_reported if host_ordinal is None else host_ordinal),
            "ordinal": ordinal_reported, "ok": ok or mode == "stale", "hip_error": 0, "mismatches": 0 if ok else 17,
            "nonce": nonce if mode != "stale" else (nonce + 1) & 0xFFFFFFFF, "xcc_id": 0, "hw_id": 0, "iters": 4,
            "dispatches": 1, "runtime": "stub", "kernel_us": 3.0, "setup_us": 1.0,
            "total_us": 5.0, "arch": "gfx950", "name": "", "uuid": "", "pci_domain": 0,
            "pci_bus": 0, "pci_device": 0, "cu_count": 256, "total_mem": 0,
            "error": "" if ok or mode == "stale" else "17/1024 MFMA results differ from host reference"}


def _perf_device(ordinal_reported, mode, nonce, host_ordinal=None):
    """Throughput-check reply (kind "perf"); modes from the control file's
    "perf" map: slow_hbm, slow_mfma, slow_xcd (one XCD at a third of the clock),
    corrupt (HBM words read back wrong); hang (the server never answers; serve mode only)."""
    xcd = [1530.0] * 8
    if mode == "slow_xcd":
        xcd[3] = 510.0
    d = {**_identity(ordinal_reported if host_ordinal is None else host_ordinal),
         "ordinal": ordinal_reported, "ok": mode != "corrupt", "hsa_error": 0, "nonce": nonce, "bytes": 4 << 30,
         "cu_count": 256, "num_xcc": 8, "hbm_write_gbps": 4600.0, "hbm_read_gbps": 1500.0 if mode == "slow_hbm" else 6000.0,
         "hbm_bad_words": 3 if mode == "corrupt" else 0, "hbm_first_bad": 4096 if mode == "corrupt" else -1,
         "mfma_iters": 65536, "mfma_grid": 512, "mfma_records_ok": 512, "mfma_checksum_mismatch": 0, "mfma_xccs": 8,
         "mfma_tflops": 400.0 if mode == "slow_mfma" else 1550.0, "clock_mhz_min": min(xcd), "clock_mhz_median": 1530.0,
         "clock_mhz_max": max(xcd), "xcd_clock_mhz": xcd, "total_us": 35000.0, "in_flight_s": 0.0,
         "error": "hbm_bad_words=3 first_bad_unit=4096" if mode == "corrupt" else ""}
    return d


def _kfd_entry():
    """Like a kept-queue server: a kfd proc entry with one queue per GPU id
    (MI355X_STUB_KFD_PROC / MI355X_STUB_KFD_GPUIDS), removed on exit.
    MI355X_STUB_KFD_ALSO="<pid>:<gid>,<gid>" adds another process' entry in the
    same instant (a pod started with the server; left in place)."""
    root, gids = os.environ.get("MI355X_STUB_KFD_PROC"), os.environ.get("MI355X_STUB_KFD_GPUIDS", "")
    if not root:
        return None
    import shutil

    def make(entry, ids):
        for i, g in enumerate(x for x in ids.split(",") if x):
            os.makedirs(os.path.join(entry, "queues", str(i)), exist_ok=True)
            with open(os.path.join(entry, "queues", str(i), "gpuid"), "w") as f:
                f.write(g + "\n")
    entry = os.path.join(root, str(os.getpid()))
    make(entry, gids)
    also = os.environ.get("MI355X_STUB_KFD_ALSO", "")
    if also:
        pid, ids = also.split(":")
        make(os.path.join(root, pid), ids)
    import atexit
    atexit.register(shutil.rmtree, entry, True)
    return entry


def _parse(line):
    """One request line: (id or None, kind, timeout_s, [(ordinal, nonce, deadline_s)])."""
    parts = line.split()
    rid = None
    if parts and parts[0].startswith("@"):
        rid, parts = int(parts[0][1:]), parts[1:]
    kind = parts[0]
    timeout = float(parts[2])
    devs = []
    for tok in parts[4:] if kind == "perf" else parts[3:]:
        f = tok.split(":")
        devs.append((f[0], int(f[1], 0), float(f[2]) if len(f) > 2 and float(f[2]) > 0 else timeout))
    return rid, kind, timeout, devs


def serve():
    import threading
    ctl = _control()
    if ctl.get("serve") == "broken":
        print(json.dumps({"serve": True, "ok": False, "hip_device_count": 0}), flush=True)
        return 2
    if ctl.get("serve") == "slow_start":   # a runtime start-up that outlasts the caller's patience
        time.sleep(float(ctl.get("serve_start_s", 30)))
    _kfd_entry()
    t = time.monotonic_ns()
    # like the real server: tagged requests are answered concurrently, as they complete
    print(json.dumps({"serve": True, "ok": True, "hip_device_count": 8, "concurrent": True, "deadlines": True,
                      "t_start_ns": t, "t_runtime_ns": t}), flush=True)
    slots = {}   # ordinal -> nonce of the kept slot's outstanding dispatch (like --keep)
    slow = {}    # ordinal -> (submitted at, nonce) of a "slow" device's outstanding dispatch
    locks = {}   # ordinal -> its kept slot's lock (requests on one device serialise, as on the real server)
    out_mu, state_mu = threading.Lock(), threading.Lock()
    # like ROCr: with ROCR_VISIBLE_DEVICES the server numbers only those GPUs
    vis = [x for x in os.environ.get("ROCR_VISIBLE_DEVICES", "").split(",") if x]
    starts_log = os.environ.get("MI355X_STUB_PROBE_LOG")
    if starts_log and vis:
        with open(starts_log, "a") as f:
            f.write("visible=" + ",".join(vis) + "\n")

    def one(kind, o, n, deadline, ctl):
        hosto = vis[int(o)] if vis and int(o) < len(vis) else o
        if kind == "perf":
            pmode = ctl.get("perf", {}).get(hosto, "ok")
            if pmode == "hang":   # a check that never finishes (the daemon stops meanwhile)
                time.sleep(3600)
            return _perf_device(int(o), pmode, n, host_ordinal=int(hosto))
        mode = ctl.get(hosto, "ok")
        if mode == "server_fail":
            mode = "fail"
        if mode == "hang":
            time.sleep(3600)
        if mode == "slow":
            # a dispatch that completes "slow_s" seconds after it was submitted:
            # a request whose deadline comes first is answered pending (the
            # dispatch stays queued), and a later one collects its late verdict
            with state_mu:
                since, first = slow.setdefault(o, (time.monotonic(), n))
            left = since + float(ctl.get("slow_s", 1.0)) - time.monotonic()
            if left > deadline:
                time.sleep(deadline)
                d = _device(int(o), "fail", n, host_ordinal=int(hosto))
                d.update(hip_error=-1, mismatches=0, pending_s=max(time.monotonic() - since, 1e-3),
                         error=f"dispatch pending for {time.monotonic() - since:.1f}s (not completed)")
                return d
            time.sleep(max(0.0, left))
            with state_mu:
                slow.pop(o, None)
            d = _device(int(o), "ok", first, host_ordinal=int(hosto))
            if first != n:
                d["late"] = 1
            return d
        if mode == "garbage":
            print("segfault-ish noise", flush=True)
            os._exit(139)
        if mode == "timeout":   # server without kept queues: the dispatch did not complete
            time.sleep(deadline)
            d = _device(int(o), "fail", n, host_ordinal=int(hosto))
            d.update(hip_error=-1, mismatches=0, error=f"dispatch did not complete within {deadline:.1f}s")
            return d
        if mode == "pending" and kind != "sweep":
            # kept-queue server: the dispatch stays queued behind other work; the
            # server waits out this device's whole deadline first, as
            # hsa_probe.cpp's wait_and_verify does
            with state_mu:
                slots.setdefault(o, n)
            if starts_log:   # a test can tell when a request is waiting on this device
                with open(starts_log, "a") as f:
                    f.write(f"pending:{hosto}\n")
            time.sleep(deadline)
            d = _device(int(o), "fail", n, host_ordinal=int(hosto))
            d.update(hip_error=-1, mismatches=0, pending_s=max(deadline, 1e-3),
                     error=f"dispatch pending for {deadline:.1f}s (not completed)")
            return d
        with state_mu:
            late = slots.pop(o, None) if kind != "sweep" else None
        if late is not None:   # the outstanding dispatch completed: its late verdict
            d = _device(int(o), mode, late, host_ordinal=int(hosto))
            d["late"] = 1
            return d
        return _device(int(o), "ok" if mode == "pending" else mode, n, host_ordinal=int(hosto))

    def answer(rid, kind, devs_in):
        ctl = _control()
        res = [None] * len(devs_in)

        def dev(i, o, n, dl):
            with state_mu:
                lk = locks.setdefault(o, threading.Lock())
            if not lk.acquire(timeout=dl):   # another request holds this device's slot past our deadline
                d = _device(int(o), "fail", n)
                d.update(hip_error=-1, mismatches=0, pending_s=dl, error="another request on this device's queue")
                res[i] = d
                return
            try:
                res[i] = one(kind, o, n, dl, ctl)
            finally:
                lk.release()
        ths = [threading.Thread(target=dev, args=(i, *x), daemon=True) for i, x in enumerate(devs_in)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        doc = {"ok": all(d["ok"] for d in res), "hip_device_count": 8, "sweep": kind == "sweep",
               "t_ready_ns": time.monotonic_ns(), "devices": res}
        if rid is not None:
            doc = {"id": rid, **doc}
        with out_mu:
            sys.stdout.write(json.dumps(doc) + "\n")
            sys.stdout.flush()

    for line in sys.stdin:
        parts = line.split()
        if not parts or parts[0] == "quit":
            break
        rid, kind, _, devs = _parse(line)
        if rid is None:
            answer(rid, kind, devs)
        else:
            threading.Thread(target=answer, args=(rid, kind, devs), daemon=True).start()
    return 0


def main(argv):
    log = os.environ.get("MI355X_STUB_PROBE_LOG")
    if log:
        with open(log, "a") as f:
            f.write(("serve" + ("+keep" if "--keep" in argv else "") if "--serve" in argv
                     else os.environ.get("ROCR_VISIBLE_DEVICES", "0")) + "\n")
    if "--serve" in argv:
        return serve()
    nonce = 0
    for i, a in enumerate(argv):
        if a == "--nonce":
            nonce = int(argv[i + 1], 0)
    ordinal = os.environ.get("ROCR_VISIBLE_DEVICES", "0").split(",")[0]
    if "--perf" in argv:
        d = _perf_device(0, _control().get("perf", {}).get(ordinal, "ok"), nonce, host_ordinal=int(ordinal))
        print(json.dumps({"ok": d["ok"], "perf": True, "hip_device_count": 1, "devices": [d]}))
        return 0 if d["ok"] else 1
    ctl = _control()
    mode = ctl.get(ordinal, "ok")
    if mode == "server_fail":
        mode = "ok"
    if mode == "slow":
        time.sleep(float(ctl.get("slow_s", 1.0)))
        mode = "ok"
    if mode in ("pending", "timeout"):   # a fresh process waits too, then gives up
        mode = "fail"
    if mode == "hang":
        time.sleep(3600)
    if mode == "garbage":
        print("segfault-ish noise")
        return 139
    t = time.monotonic_ns()
    # as a container entrypoint (bench.py --fixture): one result per --devices
    # entry; with the fake runtime's /dev view the visible GPU count is the
    # number of render nodes it allows (what ROCr's thunk would find)
    wanted = ["0"]
    if "--devices" in argv:
        wanted = [x for x in argv[argv.index("--devices") + 1].split(",") if x]
    allow = os.environ.get("MI355X_DEV_ALLOW")
    count = (sum(1 for p in allow.split(";") if "/renderD" in p) if allow is not None
             else max(1, len(wanted)))
    host = os.environ.get("ROCR_VISIBLE_DEVICES")
    devs = [_device(int(o), mode, nonce + i, host_ordinal=int(host.split(",")[int(o)])
                    if host and int(o) < len(host.split(",")) else None)
            for i, o in enumerate(wanted)]
    ok = all(d["ok"] for d in devs)
    doc = {"ok": ok, "hip_device_count": count, "identify": False, "t_start_ns": t, "t_runtime_ns": t,
           "t_ready_ns": time.monotonic_ns(), "devices": devs}
    print(json.dumps(doc))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
