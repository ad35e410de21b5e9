"""Peer-link probe wrapper (CPU: a stub executable speaking the --peer JSON)."""
import json
import os
import stat

from rocm_k8s_device_plugin_amd.health.peer import probe_peers


def _stub(tmp_path, body):
    exe = tmp_path / "probe"
    exe.write_text("#!/usr/bin/env python3\nimport json, os, sys\n" + body)
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    return str(exe)


def test_probe_peers_maps_local_indices_to_host_ordinals(tmp_path):
    exe = _stub(tmp_path, """
vis = os.environ["ROCR_VISIBLE_DEVICES"].split(",")
assert "--peer" in sys.argv
devs = [int(x) for x in sys.argv[sys.argv.index("--devices") + 1].split(",")]
pairs = [{"src": a, "dst": b, "ok": True, "link_type": 4, "bytes": 1024, "gbps_best": 40.0 + a + b,
          "mismatches": 0, "error": ""} for a in devs for b in devs if a != b]
print(json.dumps({"peer": True, "ok": True, "pairs": pairs, "vis": vis}))
""")
    rep = probe_peers([3, 5, 6], nbytes=1024, exe=exe)
    assert rep.ok and len(rep.pairs) == 6
    assert {(p["src"], p["dst"]) for p in rep.pairs} == {(a, b) for a in (3, 5, 6) for b in (3, 5, 6) if a != b}
    s = rep.summary()
    assert s["link_types"] == ["xgmi"] and s["pairs_ok"] == 6 and s["gbps_min"] == 41.0 and s["gbps_max"] == 43.0


def test_probe_peers_failure_and_garbage(tmp_path):
    bad = _stub(tmp_path, """
print(json.dumps({"peer": True, "ok": False, "pairs": [{"src": 0, "dst": 1, "ok": False, "link_type": 2,
      "bytes": 8, "gbps_best": 0, "mismatches": 2, "error": "2/2 words differ"}]}))
sys.exit(1)
""")
    rep = probe_peers([0, 1], exe=bad)
    assert not rep.ok and rep.summary()["errors"] == ["2/2 words differ"]
    (tmp_path / "g").mkdir()
    garbage = _stub(tmp_path / "g", "print('boom')\n")
    rep = probe_peers([0], exe=garbage)
    assert not rep.ok and "unparseable" in rep.error
