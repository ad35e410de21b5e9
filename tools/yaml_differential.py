#!/usr/bin/env python3
"""Exploratory native-YAML-reader vs PyYAML differential: the property tests of
tests/test_native_yaml.py (and the JSON reader's, tests/test_native_json.py)
under the "explore" Hypothesis profile (tests/conftest.py): fresh random draws,
--examples per property instead of the CI profile's fixed 300.

  python tools/yaml_differential.py --examples 10000 --out profiles/r6/yaml_differential.json

The suite itself runs derandomized; a failure found here is added to the
parametrised cases of tests/test_native_yaml.py.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROPERTIES = ["tests/test_native_yaml.py::test_native_reader_equals_pyyaml",
              "tests/test_native_yaml.py::test_hand_written_layouts_equal_pyyaml",
              "tests/test_native_yaml.py::test_shared_nodes_equal_pyyaml",
              "tests/test_native_json.py"]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--examples", type=int, default=10000, help="examples per property")
    ap.add_argument("--seed", type=int, default=None, help="Hypothesis seed (default: random)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    env = dict(os.environ, HYPOTHESIS_PROFILE="explore", MI355X_HYPOTHESIS_EXAMPLES=str(a.examples))
    seed = a.seed if a.seed is not None else int.from_bytes(os.urandom(4), "little")
    cmd = [sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", f"--hypothesis-seed={seed}",
           "--hypothesis-show-statistics", *[p for p in PROPERTIES if os.path.exists(os.path.join(REPO, p.split("::")[0]))]]
    t0 = time.monotonic()
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True)
    took = time.monotonic() - t0
    out = p.stdout + p.stderr
    # per property: "- N passing, M failing, and K invalid test cases" (--hypothesis-show-statistics)
    stats, name = {}, None
    for ln in out.splitlines():
        m = re.match(r"^(tests/\S+::\S+):$", ln.strip())
        if m:
            name = m.group(1)
        cnt = re.search(r"(\d+) passing, (\d+) failing", ln)
        if cnt and name:
            stats[name] = {"passing": int(cnt.group(1)), "failing": int(cnt.group(2))}
    res = {"examples_per_property": a.examples, "seed": seed, "returncode": p.returncode, "seconds": round(took, 1),
           "generate_phase": stats, "summary": out.strip().splitlines()[-1:],
           "command": " ".join(cmd[2:])}
    if p.returncode != 0:
        res["failure_tail"] = out[-4000:]
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return p.returncode


if __name__ == "__main__":
    sys.exit(main())
