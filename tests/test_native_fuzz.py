"""Coverage-guided fuzzing of the native parsers, short runs (tools/fuzz_native.py).

Every libFuzzer target in native/fuzz/ runs a fixed number of executions from
its seed corpus under ASan, then everything it kept is replayed under ASan + UBSan (and
under TSan for the targets that drive the threaded server or a peer thread); the
inputs that once broke a target (native/fuzz/regressions/) are replayed too.
Long campaigns: ``python tools/fuzz_native.py --seconds 600`` (profiles/r3/
fuzz_native.json). CPU only.
"""
import importlib.util
import os
import shutil
import subprocess
import tempfile
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
_spec = importlib.util.spec_from_file_location("fuzz_native", REPO / "tools" / "fuzz_native.py")
fz = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(fz)

pytestmark = pytest.mark.skipif(not fz.available(), reason="clang with libFuzzer not available")

SECONDS = float(os.environ.get("MI355X_FUZZ_SECONDS", "0"))
# a fixed number of executions per target (the seeds, then mutations), so a
# loaded machine runs the same work more slowly instead of less of it; the
# time is only a cap. MI355X_FUZZ_SECONDS > 0: fuzz for that long instead
MUTATIONS = {"sysfs": 20, "labels": 20}
RUNS_CAP_S = 240


@pytest.fixture(scope="module")
def built():
    fz.build()
    return True


def test_every_target_runs_clean_from_its_seeds(built, tmp_path):
    env = fz.make_fixtures(tmp_path / "fixtures")
    seeds = fz.make_seeds(tmp_path, env)
    from concurrent.futures import ThreadPoolExecutor
    def one(t):
        if SECONDS > 0:
            return fz.run_target(t, SECONDS, tmp_path, seeds[t], env)
        nseeds = len(list(seeds[t].iterdir()))
        return fz.run_target(t, RUNS_CAP_S, tmp_path, seeds[t], env, runs=nseeds + MUTATIONS.get(t, 500))

    with ThreadPoolExecutor(max_workers=4) as ex:
        rows = list(ex.map(one, fz.TARGETS))
    for r in rows:
        assert r["rc"] == 0 and r["replay_rc"] == 0 and not r["findings"], (r["target"], r["error_tail"])
        if r["target"] in fz.TSAN_TARGETS:    # the server's / peer's threads, under TSan
            assert r["tsan_replay_rc"] == 0, (r["target"], r["error_tail"])
        assert r["execs"] >= MUTATIONS.get(r["target"], 500), r
        # the targets reach code beyond the harness (coverage feedback works)
        assert r["coverage_edges"] and r["coverage_edges"] > 100, r
        assert r["replayed_full_ubsan"] >= r["seeds"], r


def test_regression_inputs_replay_clean(built, tmp_path):
    env = fz.make_fixtures(tmp_path / "fixtures")
    reg = REPO / "native" / "fuzz" / "regressions"
    dirs = sorted(d for d in reg.iterdir() if d.is_dir())
    assert dirs, "no regression inputs"
    for d in dirs:
        assert d.name in fz.TARGETS, d
        short = tempfile.mkdtemp(prefix="mf-reg-", dir="/tmp")  # socket paths under the sun_path limit
        e = dict(os.environ, **env, MI355X_FUZZ_TMP=short)
        if d.name in ("sysfs", "labels"):
            mut = tmp_path / "mut"
            shutil.copytree(env["MI355X_FUZZ_SYSFS_MUT"], mut, symlinks=True)
            e["MI355X_FUZZ_SYSFS_MUT"] = str(mut)
        for build in (fz.BUILD, fz.BUILD_REPLAY):
            p = subprocess.run([str(build / f"fuzz_{d.name}"), *map(str, sorted(d.iterdir()))], env=e,
                               capture_output=True, text=True, errors="replace", timeout=300)
            assert p.returncode == 0, (d.name, build.name, p.stderr[-3000:])
        shutil.rmtree(short, ignore_errors=True)
