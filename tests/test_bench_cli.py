"""bench.py's command line (CPU): ``--gpus N`` means N ranks -- refused loudly when the launcher's WORLD_SIZE
differs or fewer than N GPUs are visible, otherwise (no launcher) handed to torch.distributed.run with N ranks
-- and the roofline block, which takes PMC figures only from a summary of the same workload.  The end-to-end
``--gpus 2`` run is tests/test_gpu_multiview.py::test_bench_gpus_2_spawns_two_ranks (it needs a GPU)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_bench(args, **env):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=120)


def test_gpus_more_than_visible_fails_loudly():
    r = run_bench(["--gpus", "8"], HIP_VISIBLE_DEVICES="")
    assert r.returncode == 2 and "needs 8 visible GPUs" in r.stderr and r.stdout == ""


def test_world_size_mismatch_fails_loudly():
    r = run_bench(["--gpus", "8"], WORLD_SIZE="1")
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_check_ranks_and_launcher_argv():
    import bench
    assert bench.check_ranks(1, {}) is None
    assert bench.check_ranks(2, {"WORLD_SIZE": "2", "GSD_DIST_BACKEND": "gloo"}) is None
    assert "WORLD_SIZE=4" in bench.check_ranks(2, {"WORLD_SIZE": "4"})
    assert bench.check_ranks(0, {}) is not None
    argv = bench.launcher_argv(4, ["--gpus", "4", "--steps", "7"], 12345)
    assert argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in argv and "--master-port=12345" in argv
    assert argv[argv.index("--master-addr") + 1] == "127.0.0.1"
    assert argv[-4:] == ["--gpus", "4", "--steps", "7"] and argv[-5].endswith("bench.py")


def test_roofline_uses_only_the_same_workloads_pmc(tmp_path, monkeypatch):
    import bench
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    d = tmp_path / "profiles" / "roundX" / "pmc" / "cfg4"
    d.mkdir(parents=True)
    (d / "pmc_traffic.json").write_text(json.dumps({
        "_workload": "cfg4",
        "render_bwd": {"hbm_bytes": 300_000_000, "valu": {"instructions": 250_000_000, "issue_per_simd_cycle": 0.2,
                                                          "lds_issue_wait_frac": 0.1}}}))
    # an untagged (older) summary is never used
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps({"render_bwd": {"hbm_bytes": 1}}))
    r4 = bench.roofline("render_bwd", 0.5, 220_000_000, "cfg4")
    assert r4["traffic"] == 300_000_000 and r4["bound"] == "valu"
    assert r4["achieved"] == pytest.approx(250e6 / 0.5e-3 / 1e9, rel=1e-4)
    assert r4["frac"] == pytest.approx(r4["achieved"] / bench.VALU_PEAK_GINST, rel=1e-3)
    assert r4["hbm"]["achieved"] == pytest.approx(220e6 / 0.5e-3 / 1e9, rel=1e-4)
    r5 = bench.roofline("render_bwd", 1.5, 700_000_000, "cfg5")
    assert r5["traffic"] is None and r5["bound"] == "hbm" and "valu" not in r5
    assert r5["frac"] == pytest.approx(700e6 / 1.5e-3 / 1e9 / 8000.0, rel=1e-3)
