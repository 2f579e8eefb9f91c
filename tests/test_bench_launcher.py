"""bench.py's multi-GPU launcher and rank logic on CPU (gloo), the GPU step stubbed
(`--stub-step`): `--gpus N` spawns N ranks, each rank segments its own frame stream, the job
time is the max over ranks, and a torchrun WORLD_SIZE that disagrees with --gpus is refused.
Reference: seg_video_old_no_plot.py:157-166 (per-frame independent loop),
semantic_seg_multigpu.py:467-468 (one process per GPU, init_process_group)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

SMALL = ["--stub-step", "--steps", "3", "--warmup", "1", "--batch", "2", "--height", "16", "--width", "32"]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def test_resolve_world():
    a1 = bench.parse(["--gpus", "1"])
    a2 = bench.parse(["--gpus", "2"])
    assert bench.resolve_world(a1, {}) == (1, 0, 0)
    assert bench.resolve_world(a2, {}) is None                       # must spawn its ranks
    assert bench.resolve_world(a2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}) == (2, 1, 1)
    with pytest.raises(SystemExit):
        bench.resolve_world(a1, {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert bench.frame_seed(0) != bench.frame_seed(1)


def test_gpus2_spawns_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", *SMALL],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                            # rank 0 prints ONE line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    ranks = d["per_rank"]
    assert [p["rank"] for p in ranks] == [0, 1]
    assert ranks[0]["frame_seed"] != ranks[1]["frame_seed"]
    assert ranks[0]["frame_sum"] != ranks[1]["frame_sum"]             # different frames per rank
    job = max(p["seconds"] for p in ranks)
    # value = frames of all ranks / the slowest rank's time (barriers make them nearly equal)
    assert d["value"] == pytest.approx(2 * 2 * 3 / (d["ms_per_step"] * 3 / 1e3), rel=1e-6)
    assert d["ms_per_step"] * 3 / 1e3 == pytest.approx(job, rel=1e-6)


def test_world_mismatch_refused():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_PORT="29999")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", *SMALL],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_single_rank_stub():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *SMALL],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and len(d["per_rank"]) == 1


FT_SMALL = ["--stub-step", "--steps", "3", "--warmup", "1", "--batch", "2"]


def test_finetune_gpus2_spawns_two_ranks():
    """bench_finetune.py --gpus 2 (config C4's launcher, semantic_seg_multigpu.py:467-468) starts
    two ranks that all-reduce over the process group: the reduced sum is the sum of both ranks'
    rank-seeded tensors, and rank 0 prints one line with n_gpus = 2."""
    import torch
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench_finetune.py"), "--gpus", "2", *FT_SMALL],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    want = sum(float(torch.randn(4096, generator=torch.Generator().manual_seed(2000 + k)).sum()) for k in (0, 1))
    assert d["reduced_sum"] == pytest.approx(want, rel=1e-5, abs=1e-3)
    assert d["value"] == pytest.approx(2 * 2 * 3 / (d["ms_per_step"] * 3 / 1e3), rel=1e-6)


def test_finetune_world_mismatch_refused():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_PORT="29998")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench_finetune.py"), "--gpus", "1", *FT_SMALL],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


class _Ev:
    """a stand-in for torch.cuda.Event: elapsed_time between two host-side stamps (ms)"""
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def test_step_spread_reports_one_off_stall():
    """bench.step_spread: per-step min / median / max from the step-boundary events, the slowest
    step's index and the time spent beyond 1.5x the median (a one-off stall, not a steady cost)."""
    import bench
    steps = [5.0] * 9 + [40.0] + [5.0] * 10            # a 35-ms stall in step 9
    t, marks = 0.0, [_Ev(0.0)]
    for d in steps:
        t += d
        marks.append(_Ev(t))
    s = bench.step_spread(marks)
    assert s["steps"] == 20 and s["min"] == 5.0 and s["median"] == 5.0 and s["max"] == 40.0
    assert s["max_at_step"] == 9 and s["stall_ms"] == 35.0
    assert bench.step_spread(marks[:1]) is None


def test_newest_first_orders_rounds_numerically(tmp_path):
    """bench.newest_first: r11s_ > r11p_ > r10p_ > r9zz_ (string order would put r9zz first)."""
    import bench
    for n in ("r9zz_bf16_pmc_mfma.json", "r10p_bf16_pmc_mfma.json", "r11p_bf16_pmc_mfma.json",
              "r11s_bf16_pmc_mfma.json", "misc_pmc_mfma.json"):
        (tmp_path / n).write_text("{}")
    got = [os.path.basename(f) for f in bench.newest_first(str(tmp_path / "*_pmc_mfma.json"))]
    assert got == ["r11s_bf16_pmc_mfma.json", "r11p_bf16_pmc_mfma.json", "r10p_bf16_pmc_mfma.json",
                   "r9zz_bf16_pmc_mfma.json", "misc_pmc_mfma.json"]


def test_committed_mfma_captures_cover_every_precision_line():
    """Every precision the default bench line reports has a committed MFMA-busy capture of its exact
    workload (roofline.mfma_busy comes from it; the driver's GPU box has no rocprofv3 run)."""
    import types
    import bench
    args = types.SimpleNamespace(arch="drn_d_22", height=1024, width=2048, batch=8, precision="bf16")
    for prec in ("bf16", "fp32x", "fp32", "int8"):
        m = bench.pmc_mfma(args, prec)
        assert m.get("kernels"), prec
        busy = [v["mfma_busy"] for v in m["kernels"].values() if v.get("mfma_busy") is not None]
        assert busy and all(0.0 <= b <= 1.0 for b in busy), prec
