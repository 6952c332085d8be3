"""bench.py's multi-GPU entry point (the driver's `python bench.py --gpus N` shape, BASELINE.json
metric "1/2/4/8 MI355X").

Without a launcher around it, `--gpus N` must start N ranks itself (a child
torch.distributed.run, before any GPU call) and print rank 0's single JSON line with
n_gpus = N; under a launcher, WORLD_SIZE != --gpus is an error.  `--launch-check` runs exactly
that bring-up with gloo and no GPU work, so the CPU suite covers it; the GPU test runs the real
bench with two gloo ranks sharing cuda:0."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(PYTHONUNBUFFERED="1", **kw)
    return env


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_flag_launches_n_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout              # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == n and line["gpus_arg"] == n
    assert sorted(line["ranks"]) == [[r, r, n] for r in range(n)]


def test_world_size_mismatch_fails_loudly():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       env=_env(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode != 0
    assert "WORLD_SIZE=4" in p.stderr


def test_child_keeps_cpu_thread_budget():
    """The ranks' CPU baseline uses the thread count the parent would have used at N = 1
    (torch.distributed.run would otherwise leave OMP_NUM_THREADS=1 in every rank)."""
    sys.path.insert(0, ROOT)
    import bench
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       env=_env(OMP_NUM_THREADS="3"), capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    want = min(len(os.sched_getaffinity(0)), 3)
    assert _json_lines(p.stdout)[0]["cpu_threads"] == want
    assert bench.cpu_threads() >= 1


def test_c5_runner_cpu_baseline_is_the_fullcov_oracle():
    """scripts/bench_c5.py's rank-0 CPU baseline times the oracle on the C5 target."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    sys.path.insert(0, ROOT)
    import bench_c5
    mu, cov, s = bench_c5.c5_target()
    cpu = bench_c5.cpu_baseline(mu, cov, s, 0.05)
    assert cpu["kind"] == "port" and cpu["unit"] == "MH steps/s"
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and "C5" in cpu["sample"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
def test_bench_gloo_ranks_on_one_gpu(n):
    """The real bench over n ranks sharing cuda:0 (gloo collectives): one JSON line, n_gpus n,
    value = every rank's steps over the max-over-ranks time, cpu_baseline present on rank 0; the
    self-check block lists every rank (its device, elapsed and launch times) with the spread and
    the process group's own size; the nested replicas of all n ranks are merged."""
    cmd = [sys.executable, BENCH, "--gpus", str(n), "--steps", "2", "--warmup", "1", "--sweeps", "50",
           "--chains", "4096", "--nested-nlive", "2048", "--nested-k", "64", "--nested-nmcmc", "20",
           "--nested-seeds", "1", "--cpu-seconds", "0.1"]
    p = subprocess.run(cmd, env=_env(MCG_BENCH_BACKEND="gloo", MCG_BENCH_DEVICE="0"),
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == n
    assert line["value"] == pytest.approx(n * 4096 * 50 * 2 / (line["ms_per_step"] * 2 * 1e-3), rel=1e-9)
    assert line["cpu_baseline"] is not None and line["cpu_baseline"]["value"] > 0
    assert line["log_evidence"]["seed_sweep"]["runs"] == n
    assert line["log_evidence"]["nested_run"]["nlive"] == 2048 * n
    rk = line["ranks"]
    assert rk["rccl_world"] == n and rk["backend"] == "gloo" and rk["world_matches"]
    assert [r["rank"] for r in rk["per_rank"]] == list(range(n))
    assert all(r["device"] == 0 and r["launches"] == 2 and r["avg_launch_ms"] > 0 for r in rk["per_rank"])
    assert rk["distinct_gpus"] == 1 and not rk["one_gpu_per_rank"]       # shared card: gloo only
    assert rk["elapsed_s_max"] == pytest.approx(line["ms_per_step"] * 2 * 1e-3, rel=1e-9)
    assert rk["elapsed_s_min"] <= rk["elapsed_s_max"]


@pytest.mark.gpu
def test_bench_rccl_refuses_more_ranks_than_gpus():
    """Under RCCL (the driver's backend) a bench of more ranks than visible GPUs fails loudly
    before any GPU work instead of stacking ranks on one card."""
    import torch
    n = torch.cuda.device_count() + 1
    cmd = [sys.executable, BENCH, "--gpus", str(n), "--steps", "1", "--warmup", "1", "--sweeps", "10",
           "--chains", "1024", "--nested-nlive", "0", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode != 0
    assert "visible GPU" in p.stderr, p.stderr[-2000:]
