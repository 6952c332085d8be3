"""C5's multi-GPU form (BASELINE.json configs[4]) rehearsed on one GPU: the
sharded runner scripts/bench_c5.py launched by torch.distributed.run with 1 and 2 gloo ranks
sharing cuda:0 over the same 16,384 global chains.  Sharding by chain_offset plus the all-gather
of the 256-chain tile partials must give bit-identical moments and harmonic-mean evidence for
either rank count (the `moments_digest` of the JSON line)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(world, tmp_path, port, self_launch=False):
    """world ranks under an explicit torch.distributed.run, or (self_launch) the runner's own
    `--gpus N` child launch -- the shape the driver uses for bench.py."""
    out = tmp_path / ("c5_w%d.jsonl" % world)
    env = dict(os.environ, MCG_BENCH_BACKEND="gloo", MCG_BENCH_DEVICE="0", PYTHONUNBUFFERED="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    launcher = [] if self_launch else [
        "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
        "--master-addr", "127.0.0.1", "--master-port", str(port)]
    cmd = [sys.executable] + launcher + [
           os.path.join(ROOT, "scripts", "bench_c5.py"), "--gpus", str(world), "--total-chains", "16384",
           "--sweeps", "40", "--steps", "2", "--warmup", "1", "--out", str(out), "--no-cpu-baseline"]
    subprocess.run(cmd, env=env, check=True, timeout=100, cwd=ROOT)
    return json.loads(out.read_text().strip().splitlines()[-1])


def test_c5_sharded_runner_is_rank_count_invariant(tmp_path):
    import random
    port = 29500 + random.randint(4001, 6000)
    one = _run(1, tmp_path, port)
    two = _run(2, tmp_path, port + 1, self_launch=True)
    four = _run(4, tmp_path, port + 2, self_launch=True)
    assert one["config"]["chains_total"] == two["config"]["chains_total"] == 16384
    assert two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert one["moments_digest"] == two["moments_digest"] == four["moments_digest"]
    # the self-check block: the group's size, every rank's device and times, their spread
    rk = four["ranks"]
    assert four["n_gpus"] == 4 and rk["rccl_world"] == 4 and rk["world_matches"]
    assert [r["rank"] for r in rk["per_rank"]] == [0, 1, 2, 3]
    assert all(r["launches"] >= 2 and r["avg_launch_ms"] > 0 for r in rk["per_rank"])
    assert rk["elapsed_s_max"] == pytest.approx(four["ms_per_step"] * 2 * 1e-3, rel=1e-9)
    assert one["ranks"]["rccl_world"] == 1 and one["ranks"]["backend"] == "none"
    assert one["log_z_harmonic_mean"] == two["log_z_harmonic_mean"]
    assert one["accept_frac"] == two["accept_frac"]
    assert 0.05 < one["accept_frac"] < 0.6
    assert one["posterior_check"]["max_abs_mean_err_over_sd"] < 0.1
