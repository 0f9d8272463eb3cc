"""bench.py's multi-rank path as the driver uses it: `bench.py --gpus N`
run directly spawns N rank processes itself (torch.distributed.run, one process per GPU, before
the parent touches the GPU) and rank 0 prints ONE JSON line with n_gpus == N and config 4's
per-chunk workload.  On the one-GPU box the ranks share device 0 (GSR_BENCH_SHARE_GPU=1: gloo for
the barriers and the MAX of the elapsed time; the driver's 8-GPU runs use RCCL)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_gpus2_spawns_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["GSR_BENCH_SHARE_GPU"] = "1"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--gaussians", "200000", "--profile-steps", "1", "--train-steps", "2", "--no-config5", "--no-street",
           "--no-cpu-baseline", "--no-config3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, env=env, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 3 and d["warmup"] == 1
    c4 = d["config4"]
    assert c4["n_gpus"] == 2 and c4["value"] > 0 and len(c4["train_step_ms_per_rank"]) == 2
    assert all(v > 0 for v in c4["train_step_ms_per_rank"])


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_gpus2_trains_one_chunk_per_rank():
    """Config 4 as the product runs it (scripts/full_train.py:171-232): with --gpus 2 every rank trains
    its own synthetic street chunk (seed = rank) through the train_single.py loop (here 300 iterations
    of a small chunk); the line reports the aggregate chunk-iterations/s over the job's wall clock and
    every rank's chunk wall clock."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["GSR_BENCH_SHARE_GPU"] = "1"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--gaussians", "100000", "--profile-steps", "1", "--train-steps", "0", "--no-config5", "--no-street",
           "--no-cpu-baseline", "--chunk-iterations", "300", "--chunk-size", "384", "--chunk-positions", "8",
           "--chunk-truth", "100000", "--chunk-init", "40000"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, env=env, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-3000:]
    ch = json.loads(lines[0])["config4"]["chunks"]
    assert ch["n_gpus"] == 2 and len(ch["chunk_wall_s_per_rank"]) == 2
    assert all(w > 0 for w in ch["chunk_wall_s_per_rank"]) and ch["job_wall_s"] >= max(ch["chunk_wall_s_per_rank"])
    assert abs(ch["chunk_iterations_per_s"] - 2 * 300 / ch["job_wall_s"]) <= 0.01 * ch["chunk_iterations_per_s"] + 0.02
    assert ch["P_final_rank0"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_rccl_process_group_single_rank():
    """The collective path of the driver's multi-GPU runs on the one-GPU box: bench.py under
    torch.distributed.run with GSR_BENCH_FORCE_PG=1 initialises the RCCL ("nccl") process group
    for its one rank and times through its barriers and all-reduce (RCCL refuses two ranks on one
    device, so N > 1 cannot run here)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE", "GSR_BENCH_SHARE_GPU")}
    env["GSR_BENCH_FORCE_PG"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", "29517", os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "3",
           "--warmup", "1", "--gaussians", "200000", "--profile-steps", "1", "--metric-only"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["process_group"] == "nccl"
