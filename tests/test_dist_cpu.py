"""world_size-2 gloo tests of the multi-GPU paths on CPU:
chunk-per-rank sharding with a MAX timing reduction, and the optional data-parallel flat
all-reduce of Gaussian gradients + densify statistics."""
from __future__ import annotations

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import gsr_dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        out["chunks"] = gsr_dist.chunk_assignment(5, world, rank)
        out["max"] = gsr_dist.max_over_ranks(float(rank + 1))
        torch.manual_seed(rank)
        params = [torch.zeros(6, 3, requires_grad=True), torch.zeros(6, 16, 3, requires_grad=True),
                  torch.zeros(6, 1, requires_grad=True)]
        for p in params:
            p.grad = torch.full_like(p, float(rank + 1))
        gsr_dist.allreduce_gaussian_grads(params)
        out["grad_sums"] = [float(p.grad.unique().item()) for p in params]
        radii = torch.tensor([rank, 5 - rank, 3], dtype=torch.float32)
        acc = torch.tensor([[0.1 * rank], [0.2], [0.3 * (1 - rank)]])
        den = torch.ones(3, 1)
        gsr_dist.allreduce_densify_stats(radii, acc, den)
        out["radii"] = radii.tolist()
        out["acc"] = acc.flatten().tolist()
        out["den"] = den.flatten().tolist()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_chunk_sharding_and_dp_allreduce_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0]["chunks"] == [0, 2, 4] and res[1]["chunks"] == [1, 3]
    for r in range(world):
        assert res[r]["max"] == 2.0
        assert res[r]["grad_sums"] == [3.0, 3.0, 3.0]
        assert res[r]["radii"] == [1.0, 5.0, 3.0]
        assert res[r]["den"] == [2.0, 2.0, 2.0]
        assert abs(res[r]["acc"][0] - 0.1) < 1e-6 and abs(res[r]["acc"][2] - 0.3) < 1e-6


def test_single_process_is_a_noop():
    p = torch.zeros(3, requires_grad=True)
    p.grad = torch.ones(3)
    gsr_dist.allreduce_gaussian_grads([p])
    assert torch.equal(p.grad, torch.ones(3))
    assert gsr_dist.max_over_ranks(4.0) == 4.0
    assert gsr_dist.chunk_assignment(3, 1, 0) == [0, 1, 2]
