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


class _FakeRasterBackward(torch.autograd.Function):
    """Stands in for the rasterizer + activations backward: produces every leaf gradient through
    gsr_dist.grad_out, as _C.rasterize_gaussians_backward / gs_train.activations do."""

    @staticmethod
    def forward(ctx, xyz, features, opacity, scaling, rotation):
        ctx.keys = [t.data_ptr() for t in (xyz, features, opacity, scaling, rotation)]
        ctx.shapes = [t.shape for t in (xyz, features, opacity, scaling, rotation)]
        return (xyz.sum() + features.sum() + opacity.sum() + scaling.sum() + rotation.sum()).reshape(1)

    @staticmethod
    def backward(ctx, g):
        outs = []
        for k, (key, shape) in enumerate(zip(ctx.keys, ctx.shapes)):
            t = gsr_dist.grad_out(key, shape, g.device)
            t.copy_(g.expand(t.numel()).reshape(shape) * (k + 1))  # the "kernel" writes every element
            outs.append(t)
        return tuple(outs)


def _bucket_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        P = 1000  # rasterizer-shaped: 59 floats per Gaussian
        params = {"xyz": torch.zeros(P, 3), "features": torch.zeros(P, 16, 3), "opacity": torch.zeros(P, 1),
                  "scaling": torch.zeros(P, 3), "rotation": torch.zeros(P, 4)}
        params = {k: torch.nn.Parameter(v) for k, v in params.items()}
        bucket = gsr_dist.GradBucket(params)
        out = {"numel": bucket.flat.numel()}
        for step in range(2):
            for p in params.values():
                p.grad = None
            with bucket.capture():
                loss = _FakeRasterBackward.apply(*params.values()) * float(rank + 1)
                loss.backward()
            out[f"owned{step}"] = all(bucket.owns(p) for p in params.values())
            ptr0 = bucket.flat.data_ptr()
            bucket.allreduce()
            out[f"inplace{step}"] = bucket.flat.data_ptr() == ptr0 and all(bucket.owns(p) for p in params.values())
            out[f"vals{step}"] = [float(p.grad.unique().item()) for p in params.values()]
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_grad_bucket_flat_allreduce_gloo():
    """GradBucket: the leaf gradients land in views of one flat buffer during backward (autograd
    adopts them as .grad, no copy) and one in-place all-reduce sums them across 2 ranks."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r]["numel"] == 1000 * 59
        for step in range(2):
            assert res[r][f"owned{step}"] and res[r][f"inplace{step}"]
            # rank r contributes (r + 1) * (k + 1) for parameter k: summed over ranks 3 * (k + 1)
            assert res[r][f"vals{step}"] == [3.0, 6.0, 9.0, 12.0, 15.0]


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
