"""GPU tests of the backward work split (gsr_set_bwd_segment, render.hip): with a segment length L
the forward checkpoints every pixel's transmittance and accumulated colour / inverse depth every L
list positions of its tile, and the backward replays a tile whose last contributor lies past L as
independent segments.  The split changes only where the replay starts, so:

* forward outputs are bitwise those of the unsplit run;
* gradients meet the same oracle bars as test_gpu_parity.py (GRAD_TOL 5e-5 relative L2) and agree
  with the unsplit run to fp32 rounding (SEG_TOL);
* the record (deterministic) mode stays bitwise reproducible with segments;
* a backward uses the length its forward was made with, whatever the setting is in between.

The scenes are translucent (opacity 0.004 .. 0.012) so that tiles keep thousands of contributors:
tile work well past L, several segments per tile.
"""
from __future__ import annotations

import contextlib

import numpy as np
import pytest

from helpers import deterministic, rel_l2
from test_gpu_parity import compare, make_scene, run_hip, run_oracle, upstream_grads

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _splits_every_frame():
    """The split gate off: every frame of these tests takes the splits it is set up for."""
    from diff_gaussian_rasterization import _C
    prev = _C.set_split_gate(False)
    prev_min = _C.set_fwd_split_min(4 * 4096)  # these scenes' 22k-28k lists take the forward split
    yield
    _C.set_split_gate(prev)
    _C.set_fwd_split_min(prev_min)

SEG_TOL = 1e-5  # segmented vs unsplit gradients, relative L2 (fp32 rounding of S at the checkpoints; measured <= 2.2e-6)

CASES = [
    dict(name="seg_translucent_deg3", P=40000, W=96, H=64, deg=3, seed=21, log_scale=-2.0, opac=(0.004, 0.012)),
    dict(name="seg_translucent_odd_deg1", P=60000, W=150, H=70, deg=1, seed=22, log_scale=-2.1, opac=(0.004, 0.012)),
    dict(name="seg_no_depth", P=40000, W=96, H=64, deg=2, seed=23, log_scale=-2.0, opac=(0.004, 0.012), do_depth=False),
    # opaque splats mixed in: pixels saturate at different segments of the same tile
    dict(name="seg_mixed_opacity", P=40000, W=96, H=64, deg=3, seed=24, log_scale=-2.0, opac=(0.004, 0.012),
         opaque=0.002),
]


def seg_scene(c):
    s = make_scene(c)
    rng = np.random.default_rng(c["seed"] + 7)
    lo, hi = c["opac"]
    op = rng.uniform(lo, hi, (c["P"], 1)).astype(np.float32)
    if c.get("opaque"):
        idx = rng.random(c["P"]) < c["opaque"]
        op[idx] = rng.uniform(0.5, 0.99, (int(idx.sum()), 1)).astype(np.float32)
    s["opacities"] = op
    return s


@contextlib.contextmanager
def bwd_segment(L):
    from diff_gaussian_rasterization import _C
    prev = _C.set_bwd_segment(L)
    try:
        yield
    finally:
        _C.set_bwd_segment(prev)


@contextlib.contextmanager
def fwd_segment(L):
    from diff_gaussian_rasterization import _C
    prev = _C.set_fwd_segment(L)
    try:
        yield
    finally:
        _C.set_fwd_segment(prev)


def max_tile_work(h, c):
    nc = h["state"]["n_contrib"].reshape(c["H"], c["W"])
    gy, gx = (c["H"] + 15) // 16, (c["W"] + 15) // 16
    pad = np.zeros((gy * 16, gx * 16), nc.dtype)
    pad[:c["H"], :c["W"]] = nc
    return int(pad.reshape(gy, 16, gx, 16).max(axis=(1, 3)).max())


@pytest.mark.parametrize("L", [512, 1024])
@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_segments_vs_oracle_and_unsplit(c, L):
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    st, g = run_oracle(s, c, dcol, dinv)
    with bwd_segment(0), fwd_segment(0):
        base = run_hip(s, c, dcol, dinv)
    with bwd_segment(L), fwd_segment(0):
        h = run_hip(s, c, dcol, dinv)
    work = max_tile_work(h, c)
    print(f"{c['name']} L={L}: max tile work {work}")
    assert work > 2 * 1024, f"scene too light for the split: max tile work {work}"
    compare(c, st, g, h)
    # forward untouched (checkpoints are extra writes only)
    np.testing.assert_array_equal(h["color"], base["color"])
    np.testing.assert_array_equal(h["invdepth"], base["invdepth"])
    np.testing.assert_array_equal(h["state"]["n_contrib"], base["state"]["n_contrib"])
    for k, v in h["grads"].items():
        if v is None:
            continue
        err = rel_l2(v, base["grads"][k])
        assert err <= SEG_TOL, (k, err)


def test_segments_deterministic_mode():
    c = CASES[0]
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    st, g = run_oracle(s, c, dcol, dinv)
    with deterministic(), bwd_segment(512), fwd_segment(0):
        h1 = run_hip(s, c, dcol, dinv)
        h2 = run_hip(s, c, dcol, dinv)
    compare(c, st, g, h1)
    for k, v in h1["grads"].items():
        if v is not None:
            np.testing.assert_array_equal(v, h2["grads"][k], err_msg=k)


def test_backward_uses_the_forwards_length():
    """Forward with L = 512, setting switched to 0 (and to 1024) before the backward: the backward
    still cuts tiles at 512 (its items and checkpoints were published that way)."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    from helpers import settings, torch_inputs
    c = CASES[1]
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    st, g = run_oracle(s, c, dcol, dinv)
    dev = torch.device("cuda:0")
    setting = _C.set_bwd_segment(0)
    _C.set_bwd_segment(setting)
    for later in (0, 1024):
        inp = torch_inputs(s, dev)
        rs = settings(s, dev, c["deg"])
        with bwd_segment(512):
            color, radii, invd = GaussianRasterizer(rs)(**inp)
        with bwd_segment(later):
            loss = (color * torch.tensor(dcol, device=dev)).sum() + (invd * torch.tensor(dinv, device=dev)).sum()
            loss.backward()
        torch.cuda.synchronize()
        for hk, ok in (("means3D", "dL_dmeans3D"), ("opacities", "dL_dopacity"), ("shs", "dL_dsh"),
                       ("scales", "dL_dscales"), ("rotations", "dL_drotations")):
            err = rel_l2(inp[hk].grad.detach().cpu().numpy().reshape(g[ok].shape), g[ok])
            assert err <= 5e-5, (later, hk, err)
    assert _C.set_bwd_segment(setting) == setting


def test_set_bwd_segment_validation():
    from diff_gaussian_rasterization import _C
    prev = _C.set_bwd_segment(0)
    try:
        for bad in (-64, 64, 448, 520):
            with pytest.raises(RuntimeError):
                _C.set_bwd_segment(bad)
        assert _C.set_bwd_segment(2048) == 0
        assert _C.set_bwd_segment(512) == 2048
    finally:
        _C.set_bwd_segment(prev)


# ---------------------------------------------------------------------------------------------
# Forward segments (gsr_set_fwd_segment): tiles with lists longer than Lf blended as Lf-position
# items by a worker pool (transmittance products, per-pixel lookback, blend, ordered sum).  The
# colours are the same sums in a different association, and each item's starting transmittance is
# the product of its predecessors' instead of the running product, so the bars are stated for fp32
# reassociation: FWD_PSNR_BAR / FWD_MAXABS on colour and inverse depth, FWD_NC_TOL for n_contrib
# (an ulp of T at the 1e-4 stop test), gradients on the oracle's GRAD_TOL.
FWD_PSNR_BAR = 125.0
FWD_MAXABS = 2e-5
FWD_NC_TOL = 1e-3
GRAD_TOL = 5e-5

FWD_CASES = [
    dict(name="fseg_translucent_deg3", P=130000, W=96, H=64, deg=3, seed=31, log_scale=-2.0, opac=(0.004, 0.012)),
    dict(name="fseg_odd_deg1", P=200000, W=150, H=70, deg=1, seed=32, log_scale=-2.1, opac=(0.004, 0.012)),
    # opaque splats mixed in: pixels stop in different items of one tile
    dict(name="fseg_mixed_opacity", P=130000, W=96, H=64, deg=3, seed=34, log_scale=-2.0, opac=(0.004, 0.012),
         opaque=0.004),
    dict(name="fseg_no_depth", P=130000, W=96, H=64, deg=2, seed=33, log_scale=-2.0, opac=(0.004, 0.012),
         do_depth=False),
]



def fwd_compare(c, st, g, h, base=None):
    from helpers import psnr
    assert h["K"] == st["K"]
    np.testing.assert_array_equal(h["radii"], st["radii"])
    S = h["state"]
    np.testing.assert_array_equal(S["point_list"], st["point_list"])
    np.testing.assert_array_equal(S["ranges"], st["ranges"])
    nc_bad = float(np.mean(S["n_contrib"] != st["n_contrib"]))
    p_img = psnr(h["color"], st["color"])
    mx = float(np.abs(h["color"] - st["color"]).max())
    m = dict(nc_bad=nc_bad, psnr=p_img, maxabs=mx)
    if c.get("do_depth", True):
        m["inv_maxabs"] = float(np.abs(h["invdepth"] - st["invdepth"]).max() / max(1e-30, np.abs(st["invdepth"]).max()))
    G = h["grads"]
    for hk, ok in (("means3D", "dL_dmeans3D"), ("means2D", "dL_dmeans2D"), ("opacities", "dL_dopacity"),
                   ("shs", "dL_dsh"), ("scales", "dL_dscales"), ("rotations", "dL_drotations")):
        m["grad_" + hk] = rel_l2(G[hk].reshape(g[ok].shape), g[ok])
    print(c["name"], m)
    assert nc_bad <= FWD_NC_TOL, m
    assert p_img >= FWD_PSNR_BAR, m
    assert mx <= FWD_MAXABS, m
    if "inv_maxabs" in m:
        assert m["inv_maxabs"] <= FWD_MAXABS, m
    for k, v in m.items():
        if k.startswith("grad_"):
            assert v <= GRAD_TOL, (k, m)


@pytest.mark.parametrize("Lf", [4096, 2048])  # 2048: the default since r05 (twice the items per tile)
@pytest.mark.parametrize("bwd_L", [0, 512])
@pytest.mark.parametrize("c", FWD_CASES, ids=[c["name"] for c in FWD_CASES])
def test_fwd_segments_vs_oracle(c, bwd_L, Lf):
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    st, g = run_oracle(s, c, dcol, dinv)
    lens = np.diff(st["ranges"].astype(np.int64), axis=1)
    assert lens.max() > 4 * 4096, f"lists too short for the split (4 segments): {lens.max()}"
    with fwd_segment(Lf), bwd_segment(bwd_L):
        h = run_hip(s, c, dcol, dinv)
    fwd_compare(c, st, g, h)


def test_fwd_segments_deterministic_and_repeatable():
    """Record mode with both splits: two runs bitwise equal (the item order of the worker pool
    varies run to run; every sum is in segment order regardless)."""
    c = FWD_CASES[0]
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    st, g = run_oracle(s, c, dcol, dinv)
    with deterministic(), fwd_segment(4096), bwd_segment(512):
        h1 = run_hip(s, c, dcol, dinv)
        h2 = run_hip(s, c, dcol, dinv)
    fwd_compare(c, st, g, h1)
    np.testing.assert_array_equal(h1["color"], h2["color"])
    np.testing.assert_array_equal(h1["state"]["n_contrib"], h2["state"]["n_contrib"])
    for k, v in h1["grads"].items():
        if v is not None:
            np.testing.assert_array_equal(v, h2["grads"][k], err_msg=k)


@pytest.mark.parametrize("c", [FWD_CASES[0], FWD_CASES[2]], ids=[FWD_CASES[0]["name"], FWD_CASES[2]["name"]])
def test_fwd_workers_launched_ahead_equal_beside(c, monkeypatch):
    """GSR_FWD_EARLY_WORKERS=1 launches the worker pool before tile_order (waiting for its queue
    release); the items, their order of sums and so the frame are those of the pool launched beside
    render_fwd: record mode bitwise equal, and the oracle's bars."""
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    st, g = run_oracle(s, c, dcol, dinv)
    out = {}
    for e in ("1", "0", "1"):
        monkeypatch.setenv("GSR_FWD_EARLY_WORKERS", e)
        with deterministic(), fwd_segment(4096), bwd_segment(512):
            out.setdefault(e, []).append(run_hip(s, c, dcol, dinv))
    fwd_compare(c, st, g, out["1"][0])
    for h in (out["0"][0], out["1"][1]):
        np.testing.assert_array_equal(out["1"][0]["color"], h["color"])
        np.testing.assert_array_equal(out["1"][0]["state"]["n_contrib"], h["state"]["n_contrib"])
        for k, v in out["1"][0]["grads"].items():
            if v is not None:
                np.testing.assert_array_equal(v, h["grads"][k], err_msg=k)


def test_fwd_segments_no_backward_forward():
    """A no-grad forward (no backward state) with the forward split: same image."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizer
    from helpers import settings, torch_inputs
    c = FWD_CASES[1]
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    st, _ = run_oracle(s, c, dcol, dinv)
    dev = torch.device("cuda:0")
    inp = torch_inputs(s, dev, requires_grad=False)
    with torch.no_grad(), fwd_segment(4096):
        color, _, invd = GaussianRasterizer(settings(s, dev, c["deg"]))(**inp)
    err = float(np.abs(color.cpu().numpy() - st["color"]).max())
    assert err <= FWD_MAXABS, err


def test_set_fwd_segment_validation():
    from diff_gaussian_rasterization import _C
    prev = _C.set_fwd_segment(0)
    try:
        for bad in (-64, 512, 960, 2000, 4097):
            with pytest.raises(RuntimeError):
                _C.set_fwd_segment(bad)
        assert _C.set_fwd_segment(8192) == 0
        assert _C.set_fwd_segment(4096) == 8192
    finally:
        _C.set_fwd_segment(prev)


def test_split_gate_arms_after_a_long_list_frame():
    """Gate on: the first frame of long lists runs unsplit and reports its lengths; the frames after
    it take the tile binning split (frame_stats counts its items) and the forward split; a scene
    with short lists never arms them."""
    import torch
    from diff_gaussian_rasterization import _C
    from helpers import settings, torch_inputs
    dev = torch.device("cuda:0")

    def frame(c):
        s = seg_scene(c)
        inp = torch_inputs(s, dev, requires_grad=False)
        rs = settings(s, dev, c["deg"])
        e = torch.empty(0, device=dev)
        raw = _C.rasterize_gaussians(rs.bg, inp["means3D"], e, inp["opacities"], inp["scales"], inp["rotations"],
                                     1.0, e, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, c["H"], c["W"],
                                     inp["shs"], c["deg"], rs.campos, False, False, rs.render_indices,
                                     rs.parent_indices, rs.interpolation_weights, rs.num_node_kids, True)
        torch.cuda.synchronize()
        return _C.frame_stats(raw[4], c["P"], c["H"], c["W"]), raw[1].cpu().numpy()

    _C.set_split_gate(True)
    _C.reset_capacity_hint()
    short = dict(name="short", P=2000, W=96, H=64, deg=1, seed=5, log_scale=-3.0, opac=(0.3, 0.9))
    for _ in range(2):
        st, _ = frame(short)
        assert st["tb_split_items"] == 0
    long_ = FWD_CASES[0]
    st1, img1 = frame(long_)
    assert st1["max_sb_list"] > 16384 and st1["tb_split_items"] == 0  # the first long frame: gate closed
    st2, img2 = frame(long_)
    assert st2["tb_split_items"] > 0  # armed by the frame before
    np.testing.assert_allclose(img2, img1, rtol=0, atol=FWD_MAXABS)  # forward split: same image
    _C.reset_capacity_hint()
    st3, _ = frame(long_)
    assert st3["tb_split_items"] == 0


def test_split_frame_capacity_rerun_matches():
    """A long-list frame whose K exceeds the capacity hint, with the forward split (workers
    launched ahead of tile_order) and the superblock split armed: the first pass's workers, tile
    order and render leave at the capacity test and the frame is binned and rendered again at K.
    Record mode: bitwise the same frame as the next one, which fits the hint."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizer, _C
    from helpers import settings, torch_inputs
    dev = torch.device("cuda:0")
    c = FWD_CASES[0]
    s = seg_scene(c)
    short = seg_scene(dict(name="short", P=2000, W=96, H=64, deg=1, seed=5, log_scale=-3.0, opac=(0.3, 0.9)))

    def frame(sc, deg):
        inp = torch_inputs(sc, dev)
        for v in inp.values():
            v.requires_grad_(True)
        color, _, invd = GaussianRasterizer(settings(sc, dev, deg))(**inp)
        g = torch.Generator(device=dev).manual_seed(3)
        (color * torch.randn(color.shape, generator=g, device=dev)).sum().backward()
        torch.cuda.synchronize()
        return [color.detach(), invd.detach()] + [inp[k].grad for k in ("means3D", "shs", "opacities", "scales")]

    reruns = lambda: _C.forward_stats()["reruns"]
    with deterministic(), fwd_segment(4096), bwd_segment(512):
        _C.reset_capacity_hint()
        for _ in range(2):
            frame(short, 1)
        r0 = reruns()
        a = frame(s, c["deg"])  # K far above the hint: binned and rendered twice
        r1 = reruns()
        b = frame(s, c["deg"])
        r2 = reruns()
    assert (r1 - r0, r2 - r1) == (1, 0)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@contextlib.contextmanager
def fwd_spin_limits(ready=0, flag=0):
    from diff_gaussian_rasterization import _C
    _C.set_fwd_spin_limits(ready, flag)
    try:
        yield
    finally:
        _C.set_fwd_spin_limits(0, 0)


def test_fwd_workers_that_give_up_on_the_queue_leave_the_frame_exact(monkeypatch):
    """The early pool's workers wait for tile_order's release of the queue on another stream; if they
    give up (here: a ready-spin limit of one trip, as when the two streams do not run concurrently),
    they are counted (forward_stats) and the pool's second launch after render_fwd blends every item:
    record mode, the frame bitwise the normal one's.  ready = -1 makes every worker leave at once
    (normally tile_order has released the queue before the side stream's workers even start)."""
    from diff_gaussian_rasterization import _C
    monkeypatch.setenv("GSR_FWD_EARLY_WORKERS", "1")
    c = FWD_CASES[0]
    s = seg_scene(c)
    dcol, dinv = upstream_grads(c)
    with deterministic(), fwd_segment(4096), bwd_segment(512):
        ref = run_hip(s, c, dcol, dinv)
        g0 = _C.forward_stats()["fwd_worker_giveups"]
        with fwd_spin_limits(ready=-1):
            h = run_hip(s, c, dcol, dinv)
        g1 = _C.forward_stats()["fwd_worker_giveups"]
    assert g1 > g0, "no worker gave up: the test did not exercise the second launch"
    assert not np.isnan(h["color"]).any()
    np.testing.assert_array_equal(h["color"], ref["color"])
    np.testing.assert_array_equal(h["state"]["n_contrib"], ref["state"]["n_contrib"])
    for k, v in h["grads"].items():
        if v is not None:
            np.testing.assert_array_equal(v, ref["grads"][k], err_msg=k)


def test_fwd_worker_predecessor_timeout_fails_loudly():
    """A worker whose wait for a predecessor segment times out (never expected: a flag-spin limit of
    one trip forces it here) leaves NaN pixels in its tile and sets the sticky device error word: the
    next rasterizer call raises RuntimeError instead of training on the frame; after it, calls work."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizer
    from helpers import settings, torch_inputs
    dev = torch.device("cuda:0")
    c = FWD_CASES[0]
    s = seg_scene(c)
    inp = torch_inputs(s, dev, requires_grad=False)
    r = GaussianRasterizer(settings(s, dev, c["deg"]))
    with fwd_segment(4096):
        with fwd_spin_limits(flag=1):
            with torch.no_grad():
                color, _, _ = r(**inp)
            torch.cuda.synchronize()
        assert torch.isnan(color).any(), "no predecessor wait timed out"
        with pytest.raises(RuntimeError, match="forward split"):
            with torch.no_grad():
                r(**inp)
        with torch.no_grad():
            color2, _, _ = r(**inp)
        torch.cuda.synchronize()
    assert not torch.isnan(color2).any()
