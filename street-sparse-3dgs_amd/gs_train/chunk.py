"""TrainChunk: train_single.py's whole per-chunk loop (train_single.py:65-247 with the
OptimizationParams defaults of arguments/__init__.py:86-110) around one train step of
gs_train.harness (TrainStep, NativeTrainStep or the reference-structured ReferenceTrainStep).

Per iteration, in the reference's order:
  1. learning-rate schedules (inside the step: update_learning_rate, scene/gaussian_model.py:447-457)
  2. every `sh_interval` (1000) iterations one more SH degree, up to the model's (:104-106,
     scene/gaussian_model.py:158-160)
  3. the step's render / loss / backward / densification statistics (:108-194)
  4. while iteration < densify_until_iter: densify_and_prune every densification_interval
     iterations after densify_from_iter (:196-197, min_opacity 0.005), reset_opacity every
     opacity_reset_interval iterations (:199-201, scene/gaussian_model.py:528-532: the skybox rows
     keep theirs).  Both replace the Gaussian nn.Parameters, so the .grad the backward left is gone
     and the reference's sparse Adam does not run in that iteration (:217, :225) -- TrainStep.step's
     `between` hook reproduces exactly that
  5. the optimizers and the scale shrink (inside the step, :211-241)
  6. checkpoints at `checkpoint_iterations` (:243-245: gaussians.capture() + the iteration)

The last iteration (iteration == iterations) renders and back-propagates but the reference returns
before any update (:186-188); it changes nothing, and run() stops after iterations - 1 updates.

The densification statistics are updated every iteration here; the reference stops updating them
at densify_until_iter (:191), after which nothing reads them (only densify_and_prune does).
"""
from __future__ import annotations

import dataclasses
import math
import time

import numpy as np
import torch


@dataclasses.dataclass
class ChunkSchedule:
    """arguments/__init__.py:86-110 (OptimizationParams) + the constants train_single.py hardcodes."""
    iterations: int = 30_000
    densification_interval: int = 300
    opacity_reset_interval: int = 3000
    densify_from_iter: int = 500
    densify_until_iter: int = 15_000
    densify_grad_threshold: float = 0.015
    percent_dense: float = 0.0001
    min_opacity: float = 0.005       # train_single.py:197
    sh_interval: int = 1000          # train_single.py:105
    max_sh_degree: int = 3           # ModelParams.sh_degree
    white_background: bool = False   # ModelParams.white_background (:199: a reset at densify_from_iter)
    checkpoint_iterations: tuple = ()

    def events(self, it):
        """(densify, reset) for iteration `it` (train_single.py:191-201)."""
        if it >= self.densify_until_iter:
            return False, False
        dens = it > self.densify_from_iter and it % self.densification_interval == 0
        reset = it % self.opacity_reset_interval == 0 or (self.white_background and it == self.densify_from_iter)
        return dens, reset


def inverse_sigmoid(x):
    """utils/general_utils.py:19-20."""
    return torch.log(x / (1 - x))


def _reset_values(op, skybox):
    """The reset's new opacity column (scene/gaussian_model.py:528-532), in the reference's torch ops."""
    rest = torch.sigmoid(op[skybox:])
    return torch.cat((op[:skybox], inverse_sigmoid(torch.min(rest, torch.ones_like(rest) * 0.01))), 0)


@torch.no_grad()
def warm_event_ops(device) -> None:
    """Run the opacity reset's torch ops once on a few rows.  torch's ROCm kernels load their code
    objects on first use, ~90 ms for this op sequence (tools/first_call_cost.py, r06a: min 31 ms,
    log / division 40 ms, ...); in a fresh process the first reset (iteration 3000) paid it inside
    its iteration (config 3's slowest iteration, 116-121 ms).  TrainChunk calls this at set-up."""
    op = torch.linspace(-2.0, 2.0, 64, device=device).reshape(64, 1)
    _reset_values(op, 8)
    torch.zeros_like(op)
    torch.nn.Parameter(op.contiguous())


@torch.no_grad()
def reset_opacity(g, optimizer, skybox: int) -> None:
    """scene/gaussian_model.py:528-532 + replace_tensor_to_optimizer (:546-559) on a joined-layout
    GaussianSet and its gs_train.optim.Adam: opacities of the rows after the skybox become
    min(opacity, 0.01) (in logit space), the opacity group's moments restart at zero, its step
    count stays."""
    new = _reset_values(g._opacity.detach(), skybox)
    old = g._opacity
    newp = torch.nn.Parameter(new.contiguous())
    st = optimizer.state.pop(old, None)
    if st is not None:
        st["exp_avg"] = torch.zeros_like(new)
        st["exp_avg_sq"] = torch.zeros_like(new)
        optimizer.state[newp] = st
    for group in optimizer.param_groups:
        group["params"] = [newp if q is old else q for q in group["params"]]
    g._opacity = newp


_PARAMS = ("_xyz", "_features", "_opacity", "_scaling", "_rotation")


def _spread3(x):
    """The low 10 bits of x, two zero bits after each (int64): one axis of a 30-bit Morton code."""
    x = x & 0x3FF
    x = (x | (x << 16)) & 0x30000FF
    x = (x | (x << 8)) & 0x300F00F
    x = (x | (x << 4)) & 0x30C30C3
    x = (x | (x << 2)) & 0x9249249
    return x


def spatial_order(xyz: torch.Tensor) -> torch.Tensor:
    """A stable permutation of the rows of xyz (N, 3) by the 30-bit Morton code of their positions
    quantised to 1024 steps per axis over the rows' bounding box: rows near each other in space end
    up near each other in memory."""
    lo = xyz.min(0).values
    ext = (xyz.max(0).values - lo).clamp_min(1e-12)
    q = ((xyz - lo) / ext * 1023.0).clamp(0.0, 1023.0).to(torch.int64)
    key = _spread3(q[:, 0]) | (_spread3(q[:, 1]) << 1) | (_spread3(q[:, 2]) << 2)
    return torch.argsort(key, stable=True)


@torch.no_grad()
def reorder_rows(ts, first_row: int) -> None:
    """Permute the Gaussians after `first_row` (the skybox and scaffold rows keep their places: the
    skybox lock and the scale shrink address them by index) into spatial order (spatial_order):
    every parameter, its Adam moments and the densification statistics, replaced as densification
    replaces them.  A view then covers runs of adjacent rows instead of rows scattered over the whole
    model, so the per-row passes that touch only its visible rows (the backward's live-row chain
    rule, the sparse Adam step, the preprocess) read and write whole cache lines instead of a line
    per row.  The rendered images and every per-row update are the same up to the permutation."""
    g = ts.g
    P = g.P
    if P - first_row < 2:
        return
    dev = g._xyz.device
    perm = torch.cat((torch.arange(first_row, device=dev),
                      spatial_order(g._xyz.detach()[first_row:]) + first_row))
    opts = [o for o in (getattr(ts, "optimizer", None),) if o is not None]
    for n in _PARAMS:
        old = getattr(g, n)
        newp = torch.nn.Parameter(old.detach().index_select(0, perm).contiguous())
        for opt in opts:
            st = opt.state.pop(old, None)
            if st is not None:
                for key in ("exp_avg", "exp_avg_sq"):
                    if key in st and st[key].shape[:1] == (P,):
                        st[key] = st[key].index_select(0, perm).contiguous()
                opt.state[newp] = st
            for group in opt.param_groups:
                group["params"] = [newp if q is old else q for q in group["params"]]
        setattr(g, n, newp)
    for n in ("max_radii2D", "xyz_gradient_accum", "denom"):
        setattr(g, n, getattr(g, n).index_select(0, perm).contiguous())


def capture(ts) -> dict:
    """gaussians.capture() (scene/gaussian_model.py) for a joined-layout step: every parameter, the
    optimizers' moments and step counts, the densification statistics, the SH degree, the iteration
    and the device generator's state (the per-iteration random background) -- tensors only, so
    torch.load(..., weights_only=True) reads it back."""
    g = ts.g
    out = {"iteration": torch.tensor(ts.iteration), "active_sh_degree": torch.tensor(g.active_sh_degree),
           "rng": torch.cuda.get_rng_state(g._xyz.device)}
    for n in _PARAMS + ("_exposure",):
        out["param" + n] = getattr(g, n).detach().clone()
    for n in ("max_radii2D", "xyz_gradient_accum", "denom"):
        out[n] = getattr(g, n).clone()
    for tag, opt in (("opt", ts.optimizer), ("expopt", ts.exposure_optimizer)):
        for k, group in enumerate(opt.param_groups):
            st = opt.state.get(group["params"][0], {})
            for key in ("step", "exp_avg", "exp_avg_sq"):
                if key in st:
                    out[f"{tag}{k}.{key}"] = st[key].clone()
    return out


@torch.no_grad()
def restore(ts, state: dict) -> None:
    """Load a capture() into a step built on the same views (gaussians.restore): parameters and
    moments are replaced by new tensors, as after densification."""
    g = ts.g
    dev = g._xyz.device
    by_name = {}
    for n in _PARAMS + ("_exposure",):
        old = getattr(g, n)
        newp = torch.nn.Parameter(state["param" + n].to(dev).clone().contiguous())
        setattr(g, n, newp)
        by_name[id(old)] = newp
    for tag, opt in (("opt", ts.optimizer), ("expopt", ts.exposure_optimizer)):
        for k, group in enumerate(opt.param_groups):
            old = group["params"][0]
            newp = by_name[id(old)]
            opt.state.pop(old, None)
            group["params"] = [newp]
            st = {key: state[f"{tag}{k}.{key}"].clone() for key in ("step", "exp_avg", "exp_avg_sq")
                  if f"{tag}{k}.{key}" in state}
            for key in ("exp_avg", "exp_avg_sq"):
                if key in st:
                    st[key] = st[key].to(dev).contiguous()
            if st:
                opt.state[newp] = st
    for n in ("max_radii2D", "xyz_gradient_accum", "denom"):
        setattr(g, n, state[n].to(dev).clone())
    g.active_sh_degree = int(state["active_sh_degree"])
    ts.iteration = int(state["iteration"])
    torch.cuda.set_rng_state(state["rng"], dev)


class TrainChunk:
    """Runs a step object through train_single.py's loop.  `step` must have been built with
    iterations=schedule.iterations (its exposure / depth-weight schedules depend on it).

    normals: optional callable(iteration, n_split) -> (2 n_split, 3) tensor of the standard-normal
    draws behind the split samples (parity tests inject the same draws into two runs); by default
    each run draws them from the device generator as the reference does.
    on_checkpoint: callable(iteration, capture dict).
    spatial: keep the rows after the skybox / scaffold prefix in spatial order (reorder_rows) from the
    start and again after every densification (which appends its clones and splits at the end) --
    a row permutation the reference does not make: the images, losses and per-row updates are the
    reference's up to it, but its split draws go to the split rows in the new index order.  While
    run() runs it also switches the library's backward to its list walk of the live rows
    (gsr_set_live_list, a process-wide knob); the previous setting is restored when run() returns or
    raises, so later work in the process with rows in index order keeps the per-range walk."""

    def __init__(self, step, schedule: ChunkSchedule | None = None, normals=None, on_checkpoint=None,
                 spatial: bool = False):
        self.ts = step
        self.spatial = spatial
        if spatial:
            reorder_rows(step, self._fixed_rows())
        self.sched = schedule or ChunkSchedule()
        warm_event_ops(step.g._xyz.device)
        if getattr(step, "iterations", self.sched.iterations) != self.sched.iterations:
            raise ValueError("the step's schedules were built for a different iteration count")
        self.normals = normals
        self.on_checkpoint = on_checkpoint
        self.events = []       # one dict per densify / reset iteration
        self.event_s = 0.0     # host wall-clock inside the events (synchronised)

    def _fixed_rows(self):
        return max(int(getattr(self.ts, "skybox", 0)), int(getattr(self.ts, "scaffold", 0)))

    def _between(self, it, dens, reset):
        ts, s = self.ts, self.sched

        def run():
            t0 = time.perf_counter()
            rec = {"iteration": it, "P_before": ts.g.P}
            if dens:
                nrm = self.normals
                rec.update(ts.densify_and_prune(s.densify_grad_threshold, s.min_opacity, s.percent_dense,
                                                normals=(lambda n: nrm(it, n)) if nrm is not None else None))
                if self.spatial:
                    reorder_rows(ts, self._fixed_rows())
            t1 = time.perf_counter()
            if reset:
                ts.reset_opacity()
                rec["reset"] = True
            rec["P_after"] = ts.g.P
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rec["ms"] = round((t2 - t0) * 1e3, 3)  # host wall clock of the event (densify part to t1)
            rec["ms_densify"] = round((t1 - t0) * 1e3, 3)
            self.event_s += t2 - t0
            self.events.append(rec)
        return run

    def iteration(self):
        """One train_single.py iteration; returns the step's loss tensor."""
        ts, s = self.ts, self.sched
        it = ts.iteration
        if it % s.sh_interval == 0 and ts.g.active_sh_degree < s.max_sh_degree:
            ts.g.active_sh_degree += 1
        dens, reset = s.events(it)
        loss = ts.step(between=self._between(it, dens, reset) if (dens or reset) else None)
        if it in s.checkpoint_iterations and self.on_checkpoint is not None:
            self.on_checkpoint(it, capture(ts))
        return loss

    def run(self, until=None, callback=None):
        """Iterations from the step's current one up to `until` (default: iterations - 1, the last
        one that updates the model).  callback(iteration, loss tensor) after each."""
        last = self.sched.iterations - 1 if until is None else until
        prev = None
        if self.spatial:
            # a view's live rows come in runs: the backward walks them through one list
            from diff_gaussian_rasterization import _C
            prev = _C.set_live_list(True)
        try:
            while self.ts.iteration <= last:
                it = self.ts.iteration
                loss = self.iteration()
                if callback is not None:
                    callback(it, loss)
        finally:
            if prev is not None:
                _C.set_live_list(prev)


# ---- a synthetic Street-sparse chunk (the config-3 stand-in; the example_dataset is absent) ------

C0 = 0.28209479177387814  # utils/sh_utils.py:26


def rgb2sh(rgb):
    return (rgb - 0.5) / C0


def _yaw_camera(W, H, pos, yaw, fovx_deg):
    from .synthetic import camera
    c, s = math.cos(yaw), math.sin(yaw)
    Rc2w = np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    Rw2c = Rc2w.T
    t = -Rw2c @ np.asarray(pos, np.float64)
    return camera(W, H, fovx_deg, R=Rw2c.T, t=t)


def nerfpp_radius(campos):
    """scene/dataset_readers.py getNerfppNorm: 1.1 x the largest camera distance from their mean."""
    c = np.asarray(campos, np.float64)
    return float(np.linalg.norm(c - c.mean(0), axis=1).max() * 1.1)


def street_scene(n_truth, length, device, seed=0, half_width=7.0, height=8.0, cam_y=0.0, road_y=1.6):
    """A seeded street corridor along +z (camera frame: y down): road plane at y = road_y, facades
    at x = +-half_width up to y = road_y - height, box-shaped clutter on the road; textured colours
    (smooth patterns, so the views are learnable).  Returns activated attributes on `device`."""
    g = torch.Generator(device=device).manual_seed(seed)
    u = lambda *s: torch.rand(*s, generator=g, device=device)
    n_road, n_fac = int(0.35 * n_truth), int(0.5 * n_truth)
    n_obj = n_truth - n_road - n_fac
    z0, z1 = -10.0, length + 10.0
    road = torch.stack([(u(n_road) * 2 - 1) * half_width, torch.full((n_road,), road_y, device=device),
                        z0 + (z1 - z0) * u(n_road)], 1)
    side = torch.where(u(n_fac) < 0.5, -1.0, 1.0)
    fac = torch.stack([side * half_width + 0.05 * (u(n_fac) - 0.5), road_y - height * u(n_fac),
                       z0 + (z1 - z0) * u(n_fac)], 1)
    n_box = max(1, n_obj // 400)
    bc = torch.stack([(u(n_box) * 2 - 1) * (half_width - 2), road_y - 0.75 + 0 * u(n_box), z0 + (z1 - z0) * u(n_box)],
                     1)
    bsz = torch.stack([0.5 + 1.5 * u(n_box), 0.4 + 0.6 * u(n_box), 0.8 + 3.0 * u(n_box)], 1)
    which = torch.randint(0, n_box, (n_obj,), generator=g, device=device)
    face = torch.randint(0, 3, (n_obj,), generator=g, device=device)
    off = (u(n_obj, 3) * 2 - 1)
    off[torch.arange(n_obj, device=device), face] = torch.where(u(n_obj) < 0.5, -1.0, 1.0)
    obj = bc[which] + off * bsz[which]
    means = torch.cat([road, fac, obj])
    n = means.shape[0]
    # scales: flat discs on the road / facades, small blobs on the boxes
    base = torch.exp(-3.3 + 0.4 * torch.randn(n, 3, generator=g, device=device))
    base[:n_road, 1] *= 0.1
    base[n_road:n_road + n_fac, 0] *= 0.1
    q = torch.randn(n, 4, generator=g, device=device) * 0.15
    q[:, 0] += 1.0
    q = q / q.norm(dim=1, keepdim=True)
    opac = 0.5 + 0.45 * u(n, 1)
    p = means
    pattern = torch.stack([0.5 + 0.35 * torch.sin(0.9 * p[:, 2] + 0.7 * p[:, 1]),
                           0.5 + 0.3 * torch.sin(0.5 * p[:, 0] - 1.1 * p[:, 2]),
                           0.5 + 0.3 * torch.cos(0.8 * p[:, 1] + 0.4 * p[:, 2])], 1)
    tint = torch.cat([torch.full((n_road, 3), 0.35, device=device), torch.full((n_fac, 3), 0.6, device=device),
                      u(n_obj, 3)])
    rgb = (0.5 * pattern + 0.5 * tint + 0.05 * torch.randn(n, 3, generator=g, device=device)).clamp(0.02, 0.98)
    shs = torch.zeros(n, 16, 3, device=device)
    shs[:, 0] = rgb2sh(rgb)
    shs[:, 1:] = 0.02 * torch.randn(n, 15, 3, generator=g, device=device)
    return dict(means3D=means.contiguous(), scales=base.contiguous(), rotations=q.contiguous(),
                opacities=opac.contiguous(), shs=shs.contiguous(), rgb=rgb)


def street_chunk(step_cls=None, W=1536, H=1536, positions=48, faces=4, depth_only_every=4, n_truth=1_000_000,
                 n_init=300_000, skybox=10_000, n_scaffold=20_000, spacing=1.5, seed=0, device="cuda",
                 iterations=30_000, lidar_keep=0.3, alpha=True):
    """A synthetic Street-sparse chunk (the config-3 stand-in): `positions` camera stations along the
    street, `faces` 90-degree cube faces each (ss_utils/generate_colmap_calibration.py:476-479,572:
    W x H faces with f = W / 2), plus one depth-only view (a LiDAR-like sparse inverse-depth map,
    Street-sparse's additional depth maps) every `depth_only_every` stations.  Targets are rendered
    from a seeded truth street (street_scene); every photometric view has a mono inverse-depth map
    (5% multiplicative noise) and an alpha mask.  Views are shuffled once, as Scene does
    (scene/__init__.py:63-64), and the exposure index is the view's position in that order.

    The initial Gaussians follow create_from_pcd with a scaffold_file (scene/gaussian_model.py:
    163-278): [skybox | coarse scaffold] rows first (scaffold_points = both, skybox_points the first
    ones), then `n_init` LiDAR-like points (truth surface points + 3 cm noise) with SH DC from their
    colour, distCUDA2 scales, identity rotations and opacity 0.01.  Returns (step, info)."""
    from .harness import GaussianSet, TrainStep
    from simple_knn._C import distCUDA2
    step_cls = step_cls or TrainStep
    dev = torch.device(device)
    rng = np.random.default_rng(seed + 5)
    length = spacing * (positions - 1)
    truth = street_scene(n_truth, length, dev, seed=seed)
    # views: stations along z, cube faces by yaw; depth-only views half-way between stations
    views = []
    for k in range(positions):
        pos = (0.0, 0.0, spacing * k)
        for f in range(faces):
            views.append((_yaw_camera(W, H, pos, 2 * math.pi * f / faces, 90.0), False))
        if depth_only_every and k % depth_only_every == depth_only_every // 2:
            yaw = 2 * math.pi * rng.integers(0, faces) / faces
            views.append((_yaw_camera(W, H, (0.0, 0.0, spacing * (k + 0.5)), yaw, 90.0), True))
    order = rng.permutation(len(views))
    views = [views[i] for i in order]
    cams = [v[0] for v in views]
    donly = [v[1] for v in views]
    n = len(cams)
    # targets from the truth scene
    tg = GaussianSet(truth["means3D"].cpu().numpy(), truth["shs"].cpu().numpy(), truth["opacities"].cpu().numpy(),
                     truth["scales"].cpu().numpy(), truth["rotations"].cpu().numpy(), n_images=n, sh_degree=3,
                     device=dev, joined_features=True)
    tmp = TrainStep(tg, cams, [None] * n, W, H)
    gen = torch.Generator(device=dev).manual_seed(seed + 7)
    gts, monos, dmasks, amasks = [], [], [], []
    with torch.no_grad():
        for k in range(n):
            img, invd, _, _ = tmp.render(k, torch.zeros(3, device=dev))
            if donly[k]:
                keep = (torch.rand(invd.shape, generator=gen, device=dev) < lidar_keep).float()
                monos.append((invd * keep).contiguous())
                gts.append(None)
                amasks.append(None)
                dmasks.append(None)  # depth_mask = the alpha mask = ones (scene/cameras.py:54,80)
            else:
                gts.append(img.contiguous())
                noise = 1.0 + 0.05 * torch.randn(invd.shape, generator=gen, device=dev)
                monos.append((invd * noise).contiguous())
                am = (torch.rand(invd.shape, generator=gen, device=dev) < 0.97).float() if alpha else None
                amasks.append(am)
                dmasks.append(am)
    del tmp, tg
    # initial Gaussians: skybox + scaffold (trained coarse rows) + LiDAR-like points
    sel = torch.randperm(truth["means3D"].shape[0], generator=torch.Generator(device=dev).manual_seed(seed + 11),
                         device=dev)
    pts = truth["means3D"][sel[:n_init]] + 0.03 * torch.randn(n_init, 3, device=dev)
    col = (truth["rgb"][sel[:n_init]] + 0.05 * torch.randn(n_init, 3, device=dev)).clamp(0, 1)
    sc_idx = sel[n_init:n_init + n_scaffold]
    th = torch.rand(skybox, device=dev) * 2 * math.pi
    ph = torch.arccos(1.0 - 1.4 * torch.rand(skybox, device=dev))
    center = torch.tensor([0.0, 0.0, length / 2], device=dev)
    sky = torch.stack([200 * torch.cos(th) * torch.sin(ph), -200 * torch.cos(ph), 200 * torch.sin(th) * torch.sin(ph)],
                      1) + center
    dist2 = torch.clamp_min(distCUDA2(pts), 0.0000001)
    m = torch.cat([sky, truth["means3D"][sc_idx], pts]).contiguous()
    shs = torch.zeros(m.shape[0], 16, 3, device=dev)
    shs[:skybox, 0] = rgb2sh(torch.tensor([0.7, 0.8, 0.95], device=dev))
    shs[skybox:skybox + n_scaffold] = truth["shs"][sc_idx]
    shs[skybox:skybox + n_scaffold, 4:] = 0  # the coarse model is degree 1 (train_coarse.py:31)
    shs[skybox + n_scaffold:, 0] = rgb2sh(col)
    scales = torch.cat([torch.full((skybox, 3), 4.0, device=dev), truth["scales"][sc_idx] * 2.0,
                        torch.sqrt(dist2)[:, None].repeat(1, 3)])
    rots = torch.zeros(m.shape[0], 4, device=dev)
    rots[:, 0] = 1
    rots[skybox:skybox + n_scaffold] = truth["rotations"][sc_idx]
    opac = torch.full((m.shape[0], 1), 0.01, device=dev)
    opac[:skybox] = 0.7
    opac[skybox:skybox + n_scaffold] = truth["opacities"][sc_idx]
    campos = [c[2] for c in cams]
    extent = nerfpp_radius(campos)
    model = GaussianSet(m.cpu().numpy(), shs.cpu().numpy(), opac.cpu().numpy(), scales.cpu().numpy(),
                        rots.cpu().numpy(), n_images=n, sh_degree=0, spatial_lr_scale=extent, device=dev,
                        joined_features=getattr(step_cls, "JOINED_FEATURES", True))
    ts = step_cls(model, cams, gts, W, H, cameras_extent=extent, mono_invdepths=monos, depth_masks=dmasks,
                  alpha_masks=amasks, skybox_points=skybox, scaffold_points=skybox + n_scaffold,
                  iterations=iterations, depth_only=donly)
    info = dict(views=n, depth_only_views=int(sum(donly)), P_init=model.P, extent=extent, W=W, H=H,
                truth=int(truth["means3D"].shape[0]))
    return ts, info


@torch.no_grad()
def view_psnr(ts, n=8):
    """Mean PSNR (dB, peak 1) of the step's current model against the targets of its first `n`
    photometric views: render with the view's exposure and a black background (the targets were
    rendered over black), alpha mask applied as in the loss."""
    out = []
    dev = ts.g._xyz.device
    for k in range(len(ts.cams)):
        if ts.depth_only[k]:
            continue
        img, _, _, _ = ts.render(k, torch.zeros(3, device=dev))
        if ts.amask[k] is not None:
            img = img * ts.amask[k]
        mse = torch.mean((img - ts.gts[k]) ** 2).item()
        out.append(10 * math.log10(1.0 / mse) if mse > 0 else float("inf"))
        if len(out) == n:
            break
    return round(float(np.mean(out)), 3) if out else None
