"""Train-step harness: one iteration of the train_single.py inner loop
(train_single.py:65-247) on the MI355X path, used for the "train-step ms" half of the metric.

Per step, as the reference does it:
  1. learning-rate schedules: xyz and exposure (scene/gaussian_model.py:447-457,
     utils/general_utils.py:31-70)
  2. render(): activations of the raw parameters (scene/gaussian_model.py:39-47,125-156),
     GaussianRasterizer (drop-in), per-image exposure affine and clamp
     (gaussian_renderer/__init__.py:115-120); cameras cycle over the training views
  3. image *= alpha_mask when the view has one (train_single.py:117-119)
  4. photometric loss (1 - 0.2) L1 + 0.2 (1 - SSIM) (train_single.py:121-123), plus the masked
     inverse-depth L1 w(it) |(invDepth - mono_invdepth) * depth_mask|.mean() when the view has a
     mono depth map (train_single.py:133-141, w = depth_l1_weight: 1.0 -> 0.01 log-linear)
  5. loss.backward()
  6. densification statistics (train_single.py:193-194)
  7. exposure Adam step; the locked skybox rows' gradients zeroed (train_single.py:217-223);
     sparse Adam on rows with nonzero opacity gradient (train_single.py:225-233);
     zero_grad(set_to_none=True)
  8. shrink over-large Gaussians (train_single.py:235-241)

Every piece runs on the csrc/train.hip kernels and the step is free of host synchronisation (the
reference's .item() calls feed only its progress bar).  The reference-structured formulation of
the same step (conv2d SSIM, OurAdam gather/scatter, ...) lives in oracle/train_torch_ref.py
(ReferenceTrainStep, test infrastructure and the bench's baseline leg) and overrides the hook
methods below.  Densify/prune, opacity reset, SH degree increments and checkpointing run every
few hundred/thousand iterations: gs_train.chunk.TrainChunk runs train_single.py's whole loop around
this step (step(between=...) hands it the point between the statistics and the optimizers).

Depth-only views (Street-sparse's additional depth maps, train_single.py:69-72,145-161,203-214):
the loss is depth_l1_weight * (a * mean(clamp(mono - invD, 0)) + (1 - a) * |(invD - mono) *
mask|.mean()) with a = additional_depth_maps_weight; the image is in no loss (no colour gradient),
the SH gradients are zeroed and the exposure optimizer does not step.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

from .activations import activate, shrink_scales
from .densify import add_densification_stats
from .exposure import apply_exposure
from .loss import depth_l1_loss, depth_only_loss, photo_loss
from .optim import Adam

# arguments/__init__.py:89-109 (OptimizationParams defaults)
LR = dict(position_lr_init=0.00002, position_lr_final=0.0000002, position_lr_delay_mult=0.01,
          position_lr_max_steps=30_000, feature_lr=0.0025, opacity_lr=0.05, scaling_lr=0.005, rotation_lr=0.001,
          exposure_lr_init=0.001, exposure_lr_final=0.0001, exposure_lr_delay_steps=5000,
          exposure_lr_delay_mult=0.001, depth_l1_weight_init=1.0, depth_l1_weight_final=0.01, iterations=30_000,
          lambda_dssim=0.2)
ADDITIONAL_DEPTH_MAPS_WEIGHT = 0.9  # arguments/__init__.py:71


def expon_lr(step, lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1_000_000):
    """utils/general_utils.py:31-70 (log-linear decay with an optional cosine warm-up)."""
    if lr_init == 0 or step < 0 or (lr_init == 0.0 and lr_final == 0.0):
        return 0.0
    if lr_delay_steps > 0:
        delay = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
    else:
        delay = 1.0
    t = np.clip(step / max_steps, 0, 1)
    return float(delay * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t))


class GaussianSet:
    """The raw parameters and activations of scene/gaussian_model.py the train step touches.

    joined_features=False keeps the reference's layout: _features_dc (P,1,3) and
    _features_rest (P,15,3) parameters, concatenated by get_features every step.
    joined_features=True keeps ONE (P,16,3) parameter `_features` (_features_dc/_rest are views):
    get_features is that tensor, the rasterizer's SH gradient lands in it without a split, and
    the fused Adam applies f_dc's and f_rest's learning rates to its column blocks
    (optim.Adam column_lrs).  Same arithmetic, 384 MB less HBM traffic per 1M-Gaussian step."""

    def __init__(self, means3D, shs, opacities, scales, rotations, n_images=1, sh_degree=3, spatial_lr_scale=1.0,
                 device="cuda", joined_features=False):
        t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32, device=device).contiguous()
        shs = t(shs)
        op = t(opacities).clamp(1e-6, 1 - 1e-6)
        P = shs.shape[0]
        self._xyz = torch.nn.Parameter(t(means3D))
        self.joined = joined_features
        if joined_features:
            self._features = torch.nn.Parameter(shs.contiguous())
        else:
            self._features_dc = torch.nn.Parameter(shs[:, :1].contiguous())
            self._features_rest = torch.nn.Parameter(shs[:, 1:].contiguous())
        self._opacity = torch.nn.Parameter(torch.log(op / (1 - op)))  # inverse_sigmoid
        self._scaling = torch.nn.Parameter(torch.log(t(scales)))
        self._rotation = torch.nn.Parameter(t(rotations))
        self._exposure = torch.nn.Parameter(torch.eye(3, 4, device=device)[None].repeat(n_images, 1, 1))
        self.active_sh_degree = sh_degree
        self.spatial_lr_scale = spatial_lr_scale
        self.max_radii2D = torch.zeros(P, device=device)
        self.xyz_gradient_accum = torch.zeros((P, 1), device=device)
        self.denom = torch.zeros((P, 1), device=device)

    @property
    def P(self):
        return self._xyz.shape[0]

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self._rotation)

    @property
    def get_xyz(self):
        return self._xyz

    def __getattr__(self, name):
        # joined layout: the reference's two SH parameters as views of the one buffer
        if name in ("_features_dc", "_features_rest") and self.__dict__.get("joined"):
            f = self.__dict__["_features"]
            return f[:, :1] if name == "_features_dc" else f[:, 1:]
        raise AttributeError(name)

    @property
    def get_features(self):
        if self.joined:
            return self._features
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    def param_groups(self):
        s = self.spatial_lr_scale
        return [
            {"params": [self._xyz], "lr": LR["position_lr_init"] * s, "name": "xyz"},
            *([{"params": [self._features], "lr": LR["feature_lr"], "name": "f_dc+f_rest",
                "column_lrs": [(0, 3, LR["feature_lr"]), (3, self._features[0].numel(), LR["feature_lr"] / 20.0)]}]
              if self.joined else
              [{"params": [self._features_dc], "lr": LR["feature_lr"], "name": "f_dc"},
               {"params": [self._features_rest], "lr": LR["feature_lr"] / 20.0, "name": "f_rest"}]),
            {"params": [self._opacity], "lr": LR["opacity_lr"], "name": "opacity"},
            {"params": [self._scaling], "lr": LR["scaling_lr"], "name": "scaling"},
            {"params": [self._rotation], "lr": LR["rotation_lr"], "name": "rotation"},
        ]


class TrainStep:
    """cameras: list of (view, proj, campos, tanfovx, tanfovy) numpy tuples (synthetic.camera);
    gts: list of (3, H, W) device tensors.  Optional per view: mono_invdepths (1, H, W),
    depth_masks (1, H, W) float 0/1 (None entries = no depth supervision for that view) and
    alpha_masks (1, H, W).  skybox_points: the first rows are the locked skybox
    (scene/gaussian_model.py:73-74,182-187).  scaffold_points: the first rows are the coarse
    scaffold (scene/gaussian_model.py:224-262, loaded with a scaffold_file), which the scale shrink
    leaves alone (train_single.py:239-240: violators[:scaffold_points] = False).  depth_only: per
    view, True for a depth-only view (its gts entry may be None; it needs a mono inverse-depth map);
    dens_weight: additional_depth_maps_weight."""

    def __init__(self, gaussians: GaussianSet, cameras, gts, W, H, cameras_extent=10.0, mono_invdepths=None,
                 depth_masks=None, alpha_masks=None, skybox_points=0, scaffold_points=0,
                 iterations=LR["iterations"], depth_only=None, dens_weight=ADDITIONAL_DEPTH_MAPS_WEIGHT):
        self.g = gaussians
        self.W, self.H = W, H
        self.extent = cameras_extent
        self.gts = gts
        n = len(cameras)
        self.mono = mono_invdepths if mono_invdepths is not None else [None] * n
        self.dmask = depth_masks if depth_masks is not None else [None] * n
        self.amask = alpha_masks if alpha_masks is not None else [None] * n
        self.depth_only = [bool(v) for v in depth_only] if depth_only is not None else [False] * n
        if len(self.depth_only) != n:
            raise ValueError("depth_only: one flag per view")
        for k, d in enumerate(self.depth_only):
            if d and self.mono[k] is None:
                raise ValueError(f"view {k}: a depth-only view needs its inverse-depth map")
        self.dens_weight = float(dens_weight)
        self.skybox = int(skybox_points)
        self.scaffold = int(scaffold_points)
        dev = gaussians._xyz.device
        f = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32, device=dev)
        self.cams = [dict(view=f(v).reshape(4, 4), proj=f(p).reshape(4, 4), campos=f(c), tx=float(tx), ty=float(ty))
                     for (v, p, c, tx, ty) in cameras]
        self._make_optimizers(gaussians.param_groups())
        s = gaussians.spatial_lr_scale
        self.xyz_lr = lambda it: expon_lr(it, LR["position_lr_init"] * s, LR["position_lr_final"] * s,
                                          lr_delay_mult=LR["position_lr_delay_mult"],
                                          max_steps=LR["position_lr_max_steps"])
        self.exposure_lr = lambda it: expon_lr(it, LR["exposure_lr_init"], LR["exposure_lr_final"],
                                               lr_delay_steps=LR["exposure_lr_delay_steps"],
                                               lr_delay_mult=LR["exposure_lr_delay_mult"], max_steps=iterations)
        self.depth_weight = lambda it: expon_lr(it, LR["depth_l1_weight_init"], LR["depth_l1_weight_final"],
                                                max_steps=iterations)
        self.iterations = int(iterations)
        self.iteration = 1
        self._means2D = None
        self._one = None
        self.empty_i = torch.empty(0, dtype=torch.int32)
        self.empty_f = torch.empty(0, device=dev)
        self.empty_id = torch.empty(0, dtype=torch.int32, device=dev)

    # ---- the pieces (fused kernels here; oracle/train_torch_ref.py restates them in torch) ----
    def _make_optimizers(self, groups):
        if not self.g.joined:
            raise ValueError("the fused step keeps the SH coefficients as one (P, 16, 3) parameter")
        self.optimizer = Adam(groups, lr=0.0, eps=1e-15)
        # the reference's torch.optim.Adam on the exposures, as one dense launch of the fused kernel
        # (OurAdam's arithmetic: exp_avg by mul + add where torch's foreach Adam lerps -- an
        # ulp-level difference on 12 floats per image)
        self.exposure_optimizer = Adam([self.g._exposure], lr=LR["exposure_lr_init"], eps=1e-8)

    def _means2D_leaf(self):
        # the rasterizer never reads means2D's values (it only carries dL/dmeans2D): one zero leaf
        # per Gaussian count, its .grad reset each step
        g = self.g
        if self._means2D is None or self._means2D.shape != g._xyz.shape:
            self._means2D = torch.zeros_like(g._xyz, requires_grad=True)
        self._means2D.grad = None
        return self._means2D

    def _activations(self):
        g = self.g
        return activate(g._scaling, g._rotation, g._opacity)

    def _apply_exposure(self, color, E):
        return apply_exposure(color, E)

    def _photo_loss(self, image, gt):
        return photo_loss(image, gt, LR["lambda_dssim"])[0]

    def _depth_loss(self, invd, mono, mask, w):
        return depth_l1_loss(invd, mono, mask, w)

    def _depth_only_loss(self, invd, mono, mask, w):
        return depth_only_loss(invd, mono, mask, w, self.dens_weight)[0]

    def _zero_feature_grads(self):
        # train_single.py:203-207 (the exposure gradient of :208-209 never exists here: the image is
        # in no loss)
        g = self.g._features.grad
        if g is not None:
            g.zero_()

    def _backward(self, loss):
        if self._one is None:
            self._one = torch.ones((), device=loss.device)
        loss.backward(self._one)  # = loss.backward() without the ones_like fill launch

    def _densify_stats(self, radii, grad2d):
        g = self.g
        add_densification_stats(radii, grad2d, g.max_radii2D, g.xyz_gradient_accum, g.denom)

    def _lock_skybox(self):
        # train_single.py:217-223 zeroes all six gradients of the skybox rows.  The rows then have a
        # zero opacity gradient, so the sparse step skips them; the other gradients matter only in
        # the dense fallback (no relevant row at all), which reads every row
        for p in self.optimizer.param_groups:
            for t in p["params"]:
                if t.grad is not None and t.shape[0] == self.g.P:
                    t.grad[:self.skybox] = 0

    def _sparse_step(self):
        self.optimizer.step(relevance=self.g._opacity.grad)

    def _shrink(self):
        shrink_scales(self.g._scaling, self.extent * 0.02, first_row=self.scaffold)

    # ---- the loop's events (gs_train.chunk.TrainChunk; train_single.py:196-201) ----
    def densify_and_prune(self, max_grad, min_opacity, percent_dense, normals=None):
        """gaussians.densify_and_prune(max_grad, min_opacity, cameras_extent, False) on the device
        (gs_train.densify).  normals: callable(n_split) -> the split draws, or None."""
        from .densify import densify_and_prune
        return densify_and_prune(self.g, self.optimizer, max_grad, min_opacity, self.extent, percent_dense,
                                 first_row=self.scaffold, normals=normals)

    def reset_opacity(self):
        from .chunk import reset_opacity
        reset_opacity(self.g, self.optimizer, self.skybox)

    def render(self, cam_idx, bg):
        c = self.cams[cam_idx]
        g = self.g
        rs = GaussianRasterizationSettings(
            image_height=self.H, image_width=self.W, tanfovx=c["tx"], tanfovy=c["ty"], bg=bg, scale_modifier=1.0,
            viewmatrix=c["view"], projmatrix=c["proj"], sh_degree=g.active_sh_degree, campos=c["campos"],
            prefiltered=False, debug=False, do_depth=True, render_indices=self.empty_i, parent_indices=self.empty_i,
            interpolation_weights=self.empty_f, num_node_kids=self.empty_id)
        means2D = self._means2D_leaf()
        scales, rotations, opacities = self._activations()
        color, radii, invd = GaussianRasterizer(rs)(means3D=g.get_xyz, means2D=means2D, shs=g.get_features,
                                                    colors_precomp=None, opacities=opacities, scales=scales,
                                                    rotations=rotations, cov3D_precomp=None)
        return self._apply_exposure(color, g._exposure[cam_idx]), invd, means2D, radii

    def _view(self, cam_idx):
        return (self.iteration - 1) % len(self.cams) if cam_idx is None else cam_idx

    def step(self, cam_idx=None, between=None):
        """One iteration; returns the loss tensor (no host synchronisation on the fused path).

        between: called after the densification statistics, before the optimizers
        (train_single.py:190-201: densify_and_prune / reset_opacity).  Those replace the Gaussian
        nn.Parameters, whose .grad is then None, so the reference's sparse Adam does not run in such
        an iteration (:217, :225); neither does it here.  The scale shrink still does."""
        g = self.g
        it = self.iteration
        k = self._view(cam_idx)
        depth_only = self.depth_only[k]
        for pg in self.optimizer.param_groups:
            if pg["name"] == "xyz":
                pg["lr"] = self.xyz_lr(it)
        for pg in self.exposure_optimizer.param_groups:
            pg["lr"] = self.exposure_lr(it)
        bg = torch.rand(3, device=g._xyz.device)
        image, invd, means2D, radii = self.render(k, bg)
        w = self.depth_weight(it)
        if depth_only:
            if not w > 0:
                raise ValueError("a depth-only iteration with no depth weight has no loss (train_single.py:158-161)")
            loss = self._depth_only_loss(invd, self.mono[k], self.dmask[k], w)
        else:
            if self.amask[k] is not None:
                image = image * self.amask[k]
            loss = self._photo_loss(image, self.gts[k])
            if self.mono[k] is not None and w > 0:
                loss = loss + self._depth_loss(invd, self.mono[k], self.dmask[k], w)
        self._backward(loss)
        with torch.no_grad():
            self._densify_stats(radii, means2D.grad)
            if between is not None:
                between()
            if depth_only:
                self._zero_feature_grads()
            else:
                self.exposure_optimizer.step()
            self.exposure_optimizer.zero_grad(set_to_none=True)
            if between is None:
                if self.skybox > 0 and g._opacity.grad is not None:
                    self._lock_skybox()
                self._sparse_step()
            self.optimizer.zero_grad(set_to_none=True)
            self._shrink()  # train_single.py:235-241: shrink Gaussians larger than 2% of the extent
        self.iteration += 1
        return loss.detach()


def make_problem(P, W, H, n_views=4, seed=0, sh_degree=3, device="cuda", step_cls=None, perturb=0.02,
                 depth=True, depth_mask_frac=0.85, alpha=False, skybox_points=0, scaffold_points=0, fovx_deg=60.0,
                 depth_only=0, iterations=LR["iterations"]):
    """A synthetic Street-sparse training problem: ground-truth views and inverse-depth maps
    rendered from a seeded scene over `n_views` orbit cameras, depth masks (a random ~85% of each
    map valid, as the reference's depth_mask), optional alpha masks, and a step (TrainStep, or
    `step_cls`, e.g. oracle/train_torch_ref.ReferenceTrainStep) that starts from a perturbed copy.
    The mono depth maps are the true inverse depth with 5% multiplicative noise.  fovx_deg: 90 for
    Street-sparse's cube faces (ss_utils/generate_colmap_calibration.py:476-479: f = size / 2).
    depth_only: the last `depth_only` views are depth-only (no target image; a LiDAR-like map: the
    true inverse depth on a random 30% of the pixels, zero elsewhere)."""
    from .synthetic import orbit_cameras, synthetic_scene
    step_cls = step_cls or TrainStep
    s = synthetic_scene(P, W, H, seed=seed, sh_degree=sh_degree, fovx_deg=fovx_deg)
    cams = orbit_cameras(n_views, W, H, fovx_deg=fovx_deg)
    truth = GaussianSet(s["means3D"], s["shs"], s["opacities"], s["scales"], s["rotations"], n_images=n_views,
                        sh_degree=sh_degree, device=device, joined_features=True)
    tmp = TrainStep(truth, cams, [None] * n_views, W, H)
    gen = torch.Generator(device=device).manual_seed(seed + 7)
    gts, monos, dmasks, amasks = [], [], [], []
    with torch.no_grad():
        for k in range(n_views):
            img, invd, _, _ = tmp.render(k, torch.zeros(3, device=device))
            gts.append(img.contiguous())
            noise = 1.0 + 0.05 * torch.randn(invd.shape, generator=gen, device=device)
            monos.append((invd * noise).contiguous())
            dmasks.append((torch.rand(invd.shape, generator=gen, device=device) < depth_mask_frac).float())
            amasks.append((torch.rand(invd.shape, generator=gen, device=device) < 0.97).float())
            if k >= n_views - depth_only:
                gts[-1] = None
                monos[-1] = (invd * (torch.rand(invd.shape, generator=gen, device=device) < 0.3).float()).contiguous()
                amasks[-1] = None
    rng = np.random.default_rng(seed + 99)
    noisy = dict(means3D=s["means3D"] + perturb * rng.normal(size=s["means3D"].shape).astype(np.float32),
                 shs=s["shs"] + perturb * rng.normal(size=s["shs"].shape).astype(np.float32),
                 opacities=s["opacities"], scales=s["scales"] * np.exp(perturb * rng.normal(size=s["scales"].shape)),
                 rotations=s["rotations"])
    model = GaussianSet(noisy["means3D"], noisy["shs"], noisy["opacities"], noisy["scales"].astype(np.float32),
                        noisy["rotations"], n_images=n_views, sh_degree=sh_degree, device=device,
                        joined_features=getattr(step_cls, "JOINED_FEATURES", True))
    if depth_only and not depth:
        raise ValueError("depth-only views need depth supervision (depth=True)")
    return step_cls(model, cams, gts, W, H, mono_invdepths=monos if depth else None,
                    depth_masks=dmasks if depth else None, alpha_masks=amasks if alpha else None,
                    skybox_points=skybox_points, scaffold_points=scaffold_points, iterations=iterations,
                    depth_only=[k >= n_views - depth_only for k in range(n_views)])
