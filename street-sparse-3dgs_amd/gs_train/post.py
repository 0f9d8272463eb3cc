"""PostTrainStep: one train_post.py iteration (train_post.py:69-198) -- the per-chunk hierarchy
post-optimisation (2 x 15k of the pipeline, scripts/full_train.py:155-165) -- on the gfx950 path.

Per iteration, in the reference's order:
  1. a random LOD limit: limit = 2^(U (log2 0.1 - log2 0.005) + log2 0.005), U = torch.rand(1) on the
     host generator (:73-74)
  2. update_learning_rate (the xyz schedule; the exposures are pretrained, so no exposure
     schedule: scene/gaussian_model.py:447-457, 362-371)
  3. expand_to_size (the cut) and get_interpolation_weights (:91-113) -- gaussian_hierarchy._C
  4. render_post (gaussian_renderer/__init__.py:200-243): the LOD blend of every rendered node with
     its parent, then the skybox rows -- here ONE launch over the pre-activation parameters
     (interpolate_cut_act: exp / normalize / the hierarchy model's abs opacity,
     scene/gaussian_model.py:411-412, applied to the gathered rows only) -- then the rasterizer,
     the pretrained exposure of the view and the clamp (:280-286)
  5. (1 - l) L1 + l (1 - SSIM) of image * alpha_mask against the target (:134-140)
  6. backward: through the rasterizer and the blend's scatter into the N-row parameters
  7. the gradients of the last skybox_points rows and of the anchors zeroed (:167-181): one launch
  8. torch.optim.Adam over every row (training_setup(our_adam=False), :191-192): the fused
     kernel's dense mode (relevance None), OurAdam's arithmetic (exp_avg by mul + add where torch's
     foreach Adam lerps: ulp-level differences, checked in tests/test_gpu_post.py)
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ._native import check, lib, ptr, require_gpu, stream
from .harness import LR, expon_lr
from .loss import photo_loss
from .optim import Adam

GSR_OPACITY_SIGMOID = 1
GSR_OPACITY_ABS = 2
GSR_CUT_UNIQUE_CHILDREN = 0x100  # include/gsr_hier.h

# scripts/full_train.py:155-158 (the post-optimisation's command line) over OptimizationParams
POST_LR = dict(LR, iterations=15_000, feature_lr=0.0005, opacity_lr=0.01, scaling_lr=0.001)
LIMMAX, LIMMIN = 0.1, 0.005  # train_post.py:66-67


class _CutAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xyz, s_raw, q_raw, o_raw, shs, ri, pi, w, S, opacity_act, unique_children=False):
        require_gpu(xyz, s_raw, q_raw, o_raw, shs, ri, pi, w)
        N, M, R = xyz.shape[0], shs.shape[1], ri.shape[0]
        ins = [t.detach().float().contiguous() for t in (xyz, s_raw, q_raw, o_raw, shs)]
        ri = ri.to(torch.int32).contiguous()
        pi = pi[:R].to(torch.int32).contiguous()
        w = w.detach().float().contiguous()
        rows = R + int(S)
        outs = [torch.empty((rows,) + tuple(t.shape[1:]), dtype=torch.float32, device=xyz.device) for t in ins]
        check(lib().gsr_interpolate_cut_forward_act(N, M, R, int(S), ptr(ri), ptr(pi), ptr(w), *[ptr(t) for t in ins],
                                                    int(opacity_act), *[ptr(t) for t in outs], stream(xyz.device)),
              "gsr_interpolate_cut_forward_act")
        ctx.save_for_backward(ri, pi, w, ins[1], ins[2], ins[3])
        ctx.meta = (N, M, R, int(S), int(opacity_act) | (GSR_CUT_UNIQUE_CHILDREN if unique_children else 0),
                    [tuple(t.shape) for t in ins])
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        ri, pi, w, s_raw, q_raw, o_raw = ctx.saved_tensors
        N, M, R, S, act, shapes = ctx.meta
        dev = q_raw.device
        rows = R + S
        g = [(go if go is not None else torch.zeros((rows,) + shapes[k][1:], device=dev)).float().contiguous()
             for k, go in enumerate(gouts)]
        grads = [torch.zeros(s_, dtype=torch.float32, device=dev) for s_ in shapes]
        check(lib().gsr_interpolate_cut_backward_act(N, M, R, S, ptr(ri), ptr(pi), ptr(w), ptr(s_raw), ptr(q_raw),
                                                     ptr(o_raw), act, *[ptr(t) for t in g], *[ptr(t) for t in grads],
                                                     stream(dev)), "gsr_interpolate_cut_backward_act")
        return (*grads, None, None, None, None, None, None)


def interpolate_cut_act(xyz, scaling_raw, rotation_raw, opacity_raw, features, render_indices, parent_indices,
                        interpolation_weights, skybox_points=0, opacity_act=GSR_OPACITY_ABS, unique_children=False):
    """render_post's blend (gaussian_renderer/__init__.py:200-243) of the pre-activation parameters
    (include/gsr_hier.h gsr_interpolate_cut_forward_act): returns the R + S rows (means, scales,
    rotations, opacities, SH) the rasterizer renders, differentiable w.r.t. the five raw inputs.
    unique_children: render_indices is a cut (no row twice, none a parent row, as expand_to_size
    returns it), so the backward writes the children's gradient rows instead of accumulating them
    (GSR_CUT_UNIQUE_CHILDREN)."""
    return _CutAct.apply(xyz, scaling_raw, rotation_raw, opacity_raw, features, render_indices, parent_indices,
                         interpolation_weights, int(skybox_points), int(opacity_act), bool(unique_children))


def zero_grad_rows(tensors, tail, rows=None):
    """train_post.py:167-181: the gradient rows of the last `tail` Gaussians (the skybox) and of
    `rows` (the anchors, int64 on the device) set to zero in every tensor (one launch)."""
    import ctypes
    ts = [t for t in tensors if t is not None]
    if not ts:
        return
    require_gpu(*ts)
    N = ts[0].shape[0]
    for t in ts:
        if t.shape[0] != N or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("zero_grad_rows: contiguous float32 tensors with one row count")
    ptrs = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    widths = (ctypes.c_int64 * len(ts))(*[t.numel() // max(N, 1) for t in ts])
    r = rows.to(device=ts[0].device, dtype=torch.int64).contiguous() if rows is not None and rows.numel() else None
    check(lib().gsr_zero_grad_rows(len(ts), ptrs, widths, N, int(tail), ptr(r), 0 if r is None else r.numel(),
                                   stream(ts[0].device)), "gsr_zero_grad_rows")


class HierarchyModel:
    """The state create_from_hier builds (scene/gaussian_model.py:344-418): the hierarchy's Gaussians
    (N rows, the skybox's last), SH as ONE (N, 16, 3) parameter, opacities stored as activated
    values (abs activation), log-scales, quaternions, nodes (N_nodes, 7) int32, boxes
    (N_nodes, 2, 4), the anchors (int64 rows), the pretrained per-view exposures (3, 4) or None."""

    def __init__(self, means3D, shs, opacities, scales, rotations, nodes, boxes, skybox=0, anchors=None,
                 spatial_lr_scale=1.0, device="cuda", sh_degree=3):
        t = lambda a: torch.as_tensor(a, dtype=torch.float32, device=device).contiguous()
        self._xyz = torch.nn.Parameter(t(means3D))
        self._features = torch.nn.Parameter(t(shs))
        self._opacity = torch.nn.Parameter(t(opacities).reshape(-1, 1))
        self._scaling = torch.nn.Parameter(torch.log(t(scales)))
        self._rotation = torch.nn.Parameter(t(rotations))
        self.nodes = torch.as_tensor(nodes, dtype=torch.int32, device=device).contiguous()
        self.boxes = t(boxes)
        self.skybox_points = int(skybox)
        self.anchors = (torch.as_tensor(anchors, dtype=torch.int64, device=device) if anchors is not None
                        else torch.empty(0, dtype=torch.int64, device=device))
        self.active_sh_degree = sh_degree  # train_post.py:35
        self.max_sh_degree = sh_degree
        self.spatial_lr_scale = spatial_lr_scale

    @property
    def N(self):
        return self._xyz.shape[0]

    def param_groups(self, lr=POST_LR):
        s = self.spatial_lr_scale
        return [{"params": [self._xyz], "lr": lr["position_lr_init"] * s, "name": "xyz"},
                {"params": [self._features], "lr": lr["feature_lr"], "name": "f_dc+f_rest",
                 "column_lrs": [(0, 3, lr["feature_lr"]), (3, self._features[0].numel(), lr["feature_lr"] / 20.0)]},
                {"params": [self._opacity], "lr": lr["opacity_lr"], "name": "opacity"},
                {"params": [self._scaling], "lr": lr["scaling_lr"], "name": "scaling"},
                {"params": [self._rotation], "lr": lr["rotation_lr"], "name": "rotation"}]


class PostTrainStep:
    """cameras: (view, proj, campos, tanfovx, tanfovy) tuples (synthetic.camera); gts (3, H, W);
    alpha_masks (1, H, W) or None; exposures: per view (3, 4) pretrained exposure or None (then the
    image is only clamped, gaussian_renderer/__init__.py:280-286)."""

    def __init__(self, model: HierarchyModel, cameras, gts, W, H, alpha_masks=None, exposures=None,
                 iterations=POST_LR["iterations"], lr=POST_LR, white_background=False):
        self.m = model
        self.W, self.H = W, H
        self.gts = gts
        n = len(cameras)
        self.amask = alpha_masks if alpha_masks is not None else [None] * n
        self.expo = exposures if exposures is not None else [None] * n
        dev = model._xyz.device
        f = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32, device=dev)
        self.cams = [dict(view=f(v).reshape(4, 4), proj=f(p).reshape(4, 4), campos=f(c), campos_cpu=torch.tensor(c),
                          tx=float(tx), ty=float(ty)) for (v, p, c, tx, ty) in cameras]
        self.optimizer = Adam(model.param_groups(lr), lr=0.0, eps=1e-15)
        s = model.spatial_lr_scale
        self.xyz_lr = lambda it: expon_lr(it, lr["position_lr_init"] * s, lr["position_lr_final"] * s,
                                          lr_delay_mult=lr["position_lr_delay_mult"],
                                          max_steps=lr["position_lr_max_steps"])
        self.lambda_dssim = lr["lambda_dssim"]
        self.iterations = int(iterations)
        self.iteration = 1
        Nn = model.N
        # train_post.py:59-63: the cut buffers, one entry per Gaussian
        self.ri = torch.zeros(Nn, dtype=torch.int32, device=dev)
        self.pi = torch.zeros(Nn, dtype=torch.int32, device=dev)
        self.ni = torch.zeros(Nn, dtype=torch.int32, device=dev)
        self.w = torch.zeros(Nn, dtype=torch.float32, device=dev)
        self.kids = torch.zeros(Nn, dtype=torch.int32, device=dev)
        self.zero3 = torch.zeros(3)
        self.bg = torch.tensor([1.0, 1.0, 1.0] if white_background else [0.0, 0.0, 0.0], device=dev)
        self.empty_i = torch.empty(0, dtype=torch.int32)
        self.empty_f = torch.empty(0, device=dev)
        self.empty_id = torch.empty(0, dtype=torch.int32, device=dev)
        self.last_cut = 0
        self.limit_fn = None  # tests: a fixed limit per iteration instead of the random draw

    def _limit(self):
        if self.limit_fn is not None:
            return self.limit_fn(self.iteration)
        sample = torch.rand(1).item()  # the host generator, train_post.py:73
        return math.pow(2, sample * (math.log2(LIMMAX) - math.log2(LIMMIN)) + math.log2(LIMMIN))

    def cut(self, k, limit):
        """expand_to_size + get_interpolation_weights (train_post.py:91-113); returns the cut length."""
        from gaussian_hierarchy._C import expand_to_size, get_interpolation_weights
        c, m = self.cams[k], self.m
        n = expand_to_size(m.nodes, m.boxes, limit, c["campos"], self.zero3, self.ri, self.pi, self.ni)
        get_interpolation_weights(self.ni[:n], limit, m.nodes, m.boxes, c["campos_cpu"], self.zero3, self.w, self.kids)
        return n

    def render(self, k, n):
        """render_post (gaussian_renderer/__init__.py:200-286) of the cut's n rows + the skybox."""
        from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
        c, m = self.cams[k], self.m
        means, scales, rots, opac, shs = interpolate_cut_act(m._xyz, m._scaling, m._rotation, m._opacity, m._features,
                                                            self.ri[:n], self.pi, self.w, m.skybox_points,
                                                            unique_children=True)
        rs = GaussianRasterizationSettings(
            image_height=self.H, image_width=self.W, tanfovx=c["tx"], tanfovy=c["ty"], bg=self.bg, scale_modifier=1.0,
            viewmatrix=c["view"], projmatrix=c["proj"], sh_degree=m.active_sh_degree, campos=c["campos"],
            prefiltered=False, debug=False, do_depth=False, render_indices=self.empty_i, parent_indices=self.empty_i,
            interpolation_weights=self.empty_f, num_node_kids=self.empty_id)
        means2D = torch.zeros_like(means, requires_grad=True)
        color, radii, _ = GaussianRasterizer(rs)(means3D=means, means2D=means2D, shs=shs, colors_precomp=None,
                                                 opacities=opac, scales=scales, rotations=rots, cov3D_precomp=None)
        E = self.expo[k]
        if E is not None:
            from .exposure import apply_exposure
            return apply_exposure(color, E), radii
        return color.clamp(0, 1), radii

    def step(self, cam_idx=None):
        m = self.m
        it = self.iteration
        k = (it - 1) % len(self.cams) if cam_idx is None else cam_idx
        limit = self._limit()
        for pg in self.optimizer.param_groups:
            if pg["name"] == "xyz":
                pg["lr"] = self.xyz_lr(it)
        if it % 1000 == 0 and m.active_sh_degree < m.max_sh_degree:  # :88-89 (already at the maximum)
            m.active_sh_degree += 1
        n = self.cut(k, limit)
        self.last_cut = n
        image, _ = self.render(k, n)
        if self.amask[k] is not None:
            image = image * self.amask[k]
        loss = photo_loss(image, self.gts[k], self.lambda_dssim)[0]
        loss.backward()
        with torch.no_grad():
            zero_grad_rows([p.grad for p in (m._xyz, m._rotation, m._features, m._opacity, m._scaling)],
                           m.skybox_points, m.anchors)
            self.optimizer.step()
            self.optimizer.zero_grad(set_to_none=True)
        self.iteration += 1
        return loss.detach()


def synthetic_post_problem(leaves, W, H, n_views=4, skybox=10_000, n_anchors=1000, seed=0, device="cuda",
                           iterations=POST_LR["iterations"], perturb=0.02, step_cls=None):
    """A post-optimisation problem on a synthetic hierarchy (synthetic.synthetic_lod_hierarchy: a
    Morton-grouped tree, one Gaussian per node, skybox rows last): targets rendered from the tree
    at a mid LOD limit over `n_views` orbit cameras, pretrained exposures near identity, alpha
    masks, anchors = random interior rows; the model starts from a perturbed copy."""
    from .synthetic import orbit_cameras, synthetic_lod_hierarchy
    step_cls = step_cls or PostTrainStep
    h = synthetic_lod_hierarchy(leaves, W, H, device, seed=seed, skybox=skybox, log_scale_mean=-5.0)
    cams = orbit_cameras(n_views, W, H)
    g = torch.Generator(device=device).manual_seed(seed + 3)
    expos = []
    for _ in range(n_views):
        E = torch.eye(3, 4, device=device)
        E[:, :3] += 0.02 * torch.randn(3, 3, generator=g, device=device)
        E[:, 3] = 0.01 * torch.randn(3, generator=g, device=device)
        expos.append(E)
    truth = HierarchyModel(h["means3D"], h["shs"], h["opacities"], h["scales"], h["rotations"], h["nodes"], h["boxes"],
                           skybox=skybox, device=device)
    tmp = step_cls(truth, cams, [None] * n_views, W, H, exposures=expos, iterations=iterations)
    gts, amasks = [], []
    with torch.no_grad():
        for k in range(n_views):
            n = tmp.cut(k, 0.02)
            img, _ = tmp.render(k, n)
            gts.append(img.contiguous())
            amasks.append((torch.rand((1, H, W), generator=g, device=device) < 0.97).float())
    del tmp, truth
    p = lambda x, s: x + s * torch.randn(x.shape, generator=g, device=device)
    Nn = h["means3D"].shape[0]
    anchors = torch.randperm(Nn - skybox, generator=g, device=device)[:n_anchors]
    model = HierarchyModel(p(h["means3D"], perturb), p(h["shs"], perturb), h["opacities"],
                           h["scales"] * torch.exp(perturb * torch.randn(h["scales"].shape, generator=g, device=device)),
                           h["rotations"], h["nodes"], h["boxes"], skybox=skybox, anchors=anchors, device=device)
    return step_cls(model, cams, gts, W, H, alpha_masks=[a for a in amasks], exposures=expos, iterations=iterations)
