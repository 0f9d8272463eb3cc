"""TEST INFRASTRUCTURE / BASELINE LEG ONLY -- the reference's own torch formulation of the
train-step pieces, run on the GPU as the checker of the fused kernels (tests/) and for the bench's
side-by-side "reference-structured train-step ms" (ReferenceTrainStep).  Not the product path and
not a fallback: the fused kernels never route here, and nothing under street-sparse-3dgs_amd/
imports this module.

  photo_loss           utils/loss_utils.py:17-63 (five depthwise 11x11 conv2d) as combined at
                       train_single.py:121-123
  OurAdamTorch         scene/OurAdam.py:249-337: per-group gather of the relevant rows, the
                       update as separate torch ops, scatter back; dense when nothing is relevant
  densification_stats  train_single.py:193-194 + scene/gaussian_model.py:780-793 with the
                       nonzero()-built visibility filter of gaussian_renderer/__init__.py:124-135
  ReferenceTrainStep   gs_train.harness.TrainStep with every hook in the reference's formulation
                       (train_single.py:65-247)
  densify_and_prune    scene/gaussian_model.py:560-778 (the checker of gs_train.densify)
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

_windows = {}


def _window(C, device):
    key = (C, device)
    w = _windows.get(key)
    if w is None:
        g = torch.tensor([math.exp(-((i - 5) ** 2) / (2.0 * 1.5 ** 2)) for i in range(11)], dtype=torch.float32)
        g = g / g.sum()
        w = torch.outer(g, g).expand(C, 1, 11, 11).contiguous().to(device)
        _windows[key] = w
    return w


def ssim(img, gt):
    C = img.shape[-3]
    w = _window(C, img.device)
    blur = lambda t: F.conv2d(t, w, padding=5, groups=C)
    mu1, mu2 = blur(img), blur(gt)
    mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = blur(img * img) - mu1_sq
    s2 = blur(gt * gt) - mu2_sq
    s12 = blur(img * gt) - mu12
    m = ((2 * mu12 + 0.01 ** 2) * (2 * s12 + 0.03 ** 2)) / ((mu1_sq + mu2_sq + 0.01 ** 2) * (s1 + s2 + 0.03 ** 2))
    return m.mean()


def photo_loss(img, gt, lambda_dssim=0.2):
    return (1.0 - lambda_dssim) * torch.abs(img - gt).mean() + lambda_dssim * (1.0 - ssim(img, gt))


class OurAdamTorch(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, relevant):
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                step = st["step"].item()
                sparse = relevant.numel() > 0
                idx = relevant if sparse else slice(None)
                grad, m, v, param = p.grad[idx], st["exp_avg"][idx], st["exp_avg_sq"][idx], p[idx]
                m.mul_(b1).add_(grad, alpha=1 - b1)
                v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
                step_size = group["lr"] / (1 - b1 ** step)
                denom = (v.sqrt() / math.sqrt(1 - b2 ** step)).add_(group["eps"])
                param.addcdiv_(m, denom, value=-step_size)
                if sparse:
                    st["exp_avg"][idx] = m
                    st["exp_avg_sq"][idx] = v
                    p[idx] = param


def densification_stats(g, radii, grad2d):
    vis = (radii > 0).nonzero().flatten().long()
    g.max_radii2D[vis] = torch.max(g.max_radii2D[vis], radii[vis].float())
    n = torch.norm(grad2d[vis, :2], dim=-1, keepdim=True)
    g.xyz_gradient_accum[vis] = torch.max(n, g.xyz_gradient_accum[vis])
    g.denom[vis] += 1


# ---- densify_and_prune in the reference's own formulation (scene/gaussian_model.py:560-778,
# gt_point_cloud_constraints off), on a split-layout GaussianSet and OurAdamTorch: the side-by-side
# for gs_train.densify.densify_and_prune ----------------------------------------------------------
_ATTR = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
         "scaling": "_scaling", "rotation": "_rotation"}


def _build_rotation(r):
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device)
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - r * z)
    R[:, 0, 2] = 2 * (x * z + r * y)
    R[:, 1, 0] = 2 * (x * y + r * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - r * x)
    R[:, 2, 0] = 2 * (x * z - r * y)
    R[:, 2, 1] = 2 * (y * z + r * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def _prune_optimizer(g, opt, mask):
    for group in opt.param_groups:
        p = group["params"][0]
        st = opt.state.get(p, None)
        newp = torch.nn.Parameter(p[mask].requires_grad_(True))
        if st is not None:
            st["exp_avg"] = st["exp_avg"][mask]
            st["exp_avg_sq"] = st["exp_avg_sq"][mask]
            del opt.state[p]
            opt.state[newp] = st
        group["params"][0] = newp
        setattr(g, _ATTR[group["name"]], newp)


def _cat_to_optimizer(g, opt, ext):
    for group in opt.param_groups:
        p = group["params"][0]
        e = ext[group["name"]]
        st = opt.state.get(p, None)
        newp = torch.nn.Parameter(torch.cat((p, e), dim=0).requires_grad_(True))
        if st is not None:
            st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(e)), dim=0)
            st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(e)), dim=0)
            del opt.state[p]
            opt.state[newp] = st
        group["params"][0] = newp
        setattr(g, _ATTR[group["name"]], newp)


def _postfix(g, opt, d):
    _cat_to_optimizer(g, opt, d)
    n = g._xyz.shape[0]
    dev = g._xyz.device
    g.xyz_gradient_accum = torch.zeros((n, 1), device=dev)
    g.denom = torch.zeros((n, 1), device=dev)
    g.max_radii2D = torch.cat((g.max_radii2D, torch.zeros((d["xyz"].shape[0]), device=dev)))


def _prune_points(g, opt, mask):
    valid = ~mask
    _prune_optimizer(g, opt, valid)
    g.xyz_gradient_accum = g.xyz_gradient_accum[valid]
    g.denom = g.denom[valid]
    g.max_radii2D = g.max_radii2D[valid]


def densify_and_prune(g, opt, max_grad, min_opacity, extent, percent_dense, first_row=0, N=2):
    grads = g.xyz_gradient_accum
    grads[grads.isnan()] = 0.0
    dev = g._xyz.device
    # densify_and_clone (:708-731)
    sel = torch.where(torch.norm(grads, dim=-1) * g.max_radii2D * torch.pow(g.get_opacity.flatten(), 1 / 5.0)
                      >= max_grad, True, False)
    sel = torch.logical_and(sel, g.get_opacity.flatten() > 0.15)
    sel = torch.logical_and(sel, torch.max(g.get_scaling, dim=1).values <= percent_dense * extent)
    sel[:first_row] = False
    _postfix(g, opt, {"xyz": g._xyz[sel], "f_dc": g._features_dc[sel], "f_rest": g._features_rest[sel],
                      "opacity": g._opacity[sel], "scaling": g._scaling[sel], "rotation": g._rotation[sel]})
    # densify_and_split (:672-706)
    n_init = g._xyz.shape[0]
    padded = torch.zeros((n_init), device=dev)
    padded[:grads.shape[0]] = grads.squeeze()
    sel = torch.where(padded * g.max_radii2D * torch.pow(g.get_opacity.flatten(), 1 / 5.0) >= max_grad, True, False)
    sel = torch.logical_and(sel, g.get_opacity.flatten() > 0.15)
    sel = torch.logical_and(sel, torch.max(g.get_scaling, dim=1).values > percent_dense * extent)
    sel[:first_row] = False
    stds = g.get_scaling[sel].repeat(N, 1)
    means = torch.zeros((stds.size(0), 3), device=dev)
    samples = torch.normal(mean=means, std=stds)
    rots = _build_rotation(g._rotation[sel]).repeat(N, 1, 1)
    new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + g.get_xyz[sel].repeat(N, 1)
    new_scaling = torch.log(g.get_scaling[sel].repeat(N, 1) / (0.8 * N))
    _postfix(g, opt, {"xyz": new_xyz, "f_dc": g._features_dc[sel].repeat(N, 1, 1),
                      "f_rest": g._features_rest[sel].repeat(N, 1, 1), "opacity": g._opacity[sel].repeat(N, 1),
                      "scaling": new_scaling, "rotation": g._rotation[sel].repeat(N, 1)})
    _prune_points(g, opt, torch.cat((sel, torch.zeros(N * sel.sum(), device=dev, dtype=bool))))
    # opacity prune (:753-770)
    prune = (g.get_opacity < min_opacity).squeeze()
    prune[:first_row] = False
    _prune_points(g, opt, prune)
    g.max_radii2D = torch.zeros((g._xyz.shape[0]), device=dev)


def reset_opacity(g, opt, skybox):
    """scene/gaussian_model.py:528-532 + replace_tensor_to_optimizer (:546-559) on a split-layout set."""
    op = g.get_opacity
    x = torch.min(op[skybox:], torch.ones_like(op[skybox:]) * 0.01)
    new = torch.cat((g._opacity[:skybox], torch.log(x / (1 - x))), 0)  # inverse_sigmoid
    for group in opt.param_groups:
        if group["name"] == "opacity":
            st = opt.state.get(group["params"][0], None)
            if st is not None:
                st["exp_avg"] = torch.zeros_like(new)
                st["exp_avg_sq"] = torch.zeros_like(new)
                del opt.state[group["params"][0]]
            group["params"][0] = torch.nn.Parameter(new.detach().requires_grad_(True))
            if st is not None:
                opt.state[group["params"][0]] = st
            g._opacity = group["params"][0]


# ---- one train_single.py iteration in the reference's formulation ------------------------------
def _reference_step_cls():
    from gs_train.harness import LR, TrainStep

    class ReferenceTrainStep(TrainStep):
        """TrainStep with the reference's torch pieces: get_* activations, matmul exposure,
        conv2d SSIM, the torch depth-L1 expression, nonzero()-built filters, OurAdam's per-group
        gather/scatter, the six-gradient skybox zeroing, boolean-mask scale shrink."""
        JOINED_FEATURES = False

        def _make_optimizers(self, groups):
            if self.g.joined:
                raise ValueError("the reference-structured step needs the reference's split SH layout")
            self.optimizer = OurAdamTorch(groups, lr=0.0, eps=1e-15)
            self.exposure_optimizer = torch.optim.Adam([self.g._exposure])

        def _means2D_leaf(self):
            m = torch.zeros_like(self.g._xyz, requires_grad=True) + 0
            m.retain_grad()
            return m

        def _activations(self):
            g = self.g
            return g.get_scaling, g.get_rotation, g.get_opacity

        def _apply_exposure(self, color, E):
            image = torch.matmul(color.permute(1, 2, 0), E[:3, :3]).permute(2, 0, 1) + E[:3, 3, None, None]
            return image.clamp(0, 1)

        def _photo_loss(self, image, gt):
            return photo_loss(image, gt, LR["lambda_dssim"])

        def _depth_loss(self, invd, mono, mask, w):
            m = mask if mask is not None else torch.ones_like(invd)
            return w * torch.abs((invd - mono) * m).mean()

        def _depth_only_loss(self, invd, mono, mask, w):
            # train_single.py:152-156
            m = mask if mask is not None else torch.ones_like(invd)
            pure = torch.abs((invd - mono) * m).mean()
            dens = (mono - invd).clamp(min=0).mean()
            return (w * (self.dens_weight * dens + (1 - self.dens_weight) * pure)).clone()

        def _zero_feature_grads(self):
            # train_single.py:203-209
            g = self.g
            for p in (g._features_dc, g._features_rest, g._exposure):
                if p.grad is not None:
                    p.grad.zero_()

        def _backward(self, loss):
            loss.backward()

        def _densify_stats(self, radii, grad2d):
            densification_stats(self.g, radii, grad2d)

        def _lock_skybox(self):
            g, S = self.g, self.skybox
            for p in (g._xyz, g._rotation, g._features_dc, g._features_rest, g._opacity, g._scaling):
                if p.grad is not None:
                    p.grad[:S] = 0

        def _sparse_step(self):
            relevant = (self.g._opacity.grad.flatten() != 0).nonzero().flatten().long()
            self.optimizer.step(relevant)

        def _shrink(self):
            g = self.g
            sc = g.get_scaling
            bad = sc.max(dim=1).values > self.extent * 0.02
            bad[:self.scaffold] = False  # train_single.py:239-240
            g._scaling[bad] = torch.log(sc[bad] * 0.8)

        def densify_and_prune(self, max_grad, min_opacity, percent_dense, normals=None):
            if normals is not None:
                raise NotImplementedError("the reference formulation draws its split samples itself")
            P0 = self.g._xyz.shape[0]
            densify_and_prune(self.g, self.optimizer, max_grad, min_opacity, self.extent, percent_dense,
                              first_row=self.scaffold)
            return dict(total=self.g._xyz.shape[0], P0=P0)

        def reset_opacity(self):
            reset_opacity(self.g, self.optimizer, self.skybox)

    return ReferenceTrainStep


def __getattr__(name):
    if name == "ReferenceTrainStep":
        return _reference_step_cls()
    raise AttributeError(name)


# ---- one train_post.py iteration in the reference's formulation (the checker of gs_train.post) -----
class ReferencePostStep:
    """train_post.py:69-198 with the reference's torch pieces: the getters (exp, F.normalize,
    torch.abs -- scene/gaussian_model.py:411-412), render_post's Python gather
    (gaussian_renderer/__init__.py:200-243, interp_python=True), the matmul exposure + clamp
    (:280-286), conv2d SSIM on image * alpha (:134-140), the skybox / anchor gradient zeroing by
    indexing (:167-181) and torch.optim.Adam (training_setup(our_adam=False)) over split f_dc /
    f_rest parameters.  Built from a gs_train.post.PostTrainStep (same views, model copy); the cut
    (expand_to_size / get_interpolation_weights) is the product's, as both run it the same way."""

    def __init__(self, post):
        from gs_train.post import POST_LR
        m = post.m
        self.post = post
        P = lambda t: torch.nn.Parameter(t.detach().clone().contiguous())
        self._xyz, self._opacity, self._scaling, self._rotation = P(m._xyz), P(m._opacity), P(m._scaling), P(m._rotation)
        self._features_dc = P(m._features[:, :1])
        self._features_rest = P(m._features[:, 1:])
        lr = POST_LR
        s = m.spatial_lr_scale
        self.optimizer = torch.optim.Adam(
            [{"params": [self._xyz], "lr": lr["position_lr_init"] * s, "name": "xyz"},
             {"params": [self._features_dc], "lr": lr["feature_lr"], "name": "f_dc"},
             {"params": [self._features_rest], "lr": lr["feature_lr"] / 20.0, "name": "f_rest"},
             {"params": [self._opacity], "lr": lr["opacity_lr"], "name": "opacity"},
             {"params": [self._scaling], "lr": lr["scaling_lr"], "name": "scaling"},
             {"params": [self._rotation], "lr": lr["rotation_lr"], "name": "rotation"}], lr=0.0, eps=1e-15)
        self.iteration = 1

    def features(self):
        return torch.cat((self._features_dc, self._features_rest), 1)

    def step(self, k, limit):
        from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
        post, m = self.post, self.post.m
        for pg in self.optimizer.param_groups:
            if pg["name"] == "xyz":
                pg["lr"] = post.xyz_lr(self.iteration)
        n = post.cut(k, limit)
        c = post.cams[k]
        means3D, opacity = self._xyz, torch.abs(self._opacity)
        scales, rotations = torch.exp(self._scaling), F.normalize(self._rotation)
        shs = self.features()
        render_inds = post.ri[:n].long()
        t = post.w[:n].unsqueeze(1)
        ti = (1 - post.w[:n]).unsqueeze(1)
        pinds = post.pi[:n].long()
        m3 = (t * means3D[render_inds] + ti * means3D[pinds]).contiguous()
        sc = (t * scales[render_inds] + ti * scales[pinds]).contiguous()
        sh = (t.unsqueeze(2) * shs[render_inds] + ti.unsqueeze(2) * shs[pinds]).contiguous()
        parents = rotations[pinds]
        rots = rotations[render_inds]
        dots = torch.bmm(rots.unsqueeze(1), parents.unsqueeze(2)).flatten()
        parents[dots < 0] *= -1
        rot = ((t * rots) + ti * parents).contiguous()
        op = (t * opacity[render_inds] + ti * opacity[pinds]).contiguous()
        S = m.skybox_points
        sk = torch.arange(means3D.shape[0] - S, means3D.shape[0], device=means3D.device)
        m3, sh, op = torch.cat((m3, means3D[sk])), torch.cat((sh, shs[sk])), torch.cat((op, opacity[sk]))
        rot, sc = torch.cat((rot, rotations[sk])), torch.cat((sc, scales[sk]))
        rs = GaussianRasterizationSettings(
            image_height=post.H, image_width=post.W, tanfovx=c["tx"], tanfovy=c["ty"], bg=post.bg, scale_modifier=1.0,
            viewmatrix=c["view"], projmatrix=c["proj"], sh_degree=m.active_sh_degree, campos=c["campos"],
            prefiltered=False, debug=False, do_depth=False, render_indices=post.empty_i, parent_indices=post.empty_i,
            interpolation_weights=post.empty_f, num_node_kids=post.empty_id)
        means2D = torch.zeros_like(m3, requires_grad=True) + 0
        image, _, _ = GaussianRasterizer(rs)(means3D=m3, means2D=means2D, shs=sh, colors_precomp=None, opacities=op,
                                             scales=sc, rotations=rot, cov3D_precomp=None)
        E = post.expo[k]
        if E is not None:
            image = torch.matmul(image.permute(1, 2, 0), E[:3, :3]).permute(2, 0, 1) + E[:3, 3, None, None]
        image = image.clamp(0, 1)
        am = post.amask[k]
        img = image * am if am is not None else image
        loss = photo_loss(img, post.gts[k], post.lambda_dssim)
        loss.backward()
        with torch.no_grad():
            params = (self._xyz, self._rotation, self._features_dc, self._features_rest, self._opacity, self._scaling)
            if S:
                for p in params:
                    p.grad[-S:] = 0
            for p in params:
                p.grad[m.anchors] = 0
            self.optimizer.step()
            self.optimizer.zero_grad(set_to_none=True)
        self.iteration += 1
        return loss.detach()
