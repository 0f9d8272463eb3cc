"""Where a gradient's error against the oracle comes from (run ON the GPU box):
    python3 tools/grad_diag.py --P 1000000 --W 1536 --H 1536 --deg 1 --seed 4 --fovx 90
Per tensor: rel L2 in atomic and deterministic mode; for means3D the Gaussians with the largest
error share, with their depth, radius, tiles and gradient norms."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "street-sparse-3dgs_amd"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1536)
    ap.add_argument("--H", type=int, default=1536)
    ap.add_argument("--deg", type=int, default=1)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--fovx", type=float, default=90.0)
    a = ap.parse_args()
    import test_gpu_parity as T
    from helpers import deterministic, rel_l2
    c = dict(name="diag", P=a.P, W=a.W, H=a.H, deg=a.deg, seed=a.seed, log_scale=-4.0, fovx=a.fovx)
    s = T.make_scene(c)
    dcol, dinv = T.upstream_grads(c)
    st, g = T.run_oracle(s, c, dcol, dinv)
    h = T.run_hip(s, c, dcol, dinv)
    with deterministic():
        hd = T.run_hip(s, c, dcol, dinv)
    pairs = [("means3D", "dL_dmeans3D"), ("means2D", "dL_dmeans2D"), ("opacities", "dL_dopacity"), ("shs", "dL_dsh"),
             ("scales", "dL_dscales"), ("rotations", "dL_drotations")]
    for hk, ok in pairs:
        ga = h["grads"][hk].reshape(g[ok].shape)
        gd = hd["grads"][hk].reshape(g[ok].shape)
        print(f"{hk:10s} atomic {rel_l2(ga, g[ok]):.3e}  deterministic {rel_l2(gd, g[ok]):.3e}  "
              f"atomic-vs-det {rel_l2(ga, gd):.3e}")
    ga = h["grads"]["means3D"].reshape(-1, 3).astype(np.float64)
    go = g["dL_dmeans3D"].reshape(-1, 3).astype(np.float64)
    e = ((ga - go) ** 2).sum(1)
    tot = e.sum()
    idx = np.argsort(-e)[:12]
    print("total err^2", tot, "ref norm^2", (go ** 2).sum())
    for i in idx:
        print(f"  id {i}: share {e[i] / tot:.3f}  z {s['means3D'][i, 2]:.3f}  r {st['radii'][i]}  tiles "
              f"{st['tiles_touched'][i]}  |g| {np.linalg.norm(go[i]):.3e}  |dg| {np.sqrt(e[i]):.3e}  "
              f"hip {ga[i]}  oracle {go[i]}")
    gm2 = h["grads"]["means2D"].reshape(-1, 3).astype(np.float64)
    om2 = g["dL_dmeans2D"].reshape(-1, 3).astype(np.float64)
    for i in idx[:5]:
        print(f"  means2D {i}: hip {gm2[i]} oracle {om2[i]}")


if __name__ == "__main__":
    main()
