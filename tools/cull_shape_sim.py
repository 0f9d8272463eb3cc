"""Count the (tile instance, sub-block) pairs of the bench frame that pass the exact ellipse cull
for 16x4 sub-blocks (the blend kernels' layout) vs 8x8 blocks, from the C oracle's preprocess
(CPU only).  usage: python tools/cull_shape_sim.py 1920 1080 [fovx_deg]"""
import sys, time, numpy as np
REPO = __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))
for _p in (REPO, REPO + '/oracle', REPO + '/street-sparse-3dgs_amd'):
    sys.path.insert(0, _p)
import gs_oracle as O
from gs_train.synthetic import synthetic_scene
W, H = int(sys.argv[1]), int(sys.argv[2]); fov = float(sys.argv[3]) if len(sys.argv) > 3 else 60.0
P = 1_000_000
s = synthetic_scene(P, W, H, seed=0, sh_degree=3, fovx_deg=fov)

t0 = time.time()
st = O.forward(s["means3D"], s["opacities"], s["view"], s["proj"], s["campos"], np.zeros(3), W, H, s["tanfovx"], s["tanfovy"],
               sh_degree=3, shs=s["shs"], scales=s["scales"], rotations=s["rotations"])
print("oracle fwd", time.time() - t0, "K", st["K"], flush=True)
gx = (W + 15) // 16
keys, pl = st["keys"], st["point_list"]
tile = (keys >> np.uint64(32)).astype(np.int64)
g = pl.astype(np.int64)
xy = st["xy"].astype(np.float64); co = st["conic_opacity"].astype(np.float64)
def meets(cx, cy, a, b, c, tm, x0, x1, y0, y1):
    X0, X1, Y0, Y1 = x0 - cx, x1 - cx, y0 - cy, y1 - cy
    outx = (X0 > 0) | (X1 < 0); outy = (Y0 > 0) | (Y1 < 0)
    q = np.full(cx.shape, 3e38)
    xe = np.where(X0 > 0, X0, X1)
    ys = np.clip(-b * xe / c, Y0, Y1)
    q = np.where(outx, np.minimum(q, a * xe * xe + 2 * b * xe * ys + c * ys * ys), q)
    ye = np.where(Y0 > 0, Y0, Y1)
    xs = np.clip(-b * ye / a, X0, X1)
    q = np.where(outy, np.minimum(q, a * xs * xs + 2 * b * xs * ye + c * ye * ye), q)
    return (~outx & ~outy) | (q <= tm)
tot = {"strip16x4": 0, "block8x8": 0}
n = len(g)
for s0 in range(0, n, 2_000_000):
    sl = slice(s0, min(n, s0 + 2_000_000))
    gg, tt = g[sl], tile[sl]
    cx, cy = xy[gg, 0], xy[gg, 1]
    a, b, c, op = co[gg, 0], co[gg, 1], co[gg, 2], co[gg, 3]
    tm = 2 * np.log(np.maximum(255 * op, 1e-30))
    tx0 = (tt % gx) * 16.0; ty0 = (tt // gx) * 16.0
    for k in range(4):
        tot["strip16x4"] += meets(cx, cy, a, b, c, tm, tx0, tx0 + 15, ty0 + 4 * k, ty0 + 4 * k + 3).sum()
        bx, by = k & 1, k >> 1
        tot["block8x8"] += meets(cx, cy, a, b, c, tm, tx0 + 8 * bx, tx0 + 8 * bx + 7, ty0 + 8 * by, ty0 + 8 * by + 7).sum()
print(W, H, "K", n, {k: int(v) for k, v in tot.items()}, "ratio", tot["block8x8"] / tot["strip16x4"])
