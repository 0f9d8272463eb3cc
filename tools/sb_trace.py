"""Phase times of the local sort kernel (sb_sort_bin) per superblock, from a GSR_SB_TRACE build:
    python3 street-sparse-3dgs_amd/build_hip.py --define GSR_SB_TRACE=1 --out vlibs/sbtrace.so
    GSR_LIBRARY=vlibs/sbtrace.so python3 tools/sb_trace.py
Stamps: 0 start, 1 keys loaded + range, 2 sorted, 3 footprints gathered, 4 tile counts + bases,
5 placed.  Prints the median / p90 of each phase (us) and the kernel span."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "street-sparse-3dgs_amd"))
import bench  # noqa: E402


def main():
    import torch
    from diff_gaussian_rasterization import _C
    dev = torch.device("cuda:0")
    W, H = 1920, 1080
    s, inp, gcol, ginv = bench.make_inputs(1_000_000, W, H, 3, 0, dev)
    rs, raster = bench.rasterizer_for(s, W, H, 3, dev)
    step = bench.fwd_bwd_step(raster, inp, gcol, ginv)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    buf = (ctypes.c_int64 * (2048 * 8))()
    _C._L.gsr_debug_trace(buf, 2048 * 8, 1)
    step()
    torch.cuda.synchronize()
    _C._L.gsr_debug_trace(buf, 2048 * 8, 0)
    a = np.array(buf[:], np.int64).reshape(2048, 8)
    a = a[a[:, 0] > 0]
    t0 = a[:, 0].min()
    print("workgroups", len(a), "kernel span us", (a[:, 5].max() - t0) / 100.0)
    print("start offsets us: median %.1f p90 %.1f max %.1f" % tuple(np.percentile((a[:, 0] - t0) / 100.0, [50, 90, 100])))
    names = ["load+range", "sort", "gather fp", "counts+bases", "place"]
    for i, nme in enumerate(names):
        d = (a[:, i + 1] - a[:, i]) / 100.0
        print(f"{nme:14s} median {np.median(d):7.2f} p90 {np.percentile(d, 90):7.2f} max {d.max():7.2f} us")
    tot = (a[:, 5] - a[:, 0]) / 100.0
    print(f"{'total':14s} median {np.median(tot):7.2f} p90 {np.percentile(tot, 90):7.2f} max {tot.max():7.2f} us;"
          f" list length median {np.median(a[:, 7]):.0f} max {a[:, 7].max()}")


if __name__ == "__main__":
    main()
