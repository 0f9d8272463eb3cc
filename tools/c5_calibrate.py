"""Cut size of the synthetic config-5 hierarchy vs leaf scale and tau (GPU); picks bench defaults."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "street-sparse-3dgs_amd"))
import torch
from gaussian_hierarchy._C import expand_to_size
from gs_train.synthetic import synthetic_lod_hierarchy, tau_threshold

L = int(sys.argv[1]) if len(sys.argv) > 1 else 37_500_000
for ls in (-6.5, -6.0, -5.5, -5.0):
    h = synthetic_lod_hierarchy(L, 1920, 1080, "cuda", seed=5, log_scale_mean=ls)
    N = h["nodes"].shape[0]
    ri, pi, ni = (torch.zeros(N, dtype=torch.int32, device="cuda") for _ in range(3))
    cam = torch.tensor(h["campos"], device="cuda")
    for tau in (0.0, 3.0, 6.0, 15.0):
        n = expand_to_size(h["nodes"], h["boxes"], tau_threshold(tau, h["tanfovx"], 1920), cam, torch.zeros(3), ri, pi, ni)
        print(f"log_scale {ls} tau {tau}: cut {n} of {N} nodes", flush=True)
    del h, ri, pi, ni
    torch.cuda.empty_cache()
