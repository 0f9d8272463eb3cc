"""Bit-identity check of the streaming SSIM pass against the tiled one (GSR_SSIM_TILED=1) through
gs_train.l1_ssim forward + backward at 1080p, 1536^2 and an odd size (run ON the GPU box; a
measurement variant is checked with GSR_LIBRARY=path)."""
import os, sys, torch
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "street-sparse-3dgs_amd"))
from gs_train import l1_ssim
torch.manual_seed(0)
out = []
for tiled in ("0", "1"):
    os.environ["GSR_SSIM_TILED"] = tiled
    for H, W in ((1080, 1920), (1536, 1536), (67, 131)):
        x = torch.rand(3, H, W, device="cuda", generator=torch.Generator(device="cuda").manual_seed(H)).requires_grad_(True)
        gt = torch.rand(3, H, W, device="cuda", generator=torch.Generator(device="cuda").manual_seed(W))
        v = l1_ssim(x, gt)
        (0.8 * v[0] + 0.2 * (1 - v[1])).backward()
        out.append((v[0].item(), v[1].item(), x.grad.clone()))
n = len(out) // 2
for a, b in zip(out[:n], out[n:]):
    assert a[0] == b[0] and a[1] == b[1] and torch.equal(a[2], b[2]), (a[:2], b[:2], (a[2] - b[2]).abs().max().item())
print("ssim stream == tiled: bit-identical on", n, "shapes")
