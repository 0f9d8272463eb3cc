"""Host-issue vs device time of the fused train step, plus a cProfile of 20 steps (run on the GPU box:
`python tools/train_host_split.py`)."""
import cProfile, pstats, sys, time, io
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/street-sparse-3dgs_amd")
import torch
import bench
from gs_train.harness import GaussianSet, TrainStep
dev = torch.device("cuda", 0)
P, W, H, deg = 1_000_000, 1920, 1080, 3
s, inp, gcol, ginv = bench.make_inputs(P, W, H, deg, seed=0, device=dev)
g = GaussianSet(s["means3D"], s["shs"], s["opacities"], s["scales"], s["rotations"], n_images=1, sh_degree=deg,
                device=dev, joined_features=True)
gt = torch.rand((3, H, W), device=dev, generator=torch.Generator(device=dev).manual_seed(123))
ts = TrainStep(g, [(s["view"], s["proj"], s["campos"], s["tanfovx"], s["tanfovy"])], [gt], W, H, fused=True)
for _ in range(5):
    ts.step()
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter(); host = 0.0
    for _ in range(20):
        h0 = time.perf_counter(); ts.step(); host += time.perf_counter() - h0
    torch.cuda.synchronize()
    print(f"wall/step {(time.perf_counter()-t0)/20*1e3:.3f} ms, host issue/step {host/20*1e3:.3f} ms", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    ts.step()
e1.record(); torch.cuda.synchronize()
print(f"event/step {e0.elapsed_time(e1)/20:.3f} ms", flush=True)
pr = cProfile.Profile(); pr.enable()
for _ in range(20):
    ts.step()
torch.cuda.synchronize(); pr.disable()
st = io.StringIO(); pstats.Stats(pr, stream=st).sort_stats("tottime").print_stats(30); print(st.getvalue()[:6000])
