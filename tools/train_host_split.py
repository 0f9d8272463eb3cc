"""Host-issue vs device time of the fused train step, plus a cProfile of 20 steps (run on the GPU box:
`python tools/train_host_split.py`)."""
import cProfile, pstats, sys, time, io
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/street-sparse-3dgs_amd")
import torch
from gs_train.harness import make_problem
P, W, H = 1_000_000, 1920, 1080
ts = make_problem(P, W, H, n_views=4, seed=0, skybox_points=10_000)  # the bench's Street-sparse iteration
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
