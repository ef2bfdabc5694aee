"""Per-step wall time of the cartpole (cfg2) DP solve: plain launches vs a captured hipGraph
(kernel arguments baked into the graph).  Run with and without HIP_FORCE_DEV_KERNARG=0."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lqr.jl_amd"))
import torch
import lqrx
from lqrx.models import cartpole_batch
from lqrx.dp import to_abi

N, bt = 101, 4096
cb = cartpole_batch(bt, N, seed=1)
host = {k: to_abi(getattr(cb, k)).ravel() for k in ("A", "B", "Q", "R", "Qf")}
host["x0"] = cb.x0.ravel()
t = {k: torch.from_numpy(host[k]).cuda() for k in host}
t.update(n=4, m=1, batch=bt)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    out = lqrx.dp_solve_device(t, N, stream=s.cuda_stream)
    for _ in range(200):
        lqrx.dp_solve_device(t, N, stream=s.cuda_stream, out=out)
torch.cuda.synchronize()
n = 500
t0 = time.perf_counter()
with torch.cuda.stream(s):
    for _ in range(n):
        lqrx.dp_solve_device(t, N, stream=s.cuda_stream, out=out)
torch.cuda.synchronize()
print(f"launches: {1e6 * (time.perf_counter() - t0) / n:.1f} us/step  (DEV_KERNARG={os.environ.get('HIP_FORCE_DEV_KERNARG')})")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    for _ in range(10):
        lqrx.dp_solve_device(t, N, stream=s.cuda_stream, out=out)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n // 10):
    g.replay()
torch.cuda.synchronize()
print(f"graph (10 solves per replay): {1e6 * (time.perf_counter() - t0) / n:.1f} us/step")
