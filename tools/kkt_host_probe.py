"""Host-side cost of one lqrx_kkt_solve_ws call vs the kernel (cfg3), and a hipGraph-captured
step.  Diagnoses gaps between consecutive KKT kernels in the rocprof trace."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lqr.jl_amd"))
import torch
import lqrx.kkt as K

st = K.dubins_structure(101)
bt = 16384
pb = K.random_kkt(st, bt, seed=1, h_mode=K.H_DIAG)
t = {k: torch.from_numpy(getattr(pb, k).ravel()).cuda() for k in ("Y", "y", "H", "g")}
t["batch"] = bt
s = torch.cuda.Stream()
sh = s.cuda_stream
ws = torch.empty(K.workspace_size(st, bt, K.H_DIAG, 1), dtype=torch.uint8, device="cuda")
with torch.cuda.stream(s):
    out = K.kkt_solve_device(st, t, K.H_DIAG, 1, stream=sh, workspace=ws)
torch.cuda.synchronize()
d = st.desc(bt, K.H_DIAG, 1)
lib = K._lib.load()
import ctypes as C
p = lambda x: C.c_void_p(x.data_ptr())
args = [C.byref(d), p(t["Y"]), p(t["y"]), p(t["H"]), p(t["g"]), p(out["dz"]), p(out["lam"]), p(out["info"]), p(ws),
        ws.numel(), C.c_void_p(sh)]
for label, fn in (("python wrapper", lambda: K.kkt_solve_device(st, t, K.H_DIAG, 1, stream=sh, out=out, workspace=ws)),
                  ("raw ctypes", lambda: lib.lqrx_kkt_solve_ws(*args))):
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{label}: host {1e6 * (t1 - t0) / n:.1f} us/call, wall {1e6 * (t2 - t0) / n:.1f} us/step")
# graph capture of one solve
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    lib.lqrx_kkt_solve_ws(*args[:-1], C.c_void_p(s.cuda_stream))
torch.cuda.synchronize()
n = 50
t0 = time.perf_counter()
for _ in range(n):
    g.replay()
torch.cuda.synchronize()
print(f"graph replay: wall {1e6 * (time.perf_counter() - t0) / n:.1f} us/step")
