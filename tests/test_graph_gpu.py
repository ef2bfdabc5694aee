"""hipGraph capture of the device entry points ("a call on a caller stream
allocates nothing from the driver and never synchronises, so it can be captured").

Each test warms the entry up on a side stream (structure-table upload, LDS attribute), captures
one call with torch.cuda.graph (capture_error_mode "global": any synchronising or allocating
HIP call inside the capture fails it), overwrites the captured input buffers with a second
problem, replays, and requires the replayed outputs to equal an eager call on that second
problem bit for bit.  The entries covered are the ones a graph-based caller would put in a
control loop: lqrx_dp_solve (layout 0: MFMA kernel, quad and lane kernels), lqrx_kkt_solve_ws
(caller workspace; FIL and generic kernels) and lqrx_ls_solve (LDS-resident path).
"""
import pytest

pytestmark = pytest.mark.gpu


def _capture_and_replay(call, inputs, second):
    """call(stream) -> outputs dict; inputs: dict of device tensors the call reads;
    second: dict of same-shaped tensors copied into `inputs` before the replay."""
    import torch

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        call(side.cuda_stream)                       # warm-up: caches, attributes
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = call(torch.cuda.current_stream().cuda_stream)
    for k, v in second.items():
        inputs[k].copy_(v)
    g.replay()
    torch.cuda.synchronize()
    got = {k: v.clone() for k, v in out.items() if hasattr(v, "clone")}
    ref = call(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return got, ref


def _dev(d, keys):
    import torch

    return {k: torch.from_numpy(d[k]).cuda() for k in keys}


@pytest.mark.parametrize("n,m,N,batch", [(6, 3, 21, 96), (4, 2, 16, 200), (2, 1, 11, 130)])
def test_graph_dp(lqrx, gpu_ok, n, m, N, batch):
    from lqrx.dp import dp_solve_device

    keys = ("A", "B", "Q", "R", "Qf", "x0")
    t = _dev(lqrx.random_batch(n, m, N, batch, 11), keys)
    t.update(n=n, m=m, batch=batch)
    second = _dev(lqrx.random_batch(n, m, N, batch, 12), keys)
    got, ref = _capture_and_replay(lambda s: dp_solve_device(t, N, 1, stream=s), t, second)
    for k in ("K", "P", "X", "U", "info"):
        assert got[k].equal(ref[k]), k


@pytest.mark.parametrize("which", ["dubins", "di3"])
def test_graph_kkt_ws(lqrx, gpu_ok, which):
    import torch
    import lqrx.kkt as K

    st, bt = (K.dubins_structure(101), 300) if which == "dubins" else (K.double_integrator_structure(3, 11), 70)
    keys = ("Y", "y", "H", "g")
    mk = lambda seed: {k: torch.from_numpy(getattr(K.random_kkt(st, bt, seed=seed, h_mode=K.H_DIAG), k).ravel()).cuda()
                       for k in keys}
    t = mk(5)
    t["batch"] = bt
    ws = torch.empty(K.workspace_size(st, bt, K.H_DIAG, 1), dtype=torch.uint8, device="cuda")
    got, ref = _capture_and_replay(
        lambda s: K.kkt_solve_device(st, t, K.H_DIAG, 1, stream=s, workspace=ws), t, mk(6))
    for k in ("dz", "lam", "info"):
        assert got[k].equal(ref[k]), k


def test_graph_ls(lqrx, gpu_ok):
    from lqrx.ls import ls_solve_device

    n, m, N, batch = 4, 2, 11, 64
    keys = ("A", "B", "Q", "R", "Qf", "x0")
    t = _dev(lqrx.random_batch(n, m, N, batch, 21), keys)
    t.update(n=n, m=m, batch=batch)
    second = _dev(lqrx.random_batch(n, m, N, batch, 22), keys)
    got, ref = _capture_and_replay(lambda s: ls_solve_device(t, N, stream=s), t, second)
    for k in ("U", "X", "info"):
        assert got[k].equal(ref[k]), k


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_graph_kkt_big(lqrx, gpu_ok, dt):
    """The large-block KKT path (split: Schur, general + interior factor, backward kernels) on
    a caller workspace captured in a hipGraph, fp64 and fp32 (n=16, m=8: 4 + 1 + 1 + 1 kernels
    per chunk)."""
    import numpy as np
    import torch
    import lqrx.kkt as K

    st, bt = K.trajectory_structure(16, 8, 13), 9
    keys = ("Y", "y", "H", "g")
    tdt = torch.float64 if dt == "f64" else torch.float32
    code = lqrx.F64 if dt == "f64" else lqrx.F32
    mk = lambda seed: {k: torch.from_numpy(np.ascontiguousarray(getattr(
        K.random_kkt(st, bt, seed=seed, h_mode=K.H_DIAG, dyn="dense"), k).ravel())).to("cuda", tdt) for k in keys}
    t = mk(5)
    t["batch"] = bt
    ws = torch.empty(K.workspace_size(st, bt, K.H_DIAG, 1, dtype=code), dtype=torch.uint8, device="cuda")
    got, ref = _capture_and_replay(
        lambda s: K.kkt_solve_device(st, t, K.H_DIAG, 1, stream=s, workspace=ws), t, mk(6))
    for k in ("dz", "lam", "info"):
        assert got[k].equal(ref[k]), k
