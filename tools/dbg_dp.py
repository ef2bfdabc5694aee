import sys, numpy as np
sys.path[:0] = ['/root/repo/lqr.jl_amd', '/root/repo']
import lqrx
from lqrx.dp import abi_to_batch, from_abi
from oracle import oracle as o
np.set_printoptions(precision=4, linewidth=150)
for (n, m, N, bt, seed) in [(4,1,101,64,1000+4*7+1), (4,1,101,2,1), (4,1,20,64,1), (4,1,101,64,1)]:
    d = lqrx.random_batch(n, m, N, bt, seed=seed)
    b = abi_to_batch(d)
    got = lqrx.solve_batch(b, all_P=True)
    ref = o.dp_solve_abi(d, N, all_P=True)
    K = from_abi(ref['K'], (bt, N-1, m, n)); P = from_abi(ref['P'], (bt, N, n, n))
    e = np.abs(got['K'] - K).max(axis=(2,3))
    bad = np.argwhere(e > 1e-8)
    print(n, m, N, bt, 'maxerr', e.max(), 'n bad', len(bad), bad[:5].tolist(), 'info', got['info'][:8], ref['info'][:8])
    if len(bad):
        t, k = bad[0]
        print('K got', got['K'][t, k], '\nK ref', K[t, k])
        print('P got', got['P'][t, k+1], '\nP ref', P[t, k+1])
        print('|K| max', np.abs(K).max(), 'E diag?')
