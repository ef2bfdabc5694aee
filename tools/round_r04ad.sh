#!/bin/bash
# round 4: padded bin (8,4,8,1,8) — parity, and (8,4,101) / (7,3,101)-class lines beside the large-block path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04ad}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_pad_gpu.py -m gpu -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/pad_tests.log 2>&1 || { tail -40 gpurun_out/$T/pad_tests.log; exit 1; }
tail -3 gpurun_out/$T/pad_tests.log
B="--workload kkt --kkt-structure dense --N 101 --batch 16384 --dtype f64 --no-cpu-baseline"
TAG=${T}_t84 tools/gpu_measure.sh bench $B --n 8 --m 4 || exit 2
LQRX_KKT_PAD=0 TAG=${T}_t84big tools/gpu_measure.sh bench $B --n 8 --m 4 || exit 3
TAG=${T}_t72 tools/gpu_measure.sh bench $B --n 7 --m 2 || exit 4
LQRX_KKT_PAD=0 TAG=${T}_t72big tools/gpu_measure.sh bench $B --n 7 --m 2 || exit 5
