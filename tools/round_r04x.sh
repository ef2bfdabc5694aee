#!/bin/bash
# round 4: padded direct KKT kernel (Shape<…, PAD>) — parity tests, then (6,2,101) beside the
# exact (5,2,101) shape and the large-block path it replaces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04x}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_gpu.py tests/test_kkt_pad_gpu.py tests/test_abi.py -m gpu -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/pad_tests.log 2>&1 || { tail -40 gpurun_out/$T/pad_tests.log; exit 1; }
tail -3 gpurun_out/$T/pad_tests.log
timeout -k 10 300 python -u -m pytest tests/test_kkt_big_gpu.py tests/test_sqp.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/big_tests.log 2>&1 || { tail -40 gpurun_out/$T/big_tests.log; exit 6; }
tail -3 gpurun_out/$T/big_tests.log
B="--workload kkt --kkt-structure dense --N 101 --batch 16384 --dtype f64 --cpu-seconds 3"
TAG=${T}_t62 tools/gpu_measure.sh bench $B --n 6 --m 2 || exit 2
TAG=${T}_t52 tools/gpu_measure.sh bench $B --n 5 --m 2 || exit 3
TAG=${T}_t63 tools/gpu_measure.sh bench $B --n 6 --m 3 || exit 4
LQRX_KKT_PAD=0 TAG=${T}_t62big tools/gpu_measure.sh bench $B --n 6 --m 2 --no-cpu-baseline || exit 5
