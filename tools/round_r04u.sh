#!/bin/bash
# round 4: workgroup KKT kernel after the wg routine rework (tests + n=96 bench with prof)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04u}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_kkt_wg_gpu.py tests/test_dp_big_gpu.py tests/test_abi.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/wg_tests.log 2>&1 || { tail -40 gpurun_out/$T/wg_tests.log; exit 1; }
tail -3 gpurun_out/$T/wg_tests.log
TAG=${T}_wg tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 96 --m 48 --N 64 --batch 2048 --dtype f64 || exit 2
