#!/bin/bash
# round 4: backward KKT kernel with D2 held in registers (large-block tests + configs[4] KKT prof)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04w}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_big_gpu.py tests/test_abi.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/big_tests.log 2>&1 || { tail -40 gpurun_out/$T/big_tests.log; exit 1; }
tail -3 gpurun_out/$T/big_tests.log
TAG=${T}_kkt tools/gpu_measure.sh prof --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
