#!/bin/bash
# round 4: dp_big on the blocked workgroup factor/solves (tests + the §3.8 bench lines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04v}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_dp_big_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$T/big_tests.log 2>&1 || { tail -40 gpurun_out/$T/big_tests.log; exit 1; }
tail -3 gpurun_out/$T/big_tests.log
TAG=${T}_n128 tools/gpu_measure.sh bench --n 128 --m 64 --N 64 --batch 2048 --dtype f64 || exit 2
TAG=${T}_n96 tools/gpu_measure.sh bench --n 96 --m 48 --N 256 --batch 4096 --dtype f64 || exit 3
