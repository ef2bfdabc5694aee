#!/bin/bash
# round 4: backward KKT kernel with partial D2 hold (fp64 32 columns, fp32 wide knots)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04ae}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_big_gpu.py tests/test_full_size_gpu.py -m gpu -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/big_tests.log 2>&1 || { tail -40 gpurun_out/$T/big_tests.log; exit 1; }
tail -3 gpurun_out/$T/big_tests.log
TAG=${T}_kkt64 tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 4096 --dtype f64 --no-cpu-baseline || exit 2
TAG=${T}_kkt tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 --no-cpu-baseline || exit 3
