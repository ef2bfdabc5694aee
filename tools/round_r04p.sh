#!/bin/bash
# round 4: workgroup KKT kernel tests, large-block KKT tests (bwd LDS trim), configs[4] KKT
# fp32 prof + fp64 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04p}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_kkt_wg_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/$T/wg_tests.log 2>&1
rc=$?
tail -15 gpurun_out/$T/wg_tests.log
case $rc in 0|1) ;; *) echo "wg tests rc=$rc: stopping"; exit 9 ;; esac
timeout -k 10 600 python -u -m pytest tests/test_kkt_big_gpu.py tests/test_full_size_gpu.py -m gpu -x -q -k "kkt" \
    --timeout 300 --timeout-method thread > gpurun_out/$T/big_tests.log 2>&1 || { tail -30 gpurun_out/$T/big_tests.log; exit 1; }
tail -3 gpurun_out/$T/big_tests.log
TAG=${T}_kkt tools/gpu_measure.sh prof --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
TAG=${T}_kkt64 tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 4096 --dtype f64 || exit 3
