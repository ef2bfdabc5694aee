#!/bin/bash
# round 4: leaf triangular inverse without LDS round trips (large-block KKT), dense-H DI bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04y}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_big_gpu.py tests/test_kkt_wg_gpu.py -m gpu -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/big_tests.log 2>&1 || { tail -40 gpurun_out/$T/big_tests.log; exit 1; }
tail -3 gpurun_out/$T/big_tests.log
TAG=${T}_kkt tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 --no-cpu-baseline || exit 2
TAG=${T}_kkt64 tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 4096 --dtype f64 --no-cpu-baseline || exit 3
TAG=${T}_di0 tools/gpu_measure.sh bench --workload kkt --kkt-structure di --N 101 --batch 16384 --kkt-hmode 0 --cpu-seconds 3 || exit 4
TAG=${T}_di2 tools/gpu_measure.sh bench --workload kkt --kkt-structure di --N 101 --batch 16384 --no-cpu-baseline || exit 5
# cfg3 layout 0: staging DMA with the non-temporal policy (A/B library tools/abl/liblqrx_nt.so)
TAG=${T}_cfg3 tools/gpu_measure.sh prof --workload kkt --no-cpu-baseline || exit 6
LQRX_LIB=$PWD/tools/abl/liblqrx_nt.so TAG=${T}_cfg3nt tools/gpu_measure.sh prof --workload kkt --no-cpu-baseline || exit 7
