#!/bin/bash
# round 4: layout-0 output ring in the staged FIL kernel — parity, cfg3 layout 0 prof, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04ag}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_gpu.py tests/test_sqp.py tests/test_golden.py tests/test_graph_gpu.py -m gpu -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/kkt_tests.log 2>&1 || { tail -40 gpurun_out/$T/kkt_tests.log; exit 1; }
tail -3 gpurun_out/$T/kkt_tests.log
TAG=${T}_cfg3 tools/gpu_measure.sh prof --workload kkt --no-cpu-baseline || exit 2
LQRX_LIB=$PWD/tools/abl/liblqrx_noring.so TAG=${T}_cfg3old tools/gpu_measure.sh bench --workload kkt --no-cpu-baseline || exit 3
TAG=${T}_cfg3b tools/gpu_measure.sh bench --workload kkt --no-cpu-baseline || exit 4
