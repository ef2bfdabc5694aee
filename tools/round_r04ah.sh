#!/bin/bash
# round 4: DP rollout of the linear-term variants on compiler-tracked loads (race fix) — tests,
# the linear-terms bench line and the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04ah}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_dp_linear_gpu.py tests/test_dp_gpu.py tests/test_full_size_gpu.py -m gpu -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/dp_tests.log 2>&1 || { tail -40 gpurun_out/$T/dp_tests.log; exit 1; }
tail -3 gpurun_out/$T/dp_tests.log
TAG=${T}_lin tools/gpu_measure.sh bench --linear --no-cpu-baseline || exit 2
TAG=${T}_cfg4 tools/gpu_measure.sh bench --no-cpu-baseline || exit 3
