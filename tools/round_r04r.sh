#!/bin/bash
# round 4: small-n DP hex kernel tests + cfg2 bench/prof; KKT layout-1 staging; full suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04r}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_dp_lane_gpu.py tests/test_layout_gpu.py tests/test_dp_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/small_tests.log 2>&1 || { tail -40 gpurun_out/$T/small_tests.log; exit 1; }
tail -3 gpurun_out/$T/small_tests.log
TAG=${T}_cfg2 tools/gpu_measure.sh prof --workload cartpole || exit 2
LQRX_DP_SMALL=quad timeout -k 10 300 python -u bench.py --workload cartpole > gpurun_out/$T/cfg2_quad.json 2>gpurun_out/$T/cfg2_quad.err || exit 3
tail -c 400 gpurun_out/$T/cfg2_quad.json
timeout -k 10 600 python -u -m pytest tests/test_kkt_gpu.py -m gpu -x -q -k "layout1" --timeout 300 \
    --timeout-method thread > gpurun_out/$T/layout1_tests.log 2>&1 || { tail -40 gpurun_out/$T/layout1_tests.log; exit 4; }
tail -3 gpurun_out/$T/layout1_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 5; }
tail -3 gpurun_out/$T/gpu_tests.log
