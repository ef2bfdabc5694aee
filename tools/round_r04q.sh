#!/bin/bash
# round 4: KKT layout-1 staging (every structure), workgroup + large-block KKT tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04q}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_gpu.py -m gpu -x -q -k "layout1" --timeout 300 \
    --timeout-method thread > gpurun_out/$T/layout1_tests.log 2>&1 || { tail -40 gpurun_out/$T/layout1_tests.log; exit 1; }
tail -3 gpurun_out/$T/layout1_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 2; }
tail -3 gpurun_out/$T/gpu_tests.log
