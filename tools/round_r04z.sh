#!/bin/bash
# round 4: dense-H passes with closed-form U offsets — parity, DI(3) dense-H profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04z}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_pad_gpu.py -m gpu -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/pad_tests.log 2>&1 || { tail -40 gpurun_out/$T/pad_tests.log; exit 1; }
tail -3 gpurun_out/$T/pad_tests.log
TAG=${T}_di0 tools/gpu_measure.sh prof --workload kkt --kkt-structure di --N 101 --batch 16384 --kkt-hmode 0 --cpu-seconds 3 || exit 2
