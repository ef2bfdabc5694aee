#!/bin/bash
# Linear-cost-term DP parity first (new kernels), then the round-2 measurement set
# (tools/gpu_round2.sh).  A parity failure is reported and the set still runs; a time
# limit, abort or fault (exit 124/134/137/139) ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r2_${TAG:-h}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dp_linear_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/lin_tests.log 2>&1
rc=$?
tail -15 $OUT/lin_tests.log
case $rc in 124|134|137|139) echo "linear tests ended with $rc"; exit $rc;; esac
[ -n "$LIN_ONLY" ] && exit $rc
bash tools/gpu_round2.sh
