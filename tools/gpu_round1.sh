#!/bin/bash
# first GPU contact: parity tests, MFMA probe, short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_dp_gpu.py -x -q > gpurun_out/t1.log 2>&1; rc=$?
tail -30 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/mfma_probe > gpurun_out/probe.log 2>&1 || exit 3
cat gpurun_out/probe.log
timeout -k 10 300 python bench.py --batch 8192 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b1.log 2>&1 || { cat gpurun_out/b1.log; exit 4; }
cat gpurun_out/b1.log
