#!/bin/bash
# LS / sparse formulation: GPU parity tests, bench line, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ls_${TAG:-x}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ls.py tests/test_golden.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -8 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload ls --steps 10 --warmup 3 --cpu-seconds 4 > $OUT/ls.json 2> $OUT/ls.err || { tail -20 $OUT/ls.err; exit 3; }
cat $OUT/ls.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ls --output-format csv -- python bench.py --workload ls --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 4; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
