#!/bin/bash
# KKT (cfg3) iteration loop: KKT parity tests on the in-tree library, then A/B timing of the
# kkt workload — in-tree liblqrx.so (A) vs lqr.jl_amd/lqrx/liblqrx_alt.so (B), alternating —
# and rocprofv3 kernel stats of A.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/kab_${TAG:-x}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kkt_gpu.py tests/test_sqp.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
ALT=$PWD/lqr.jl_amd/lqrx/liblqrx_alt.so
for i in $(seq ${REPS:-3}); do
  for v in A B; do
    if [ $v = B ]; then export LQRX_LIB=$ALT; else unset LQRX_LIB; fi
    timeout -k 10 120 python bench.py --workload kkt --steps 20 --warmup 20 --no-cpu-baseline ${BARGS:-} > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -5 $OUT/$v$i.err; exit 2; }
    python -c "import json; d=json.load(open('$OUT/$v$i.json')); print('$v', $i, round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],4), d['check']['sampled_parity']['pass'])"
  done
done
unset LQRX_LIB
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --workload kkt --steps 20 --warmup 20 --no-cpu-baseline > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 3; }
find $OUT/kt -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -8
