#!/bin/bash
# A/B timing of the headline DP workload: in-tree liblqrx.so (A) vs lqr.jl_amd/lqrx/liblqrx_alt.so (B),
# alternating, REPS times each.  Extra bench args in BARGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/ab_${TAG:-x}
mkdir -p $OUT
ALT=$PWD/lqr.jl_amd/lqrx/liblqrx_alt.so
for i in $(seq ${REPS:-2}); do
  for v in A B; do
    if [ $v = B ]; then export LQRX_LIB=$ALT; else unset LQRX_LIB; fi
    timeout -k 10 300 python bench.py ${BARGS:-} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -5 $OUT/$v$i.err; exit 2; }
    python -c "import json; d=json.load(open('$OUT/$v$i.json')); print('$v', $i, round(d['roofline']['kernel_ms'],3), 'ms', round(d['value']), round(d['roofline']['frac'],4))"
  done
done
