#!/bin/bash
# A/B of liblqrx.so (A) vs liblqrx_alt.so (B) on several workloads (WL), then the DP parity
# tests against B.  Each GPU step under its own timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ab_${TAG:-x}
mkdir -p $OUT
ALT=$PWD/lqr.jl_amd/lqrx/liblqrx_alt.so
if [ -n "$TESTS" ]; then
  LQRX_LIB=$ALT timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
IFS=';' read -ra W <<< "${WL:---steps 5 --warmup 1}"
for i in $(seq ${REPS:-2}); do
  for w in "${W[@]}"; do
    for v in A B; do
      if [ $v = B ]; then export LQRX_LIB=$ALT; else unset LQRX_LIB; fi
      timeout -k 10 300 python bench.py $w --no-cpu-baseline > $OUT/r.json 2> $OUT/r.err || { tail -5 $OUT/r.err; exit 2; }
      python -c "import json; d=json.load(open('$OUT/r.json')); print('$v', $i, '$w', round(d['roofline']['kernel_ms'],4), 'ms', round(d['value']), round(d['roofline']['frac'],4), d['check']['sampled_parity'] and d['check']['sampled_parity']['pass'])"
    done
  done
done
