#!/bin/bash
# Time one workload under several builds of liblqrx.so (LIBS = names under lqr.jl_amd/lqrx/,
# "main" = the in-tree liblqrx.so), alternating, REPS rounds.  Ablation / A-B studies.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/libs_${TAG:-x}
mkdir -p $OUT
for i in $(seq ${REPS:-2}); do
  for L in ${LIBS:-main}; do
    if [ $L = main ]; then unset LQRX_LIB; else export LQRX_LIB=$PWD/lqr.jl_amd/lqrx/$L.so; fi
    timeout -k 10 120 python bench.py --workload ${WL:-kkt} --steps 20 --warmup 20 --no-cpu-baseline ${BARGS:-} > $OUT/$L$i.json 2> $OUT/$L$i.err || { tail -5 $OUT/$L$i.err; exit 2; }
    python -c "import json; d=json.load(open('$OUT/$L$i.json')); print('$L', $i, round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],4))"
  done
done
