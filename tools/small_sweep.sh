#!/bin/bash
# lane vs quad small-n DP kernel across batch sizes (cartpole n=4 m=1 N=101)
cd "$GRAFT_REPO_ROOT" || exit 1
for B in 16384 32768 65535; do
  for mode in lane quad; do
    LQRX_DP_SMALL=$mode timeout -k 10 120 python bench.py --workload cartpole --batch $B --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/sw_${mode}_$B.json 2>/dev/null || exit 3
    python -c "import json; d=json.load(open('gpurun_out/sw_${mode}_$B.json')); print('$mode', $B, d['value'], d['roofline']['kernel_ms'])"
  done
done
