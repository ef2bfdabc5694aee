#!/bin/bash
# quad-per-trajectory DP kernel: lane-kernel parity tests in both small-batch modes, cfg2 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/quad_${TAG:-x}
mkdir -p $OUT
LQRX_DP_SMALL=quad timeout -k 10 300 python -u -m pytest tests/test_dp_lane_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t_quad.log 2>&1; rc=$?
tail -3 $OUT/t_quad.log
[ $rc -eq 0 ] || exit $rc
for mode in lane quad; do
  LQRX_DP_SMALL=$mode timeout -k 10 200 python bench.py --workload cartpole --steps 20 --warmup 20 --no-cpu-baseline > $OUT/b_$mode.json 2> $OUT/b_$mode.err || { tail -20 $OUT/b_$mode.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/b_$mode.json')); print('$mode', d['value'], d['roofline']['kernel_ms'])"
done
for B in 16384 65536; do
for mode in lane quad; do
  LQRX_DP_SMALL=$mode timeout -k 10 200 python bench.py --workload cartpole --batch $B --steps 20 --warmup 20 --no-cpu-baseline > $OUT/b_${mode}_$B.json 2> $OUT/b_$mode.err || { tail -20 $OUT/b_$mode.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/b_${mode}_$B.json')); print('$mode $B', d['value'], d['roofline']['kernel_ms'])"
done
done
