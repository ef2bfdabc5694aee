#!/bin/bash
# Linear-cost-term DP: parity tests, then bench lines (cfg4 shape plain vs linear, cartpole
# plain vs linear, time-varying linear).  Each GPU step under its own timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r2_${TAG:-lin}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dp_linear_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/lin_tests.log 2>&1 || { tail -30 $OUT/lin_tests.log; exit 1; }
tail -2 $OUT/lin_tests.log
bench() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$nm.json 2> $OUT/bench_$nm.err || { tail -20 $OUT/bench_$nm.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/bench_$nm.json')); r=d['roofline']; print('$nm', round(d['value']), round(d['ms_per_step'],4), 'ms', r['bound'], round(r['frac'],4), (d.get('check') or {}).get('sampled_parity',{}) and d['check']['sampled_parity'].get('pass'))"
}
bench cfg4 --no-cpu-baseline
bench lin --linear --no-cpu-baseline
bench lin_tv --linear --tv --no-cpu-baseline
bench cartpole --workload cartpole --steps 20 --warmup 20 --no-cpu-baseline
bench lin_cp --workload cartpole --linear --steps 20 --warmup 20 --no-cpu-baseline
[ -n "$PROF" ] || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/lin_kt -o kt --output-format csv -- python bench.py --linear --steps 3 --warmup 1 --no-cpu-baseline > $OUT/lin_kt.log 2>&1 || { tail -20 $OUT/lin_kt.log; exit 4; }
