#!/bin/bash
# Lane-per-trajectory SQP kernels (SoA loop for Dubins / cartpole): GPU tests, bench lines,
# kernel-trace stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r2_${TAG:-f}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_sqp.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bench() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$nm.json 2> $OUT/bench_$nm.err || { tail -20 $OUT/bench_$nm.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/bench_$nm.json')); r=d['roofline']; print('$nm', round(d['value']), round(d['ms_per_step'],4), 'ms', round(r['frac'],4), (d.get('check') or {}).get('sampled_parity'))"
}
bench sqp --workload sqp --steps 3 --warmup 1 --cpu-seconds 4
bench sqp_cp --workload sqp --sqp-model cartpole --steps 3 --warmup 1 --cpu-seconds 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sqp_kt -o kt --output-format csv -- python bench.py --workload sqp --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sqp_kt.log 2>&1 || { tail -20 $OUT/sqp_kt.log; exit 4; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sqp_cp_kt -o kt --output-format csv -- python bench.py --workload sqp --sqp-model cartpole --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sqp_cp_kt.log 2>&1 || { tail -20 $OUT/sqp_cp_kt.log; exit 5; }
