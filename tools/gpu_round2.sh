#!/bin/bash
# Round-2 measurement set on one MI355X: full GPU parity suite, smoke, the bench line of every
# workload (headline cfg4 first), rocprofv3 kernel-trace stats and separate PMC FETCH_SIZE /
# WRITE_SIZE passes for the dominant kernels.  Every GPU step has its own timeout; the first
# failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r2_${TAG:-x}
mkdir -p $OUT
nproc > $OUT/host.txt; lscpu | head -20 >> $OUT/host.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 2; }
  cat $OUT/smoke.log
fi
bench() {  # name, args...
  local nm=$1; shift
  timeout -k 10 400 python bench.py "$@" > $OUT/bench_$nm.json 2> $OUT/bench_$nm.err || { tail -20 $OUT/bench_$nm.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/bench_$nm.json')); r=d['roofline']; print('$nm', round(d['value']), round(d['ms_per_step'],4), 'ms', r['bound'], round(r['frac'],4), (d.get('check') or {}).get('sampled_parity',{}) and d['check']['sampled_parity'].get('pass'))"
}
bench cfg4 --cpu-seconds ${CPUS:-10}
bench cfg5 --n 64 --m 32 --N 512 --batch 8192 --dtype f32 --no-cpu-baseline
bench kkt --workload kkt --steps 20 --warmup 20 --cpu-seconds 6
bench kkt_di --workload kkt --kkt-structure di --steps 20 --warmup 20 --cpu-seconds 6
bench kkt_soa --workload kkt --kkt-layout 1 --steps 20 --warmup 20 --cpu-seconds 6
bench cartpole --workload cartpole --steps 20 --warmup 20 --cpu-seconds 6
bench tv --tv --no-cpu-baseline
bench ls --workload ls --steps 10 --warmup 5 --cpu-seconds 4
bench sqp --workload sqp --steps 3 --warmup 1 --cpu-seconds 4
bench sqp_cp --workload sqp --sqp-model cartpole --steps 3 --warmup 1
bench lin --linear --no-cpu-baseline
bench lin_cp --workload cartpole --linear --steps 20 --warmup 20 --no-cpu-baseline
[ -n "$SKIP_PROF" ] && exit 0
prof() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${nm}_kt -o kt --output-format csv -- python bench.py "$@" --no-cpu-baseline > $OUT/${nm}_kt.log 2>&1 || { tail -20 $OUT/${nm}_kt.log; exit 4; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${nm}_fetch -o fetch --output-format csv -- python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > $OUT/${nm}_fetch.log 2>&1 || { tail -20 $OUT/${nm}_fetch.log; exit 5; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${nm}_write -o write --output-format csv -- python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > $OUT/${nm}_write.log 2>&1 || { tail -20 $OUT/${nm}_write.log; exit 6; }
}
prof cfg4 --steps 5 --warmup 1
prof kkt --workload kkt --steps 20 --warmup 20
prof kkt_soa --workload kkt --kkt-layout 1 --steps 20 --warmup 20
prof cartpole --workload cartpole --steps 20 --warmup 20
prof tv --tv --steps 3 --warmup 1
prof ls --workload ls --steps 5 --warmup 2
prof lin --linear --steps 3 --warmup 1
prof lin_cp --workload cartpole --linear --steps 20 --warmup 20
profkt() {  # kernel trace only (whole-step workloads of several kernels)
  local nm=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${nm}_kt -o kt --output-format csv -- python bench.py "$@" --no-cpu-baseline > $OUT/${nm}_kt.log 2>&1 || { tail -20 $OUT/${nm}_kt.log; exit 7; }
}
profkt sqp --workload sqp --steps 3 --warmup 1
profkt sqp_cp --workload sqp --sqp-model cartpole --steps 3 --warmup 1
find $OUT -name "*kernel_stats.csv" | sort
