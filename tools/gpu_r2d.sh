#!/bin/bash
# KKT ABI layout 1 (batch-fastest SoA) on the compile-time-shaped kernel: GPU tests, bench
# lines for both layouts (alternating), kernel stats and PMC traffic of the SoA launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r2_${TAG:-d}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kkt_gpu.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for s in dubins di; do for L in 0 1; do timeout -k 10 200 python bench.py --workload kkt --kkt-structure $s --kkt-layout $L --steps 20 --warmup 20 --no-cpu-baseline > $OUT/b_${s}_$L.json 2>/dev/null && python -c "import json; d=json.load(open('$OUT/b_${s}_$L.json')); r=d['roofline']; print('$s layout $L', round(r['kernel_ms'],4), round(r['frac'],4), d['check']['sampled_parity']['pass'])" || exit 2; done; done
exit 0
for i in 1 2; do
  for L in 0 1; do
    timeout -k 10 200 python bench.py --workload kkt --kkt-layout $L --steps 20 --warmup 20 --no-cpu-baseline > $OUT/bench_kkt_l$L.$i.json 2> $OUT/bench_kkt_l$L.$i.err || { tail -20 $OUT/bench_kkt_l$L.$i.err; exit 3; }
    python -c "import json; d=json.load(open('$OUT/bench_kkt_l$L.$i.json')); r=d['roofline']; print('layout $L', round(d['value']), round(r['kernel_ms'],4), 'ms', round(r['frac'],4), d['check']['sampled_parity']['pass'])"
  done
done
timeout -k 10 200 python bench.py --workload kkt --kkt-layout 1 --steps 20 --warmup 20 --cpu-seconds 4 > $OUT/bench_kkt_soa.json 2> $OUT/bench_kkt_soa.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/soa_kt -o kt --output-format csv -- python bench.py --workload kkt --kkt-layout 1 --steps 20 --warmup 20 --no-cpu-baseline > $OUT/soa_kt.log 2>&1 || { tail -20 $OUT/soa_kt.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/soa_fetch -o fetch --output-format csv -- python bench.py --workload kkt --kkt-layout 1 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/soa_fetch.log 2>&1 || { tail -20 $OUT/soa_fetch.log; exit 5; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/soa_write -o write --output-format csv -- python bench.py --workload kkt --kkt-layout 1 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/soa_write.log 2>&1 || { tail -20 $OUT/soa_write.log; exit 6; }
for b in 4096 32768; do
  timeout -k 10 120 python bench.py --workload kkt --kkt-layout 1 --batch $b --steps 20 --warmup 20 --no-cpu-baseline > $OUT/scan_$b.json 2>/dev/null && python -c "import json; d=json.load(open('$OUT/scan_$b.json')); print('soa batch $b', round(d['roofline']['kernel_ms'],4))" || exit 7
done
