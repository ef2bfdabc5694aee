#!/bin/bash
# cartpole (dp_quad_kernel) and LS (ls_condensed_kernel): kernel stats + HBM traffic passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/small_${TAG:-x}
mkdir -p $OUT
for wl in cartpole ls; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 20 --cpu-seconds 4 > $OUT/$wl.json 2> $OUT/$wl.err || { tail -20 $OUT/$wl.err; exit 2; }
  cat $OUT/$wl.json
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt_$wl -o kt --output-format csv -- python bench.py --workload $wl --steps 20 --warmup 20 --no-cpu-baseline > $OUT/kt_$wl.log 2>&1 || { tail -20 $OUT/kt_$wl.log; exit 3; }
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_$wl -o f --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > $OUT/f_$wl.log 2>&1 || { tail -5 $OUT/f_$wl.log; exit 4; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_$wl -o w --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > $OUT/w_$wl.log 2>&1 || { tail -5 $OUT/w_$wl.log; exit 5; }
done
