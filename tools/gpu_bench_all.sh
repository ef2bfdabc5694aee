#!/bin/bash
# Bench every BASELINE config this build covers (1 GPU), plus rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/bench_${TAG:-x}
mkdir -p $OUT
for wl in kkt cartpole; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --cpu-seconds ${CPUS:-8} > $OUT/$wl.json 2> $OUT/$wl.err || { tail -20 $OUT/$wl.err; exit 2; }
  cat $OUT/$wl.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$wl -o kt --output-format csv -- python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > $OUT/kt_$wl.log 2>&1 || { tail -20 $OUT/kt_$wl.log; exit 3; }
done
