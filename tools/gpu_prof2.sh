#!/bin/bash
# Round profile set: for each workload, the bench line (CPU baseline on dp), rocprofv3
# kernel-trace stats of the same command, and separate FETCH_SIZE / WRITE_SIZE PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-x}
mkdir -p $OUT
nproc > $OUT/host.txt; lscpu | head -20 >> $OUT/host.txt
for wl in ${WLS:-dp kkt cartpole}; do
  CB="--cpu-seconds ${CPUS:-10}"
  timeout -k 10 400 python bench.py --workload $wl --steps ${STEPS:-5} --warmup 1 $CB > $OUT/${wl}_bench.json 2> $OUT/${wl}_bench.err || { tail -20 $OUT/${wl}_bench.err; exit 2; }
  cat $OUT/${wl}_bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${wl}_kt -o kt --output-format csv -- python bench.py --workload $wl --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > $OUT/${wl}_kt.log 2>&1 || { tail -20 $OUT/${wl}_kt.log; exit 3; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/${wl}_fetch -o fetch --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > $OUT/${wl}_fetch.log 2>&1 || { tail -20 $OUT/${wl}_fetch.log; exit 4; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/${wl}_write -o write --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > $OUT/${wl}_write.log 2>&1 || { tail -20 $OUT/${wl}_write.log; exit 5; }
done
find $OUT -name "*stats.csv" | head -20
