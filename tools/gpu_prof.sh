#!/bin/bash
# Full-size bench + rocprofv3 kernel-trace stats + separate PMC passes for HBM bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r01}
mkdir -p $OUT
nproc > $OUT/host.txt; lscpu | head -20 >> $OUT/host.txt
timeout -k 10 400 python bench.py --steps ${STEPS:-5} --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 4; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 5; }
find $OUT -name "*.csv" | head -20
