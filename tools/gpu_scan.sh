#!/bin/bash
# batch-size scan of the small workloads (latency- vs throughput-bound diagnosis)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/scan_${TAG:-x}
mkdir -p $OUT
for wl in ${WLS:-kkt cartpole}; do
  for b in ${BATCHES:-1024 4096 16384 65536 262144}; do
    timeout -k 10 120 python bench.py --workload $wl --batch $b --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${wl}_$b.json 2> $OUT/${wl}_$b.err || { tail -20 $OUT/${wl}_$b.err; exit 2; }
    python -c "import json,sys; d=json.load(open('$OUT/${wl}_$b.json')); print('$wl', $b, round(d['roofline']['kernel_ms'],4), 'ms', round(d['value']/1e6,3), 'M/s')"
  done
done
