#!/bin/bash
# Re-entry check: full GPU parity suite, then headline + kkt + cartpole bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/check_${TAG:-x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 5; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py --cpu-seconds ${CPUS:-6} > $OUT/dp.json 2> $OUT/dp.err || { tail -20 $OUT/dp.err; exit 2; }
cat $OUT/dp.json
for wl in kkt cartpole; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --cpu-seconds ${CPUS:-6} > $OUT/$wl.json 2> $OUT/$wl.err || { tail -20 $OUT/$wl.err; exit 3; }
  cat $OUT/$wl.json
done
