#!/bin/bash
# round 4 closing measurement set at HEAD (profiles/r04/f): smoke, every bench line of
# DESIGN §5 with rocprof stats (+ FETCH/WRITE) for the BASELINE configs, the new workgroup
# KKT and fp64 n=64 DP lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04t}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { cat gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
TAG=${T}_cfg4 tools/gpu_measure.sh prof || exit 2
TAG=${T}_cfg5 tools/gpu_measure.sh prof --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 3
TAG=${T}_cfg3 tools/gpu_measure.sh prof --workload kkt || exit 4
TAG=${T}_cfg3soa tools/gpu_measure.sh bench --workload kkt --kkt-layout 1 || exit 5
TAG=${T}_cfg2 tools/gpu_measure.sh prof --workload cartpole || exit 6
TAG=${T}_tv tools/gpu_measure.sh bench --tv --batch 16384 || exit 7
TAG=${T}_lin tools/gpu_measure.sh bench --linear || exit 8
TAG=${T}_di tools/gpu_measure.sh bench --workload kkt --kkt-structure di || exit 9
TAG=${T}_sqp tools/gpu_measure.sh bench --workload sqp || exit 10
TAG=${T}_sqpc tools/gpu_measure.sh bench --workload sqp --sqp-model cartpole || exit 11
TAG=${T}_ls tools/gpu_measure.sh bench --workload ls || exit 12
TAG=${T}_dp64 tools/gpu_measure.sh bench --n 64 --m 32 --N 512 --batch 8192 --dtype f64 || exit 13
TAG=${T}_wg tools/gpu_measure.sh prof --workload kkt --kkt-structure dense --n 96 --m 48 --N 64 --batch 2048 --dtype f64 || exit 14
