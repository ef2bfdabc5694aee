#!/bin/bash
# validation + measurement set for round 4 (run on the GPU box via gpurun):
#   TAG=r04a tools/round_r04.sh          tests, smoke, cfg4 bench + rocprof, configs[4] KKT bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04}
mkdir -p gpurun_out/$T
TAG=$T tools/gpu_measure.sh tests || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 2
tail -2 gpurun_out/$T/smoke.log
TAG=${T}_cfg4 tools/gpu_measure.sh prof || exit 3
TAG=${T}_cfg5kkt tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 4
