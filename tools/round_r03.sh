#!/bin/bash
# full validation + measurement set for round 3 (run on the GPU box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=r03e tools/gpu_measure.sh tests || exit 1
TAG=r03e_cfg5kkt tools/gpu_measure.sh prof --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
TAG=r03e_cfg4 tools/gpu_measure.sh bench || exit 3
TAG=r03e_cfg3 tools/gpu_measure.sh bench --workload kkt || exit 4
TAG=r03e_cfg2 tools/gpu_measure.sh bench --workload cartpole || exit 5
TAG=r03e_cfg5 tools/gpu_measure.sh bench --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 6
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03e/smoke.log 2>&1 || exit 7
tail -2 gpurun_out/r03e/smoke.log
