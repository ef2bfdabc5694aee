#!/bin/bash
# round 4: sub-millisecond lines with one HIP graph replayed per step (bench --graph) beside eager
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04aj}
TAG=${T}_cfg2g tools/gpu_measure.sh bench --workload cartpole --graph --no-cpu-baseline || exit 1
TAG=${T}_cfg2 tools/gpu_measure.sh bench --workload cartpole --no-cpu-baseline || exit 2
TAG=${T}_cfg3g tools/gpu_measure.sh bench --workload kkt --graph --no-cpu-baseline || exit 3
TAG=${T}_cfg3soag tools/gpu_measure.sh bench --workload kkt --kkt-layout 1 --graph --no-cpu-baseline || exit 4
TAG=${T}_cfg4g tools/gpu_measure.sh bench --graph --no-cpu-baseline || exit 5
