#!/bin/bash
# round 4: tiny trajectory structures — padded direct kernel vs the runtime-shaped generic kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04af}
mkdir -p gpurun_out/$T
B="--workload kkt --kkt-structure dense --N 101 --batch 16384 --dtype f64 --no-cpu-baseline"
for nm in "2 1" "3 1" "4 2"; do
    set -- $nm
    TAG=${T}_t$1$2 tools/gpu_measure.sh bench $B --n $1 --m $2 || exit 1
    LQRX_KKT_PAD=0 TAG=${T}_t$1$2gen tools/gpu_measure.sh bench $B --n $1 --m $2 || exit 2
done
