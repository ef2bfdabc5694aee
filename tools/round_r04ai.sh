#!/bin/bash
# round 4: PMC traffic for the padded / direct small-KKT lines (prof: stats + FETCH + WRITE)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04ai}
B="--workload kkt --kkt-structure dense --N 101 --batch 16384 --dtype f64 --no-cpu-baseline"
TAG=${T}_t62 KREGEX=kkt_ tools/gpu_measure.sh prof $B --n 6 --m 2 || exit 1
TAG=${T}_t84 KREGEX=kkt_ tools/gpu_measure.sh prof $B --n 8 --m 4 || exit 2
TAG=${T}_di KREGEX=kkt_ tools/gpu_measure.sh prof --workload kkt --kkt-structure di --no-cpu-baseline || exit 3
