#!/bin/bash
# round 4 (late): the whole -m gpu suite and smoke() at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04full}
mkdir -p gpurun_out/$T
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$T/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/$T/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 3; }
tail -3 gpurun_out/$T/smoke.log
