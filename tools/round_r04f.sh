#!/bin/bash
# round 4: large-block KKT after a kernel change — parity (big + full-size KKT), the configs[4]
# KKT line with rocprof stats + FETCH/WRITE, and the SQ counters of the fused kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04f}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_kkt_big_gpu.py tests/test_full_size_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/t.log 2>&1
rc=$?; tail -3 gpurun_out/$T/t.log; [ $rc -eq 0 ] || exit 1
TAG=${T}_kkt tools/gpu_measure.sh prof --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
[ -n "$NOPMC" ] && exit 0
TAG=${T}_kktpmc PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY" tools/gpu_measure.sh pmc --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 3
