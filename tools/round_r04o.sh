#!/bin/bash
# round 4: workgroup KKT kernel tests first, then the full GPU suite (without them), configs[4]
# KKT prof + FETCH/WRITE, fp64 KKT bench, cfg4 DP SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04o}
mkdir -p gpurun_out/${T}_wg
timeout -k 10 400 python -u -m pytest tests/test_kkt_wg_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_wg/wg_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${T}_wg/wg_tests.log
case $rc in 0|1) ;; *) echo "wg tests rc=$rc: stopping"; exit 9 ;; esac
mkdir -p gpurun_out/$T
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --ignore tests/test_kkt_wg_gpu.py > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$T/gpu_tests.log
TAG=${T}_kkt tools/gpu_measure.sh prof --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
TAG=${T}_kkt64 tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 4096 --dtype f64 || exit 3
TAG=${T}_dppmc PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY;SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT" tools/gpu_measure.sh pmc || exit 4
