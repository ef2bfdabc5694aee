#!/bin/bash
# round 4: FETCH_SIZE calibration per load width (tools/fetch_calib) and SQ counters of the
# committed configs[4] KKT kernels (kb_fuse_mid_kernel, kb_bwd_kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04ac}
mkdir -p gpurun_out/$T
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$T/calib -o fc --output-format csv -- ./tools/fetch_calib \
    > gpurun_out/$T/calib.log 2>&1 || { tail -20 gpurun_out/$T/calib.log; exit 1; }
tail -2 gpurun_out/$T/calib.log
KREGEX="kb_" PMC="SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES" \
    TAG=${T}_sq tools/gpu_measure.sh pmc --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
find gpurun_out/${T}_sq -name "*counter_collection.csv"
