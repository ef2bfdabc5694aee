#!/bin/bash
# round 4: full GPU suite at HEAD, configs[4] KKT prof + FETCH/WRITE, cfg4 DP SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04n}
TAG=$T tools/gpu_measure.sh tests || exit 1
TAG=${T}_kkt tools/gpu_measure.sh prof --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
TAG=${T}_kkt64 tools/gpu_measure.sh bench --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 4096 --dtype f64 || exit 3
TAG=${T}_dppmc PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY;SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT" tools/gpu_measure.sh pmc || exit 4
