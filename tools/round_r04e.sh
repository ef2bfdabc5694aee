set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=r04e tools/gpu_measure.sh tests || exit 1
TAG=r04e_cfg4 tools/gpu_measure.sh prof || exit 2
TAG=r04e_cfg5 tools/gpu_measure.sh bench --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 3
TAG=r04e_kktpmc PMC="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" tools/gpu_measure.sh pmc --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 4
