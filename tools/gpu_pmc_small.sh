#!/bin/bash
# SQ counters for dp_quad_kernel (cartpole) and ls_condensed_kernel (separate --pmc passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmcs_${TAG:-x}
mkdir -p $OUT
for wl in cartpole ls; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/${wl}_p$i -o p$i --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > $OUT/${wl}_p$i.log 2>&1 || { tail -5 $OUT/${wl}_p$i.log; exit 3; }
  done
done
mkdir -p $OUT/c $OUT/l
cp -r $OUT/cartpole_p* $OUT/c/ && cp -r $OUT/ls_p* $OUT/l/
python tools/pmc_summary.py $OUT/c dp_quad > $OUT/quad_summary.txt && python tools/pmc_summary.py $OUT/l ls_condensed > $OUT/ls_summary.txt
cat $OUT/quad_summary.txt $OUT/ls_summary.txt
