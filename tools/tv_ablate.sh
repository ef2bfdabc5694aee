#!/bin/bash
# Build (here, on the CPU) liblqrx variants for A/B runs (the bench runs on each with
# LQRX_LIB=tools/abl/liblqrx_<name>.so).  Large-block KKT ablations:
#   SRC=lqrx_kkt_big.hip tools/tv_ablate.sh noleaf:-DKB_ABL=1 noschur:-DKB_ABL=2 ...  One source (SRC, default lqrx_dp.hip) is rebuilt with extra defines; the
# others are linked from the in-tree build.  Arguments: name:defines ...  Defaults (SRC =
# lqrx_dp.hip): the time-varying DP ablation of profiles/r02/dp_tv_ablation_r02.txt —
#   TVABL bit 1: Q_k re-read from knot 1 (cache-resident); bit 2: A_k/B_k/R_k likewise
#   TVEXTRA 4: no rollout (VAR_NOROLL);  TVKD / TVAD: rollout prefetch depths
set -e
cd "$(dirname "$0")/../lqr.jl_amd/csrc"
SRC=${SRC:-lqrx_dp.hip}
OBJS=""
for f in $(sed -n 's/^SRCS *= *//p' Makefile); do
  [ $f = $SRC ] || OBJS="$OBJS build/$f.o"
done
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../../include -munsafe-fp-atomics"
mk() {  # name, defines
  /opt/rocm/bin/hipcc $FL $2 -c $SRC -o build/abl_$1.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/abl/liblqrx_$1.so build/abl_$1.o $OBJS -lpthread
}
if [ $# -eq 0 ]; then set -- q:-DLQRX_DP_TVABL=1 abr:-DLQRX_DP_TVABL=2 all:-DLQRX_DP_TVABL=3 \
    noroll:-DLQRX_DP_TVEXTRA=4 "noroll_all:-DLQRX_DP_TVEXTRA=4 -DLQRX_DP_TVABL=3"; fi
mkdir -p ../../tools/abl
for v in "$@"; do mk "${v%%:*}" "${v#*:}" & done   # name:defines
wait
