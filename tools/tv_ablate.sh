#!/bin/bash
# Build (here, on the CPU) liblqrx variants whose time-varying DP kernel drops one source of
# work each, for the A/B of DESIGN.md §3.1 (VAR_TV).  Run the bench on each with LQRX_LIB.
#   TVABL bit 1: Q_k re-read from knot 1 (cache-resident); bit 2: A_k/B_k/R_k likewise
#   TVEXTRA 4: no rollout (VAR_NOROLL)
set -e
cd "$(dirname "$0")/../lqr.jl_amd/csrc"
OBJS="build/lqrx_dp_lane.hip.o build/lqrx_layout.hip.o build/lqrx_kkt.hip.o build/lqrx_kkt_fil.hip.o build/lqrx_sqp.hip.o build/lqrx_ls.hip.o build/lqrx_api.cpp.o"
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../../include -munsafe-fp-atomics"
mk() {  # name, defines
  /opt/rocm/bin/hipcc $FL $2 -c lqrx_dp.hip -o build/dp_$1.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/abl/liblqrx_$1.so build/dp_$1.o $OBJS -lpthread
}
#   TVKD / TVAD: rollout prefetch depth (knots) of K_k and of the A_k/B_k rows
if [ $# -eq 0 ]; then set -- q:-DLQRX_DP_TVABL=1 abr:-DLQRX_DP_TVABL=2 all:-DLQRX_DP_TVABL=3 \
    noroll:-DLQRX_DP_TVEXTRA=4 "noroll_all:-DLQRX_DP_TVEXTRA=4 -DLQRX_DP_TVABL=3"; fi
for v in "$@"; do mk "${v%%:*}" "${v#*:}" & done   # name:defines
wait
