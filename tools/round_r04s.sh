#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r04s
timeout -k 10 300 python -u tools/hex_diag.py > gpurun_out/r04s/hex_diag.log 2>&1
rc=$?; cat gpurun_out/r04s/hex_diag.log | tail -20
case $rc in 0|1) ;; *) exit 9 ;; esac
TAG=r04s tools/round_r04r.sh
