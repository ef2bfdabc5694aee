#!/bin/bash
# gpu_measure.sh — the measurement recipe behind profiles/ (run on the GPU box via gpurun).
#
#   TAG=r03a tools/gpu_measure.sh tests                 full `-m gpu` parity suite
#   TAG=r03a tools/gpu_measure.sh bench  [bench args]   one bench.py line → $OUT/bench.json
#   TAG=r03a tools/gpu_measure.sh prof   [bench args]   bench line, then rocprofv3 --kernel-trace
#                                                       --stats of the same command, then the
#                                                       FETCH_SIZE and WRITE_SIZE PMC passes
#                                                       (separately, as MI355X_MICROARCH.md says)
#   TAG=r03a PMC="SQ_WAVES SQ_INSTS_VALU;SQ_INSTS_LDS" tools/gpu_measure.sh pmc [bench args]
#                                                       one rocprofv3 --pmc pass per ';' group
#
# $OUT = gpurun_out/$TAG.  KREGEX (default "lqrx") restricts the PMC passes to the library's
# kernels; only the stats / counter CSVs are kept (gpurun copies back ≤ 64 MiB).  Every GPU step runs under its own timeout and the script stops at
# the first failure (no retries).  On the CPU side afterwards: tools/traffic_json.py turns the
# FETCH/WRITE CSVs into profiles/traffic_*.json (gfx950 FETCH×2 correction), tools/
# pmc_summary.py summarises SQ passes; copy what is judged into profiles/<round>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
MODE=${1:?mode: tests|bench|prof|pmc}
shift
OUT=gpurun_out/${TAG:-run}
KREGEX=${KREGEX:-lqrx}
trim() { find "$OUT" -type f \( -name "*.csv" -o -name "*.json" -o -name "*.db" \) ! -name "*stats.csv" ! -name "*counter_collection.csv" ! -name "bench.json" -delete 2>/dev/null; true; }
one_rank() {   # rocprofv3 modes profile ONE rank: a --gpus N > 1 bench would start its ranks
               # from a process the profiler's preload has already GPU-initialised
    local prev=""
    for a in "$@"; do
        if [ "$prev" = "--gpus" ] && [ "$a" != "1" ]; then echo "gpu_measure.sh: $MODE profiles one rank; drop --gpus $a" >&2; exit 1; fi
        case "$a" in --gpus=*) [ "${a#--gpus=}" != "1" ] && { echo "gpu_measure.sh: $MODE profiles one rank" >&2; exit 1; } ;; esac
        prev=$a
    done
}
case "$MODE" in prof|pmc) one_rank "$@" ;; esac
mkdir -p "$OUT"
nproc > "$OUT/host.txt"
lscpu | head -20 >> "$OUT/host.txt"
case "$MODE" in
tests)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1
    rc=$?
    tail -5 "$OUT/gpu_tests.log"
    exit $rc ;;
bench)
    timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 2; }
    cat "$OUT/bench.json" ;;
prof)
    timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 2; }
    cat "$OUT/bench.json"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
        python bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 3; }
    trim
    timeout -k 10 400 rocprofv3 --kernel-include-regex "$KREGEX" --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
        python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/fetch.log" 2>&1 || { tail -20 "$OUT/fetch.log"; exit 4; }
    timeout -k 10 400 rocprofv3 --kernel-include-regex "$KREGEX" --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
        python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/write.log" 2>&1 || { tail -20 "$OUT/write.log"; exit 5; }
    trim
    find "$OUT" -name "*stats.csv" ;;
pmc)
    i=0
    IFS=';' read -ra GROUPS_ <<< "${PMC:?PMC=\"COUNTERS;COUNTERS\"}"
    for grp in "${GROUPS_[@]}"; do
        i=$((i + 1))
        timeout -s KILL 300 rocprofv3 --kernel-include-regex "$KREGEX" --pmc $grp -d "$OUT/pmc$i" -o pmc$i --output-format csv -- \
            python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc$i.log" 2>&1 || { tail -20 "$OUT/pmc$i.log"; exit 6; }
    done
    trim ;;
*)
    echo "unknown mode $MODE" >&2; exit 1 ;;
esac
