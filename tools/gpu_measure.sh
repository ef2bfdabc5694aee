#!/bin/bash
# gpu_measure.sh — the measurement recipe behind profiles/ (run on the GPU box via gpurun).
#
#   TAG=r05a tools/gpu_measure.sh tests                 full `-m gpu` parity suite + smoke()
#   TAG=r05a tools/gpu_measure.sh pytest FILES…         a subset of the -m gpu suite
#   TAG=r05a tools/gpu_measure.sh bench  [bench args]   one bench.py line → $OUT/bench.json
#   TAG=r05a tools/gpu_measure.sh kt     [bench args]   bench line, then rocprofv3 --kernel-trace
#                                                       --stats of the same command
#   TAG=r05a tools/gpu_measure.sh prof   [bench args]   kt, then the FETCH_SIZE and WRITE_SIZE PMC
#                                                       passes (separately, as MI355X_MICROARCH.md says)
#   TAG=r05a PMC="SQ_WAVES SQ_INSTS_VALU;SQ_INSTS_LDS" tools/gpu_measure.sh pmc [bench args]
#                                                       one rocprofv3 --pmc pass per ';' group
#   TAG=r05a tools/gpu_measure.sh recipe NAME           a named sequence of the modes above
#                                                       (recipe_* functions below; `recipe list`)
#
# $OUT = gpurun_out/$TAG.  Every mode writes $OUT/RECIPE.txt: the exact command, the commit it
# was launched from (GIT_HEAD, passed in by the caller: the box has no .git), the library's
# compiled-in source hash and the code digest of every kernel source in the tree — the provenance
# tools/traffic_json.py stamps into profiles/traffic_*.json and bench.py checks before it
# reports a traffic figure.  KREGEX (default "lqrx") restricts the PMC passes to the library's
# kernels; only the stats / counter CSVs are kept (gpurun copies back ≤ 64 MiB).  Every GPU step
# runs under its own timeout and the script stops at the first failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
MODE=${1:?mode: tests|bench|kt|prof|pmc|recipe}
shift
OUT=gpurun_out/${TAG:-run}
KREGEX=${KREGEX:-lqrx}
trim() { find "$OUT" -type f \( -name "*.csv" -o -name "*.json" -o -name "*.db" \) ! -name "*stats.csv" ! -name "*counter_collection.csv" ! -name "bench.json" ! -name "sources.json" -delete 2>/dev/null; true; }
one_rank() {   # rocprofv3 modes profile ONE rank: a --gpus N > 1 bench would start its ranks
               # from a process the profiler's preload has already GPU-initialised
    local prev=""
    for a in "$@"; do
        if [ "$prev" = "--gpus" ] && [ "$a" != "1" ]; then echo "gpu_measure.sh: $MODE profiles one rank; drop --gpus $a" >&2; exit 1; fi
        case "$a" in --gpus=*) [ "${a#--gpus=}" != "1" ] && { echo "gpu_measure.sh: $MODE profiles one rank" >&2; exit 1; } ;; esac
        prev=$a
    done
}
provenance() {   # $OUT/RECIPE.txt + $OUT/sources.json
    mkdir -p "$OUT"
    {
        echo "command: TAG=${TAG:-run} ${RECIPE_CMD:-tools/gpu_measure.sh $MODE $*}"
        echo "launched_from_commit: ${GIT_HEAD:-unknown}"
        echo "date_utc: $(date -u +%FT%TZ)"
    } > "$OUT/RECIPE.txt"
    python - "$OUT/sources.json" >> "$OUT/RECIPE.txt" <<'EOF'
import ctypes, glob, hashlib, importlib.util, json, os, sys
spec = importlib.util.spec_from_file_location("lqrx_lib", "lqr.jl_amd/lqrx/_lib.py")
L = importlib.util.module_from_spec(spec)
spec.loader.exec_module(L)
srcs = sorted(glob.glob("lqr.jl_amd/csrc/*.hip") + glob.glob("lqr.jl_amd/csrc/*.h")
              + glob.glob("lqr.jl_amd/csrc/*.cpp") + ["include/lqrx.h"])
lib = ctypes.CDLL("lqr.jl_amd/lqrx/liblqrx.so")
lib.lqrx_build_info.restype = ctypes.c_char_p
info = lib.lqrx_build_info().decode()
json.dump({"library_build_info": info, "git_head": os.environ.get("GIT_HEAD"),
           "library_matches_tree": info.split(" ")[0] == "src_sha256=" + L.source_hash("."),
           "code_digests": {s: L._code_digest(s) for s in srcs},
           "sha256": {s: hashlib.sha256(open(s, "rb").read()).hexdigest()[:16] for s in srcs}},
          open(sys.argv[1], "w"), indent=1)
print("library: " + info)
EOF
}
case "$MODE" in prof|pmc|kt) one_rank "$@" ;; esac
mkdir -p "$OUT"
nproc > "$OUT/host.txt"
lscpu | head -20 >> "$OUT/host.txt"

kt_pass() {
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
        python bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; return 3; }
    trim
}
bench_line() {
    timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; return 2; }
    cut -c1-240 "$OUT/bench.json"
}

# ---- named recipes (each profiles/<round>/<dir>/RECIPE.txt names the one that produced it) ----
sub() {   # sub TAG_SUFFIX MODE ARGS… — one mode into gpurun_out/${TAG}_SUFFIX
    local s=$1; shift
    RECIPE_CMD="tools/gpu_measure.sh recipe $RECIPE (step $s: $*)" TAG=${TAG:-run}_$s "$0" "$@"
}
SQ1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
SQ2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT"
CFG4KKT="--workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32"
CFG4KKT64="--workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 4096 --dtype f64"
WG96="--workload kkt --kkt-structure dense --n 96 --m 48 --N 64 --batch 2048 --dtype f64"
recipe_tests() { sub t tests; }
recipe_close() {   # the BASELINE lines with rocprof kernel stats
    sub cfg4 kt && sub cfg5 kt --n 64 --m 32 --N 512 --batch 8192 --dtype f32 && sub cfg3 kt --workload kkt &&
    sub cfg3soa kt --workload kkt --kkt-layout 1 && sub cfg2 kt --workload cartpole && sub kkt32 kt $CFG4KKT &&
    sub kkt64 kt $CFG4KKT64
}
recipe_evidence() {   # traffic at HEAD for the non-headline lines + cfg2 SQ counters
    sub cfg2 prof --workload cartpole && KREGEX=dp_quad PMC="$SQ1;$SQ2" sub cfg2sq pmc --workload cartpole &&
    sub cfg3 prof --workload kkt && sub kkt64 prof $CFG4KKT64 && sub wg96 prof $WG96
}
recipe_kktsq() {   # configs[4] KKT half: prof + SQ counters of the fused interior-knot kernel
    sub kkt32 prof $CFG4KKT && KREGEX=kb_ PMC="$SQ1;$SQ2" sub kkt32sq pmc $CFG4KKT
}
recipe_check() {   # after a kernel change: the -m gpu suite + smoke, then the lines it touches
    sub t tests && sub cfg4 kt && sub cfg3 kt --workload kkt && sub cfg3soa kt --workload kkt --kkt-layout 1 &&
    sub lin kt --linear && sub cfg2 kt --workload cartpole && sub di kt --workload kkt --kkt-structure di
}
recipe_wg() {   # the workgroup KKT kernel (blocks past 64 rows): its tests, then the n=96 line
    sub t pytest tests/test_kkt_wg_gpu.py tests/test_dp_big_gpu.py && sub wg96 prof $WG96 &&
    sub big128 kt --n 128 --m 64 --N 64 --batch 2048
}
recipe_kkt() {   # the large-block KKT path (configs[4]'s KKT half): its tests, then the fp32 / fp64 lines
    sub t pytest tests/test_kkt_big_gpu.py tests/test_full_size_gpu.py tests/test_kkt_pad_gpu.py &&
    sub kkt32 kt $CFG4KKT && sub kkt64 kt $CFG4KKT64
}
recipe_r5a() {   # round-5 closing set, part 1: suite + smoke, the DP lines and cfg2/cfg3 with traffic
    sub t tests && sub cfg4 prof && sub cfg5 prof --n 64 --m 32 --N 512 --batch 8192 --dtype f32 &&
    sub dp64 prof --n 64 --m 32 --N 512 --batch 8192 --dtype f64 && sub cfg2 prof --workload cartpole &&
    KREGEX=dp_quad PMC="$SQ1;$SQ2" sub cfg2sq pmc --workload cartpole &&
    sub cfg3 prof --workload kkt && sub cfg3soa prof --workload kkt --kkt-layout 1
}
recipe_r5b() {   # part 2: the large-block / workgroup / small-structure KKT lines with traffic + SQ
    sub kkt32 prof $CFG4KKT && KREGEX=kb_ PMC="$SQ1;$SQ2" sub kkt32sq pmc $CFG4KKT &&
    sub kkt64 prof $CFG4KKT64 && sub wg96 prof $WG96 &&
    sub t62 prof --workload kkt --kkt-structure dense --n 6 --m 2 --N 101 --batch 16384 --dtype f64 &&
    sub t84 prof --workload kkt --kkt-structure dense --n 8 --m 4 --N 101 --batch 16384 --dtype f64
}
recipe_r5lines() {   # the closing lines again, now that traffic_r05.json holds their HEAD entries
    sub cfg4 bench && sub cfg5 bench --n 64 --m 32 --N 512 --batch 8192 --dtype f32 &&
    sub dp64 bench --n 64 --m 32 --N 512 --batch 8192 --dtype f64 && sub cfg2 bench --workload cartpole &&
    sub cfg3 bench --workload kkt && sub cfg3soa bench --workload kkt --kkt-layout 1 &&
    sub kkt32 bench $CFG4KKT && sub kkt64 bench $CFG4KKT64 && sub wg96 bench $WG96 &&
    sub t62 bench --workload kkt --kkt-structure dense --n 6 --m 2 --N 101 --batch 16384 --dtype f64 &&
    sub t84 bench --workload kkt --kkt-structure dense --n 8 --m 4 --N 101 --batch 16384 --dtype f64
}
recipe_r5dp() {   # after a change in lqrx_dp.hip: its suite files, then the three DP lines with traffic
    sub t pytest tests/test_dp_gpu.py tests/test_dp_linear_gpu.py tests/test_layout_gpu.py &&
    sub cfg4 prof && sub cfg5 prof --n 64 --m 32 --N 512 --batch 8192 --dtype f32 &&
    sub dp64 prof --n 64 --m 32 --N 512 --batch 8192 --dtype f64 &&
    KREGEX=dp_wg4 PMC="$SQ1;$SQ2" sub dp64sq pmc --n 64 --m 32 --N 512 --batch 8192 --dtype f64
}
DP64="--n 64 --m 32 --N 512 --batch 8192 --dtype f64"
DP64TV="--n 64 --m 32 --N 512 --batch 2048 --dtype f64 --tv"
recipe_r6lines() {   # the lines whose kernels changed in round 5 (TV / LIN rollout,
                     # DoubleIntegrator(3) KKT) with traffic, and the fp64 n = 64 TV / LIN lines
    sub tv prof --tv && sub lin prof --linear && sub di prof --workload kkt --kkt-structure di &&
    sub tv64 kt $DP64TV && sub lin64 kt $DP64 --linear
}
recipe_r6dp64() {   # the fp64 n = 64 DP surface: its tests, then plain / TV / LIN lines with traffic
    sub t pytest tests/test_dp_gpu.py tests/test_dp_wg4_gpu.py tests/test_dp_linear_gpu.py tests/test_dp_lane_gpu.py \
        tests/test_full_size_gpu.py::test_dp64_wg4_full_batch_parity &&
    sub dp64 prof $DP64 && sub tv64 prof $DP64TV && sub lin64 prof $DP64 --linear
}
recipe_r6close() {   # round-6 closing set: suite + smoke, every line whose kernel source changed this
                     # round (lqrx_dp.hip, lqrx_dp_lane.hip, lqrx_kkt_wg.hip) with traffic, cfg3 for the record
    sub t tests && sub cfg4 prof && sub cfg5 prof --n 64 --m 32 --N 512 --batch 8192 --dtype f32 &&
    sub dp64 prof $DP64 && sub cfg2 prof --workload cartpole && sub tv prof --tv && sub lin prof --linear &&
    sub wg96 prof $WG96 && sub cfg3 kt --workload kkt && sub kkt32 kt $CFG4KKT
}
recipe_r6kkt() {   # configs[4] KKT half after the round-6 fused-kernel changes (leaf rsqrt, zero-C peel):
                   # its tests, fp32 with traffic + SQ counters, fp64 with traffic
    sub t pytest tests/test_kkt_big_gpu.py tests/test_full_size_gpu.py && sub kkt32 prof $CFG4KKT &&
    KREGEX=kb_ PMC="$SQ1;$SQ2" sub kkt32sq pmc $CFG4KKT && sub kkt64 prof $CFG4KKT64
}
recipe_r6final() {   # round-6 final closing set at HEAD: suite + smoke, every bench line with traffic
                     # (lqrx_internal.h's DpArgs changed, so every traffic_r06.json entry is re-measured)
    sub t tests && sub cfg4 prof && sub cfg5 prof --n 64 --m 32 --N 512 --batch 8192 --dtype f32 &&
    sub dp64 prof $DP64 && sub lin64 prof $DP64 --linear && sub tv64 prof $DP64TV &&
    sub kkt32 prof $CFG4KKT && sub kkt64 prof $CFG4KKT64 && sub cfg2 prof --workload cartpole &&
    sub tv prof --tv && sub lin prof --linear && sub wg96 prof $WG96 &&
    sub cfg3 prof --workload kkt && sub cfg3soa kt --workload kkt --kkt-layout 1 &&
    sub di prof --workload kkt --kkt-structure di &&
    sub t62 prof --workload kkt --kkt-structure dense --n 6 --m 2 --N 101 --batch 16384 --dtype f64 &&
    sub t84 prof --workload kkt --kkt-structure dense --n 8 --m 4 --N 101 --batch 16384 --dtype f64
}
recipe_r6kkt2() {   # after the fused kernel's H/g ping-pong + prefetch: suite + smoke, the configs[4] KKT
                    # lines with traffic and SQ counters, the headline for the record
    sub t tests && sub kkt32 prof $CFG4KKT && KREGEX=kb_ PMC="$SQ1;$SQ2" sub kkt32sq pmc $CFG4KKT &&
    sub kkt64 prof $CFG4KKT64 && sub cfg4 bench
}
recipe_list() { declare -F | sed -n 's/^declare -f recipe_//p'; }

case "$MODE" in
tests)
    provenance
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1
    rc=$?
    tail -5 "$OUT/gpu_tests.log"
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 7; }
    tail -2 "$OUT/smoke.log" ;;
pytest)        # a subset of the -m gpu suite: the test files / -k expression given
    provenance "$@"
    timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1
    rc=$?
    tail -5 "$OUT/gpu_tests.log"
    exit $rc ;;
bench)
    provenance "$@"
    bench_line "$@" || exit 2 ;;
kt)
    provenance "$@"
    bench_line "$@" || exit 2
    kt_pass "$@" || exit 3
    find "$OUT" -name "*stats.csv" ;;
prof)
    provenance "$@"
    bench_line "$@" || exit 2
    kt_pass "$@" || exit 3
    timeout -k 10 400 rocprofv3 --kernel-include-regex "$KREGEX" --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
        python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/fetch.log" 2>&1 || { tail -20 "$OUT/fetch.log"; exit 4; }
    timeout -k 10 400 rocprofv3 --kernel-include-regex "$KREGEX" --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
        python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/write.log" 2>&1 || { tail -20 "$OUT/write.log"; exit 5; }
    trim
    find "$OUT" -name "*stats.csv" ;;
pmc)
    provenance "$@"
    i=0
    IFS=';' read -ra GROUPS_ <<< "${PMC:?PMC=\"COUNTERS;COUNTERS\"}"
    for grp in "${GROUPS_[@]}"; do
        i=$((i + 1))
        timeout -s KILL 300 rocprofv3 --kernel-include-regex "$KREGEX" --pmc $grp -d "$OUT/pmc$i" -o pmc$i --output-format csv -- \
            python bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc$i.log" 2>&1 || { tail -20 "$OUT/pmc$i.log"; exit 6; }
    done
    trim ;;
recipe)
    RECIPE=${1:?recipe name (tools/gpu_measure.sh recipe list)}
    declare -F "recipe_$RECIPE" > /dev/null || { echo "no recipe '$RECIPE'; recipes: $(recipe_list | tr '\n' ' ')" >&2; exit 1; }
    "recipe_$RECIPE" ;;
*)
    echo "unknown mode $MODE" >&2; exit 1 ;;
esac
