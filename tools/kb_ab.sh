#!/bin/bash
# kb_ab.sh — large-block KKT A/B on the GPU box: the bench line (configs[4] KKT half) for each
# library variant under tools/abl/ given as arguments (built by tools/tv_ablate.sh), then a
# rocprofv3 kernel-trace of the in-tree library.  Output under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-kb_ab}
mkdir -p "$OUT"
ARGS=${KB_ARGS:---workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 8192 --dtype f32}
case " $ARGS " in *" --gpus "[2-9]*|*" --gpus="[2-9]*) echo "kb_ab.sh: one rank only (rocprofv3 below)" >&2; exit 1 ;; esac
for v in "" "$@"; do
    name=${v:-base}
    lib=""
    [ -n "$v" ] && lib=tools/abl/liblqrx_$v.so
    LQRX_LIB=$lib timeout -k 10 300 python -u bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline \
        > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 2; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms')" "$OUT/$name.json" "$name"
    grep -A5 KB_PROF "$OUT/$name.err" | head -8
done
if [ -z "$NOPROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 3; }
find "$OUT/kt" -type f ! -name "*stats.csv" -delete
cat $(find "$OUT/kt" -name "*kernel_stats.csv") | cut -d, -f1-4 | head -8
fi
