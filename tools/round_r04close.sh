#!/bin/bash
# round 4 closing set at HEAD: the BASELINE bench lines with rocprof kernel stats (cfg4 default,
# cfg5, cfg3 layouts 0/1, cfg2) and the fp64 configs[4]-shape KKT line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r04close}
mkdir -p gpurun_out/$T
kt() {   # name, bench args: the bench line, then a rocprofv3 kernel-trace/stats run of it
    local n=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > gpurun_out/$T/${n}_bench.json 2> gpurun_out/$T/${n}_bench.err || { tail -20 gpurun_out/$T/${n}_bench.err; return 1; }
    cat gpurun_out/$T/${n}_bench.json | cut -c1-200
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/${n}_kt -o kt --output-format csv -- \
        python bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/${n}_kt.log 2>&1 || { tail -20 gpurun_out/$T/${n}_kt.log; return 1; }
    find gpurun_out/$T/${n}_kt -type f ! -name "*stats.csv" -delete
}
kt cfg4 || exit 1
kt cfg5 --n 64 --m 32 --N 512 --batch 8192 --dtype f32 || exit 2
kt cfg3 --workload kkt || exit 3
kt cfg3soa --workload kkt --kkt-layout 1 || exit 4
kt cfg2 --workload cartpole || exit 5
kt kkt64 --workload kkt --kkt-structure dense --n 64 --m 32 --N 512 --batch 4096 --dtype f64 || exit 6
