#!/bin/bash
# Round-2 check: full-size cfg4/cfg5 parity tests, then bench lines (cfg4, cfg5, kkt, cartpole) with the output checks.
set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 400 python -u -m pytest tests/test_full_size_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02b/full.log 2>&1 && \
timeout -k 10 240 python bench.py > gpurun_out/r02b/bench_cfg4.json 2> gpurun_out/r02b/bench_cfg4.err && \
timeout -k 10 240 python bench.py --n 64 --m 32 --N 512 --batch 8192 --dtype f32 --no-cpu-baseline > gpurun_out/r02b/bench_cfg5.json 2>> gpurun_out/r02b/bench.err && \
timeout -k 10 240 python bench.py --workload kkt --warmup 20 --steps 20 > gpurun_out/r02b/bench_kkt.json 2>> gpurun_out/r02b/bench.err && \
timeout -k 10 240 python bench.py --workload cartpole --warmup 20 --steps 20 > gpurun_out/r02b/bench_cartpole.json 2>> gpurun_out/r02b/bench.err
