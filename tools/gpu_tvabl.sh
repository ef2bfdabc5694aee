#!/bin/bash
# GPU side of tools/tv_ablate.sh: the --tv bench on the product library and each variant
cd "$(dirname "$0")/.."
run() {  # name, lib
  LQRX_LIB=$2 timeout -k 10 150 python bench.py ${ARGS:---tv --steps 5 --warmup 2} --cpu-seconds 0 > gpurun_out/tvabl_$1.json 2> gpurun_out/tvabl_$1.err
  rc=$?; if [ $rc -gt 1 ]; then echo "stop: $1 rc=$rc"; exit $rc; fi
  python -c "import json;d=json.loads(open('gpurun_out/tvabl_$1.json').read().strip().splitlines()[-1]);print('$1', '$ARGS', round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d['check'].get('sampled_parity',{}).get('pass'), d['check'].get('nonfinite'))"
}
[ -n "$NOBASE" ] || run base lqr.jl_amd/lqrx/liblqrx.so
for v in ${@:-q abr all noroll noroll_all}; do if [ $v = base ]; then run base lqr.jl_amd/lqrx/liblqrx.so; else run $v tools/abl/liblqrx_$v.so; fi; done
