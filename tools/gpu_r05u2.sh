#!/bin/bash
# round 5: FMA-mode WPT forward couples with the four fma chains interleaved (ff1) vs two fwd_pair calls (ff0)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "wpt" > gpurun_out/r05u2_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05u2_parity.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do for L in ab_ff0 ab_ff1; do
  JWAVE_AMD_LIB=jwave_amd/lib/$L.so timeout -k 10 180 python bench.py --workload wpt --math fma --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab/wptfma.$L.$i.json 2>gpurun_out/ab/wptfma.$L.$i.err || { echo "bench $L failed"; tail -5 gpurun_out/ab/wptfma.$L.$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roundtrip_max_abs_err'], {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" gpurun_out/ab/wptfma.$L.$i.json "wpt-fma $L"
done; done 2>&1 | tee gpurun_out/r05u2_ab.txt
