#!/bin/bash
# chain kernels: parity subset, then config-2 microbench with/without chains
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-chain}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for ch in 1 0; do  # reverse chain on / off
  echo "JWV_CHAIN=$ch"
  JWV_CHAIN=$ch timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 exact fma 2>&1 | tail -2 || exit 2
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_fwt1d.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 3; }
cat $O/bench_fwt1d.json
