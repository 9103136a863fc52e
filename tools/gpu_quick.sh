#!/bin/bash
# tests (gpu) -> microbench -> bench fwt1d
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python tools/microbench.py exact fma > $O/micro.log 2>&1 || { echo MICRO FAILED; tail $O/micro.log; exit 2; }
cat $O/micro.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { echo BENCH FAILED; tail $O/bench_fwt1d.err; exit 3; }
cat $O/bench_fwt1d.json
