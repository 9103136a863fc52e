#!/bin/bash
# Standard GPU iteration: parity tests, then benches, then a rocprofv3 kernel trace.
# usage: tools/gpu_cycle.sh TAG [tests|notests] [workloads...]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-x}; MODE=${2:-tests}; shift 2; WLS=${@:-fwt1d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$MODE" = "tests" ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
for wl in $WLS; do
  timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "BENCH $wl FAILED"; tail -20 $O/bench_$wl.err; exit 2; }
  timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 5 --math fma --no-cpu-baseline > $O/bench_${wl}_fma.json 2> $O/bench_${wl}_fma.err || { echo "BENCH fma $wl FAILED"; tail -20 $O/bench_${wl}_fma.err; exit 3; }
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "ROCPROF FAILED"; tail -20 $O/prof.log; exit 4; }
echo done
