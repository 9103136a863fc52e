#!/bin/bash
# round-1 checkpoint: full GPU parity suite + the default bench line (with cpu_baseline)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r1d; mkdir -p $O; cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "BENCH FAILED"; tail -20 $O/bench_default.err; exit 2; }
cat $O/bench_default.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 3; }
cat $O/smoke.log
