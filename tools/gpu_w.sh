#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-w}; mkdir -p $O; cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in exact fma; do
timeout -k 10 300 python bench.py --workload wpt --math $m --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_wpt_$m.json 2>$O/bench_wpt_$m.err || exit 4
done
python tools/show_bench.py $O
