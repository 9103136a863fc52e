#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-m}; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "modwt" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in exact fma; do
timeout -k 10 300 python bench.py --workload modwt --math $m --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_modwt_$m.json 2>$O/bench_modwt_$m.err || exit 4
done
python tools/show_bench.py $O
