#!/bin/bash
# full GPU parity suite + benches of the given workloads (exact and fma)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-full}; shift; mkdir -p $O; cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in "$@"; do for m in exact fma; do
timeout -k 10 300 python bench.py --workload $wl --math $m --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_${wl}_$m.json 2>$O/bench_${wl}_$m.err || { echo "BENCH $wl $m FAILED"; tail -5 $O/bench_${wl}_$m.err; exit 4; }
done; done
python tools/show_bench.py $O
