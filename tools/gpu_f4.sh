#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-f4}; mkdir -p $O; cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 fwt_d4_2^18 fwt_d4_b64x65536 exact fma || exit 2
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_fwt1d.json 2>$O/bench_fwt1d.err || exit 4
python tools/show_bench.py $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "ROCPROF FAILED"; tail -20 $O/prof.log; exit 4; }
python tools/trace_summary.py $O/prof
