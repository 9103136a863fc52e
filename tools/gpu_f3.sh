#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-f3}; mkdir -p $O; cd $R
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { echo "== $*"; env "$@" timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 fwt_d4_4096 fwt_d4_b64x65536 fwt_d8_rows8192 exact || exit 2; }
run JWV_FWT1=1
run JWV_FWD1_T=2048
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_fwt1d.json 2>$O/bench_fwt1d.err || exit 4
timeout -k 10 300 python bench.py --workload fwt2d --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_fwt2d.json 2>$O/bench_fwt2d.err || exit 4
python tools/show_bench.py $O
