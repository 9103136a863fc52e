#!/bin/bash
# quick: fwt parity subset + microbench + kernel trace of the default bench
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-q}; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fwt or axis" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 fwt_d4_b64x65536 exact || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "ROCPROF FAILED"; tail -20 $O/prof.log; exit 4; }
python tools/trace_summary.py $O/prof | head -8
