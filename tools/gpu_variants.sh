#!/bin/bash
# Compare runtime-selectable tile variants on config 2 (microbench, exact + fma).
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-var}; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fwt and not fwt2d" > $O/t.log 2>&1 || { echo TESTS FAILED; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
JWV_REV_PREF=1 JWV_REV_T=2048 JWV_FWD_T=2048 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fwt_large or config2" > $O/t2.log 2>&1 || { echo TESTS2 FAILED; tail -20 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for v in "4096 4096 0" "4096 4096 1" "2048 2048 0" "2048 2048 1" "2048 4096 1"; do
  set -- $v
  echo "FWD_T=$1 REV_T=$2 PREF=$3"
  JWV_FWD_T=$1 JWV_REV_T=$2 JWV_REV_PREF=$3 timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 fwt_d4_2^18 exact fma 2>/dev/null || exit 2
done
