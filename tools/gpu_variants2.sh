#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-var}; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fwt and not fwt2d" > $O/t.log 2>&1 || { echo TESTS FAILED; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
JWV_FWD_T=2048 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fwt_large or config2 or batch" > $O/t2.log 2>&1 || { echo TESTS2 FAILED; tail -20 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for v in "4096 2" "2048 2" "2048 3" "2048 4" "4096 1"; do
  set -- $v
  echo "FWD_T=$1 BPC=$2"
  JWV_FWD_T=$1 JWV_STREAM_BPC=$2 timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 fwt_d4_b64x65536 exact fma 2>/dev/null || exit 2
done
echo "no-stream"
JWV_FWD_STREAM=0 timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 exact 2>/dev/null
