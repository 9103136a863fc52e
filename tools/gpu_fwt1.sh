#!/bin/bash
# fwt1 kernels: parity subset, then tuning variants (microbench, events per kernel kind)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-f1}; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fwt or axis or facade or device" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { echo "== $*"; env "$@" timeout -k 10 120 python tools/microbench.py fwt_d4_2^24 fwt_d4_b64x65536 exact fma || exit 2; }
run JWV_FWT1=0
run JWV_FWT1=1
run JWV_FWD1_T=2048
run JWV_FWD1_NT=512
run JWV_REV1_T=4096
run JWV_REV1_NT=128
