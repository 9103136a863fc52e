#!/bin/bash
# round 5: WPT couples with the products of G taps / terms issued ahead of
# their adds (forward fwd_couple_pipe, JWV_WPT_FPIPE = G; reverse
# rev_couple_pipe, JWV_WPT_RPIPE = G; p0 = the round-4 forms).  Parity of the
# WPT cases per build, then config 4 A/B.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
O=gpurun_out/r05j; mkdir -p $O
L=jwave_amd/lib
for v in ab_p2 ab_p4 ab_p1 ab_p2r2 ab_p2r1 ab_p2r4; do
  JWAVE_AMD_LIB=$L/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wpt" > $O/pytest_$v.log 2>&1 || { echo "parity $v failed"; grep -E "FAILED|Error" $O/pytest_$v.log | head; exit 1; }
  tail -1 $O/pytest_$v.log
done
bash tools/gpu_ab_libs.sh wpt 3 $L/ab_p0.so $L/ab_p2.so $L/ab_p4.so $L/ab_p1.so $L/ab_p2r2.so $L/ab_p2r1.so $L/ab_p2r4.so
