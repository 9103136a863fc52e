#!/bin/bash
# round 5: array-head pairs of the one-pair-per-lane reverse levels from LDS taps (rev_pair_rot_t) for the head lanes only
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "fwt or decompose or aed or denoise or in_place or rows_chunked" > gpurun_out/r05t_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05t_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh fwt1d 5 jwave_amd/lib/ab_h0.so jwave_amd/lib/ab_h1.so 2>&1 | tee gpurun_out/r05t_ab.txt && \
bash tools/gpu_ab_libs.sh fwt2d 2 jwave_amd/lib/ab_h0.so jwave_amd/lib/ab_h1.so 2>&1 | tee -a gpurun_out/r05t_ab.txt
