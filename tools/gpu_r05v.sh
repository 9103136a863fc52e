#!/bin/bash
# round 5: WPT reverse head pairs via LDS taps (rev_pair_rot_t) vs rev_pair_head
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "wpt" > gpurun_out/r05v_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05v_parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh wpt ${1:-3} jwave_amd/lib/ab_headt0.so jwave_amd/lib/ab_headt1.so 2>&1 | tee gpurun_out/r05v_ab.txt
