#!/bin/bash
# round-4: 512-thread 16-column tiles (B: forward, C: reverse) against 256 (A)
set -o pipefail
L=jwave_amd/lib
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_B.so fwt2d 2 "2d or 3d or axis" && cp gpurun_out/ab/pytest.txt gpurun_out/ab/pytestB.txt && \
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_C.so fwt2d 2 "2d or 3d or axis"
