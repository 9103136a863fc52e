#!/bin/bash
# round-4: B = row reverse tile at waves_per_eu 7; C = 256-row forward column tiles
set -o pipefail
L=jwave_amd/lib
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_B.so fwt2d 2 "fwt and not 2d and not 3d" && \
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_C.so fwt2d 2 "2d or 3d or axis"
