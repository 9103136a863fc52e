#!/bin/bash
# round-4: row reverse resident cap 512 (B) / 2048 (C) against 1024 (A)
set -o pipefail
L=jwave_amd/lib
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_B.so fwt2d 2 "2d or batch or rows" && \
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_C.so fwt2d 2 "2d or batch or rows"
