#!/bin/bash
# round-4: wave-per-row tails with LDS sized to the row (B) against 1024 doubles per row (A)
set -o pipefail
L=jwave_amd/lib
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_B.so fwt2d 3 "2d or batch or rows or small"
