#!/bin/bash
# round-4: forward column tail (fwt_fwd_res, C = 8) at 512 threads (B) against 256 (A)
set -o pipefail
L=jwave_amd/lib
bash tools/gpu_ab_lib.sh $L/ab_A.so $L/ab_B.so fwt2d 3 "2d or 3d or axis"
