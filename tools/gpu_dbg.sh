#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
JWV_MODWT_FSTREAM=1 timeout -k 10 200 python tools/exp/modwt_fdbg.py
