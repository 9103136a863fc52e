#!/bin/bash
# round-4: MODWT tile time split (tools/diag/diag_modwt_*: diagnostic builds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for v in base nobar nowf nofp nbnf; do
  timeout -k 10 120 tools/diag/diag_modwt_$v || exit 1
done 2>&1 | tee gpurun_out/r04d_diag_modwt.txt
