#!/bin/bash
# round-4: XCD-paired slabs in the generic resident column kernels
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "2d or 3d or axis or column" > gpurun_out/r04q_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r04q_tests.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04q_tests.txt | head; exit 1; }
bash tools/gpu_kstats.sh r04q_ks fwt2d > gpurun_out/r04q_ks.txt 2>&1 || { cat gpurun_out/r04q_ks.txt; exit 3; }
head -10 gpurun_out/r04q_ks.txt
bash tools/gpu_pmc.sh r04q_pmc exact fwt2d || exit 4
