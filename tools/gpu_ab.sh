#!/bin/bash
# Parity subset for each library build, then an alternating A/B of them on one
# bench workload (one box).  usage: gpu_ab.sh WORKLOAD ROUNDS "PYTEST -k EXPR" LIB...
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab
WL=$1; N=$2; K=$3; shift 3
for L in "$@"; do
  t=$(basename $L .so)
  JWAVE_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/ab/pytest.$t.log 2>&1 || { echo "parity $t FAILED"; tail -5 gpurun_out/ab/pytest.$t.log; exit 1; }
  echo "parity $t: $(tail -1 gpurun_out/ab/pytest.$t.log)"
done
exec_ab() { bash tools/gpu_ab_libs.sh "$WL" "$N" "$@"; }
exec_ab "$@"
