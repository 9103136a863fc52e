#!/bin/bash
# 2-D rows through tile passes: parity (2D/3D/batch subset) + fwt2d bench per JWV_ROWCAP
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-rowcap}; mkdir -p $O; cd $R
shift
for rc in "$@"; do
  JWV_ROWCAP=$rc timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "2d or 3d or batch or axis" > $O/t$rc.log 2>&1 || { echo TESTS $rc FAILED; tail -30 $O/t$rc.log; exit 1; }
  echo "rowcap=$rc: $(tail -1 $O/t$rc.log)"
  JWV_ROWCAP=$rc timeout -k 10 300 python bench.py --workload fwt2d --steps 10 --warmup 3 --no-cpu-baseline > $O/b$rc.json 2> $O/b$rc.err || { echo BENCH FAILED; tail $O/b$rc.err; exit 2; }
  python -c "
import json;r=json.load(open('$O/b$rc.json'));print('  ms/step',r['ms_per_step'],r['kernels_profiled_pass'])"
done
