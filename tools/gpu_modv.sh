#!/bin/bash
# MODWT tile variants: parity subset + config-5 microbench per (fwd, inv) variant pair
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-modv}; mkdir -p $O; cd $R
shift
for pr in "$@"; do
  f=${pr%,*}; i=${pr#*,}
  JWV_MODFWD=$f JWV_MODINV=$i timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "modwt or MODWT" > $O/t$f$i.log 2>&1 || { echo TESTS $pr FAILED; tail -30 $O/t$f$i.log; exit 1; }
  echo "variant fwd=$f inv=$i: $(tail -1 $O/t$f$i.log)"
  JWV_MODFWD=$f JWV_MODINV=$i timeout -k 10 120 python tools/microbench.py modwt_d4_1e7 exact fma 2>&1 | grep case || exit 2
done
