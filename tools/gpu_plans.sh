#!/bin/bash
# pass plans (JWV_PLAN bits) x sizes, per-call microbench; then GPU tests of the chain plans
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-plans}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "chain or config2" > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for p in 0 4 1 3; do
  echo "JWV_PLAN=$p"
  JWV_PLAN=$p timeout -k 10 120 python tools/microbench.py fwt_d4_2^18 fwt_d4_2^20 fwt_d4_2^22 fwt_d4_2^24 exact 2>&1 | python -c "
import json,sys
for l in sys.stdin:
    try: r=json.loads(l)
    except Exception: continue
    print('  %-12s step %8.2f us  %s' % (r['case'], r['step_us_no_events'], r['us_per_call']))" || exit 2
done
