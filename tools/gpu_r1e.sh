#!/bin/bash
# re-entry check: full GPU parity suite, pass-plan microbench, default bench line
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r1e}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for p in 4 5 7 3; do
  echo "JWV_PLAN=$p"
  JWV_PLAN=$p timeout -k 10 120 python tools/microbench.py fwt_d4_2^20 fwt_d4_2^24 exact 2>&1 | python -c "
import json,sys
for l in sys.stdin:
    try: r=json.loads(l)
    except Exception: continue
    print('  %-12s step %8.2f us  %s' % (r['case'], r['step_us_no_events'], r['us_per_call']))" || exit 2
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_fwt1d.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 3; }
cat $O/bench_fwt1d.json
