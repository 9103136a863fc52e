#!/bin/bash
# Store-policy experiment (config 2): parity tests, then the bench with
# JWV_STPOL = 0 / 1 / 2 and a kernel trace of the default.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-stpol}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -20
[ $rc -eq 0 ] || { echo PYTEST rc=$rc; exit 1; }
for p in 0 1 2 1 0; do
  JWV_STPOL=$p timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_sp$p.json 2> $O/bench_sp$p.err || { echo BENCH FAILED; tail $O/bench_sp$p.err; exit 2; }
  python - $O/bench_sp$p.json $p <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("STPOL", sys.argv[2], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"], {k:v["avg_us"] for k,v in d["kernels_profiled_pass"].items()})
PY
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "ROCPROF FAILED"; tail -20 $O/prof.log; exit 4; }
python tools/trace_summary.py $O/prof
