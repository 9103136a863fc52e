#!/bin/bash
# Round-2 GPU cycle: parity tests (-m gpu), then the default bench line.
# usage: gpu_r2.sh TAG [pytest -k expr]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-r2}; K=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread "${KA[@]}" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -20
[ $rc -eq 0 ] || { echo PYTEST rc=$rc; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { echo BENCH FAILED; tail $O/bench_fwt1d.err; exit 2; }
cat $O/bench_fwt1d.json
