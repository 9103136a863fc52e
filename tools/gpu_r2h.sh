#!/bin/bash
# Closing check: full GPU parity + smoke, bench lines for configs 2 and 3,
# kernel stats for config 3.  usage: gpu_r2h.sh TAG
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-r02h}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 2; }
grep smoke $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { echo BENCH fwt1d FAILED; tail $O/bench_fwt1d.err; exit 3; }
timeout -k 10 300 python bench.py --workload fwt2d --steps 30 --warmup 10 > $O/bench_fwt2d.json 2> $O/bench_fwt2d.err || { echo BENCH fwt2d FAILED; tail $O/bench_fwt2d.err; exit 4; }
python tools/show_bench.py $O
bash tools/gpu_kstats.sh $TAG/ks_fwt2d fwt2d > $O/ks_fwt2d.txt && cat $O/ks_fwt2d.txt || exit 5
