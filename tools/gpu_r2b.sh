#!/bin/bash
# Round-2 measurement cycle: full GPU parity, then every workload's bench line
# (with its CPU baseline), then per-workload PMC traffic.  usage: gpu_r2b.sh TAG [skip_tests]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-r2b}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { echo BENCH fwt1d FAILED; tail $O/bench_fwt1d.err; exit 2; }
for WL in fwt2d wpt modwt; do
  timeout -k 10 300 python bench.py --workload $WL --steps 30 --warmup 10 > $O/bench_$WL.json 2> $O/bench_$WL.err || { echo BENCH $WL FAILED; tail $O/bench_$WL.err; exit 3; }
done
python tools/show_bench.py $O
bash tools/gpu_pmc.sh $TAG/pmc exact fwt1d fwt2d wpt modwt || exit 4
