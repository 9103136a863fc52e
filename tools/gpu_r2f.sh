#!/bin/bash
# Round-2 closing measurement: GPU parity, every workload's bench line (with
# its CPU baseline and build provenance), rocprofv3 kernel stats for the
# listed workloads.  usage: gpu_r2f.sh TAG [WORKLOAD...] (default fwt1d modwt)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-r02f}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 2; }
cat $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { echo BENCH fwt1d FAILED; tail $O/bench_fwt1d.err; exit 3; }
for WL in fwt2d wpt modwt; do
  timeout -k 10 300 python bench.py --workload $WL --steps 30 --warmup 10 > $O/bench_$WL.json 2> $O/bench_$WL.err || { echo BENCH $WL FAILED; tail $O/bench_$WL.err; exit 4; }
done
python tools/show_bench.py $O
shift
KS="$@"; [ -n "$KS" ] || KS="fwt1d modwt"
for WL in $KS; do
  bash tools/gpu_kstats.sh $TAG/ks_$WL $WL > $O/ks_$WL.txt && cat $O/ks_$WL.txt || exit 5
done
