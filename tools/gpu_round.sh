#!/bin/bash
# Full measurement set for the round: bench lines for every workload, rocprofv3
# kernel stats of the default bench, and FETCH/WRITE PMC passes.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { echo B1 FAILED; tail $O/bench_fwt1d.err; exit 1; }
cat $O/bench_fwt1d.json
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --math fma --no-cpu-baseline > $O/bench_fwt1d_fma.json 2> $O/bench_fwt1d_fma.err || { echo B2 FAILED; exit 2; }
for wl in fwt2d wpt modwt; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo B3 $wl FAILED; tail $O/bench_$wl.err; exit 3; }
  cat $O/bench_$wl.json
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --warmup-seconds 0 > $O/prof.log 2>&1 || { echo ROCPROF FAILED; tail -20 $O/prof.log; exit 4; }
python tools/trace_summary.py $O/prof
bash tools/gpu_pmc.sh $TAG/pmc exact fwt1d fwt2d wpt modwt || exit 5

