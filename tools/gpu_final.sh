#!/bin/bash
# Round-end evidence set, in two parts (each fits one gpurun call):
#   gpu_final.sh TAG a   GPU parity suite + smoke, bench lines for every
#                        workload (driver-shaped 20/5 for config 2, FMA line),
#                        rocprofv3 kernel stats per workload
#   gpu_final.sh TAG b   PMC FETCH/WRITE traffic per workload (+ FMA WPT), SQ
#                        counters of the MODWT, WPT and 2-D FWT kernels
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-final}; PART=${2:-a}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
if [ "$PART" = a ]; then
  bash tools/gpu_tests.sh $TAG/tests || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { echo B1 FAILED; tail $O/bench_fwt1d.err; exit 2; }
  tail -1 $O/bench_fwt1d.json
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --math fma --no-cpu-baseline > $O/bench_fwt1d_fma.json 2> $O/bench_fwt1d_fma.err || { echo B2 FAILED; exit 3; }
  for wl in fwt2d wpt modwt; do
    timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo B3 $wl FAILED; tail $O/bench_$wl.err; exit 4; }
    tail -1 $O/bench_$wl.json
  done
  for wl in fwt1d fwt2d wpt modwt; do
    bash tools/gpu_kstats.sh $TAG/ks_$wl $wl > $O/ks_$wl.txt 2>&1 || { echo KS $wl FAILED; tail $O/ks_$wl.txt; exit 5; }
    head -6 $O/ks_$wl.txt
  done
else
  bash tools/gpu_pmc.sh $TAG/pmc exact fwt1d fwt2d wpt modwt || exit 6
  bash tools/gpu_pmc.sh $TAG/pmc_fma fma wpt || exit 6
  for wl in modwt wpt fwt2d; do
    bash tools/gpu_sqpmc_wl.sh $TAG/sq_$wl $wl > $O/sq_$wl.txt 2>&1 || { echo SQ $wl FAILED; tail $O/sq_$wl.txt; exit 7; }
  done
  bash tools/gpu_sqpmc_wl.sh $TAG/sq_wpt_fma wpt fma > $O/sq_wpt_fma.txt 2>&1 || { echo SQ wpt fma FAILED; tail $O/sq_wpt_fma.txt; exit 7; }
  echo part b done
fi
