#!/bin/bash
# First-round measurement script (run through gpurun on a 1-GPU MI355X box).
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || exit 1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --math fma --no-cpu-baseline > $O/bench_fwt1d_fma.json 2> $O/bench_fwt1d_fma.err || exit 2
for wl in fwt2d wpt modwt; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || exit 3
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fwt1d -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_fwt1d.log 2>&1 || exit 4
echo done
