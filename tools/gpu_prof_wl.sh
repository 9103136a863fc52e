#!/bin/bash
# rocprofv3 kernel trace of one bench workload: per-(kernel, grid) durations
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-profwl}; WL=${2:-fwt2d}; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "ROCPROF FAILED"; tail -20 $O/prof.log; exit 4; }
python tools/trace_summary.py $O/prof 14
