#!/bin/bash
# round-4: profiled-pass timing with in-packet events (hipExtLaunchKernelGGL)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for wl in fwt1d modwt wpt fwt2d; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04m_$wl.json 2>gpurun_out/r04m_$wl.err || { tail gpurun_out/r04m_$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" gpurun_out/r04m_$wl.json
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/r04m_tests.txt; exit $rc
