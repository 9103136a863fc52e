#!/bin/bash
# round-4: roofline timing check against rocprofv3 (bench region B, all kinds evented)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for wl in fwt1d modwt wpt fwt2d; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04n_$wl.json 2>gpurun_out/r04n_$wl.err || { tail gpurun_out/r04n_$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], r.get('traffic_source'), {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" gpurun_out/r04n_$wl.json
done
