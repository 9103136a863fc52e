#!/bin/bash
# Box-level spread of the default (config 2) bench line in the driver's shape
# (five back-to-back runs of --steps 20 --warmup 5) and FMA-mode lines of
# configs 3-5.  usage: gpu_reps.sh TAG
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-reps}; mkdir -p $O; cd $R
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['roofline']['frac'], d.get('roundtrip_max_abs_err'), d.get('kernels_profiled_pass'))" "$1"; }
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/rep$i.json 2>$O/rep$i.err || { tail $O/rep$i.err; exit 1; }
  show $O/rep$i.json
done
for wl in wpt modwt fwt2d; do
  timeout -k 10 300 python bench.py --workload $wl --math fma --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_${wl}_fma.json 2>$O/$wl.err || { tail $O/$wl.err; exit 2; }
  show $O/bench_${wl}_fma.json
done
