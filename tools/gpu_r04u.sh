#!/bin/bash
# round-4: bench with the round-trip check after the timed regions
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r04u
for WL in fwt2d fwt1d modwt wpt fwt1d fwt2d; do
  timeout -k 10 240 python bench.py --workload $WL --steps 20 --warmup 5 > gpurun_out/r04u/$WL.json 2> gpurun_out/r04u/$WL.err || { echo "bench $WL failed"; tail gpurun_out/r04u/$WL.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d[\"ms_per_step\"], d[\"roofline\"][\"kernel\"], d[\"roofline\"][\"avg_launch_us\"], d[\"roundtrip_max_abs_err\"])" gpurun_out/r04u/$WL.json $WL
done
bash tools/gpu_kstats.sh r04u_ks fwt2d > gpurun_out/r04u/ks.txt 2>&1 || { tail gpurun_out/r04u/ks.txt; exit 3; }
