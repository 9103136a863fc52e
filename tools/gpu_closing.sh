#!/bin/bash
# Closing check: GPU parity suite + smoke with the default library, the
# config-2 bench line in the driver's shape, then an A/B of one env knob on
# the config-4 workload (its parity tests under both settings first).
# usage: gpu_closing.sh TAG "ENV_A" "ENV_B"
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-closing}; R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
bash tools/gpu_tests.sh $TAG/tests || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_fwt1d.json 2> $O/bench_fwt1d.err || { tail $O/bench_fwt1d.err; exit 2; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('config 2', d['ms_per_step'], d['roofline']['frac'], d['build']['lib_sha256'])" $O/bench_fwt1d.json
bash tools/gpu_ab_multi.sh wpt 3 wpt "$2" "$3" || exit 3
