#!/bin/bash
# GPU parity (all -m gpu tests), then an A/B/C/D of the big-pass tile walk
# (JWV_TILE_DESC 0..3) on config 2, alternating on one box.
# usage: gpu_desc.sh TAG [skip_tests] [rounds]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-desc}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
fi
N=${3:-3}
for i in $(seq 1 $N); do
  for D in 0 1 2 3; do
    JWV_TILE_DESC=$D timeout -k 10 180 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-secondary > $O/d$D.$i.json 2> $O/d$D.$i.err || { echo "bench desc=$D failed"; tail -5 $O/d$D.$i.err; exit 2; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" $O/d$D.$i.json "desc=$D"
  done
done
