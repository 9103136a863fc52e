#!/bin/bash
# A/B/C... of env settings on one bench workload (same box, alternating rounds):
# usage gpu_ab_multi.sh WORKLOAD ROUNDS "PYTEST_K|-" "ENV_1" "ENV_2" ...
# With a pytest -k filter the GPU parity tests run once under every setting first.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab
WL=$1; N=$2; K="$3"; shift 3
if [ "$K" != "-" ]; then
  for E in "$@"; do
    env $E timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab/tests.log 2>&1
    rc=$?; echo "[$E] $(tail -1 gpurun_out/ab/tests.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/ab/tests.log | head; exit 1; }
  done
fi
for i in $(seq 1 $N); do
  v=0
  for E in "$@"; do
    v=$((v+1))
    env $E timeout -k 10 180 python bench.py --workload $WL --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab/v$v.$i.json 2>/dev/null || { echo "bench [$E] failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" gpurun_out/ab/v$v.$i.json "[$E]"
  done
done
