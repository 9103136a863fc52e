#!/bin/bash
# A/B of env settings on one bench workload (same box, alternating):
# usage gpu_ab_wl.sh WORKLOAD "ENV_A" "ENV_B" [rounds] [pytest -k filter]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab
WL=$1; A="$2"; B="$3"; N=${4:-3}; K="$5"
if [ -n "$K" ]; then
  for E in "$A" "$B"; do
    env $E timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" 2>&1 | tail -1
    [ ${PIPESTATUS[0]} -eq 0 ] || { echo "tests failed under [$E]"; exit 1; }
  done
fi
for i in $(seq 1 $N); do
  for tag in A B; do
    if [ $tag = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 180 python bench.py --workload $WL --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab/$tag$i.json 2>/dev/null || { echo "bench $tag failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" gpurun_out/ab/$tag$i.json "$tag [$E]"
  done
done
