#!/bin/bash
# A/B of env settings on the default bench (same box, alternating, no CPU
# baseline, no secondary): usage gpu_ab.sh "ENV_A" "ENV_B" [rounds]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab
A="$1"; B="$2"; N=${3:-4}
for i in $(seq 1 $N); do
  for tag in A B; do
    if [ $tag = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-secondary > gpurun_out/ab/$tag$i.json 2>/dev/null || { echo "bench $tag failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k:v['avg_us'] for k,v in d.get('kernels_profiled_pass',{}).items()})" gpurun_out/ab/$tag$i.json "$tag [$E]"
  done
done
