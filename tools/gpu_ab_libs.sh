#!/bin/bash
# A/B/C... of several builds of the library on one bench workload (same box,
# alternating rounds).  usage: [MATH=fma] gpu_ab_libs.sh WORKLOAD ROUNDS LIB...
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab
WL=$1; N=$2; shift 2
for i in $(seq 1 $N); do
  for L in "$@"; do
    t=$(basename $L .so)
    JWAVE_AMD_LIB=$L timeout -k 10 180 python bench.py --workload $WL --math ${MATH:-exact} --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab/$WL.$t.$i.json 2>gpurun_out/ab/$WL.$t.$i.err || { echo "bench $WL $t failed"; tail -5 gpurun_out/ab/$WL.$t.$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" gpurun_out/ab/$WL.$t.$i.json "$WL $t"
  done
done
