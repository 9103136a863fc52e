#!/bin/bash
# A/B of two builds of the library on bench workloads (same box, alternating):
# usage gpu_ab_lib.sh LIB_A LIB_B "WORKLOADS" [rounds] [pytest -k filter for LIB_B]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab
A=$1; B=$2; WLS="$3"; N=${4:-3}; K="$5"
if [ -n "$K" ]; then
  JWAVE_AMD_LIB=$B timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab/pytest.txt 2>&1
  rc=$?; tail -1 gpurun_out/ab/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/ab/pytest.txt | head; exit 1; }
fi
for i in $(seq 1 $N); do
  for WL in $WLS; do
    for tag in A B; do
      if [ $tag = A ]; then L=$A; else L=$B; fi
      JWAVE_AMD_LIB=$L timeout -k 10 180 python bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab/$WL.$tag$i.json 2>/dev/null || { echo "bench $WL $tag failed"; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels_profiled_pass'].items()})" gpurun_out/ab/$WL.$tag$i.json "$WL $tag"
    done
  done
done
