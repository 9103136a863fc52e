#!/bin/bash
# kernel traces of the config-3 step: serial schedule vs the overlapped one (G=2, G=4)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1 TMPDIR=/tmp
L=jwave_amd/lib
for t in ab_ser ab_g2 libjwave_hip; do
  JWAVE_AMD_LIB=$L/$t.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05c/$t -o run -- python bench.py --workload fwt2d --steps 6 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/r05c/$t.log 2>&1 || { echo "trace $t failed"; tail -5 gpurun_out/r05c/$t.log; exit 1; }
  tail -1 gpurun_out/r05c/$t.log | cut -c1-200
done
