#!/bin/bash
# round-4: pageable host entry with 32 MiB staging slots
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "host or jni or staging or thread or pinned or pageable" > gpurun_out/r04o_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/r04o_tests.txt; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04o_b$i.json 2>gpurun_out/r04o_b$i.err || { tail gpurun_out/r04o_b$i.err; exit 2; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_entry']; print(d['ms_per_step'], h['pageable_over_pcie'], h['pinned_over_pcie'], h['ring'])" gpurun_out/r04o_b$i.json
done
