#!/bin/bash
# the driver's default bench command (config 2 + secondaries incl. configs 3-5)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
mkdir -p gpurun_out/r05e
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r05e/bench_default.json 2> gpurun_out/r05e/bench_default.err || { tail -20 gpurun_out/r05e/bench_default.err; exit 1; }
python3 - gpurun_out/r05e/bench_default.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("config 2", d["ms_per_step"], d["roofline"]["frac"])
for k, v in d.get("configs", {}).items():
    print(k, v.get("ms_per_step"), (v.get("roofline") or {}).get("frac"), (v.get("roofline_fp64") or {}).get("frac"), v.get("error", ""))
print("wpt strong", d["batched_wpt_strong"]["ms_per_step"], "host", d["host_entry"]["pageable_over_pcie"], d["host_entry"]["pinned_over_pcie"])
PY
