#!/bin/bash
# round 6: host staging tests + default bench line (config CPU legs, host_entry pool report)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
O=gpurun_out/${1:-r06c}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_multi.py -x -v --timeout 200 --timeout-method thread -k "host_entry or multi or staging" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("config2", d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"])
for k, v in d["configs"].items():
    print(k, v.get("ms_per_step"), (v.get("roofline") or {}).get("frac"), (v.get("cpu_baseline") or {}).get("value"), (v.get("cpu_baseline") or {}).get("sample", "")[:80])
print("host_entry", json.dumps(d["host_entry"]))
PY
