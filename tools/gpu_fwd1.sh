#!/bin/bash
# Config-2 geometry sweep: forward first-pass tile/levels and tail (env), each
# with the default bench (no CPU baseline); parity tests of the 1-D paths first.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-fwd1}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fwt and not 2d and not 3d" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
timeout -k 10 60 tools/diag/diag_tails > $O/tails.txt 2>&1 && grep -E "rev head|rev res" $O/tails.txt
i=0
for v in "JWV_FWD1T=2048" "JWV_FWD1T=1024 JWV_FWD1K=5" "JWV_FWD1T=1024 JWV_FWD1K=5 JWV_FWD1TAIL=1024" "JWV_FWD1T=1024 JWV_FWD1K=4" "JWV_FWD1T=1024 JWV_FWD1K=6" "JWV_FWD1T=2048 JWV_FWD1TAIL=1024" "JWV_FWD1T=2048"; do
  i=$((i+1))
  env $v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || { echo BENCH FAILED; tail $O/b$i.err; exit 2; }
  python - $O/b$i.json "$v" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-52s ms/step %.4f  %s" % (sys.argv[2], d["ms_per_step"], {k:v["avg_us"] for k,v in d["kernels_profiled_pass"].items()}))
PY
done
