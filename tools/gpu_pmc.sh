#!/bin/bash
# HBM traffic per (workload, kernel kind): rocprofv3 --pmc FETCH_SIZE and
# WRITE_SIZE in separate passes (never combined with tracing), each with the
# library's launch log for attribution.  usage: gpu_pmc.sh TAG MATH WORKLOAD...
set -o pipefail
export JWAVE_AMD_NO_BUILD=1 JWV_LAUNCH_LOG=1
TAG=${1:-pmc}; MATH=${2:-exact}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
for WL in "$@"; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$WL.fetch -o run -- python3 tools/pmc_driver.py $WL $MATH 3 > $O/$WL.fetch.log 2>&1 || { echo "$WL FETCH FAILED"; tail $O/$WL.fetch.log; exit 2; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$WL.write -o run -- python3 tools/pmc_driver.py $WL $MATH 3 > $O/$WL.write.log 2>&1 || { echo "$WL WRITE FAILED"; tail $O/$WL.write.log; exit 3; }
  python3 tools/pmc_traffic.py $WL $MATH $O/$WL.fetch $O/$WL.fetch.log $O/$WL.write $O/$WL.write.log $O/pmc_$WL.json > $O/$WL.parse.log 2>&1 || { echo "$WL PARSE FAILED"; tail $O/$WL.parse.log; exit 4; }
  python3 - $O/pmc_$WL.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["workload"], "calib", round(d["calibration"]["fetch_factor"],3), round(d["calibration"]["write_factor"],3))
for k,v in d["kernels"].items():
    print("  %-36s launches %3d  hbm %.4g B  alg %.4g B  ratio %s" % (k, v["launches"], v["hbm_bytes_per_launch"] or 0, v["algorithmic_bytes_per_launch"], v["traffic_over_algorithmic"] and round(v["traffic_over_algorithmic"],3)))
PY
done
echo done
