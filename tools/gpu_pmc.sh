#!/bin/bash
# HBM traffic per kernel: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate
# passes (never combined with tracing), plus a kernel trace of the same driver.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-pmc}; MATH=${2:-exact}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/pmc_driver.py $MATH 3 > $O/trace.log 2>&1 || { echo TRACE FAILED; tail $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python tools/pmc_driver.py $MATH 3 > $O/fetch.log 2>&1 || { echo FETCH FAILED; tail $O/fetch.log; exit 2; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python tools/pmc_driver.py $MATH 3 > $O/write.log 2>&1 || { echo WRITE FAILED; tail $O/write.log; exit 3; }
python tools/pmc_traffic.py $O/fetch $O/write $O/pmc.json > $O/pmc_parse.log 2>&1 || { echo PARSE FAILED; tail $O/pmc_parse.log; exit 4; }
echo done
