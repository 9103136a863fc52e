#!/bin/bash
# round 5: FETCH_SIZE correction vs footprint (tools/pmc_footprint.py)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/pmc_footprint.py > $O/fetch.log 2>&1 || { echo FETCH FAILED; tail $O/fetch.log; exit 2; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/pmc_footprint.py > $O/write.log 2>&1 || { echo WRITE FAILED; tail $O/write.log; exit 3; }
python3 tools/pmc_footprint.py parse $O/fetch $O/write > $O/footprint.json && cat $O/footprint.json
