#!/bin/bash
# round 5: fused forward tail with XCD-contiguous units -- parity, PMC
# footprint/tail traffic, config 2 A/B (tailrr = round-robin units, as before)
set -o pipefail
export JWAVE_AMD_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "config2 or chain or fwt_large" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/pmc_footprint.py > $O/fetch.log 2>&1 || { echo FETCH FAILED; tail $O/fetch.log; exit 2; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/pmc_footprint.py > $O/write.log 2>&1 || { echo WRITE FAILED; tail $O/write.log; exit 3; }
python3 tools/pmc_footprint.py parse $O/fetch $O/write > $O/footprint.json && python3 -c "import json; d=json.load(open('$O/footprint.json')); print(json.dumps(d['config2']['fwt_fwd_tail1']))"
L=jwave_amd/lib
bash tools/gpu_ab_libs.sh fwt1d 5 $L/ab_tailrr.so $L/libjwave_hip.so
