#!/bin/bash
# round 5: chunked row passes (sharded 2-D exchange without pack/unpack)
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "rows_chunked" \
  > gpurun_out/r05n_parity.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_distributed.py -m gpu > gpurun_out/r05n_dist.log 2>&1
rc=$?
tail -3 gpurun_out/r05n_parity.log; tail -3 gpurun_out/r05n_dist.log 2>/dev/null
exit $rc
