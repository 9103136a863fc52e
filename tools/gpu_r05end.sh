#!/bin/bash
# round 5 end: the tree as the driver runs it (prebuilt library): GPU suite, smoke, default bench line
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
mkdir -p gpurun_out/r05end
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05end/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r05end/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05end/smoke.log 2>&1 || { tail -5 gpurun_out/r05end/smoke.log; exit 1; }
tail -1 gpurun_out/r05end/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r05end/bench.json 2> gpurun_out/r05end/bench.err || { tail -5 gpurun_out/r05end/bench.err; exit 1; }
tail -1 gpurun_out/r05end/bench.json | cut -c1-300
