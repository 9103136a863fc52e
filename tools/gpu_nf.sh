#!/bin/bash
# round 6: MODWT non-finite parity + MODWT/2-D regression tests + config-5 bench
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
O=gpurun_out/${1:-r06b}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "nonfinite or modwt or alternating or stream or tail or chain" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload modwt --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_modwt.json 2> $O/bench_modwt.err || { tail -5 $O/bench_modwt.err; exit 1; }
tail -1 $O/bench_modwt.json | cut -c1-300
