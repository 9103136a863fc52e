#!/bin/bash
# C = 8 column-slab kernels (fwt8) + MODWT XCD tile order: parity subset first,
# then the full GPU suite, then fwt2d (JWV_FWT8 = 1 / 0) and modwt bench lines.
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-fwt8}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "2d or 3d or axis or modwt or MODWT" > $O/t_sub.log 2>&1 || { echo SUBSET FAILED; tail -40 $O/t_sub.log; exit 1; }
echo "subset: $(tail -1 $O/t_sub.log)"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { echo FULL FAILED; tail -40 $O/t_all.log; exit 2; }
echo "full: $(tail -1 $O/t_all.log)"
for v in 1 0; do
  JWV_FWT8=$v timeout -k 10 300 python bench.py --workload fwt2d --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_fwt2d_fwt8_$v.json 2> $O/b2d_$v.err || { echo BENCH2D $v FAILED; tail $O/b2d_$v.err; exit 3; }
done
timeout -k 10 300 python bench.py --workload modwt --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_modwt.json 2> $O/bm.err || { echo BENCHM FAILED; tail $O/bm.err; exit 4; }
python tools/show_bench.py $O
