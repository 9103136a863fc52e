#!/bin/bash
# Per-kernel (template-resolved) stats of one bench workload, steady state
# (the bench's warmup runs >= 0.25 s of steps before its timed ones):
# usage gpu_kstats.sh TAG WORKLOAD [extra bench args]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=${1:-ks}; WL=${2:-fwt2d}; shift 2
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline --no-secondary "$@" > $O/b.log 2>&1 || { echo "rocprof failed"; tail $O/b.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:14]:
    print(f"{float(r['AverageNs'])/1e3:9.2f} us x{int(r['Calls']):4d}  {r['Name'][:150]}")
PY
