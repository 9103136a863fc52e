#!/bin/bash
# Effective shader clock per kernel kind of one workload: GRBM_GUI_ACTIVE
# (GPU busy cycles) over the kernel's duration, in a --pmc pass of its own.
# usage: gpu_clock.sh TAG WORKLOAD [MATH]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; WL=$2; M=${3:-exact}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/$WL -o run -- python bench.py --workload $WL --math $M --steps 4 --warmup 2 --no-cpu-baseline --warmup-seconds 0.2 > $O/$WL.log 2>&1 || { echo "pmc failed"; tail $O/$WL.log; exit 1; }
python3 - $O/$WL <<'PY'
import csv, glob, sys, re
from collections import defaultdict
d = sys.argv[1]
cc = glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0]
acc = defaultdict(list)
for r in csv.DictReader(open(cc)):
    m = re.search(r'jwv::(\w+)<', r['Kernel_Name'])
    if not m: continue
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) if 'End_Timestamp' in r else None
    acc[m.group(1)].append((float(r['Counter_Value']), dur))
for k, v in acc.items():
    v = v[-8:]
    cyc = sum(a for a, _ in v) / len(v)
    durs = [b for _, b in v if b]
    if durs:
        dur = sum(durs) / len(durs)
        print("%-24s cycles %.4g  dur %.1f us  clock %.2f GHz" % (k, cyc, dur / 1e3, cyc / dur))
    else:
        print("%-24s cycles %.4g (no timestamps)" % (k, cyc))
PY
