#!/bin/bash
# round 5: pageable host entry, process-wide copy pool (newpool) vs the
# per-context pool of round 4 (oldpool), alternating, 4 rounds; then the
# bench's own host_entry object with the current library
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
for i in 1 2 3 4; do
  for v in oldpool newpool; do
    timeout -k 10 120 python3 tools/host_entry_ab.py jwave_amd/lib/ab_$v.so 5 >> $O/ab.jsonl 2>$O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
    tail -1 $O/ab.jsonl
  done
done
