#!/bin/bash
# SQ / LDS / TCC counters for one bench workload (separate --pmc passes)
# usage: gpu_sqpmc_wl.sh TAG WORKLOAD [MATH]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-sqw}; WL=${2:-wpt}; M=${3:-exact}; mkdir -p $O; cd $R
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU"
P3="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INST_CYCLES_VALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python bench.py --workload $WL --math $M --steps 2 --warmup 1 --no-cpu-baseline --warmup-seconds 0 > $O/p$i.log 2>&1 || { echo "PMC $i FAILED"; tail $O/p$i.log; exit $i; }
done
python tools/pmc_summary.py $O
