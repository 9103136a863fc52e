#!/bin/bash
# SQ / LDS / TCC counters for the config-2 kernels vs the copy kernel (separate --pmc passes).
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-sq}; mkdir -p $O; cd $R
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU"
P3="TCC_EA0_WRREQ_STALL TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_BUSY TA_BUSY"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python tools/pmc_driver.py exact 2 > $O/p$i.log 2>&1 || { echo "PMC $i FAILED"; tail $O/p$i.log; exit $i; }
done
python tools/pmc_summary.py $O
