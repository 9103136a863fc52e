#!/bin/bash
# builds tools/diag/diag_modwt_{base,nobar,nowf,nofp,all} (hipcc, gfx950)
set -e
cd "$(dirname "$0")"
F="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950"
hipcc $F -DTAG='"base"' diag_modwt.hip -o diag_modwt_base &
hipcc $F -DTAG='"nobar"' -DJWV_EXP_MOD_NOBAR diag_modwt.hip -o diag_modwt_nobar &
hipcc $F -DTAG='"nowf"' -DJWV_EXP_MOD_NOWF diag_modwt.hip -o diag_modwt_nowf &
hipcc $F -DTAG='"nofp"' -DJWV_EXP_MOD_NOFP diag_modwt.hip -o diag_modwt_nofp &
hipcc $F -DTAG='"nb+nf"' -DJWV_EXP_MOD_NOBAR -DJWV_EXP_MOD_NOFP diag_modwt.hip -o diag_modwt_nbnf &
wait
