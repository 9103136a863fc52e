#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
JWV_MODWT_STREAM=0 timeout -k 10 200 python tools/exp/modwt_dbg2.py tile && JWV_MODWT_STREAM=1 timeout -k 10 200 python tools/exp/modwt_dbg2.py stream && python -c "
import numpy as np
a=np.load('gpurun_out/dbg2_tile.npy'); b=np.load('gpurun_out/dbg2_stream.npy'); d=np.nonzero(a!=b)[0]
print('tile vs stream differ', d.size, d[:10].tolist(), sorted(set((d//512).tolist()))[:20])
" && rm -f gpurun_out/dbg2_*.npy
