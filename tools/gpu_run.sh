#!/bin/bash
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
mkdir -p gpurun_out/r06a
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err || { tail -5 gpurun_out/r06a/bench.err; exit 1; }
tail -1 gpurun_out/r06a/bench.json | cut -c1-400
