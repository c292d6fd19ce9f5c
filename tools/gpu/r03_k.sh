#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GSC_FRAME_STATS=1 timeout -k 10 300 python -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r03_k_c4.log 2>&1 || exit 3
grep "^frame" gpurun_out/r03_k_c4.log | sort -t+ -k2 -n | tail -8
