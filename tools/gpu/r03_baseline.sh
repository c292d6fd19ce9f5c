#!/bin/bash
# round-3 baseline: default bench (no CPU leg) with the host stage timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_base.log 2>&1 || exit 3
tail -3 gpurun_out/r03_base.log
