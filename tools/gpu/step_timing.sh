#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BENCH_STEP_TIMING=1 GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/steptiming.log 2>&1 || exit 2
grep -E "^step|host timing" gpurun_out/steptiming.log; tail -1 gpurun_out/steptiming.log | cut -c1-200
