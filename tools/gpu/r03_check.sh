#!/bin/bash
# GPU parity suite, then the default bench with host stage timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/r03_gputest.log
[ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_base.log 2>&1 || exit 3
tail -3 gpurun_out/r03_base.log
