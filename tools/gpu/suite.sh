#!/bin/bash
# the full -m gpu suite, smoke(), then the default C2 bench (1024 s) without the CPU leg
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1
rc=$?; tail -3 gpurun_out/suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
tail -1 gpurun_out/smoke.log
[ -n "$NOBENCH" ] && exit 0
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c2.log 2>&1 || exit 4
tail -1 gpurun_out/c2.log | cut -c1-400
