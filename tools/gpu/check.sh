#!/bin/bash
# round-3 final check: the full -m gpu suite, then smoke()
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final_test.log 2>&1
rc=$?; tail -3 gpurun_out/final_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit 3
tail -1 gpurun_out/final_smoke.log
