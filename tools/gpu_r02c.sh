#!/bin/bash
# round-2 state check: the whole -m gpu suite, the default bench line, a C3 bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gputests.log | tail -80
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 > gpurun_out/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2.log; exit 3; }
tail -3 gpurun_out/bench_c2.log
timeout -k 10 600 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail -20 gpurun_out/bench_c3.log; exit 4; }
tail -3 gpurun_out/bench_c3.log
exit $rc
