#!/bin/bash
# round-2 re-entry check: whole -m gpu suite, one default bench line with the host timing breakdown
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests.log | tail -30
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
GSC_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 3; }
grep -E "scan tail|pass" gpurun_out/bench_c2.log | tail -8
tail -1 gpurun_out/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['realtime_x'], d['stages_ms'], d['roofline']['frac'])"
exit $rc
