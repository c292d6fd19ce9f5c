#!/bin/bash
# round-2 final check: the whole -m gpu suite, smoke(), then the default bench line (with the CPU baseline)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputests_k.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_k.log | tail -20
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_k.log 2>&1 || { tail -20 gpurun_out/smoke_k.log; exit 2; }
tail -1 gpurun_out/smoke_k.log
GSC_HOST_TIMING=1 timeout -k 10 400 python -u bench.py > gpurun_out/bench_k.log 2>&1 || { tail -20 gpurun_out/bench_k.log; exit 3; }
grep -E "host timing" gpurun_out/bench_k.log | tail -1
tail -1 gpurun_out/bench_k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['realtime_x'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
