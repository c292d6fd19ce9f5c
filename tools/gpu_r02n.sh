#!/bin/bash
# attenuation producer waves: DSP parity, whole-file goldens + corpus, bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_dsp.py tests/test_gpu_parity.py -m gpu -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "dsp or gsc_matches or corpus" > gpurun_out/gputests_n.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_n.log | tail -30
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
GSC_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n.log 2>&1 || { tail -20 gpurun_out/bench_n.log; exit 3; }
grep -E "host timing" gpurun_out/bench_n.log | tail -1
tail -1 gpurun_out/bench_n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['realtime_x'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
