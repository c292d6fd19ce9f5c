#!/bin/bash
# yakmo compose/no-SLP + staged atten: DSP + yakmo parity, goldens, bench, stamps, and the no-compose variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsp.py tests/test_gpu_parity.py tests/test_gpu_scan.py tests/test_gpu_abi.py -m gpu -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "dsp or yakmo or gsc_matches" --durations=10 > gpurun_out/gputests_h.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_h.log | tail -30
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
GSC_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_h.log 2>&1 || { tail -20 gpurun_out/bench_h.log; exit 3; }
grep -E "host timing" gpurun_out/bench_h.log | tail -2
tail -1 gpurun_out/bench_h.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['realtime_x'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_stamps_h.log 2>&1 || { tail -20 gpurun_out/bench_stamps_h.log; exit 4; }
grep -E "yakmo stamps" gpurun_out/bench_stamps_h.log
GSC_LIB=soundchunks_amd/lib/varnc/libsoundchunks_amd.so GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_varnc.log 2>&1 || { tail -20 gpurun_out/bench_varnc.log; exit 5; }
echo "varnc:"; grep -E "host timing" gpurun_out/bench_varnc.log | tail -1
GSC_LIB=soundchunks_amd/lib/varks/libsoundchunks_amd.so GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_varks.log 2>&1 || { tail -20 gpurun_out/bench_varks.log; exit 6; }
echo "varks:"; grep -E "host timing" gpurun_out/bench_varks.log | tail -1
tail -1 gpurun_out/bench_varks.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'])"
