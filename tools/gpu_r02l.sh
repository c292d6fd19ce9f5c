#!/bin/bash
# yakmo one-slot X look-ahead: yakmo parity + goldens, bench, stamps, deeper variant (prefetch 6 / look-ahead 3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scan.py tests/test_gpu_abi.py -m gpu -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "yakmo or gsc_matches" > gpurun_out/gputests_l.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_l.log | tail -30
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
GSC_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_l.log 2>&1 || { tail -20 gpurun_out/bench_l.log; exit 3; }
grep -E "host timing" gpurun_out/bench_l.log | tail -1
tail -1 gpurun_out/bench_l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['realtime_x'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_stamps_l.log 2>&1 || { tail -20 gpurun_out/bench_stamps_l.log; exit 4; }
grep -E "yakmo stamps" gpurun_out/bench_stamps_l.log
GSC_LIB=soundchunks_amd/lib/v63/libsoundchunks_amd.so GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_v63.log 2>&1 || { tail -20 gpurun_out/bench_v63.log; exit 5; }
echo "v63:"; grep -E "host timing" gpurun_out/bench_v63.log | tail -1
