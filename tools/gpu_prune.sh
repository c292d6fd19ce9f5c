#!/bin/bash
# A1 pruning: scan parity + goldens, stamps on one C2 frame, default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_parity.py -k "scan or golden" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/prune_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/prune_tests.log | tail -40
[ $rc -eq 0 ] || { tail -60 gpurun_out/prune_tests.log; exit $rc; }
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 200 python -u tools/scan_stamps.py 100 > gpurun_out/stamps_prune.log 2>&1 || { cat gpurun_out/stamps_prune.log; exit 5; }
cat gpurun_out/stamps_prune.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prune.log 2>&1 || { tail -20 gpurun_out/bench_prune.log; exit 3; }
tail -1 gpurun_out/bench_prune.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('PRUNE', d['value'], d['realtime_x'], d['stages_ms'], d['scan'], d['roofline']['frac'])"
