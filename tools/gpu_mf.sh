#!/bin/bash
# MFMA-layout scan: parity (scan stages + whole-file goldens), then bench MF vs lane layout
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_parity.py -k "scan or golden" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/mf_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/mf_tests.log | tail -40
[ $rc -eq 0 ] || { tail -60 gpurun_out/mf_tests.log; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_mf.log 2>&1 || { tail -20 gpurun_out/bench_mf.log; exit 3; }
tail -1 gpurun_out/bench_mf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('MF', d['value'], d['stages_ms'], d['scan'], d['roofline']['frac'])"
GSC_SCAN_LANE_LAYOUT=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_lane.log 2>&1 || { tail -20 gpurun_out/bench_lane.log; exit 4; }
tail -1 gpurun_out/bench_lane.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('LANE', d['value'], d['stages_ms'], d['scan'], d['roofline']['frac'])"
