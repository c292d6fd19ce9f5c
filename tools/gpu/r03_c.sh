#!/bin/bash
# scan kernel changes (parallel vp scan, half-dimension A1): exactness, then A/B timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 \
  --timeout-method thread -k "scan or gsc_matches_golden or yakmo" > gpurun_out/r03_c_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_c_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_c_half.log 2>&1 || exit 3
grep -E "host timing|passes histogram" gpurun_out/r03_c_half.log | tail -2; tail -1 gpurun_out/r03_c_half.log | cut -c1-400
GSC_SCAN_FULL_A1=1 GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_c_full.log 2>&1 || exit 4
grep -E "host timing" gpurun_out/r03_c_full.log | tail -1; tail -1 gpurun_out/r03_c_full.log | cut -c1-400
