#!/bin/bash
# frames over 262,144 chunks (yakmo state in HBM): yakmo stage parity at N = 270k / 300k, the 13-s-frame golden;
# yakmo + scan timing of the default bench (LDS path unchanged)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "yakmo or syn13s or gsc_matches_golden" > gpurun_out/long_test.log 2>&1
rc=$?; grep -E "300000|270000|syn13s" gpurun_out/long_test.log; tail -2 gpurun_out/long_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/long_c2.log 2>&1 || exit 3
grep -E "host timing" gpurun_out/long_c2.log | tail -1
