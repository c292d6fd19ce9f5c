#!/bin/bash
# NaN-aware generic scan (first-leaf shortcut, NaN-safe certificate): parity on the NaN cases + corpus;
# c4 bench; D = 16 split-layout A/B (parity first); stamps of both layouts
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "silence or quiet or corpus or generic or gsc_matches_golden or scan_reduce" > gpurun_out/r03_h_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_h_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_h_c4.log 2>&1 || exit 3
tail -1 gpurun_out/r03_h_c4.log | cut -c1-300
GSC_SCAN_SPLIT16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "k4096 and not d32" > gpurun_out/r03_h_split_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_h_split_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_h_c2.log 2>&1 || exit 4
grep -E "host timing" gpurun_out/r03_h_c2.log | tail -1
GSC_SCAN_SPLIT16=1 GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_h_c2s.log 2>&1 || exit 5
grep -E "host timing" gpurun_out/r03_h_c2s.log | tail -1
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 > gpurun_out/r03_h_stamps.log 2>&1 || exit 6
tail -1 gpurun_out/r03_h_stamps.log
GSC_SCAN_SPLIT16=1 GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 > gpurun_out/r03_h_stamps_s.log 2>&1 || exit 7
tail -1 gpurun_out/r03_h_stamps_s.log
