#!/bin/bash
# split layout (D = 32, K > 2048 on one CU) + parallel ANN builds: parity; stamps; c3 / c2 / c4 benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "d32 or c3 or cs16 or corpus_as_one_batch or two_rank_hip or stale_tree or overflow or knnfit or drains" > gpurun_out/r03_f_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_f_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_f_c3.log 2>&1 || exit 4
grep -E "host timing|passes histogram" gpurun_out/r03_f_c3.log | tail -2; tail -1 gpurun_out/r03_f_c3.log | cut -c1-400
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_f_c2.log 2>&1 || exit 5
grep -E "host timing|prepare \[ms\]" gpurun_out/r03_f_c2.log | tail -2; tail -1 gpurun_out/r03_f_c2.log | cut -c1-400
GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_f_c4.log 2>&1 || exit 6
grep -c "KNNFit overflow" gpurun_out/r03_f_c4.log; tail -1 gpurun_out/r03_f_c4.log | cut -c1-400
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 > gpurun_out/r03_f_stamps.log 2>&1 || exit 7
tail -1 gpurun_out/r03_f_stamps.log
