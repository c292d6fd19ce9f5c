#!/bin/bash
# NaN-pass exact DFS (dfs_parallel_nan) on LIB: NaN / corpus parity, stamps of the corpus' NaN and quiet frames,
# c4 corpus batch with per-frame finish times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=soundchunks_amd/lib/variants/${V:-v5}/libsoundchunks_amd.so
S=soundchunks_amd/lib/variants/${V:-v5}stamps/libsoundchunks_amd.so
GSC_LIB=$L timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "silence or quiet or corpus or nan or generic or scan" > gpurun_out/nan_test.log 2>&1
rc=$?; tail -2 gpurun_out/nan_test.log; [ $rc -ne 0 ] && exit $rc
export GSC_SCAN_DEBUG=1
GSC_LIB=$S timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 tests/golden/lame_test/60.wav 1 > gpurun_out/nan_60.log 2>&1 || exit 3
GSC_LIB=$S timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 tests/golden/lame_test/velvet.wav 1 > gpurun_out/nan_velvet.log 2>&1 || exit 3
unset GSC_SCAN_DEBUG
grep "^scan:" gpurun_out/nan_60.log; tail -1 gpurun_out/nan_60.log; grep "^scan:" gpurun_out/nan_velvet.log; tail -1 gpurun_out/nan_velvet.log
GSC_LIB=$L GSC_FRAME_STATS=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/nan_c4.log 2>&1 || exit 4
grep "^frame" gpurun_out/nan_c4.log | tail -76 | sort -t+ -k2 -n | tail -4; tail -1 gpurun_out/nan_c4.log | cut -c1-250
