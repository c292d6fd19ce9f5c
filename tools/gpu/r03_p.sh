#!/bin/bash
# stamps of the corpus' slowest frames: velvet.wav frame 1 (restart-heavy), 60.wav frame 1 (NaN centroids)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1
timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 tests/golden/lame_test/velvet.wav 1 > gpurun_out/r03_p_velvet.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 tests/golden/lame_test/60.wav 1 > gpurun_out/r03_p_60.log 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/r03_p_velvet.log gpurun_out/r03_p_60.log
