#!/bin/bash
# scan phase stamps + A1 pruning counters: C2 frame (K = 4096) and K = 512
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1
timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 > gpurun_out/r03_m_k4096.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/scan_stamps.py 100 8 512 > gpurun_out/r03_m_k512.log 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/r03_m_k4096.log gpurun_out/r03_m_k512.log
