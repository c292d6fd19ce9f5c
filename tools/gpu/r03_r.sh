#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GSC_LIB=soundchunks_amd/lib/variants/prep/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 > gpurun_out/r03_r.log 2>&1 || exit 2
grep -A9 "^stamps" gpurun_out/r03_r.log
