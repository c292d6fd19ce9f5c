#!/bin/bash
# scan phase stamps on one C2 frame (stamps build), 100 passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 300 python -u tools/scan_stamps.py 100 8 > gpurun_out/scan_stamps.log 2>&1
rc=$?
tail -14 gpurun_out/scan_stamps.log
exit $rc
