#!/bin/bash
# A1 pruning A/B: stamps (K = 4096, 512) and 256-s C2 bench with and without GSC_SCAN_NO_PRUNE
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "" 1; do
  GSC_SCAN_NO_PRUNE=$v GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 > gpurun_out/r03_n_k4096_$v.log 2>&1 || exit 2
  GSC_SCAN_NO_PRUNE=$v GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 512 > gpurun_out/r03_n_k512_$v.log 2>&1 || exit 3
  tail -1 gpurun_out/r03_n_k4096_$v.log; tail -1 gpurun_out/r03_n_k512_$v.log
done
for v in "" 1; do
  GSC_SCAN_NO_PRUNE=$v GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_n_c2_$v.log 2>&1 || exit 4
  grep -E "host timing" gpurun_out/r03_n_c2_$v.log | tail -1
done
