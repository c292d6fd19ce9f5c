#!/bin/bash
# yakmo prefetch depth 4 vs 3 (A/B, bench only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q3.log 2>&1 || exit 3
echo "p3:"; grep -E "host timing" gpurun_out/bench_q3.log | tail -1
GSC_LIB=soundchunks_amd/lib/vp4/libsoundchunks_amd.so GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q4.log 2>&1 || exit 4
echo "p4:"; grep -E "host timing" gpurun_out/bench_q4.log | tail -1
