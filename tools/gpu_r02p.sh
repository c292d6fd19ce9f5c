#!/bin/bash
# C5 signal (48 kHz stereo, K = 4096) at -cs8 and -cs4 on one GPU
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 3; }
tail -1 gpurun_out/bench_c5.log | cut -c1-300
timeout -k 10 400 python -u bench.py --config c5cs4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5cs4.log 2>&1 || { tail -20 gpurun_out/bench_c5cs4.log; exit 4; }
tail -1 gpurun_out/bench_c5cs4.log | cut -c1-300
