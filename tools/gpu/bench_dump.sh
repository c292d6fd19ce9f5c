#!/bin/bash
# the default bench workload's output, dumped with its per-frame sizes (bit-exactness diagnosis)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/dump
BENCH_DUMP=gpurun_out/dump/c2_1024 timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline ${ARGS} > gpurun_out/dump/bench.log 2>&1
grep "differs" gpurun_out/dump/bench.log; tail -1 gpurun_out/dump/bench.log | cut -c1-200; ls -la gpurun_out/dump
