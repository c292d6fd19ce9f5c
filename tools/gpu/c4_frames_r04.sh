#!/bin/bash
# round-4: per-frame scan finish times of the c4 corpus batch (GSC_FRAME_STATS), final build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GSC_FRAME_STATS=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_frames.log 2>&1 || exit 4
grep "^frame" gpurun_out/c4_frames.log | tail -76 | sort -t+ -k2 -n | tail -4; tail -1 gpurun_out/c4_frames.log | cut -c1-250
