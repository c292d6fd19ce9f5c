#!/bin/bash
# Round-3 config lines with CPU baselines: c3, c4 corpus batch, br128 (1024 s), C5 at its stated 3600 s (cs8, cs4)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 400 python3 -u bench.py --config c3 --steps 2 > $O/bench_c3.log 2>&1 || exit 2
tail -1 $O/bench_c3.log | cut -c1-200
timeout -k 10 400 python3 -u bench.py --config c4 --steps 2 > $O/bench_c4.log 2>&1 || exit 3
tail -1 $O/bench_c4.log | cut -c1-200
timeout -k 10 400 python3 -u bench.py --config br128 --steps 2 > $O/bench_br128.log 2>&1 || exit 4
tail -1 $O/bench_br128.log | cut -c1-200
timeout -k 10 500 python3 -u bench.py --config c5 --seconds 3600 --steps 1 --warmup 1 > $O/bench_c5_3600.log 2>&1 || exit 5
tail -1 $O/bench_c5_3600.log | cut -c1-200
timeout -k 10 500 python3 -u bench.py --config c5cs4 --seconds 3600 --steps 1 --warmup 1 > $O/bench_c5cs4_3600.log 2>&1 || exit 6
tail -1 $O/bench_c5cs4_3600.log | cut -c1-200
