#!/bin/bash
# round-4 config lines with CPU baselines and bit-exactness: c3, c4 corpus batch, br128 (1024 s), C5 at 3600 s (cs8, cs4)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
for c in ${CONFIGS:-c3 c4 br128}; do
  timeout -k 10 500 python3 -u bench.py --config $c --steps 2 > $O/bench_$c.log 2>&1 || exit 3
  tail -1 $O/bench_$c.log | cut -c1-220
done
for c in ${C5:-c5 c5cs4}; do
  timeout -k 10 600 python3 -u bench.py --config $c --seconds 3600 --steps 1 --warmup 1 > $O/bench_${c}_3600.log 2>&1 || exit 5
  tail -1 $O/bench_${c}_3600.log | cut -c1-220
done
