#!/bin/bash
# config lines with CPU baselines and bit-exactness: RUNS = "config:seconds:steps ..." (seconds 0 =
# the config's own workload: c4 / c4d corpus); logs in gpurun_out/prof/bench_<config>_<seconds>.log
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
for r in ${RUNS:-c2:600:3 c3:1024:2 c4:0:2 c4d:0:2 br128:1024:2}; do
  IFS=: read c s n <<< "$r"
  args="--config $c --steps $n --warmup 1"; [ "$s" != 0 ] && args="$args --seconds $s"
  timeout -k 10 900 python3 -u bench.py $args $EXTRA > $O/bench_${c}_$s.log 2>&1 || exit 3
  tail -1 $O/bench_${c}_$s.log | cut -c1-200
done
