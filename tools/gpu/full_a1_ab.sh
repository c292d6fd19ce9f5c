#!/bin/bash
# scan A/B: half-dimension A1 bounds (default) vs full-dimension (GSC_SCAN_FULL_A1=1), ABAB on C5 -cs4,
# the c4d corpus and C2; scan ms and bit_exact per run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in half full; do
    for cfg in c5cs4:128 c4d:0 c2:256; do
      c=${cfg%%:*}; s=${cfg##*:}
      args="--config $c --steps 2 --warmup 1 --no-cpu-baseline"; [ "$s" != 0 ] && args="$args --seconds $s"
      if [ $v = full ]; then export GSC_SCAN_FULL_A1=1; else unset GSC_SCAN_FULL_A1; fi
      timeout -k 10 300 python -u bench.py $args > gpurun_out/fa_${v}_${c}_$r.log 2>&1 || exit 3
      echo "$v $c r$r: $(tail -1 gpurun_out/fa_${v}_${c}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stages_ms"]["gpu_scan_ms"], d["bit_exact"])')"
    done
  done
done
