#!/bin/bash
# round 5: queries per speculative batch (GSC_SCAN_KB < 32) on C2 (256 s) and the c4d corpus
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for kb in ${KBS:-32 24 16}; do
  for cfg in ${CFGS:-c2:256 c4d:0}; do
    c=${cfg%%:*}; s=${cfg##*:}
    args="--config $c --steps 2 --warmup 1 --no-cpu-baseline"; [ "$s" != 0 ] && args="$args --seconds $s"
    GSC_SCAN_KB=$kb timeout -k 10 300 python -u bench.py $args > gpurun_out/kb_${kb}_$c.log 2>&1 || exit 3
    echo "kb $kb $c: $(tail -1 gpurun_out/kb_${kb}_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stages_ms"]["gpu_scan_ms"], d["bit_exact"], d["scan"])')"
  done
done
