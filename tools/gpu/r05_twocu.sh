#!/bin/bash
# round 5: idle-CU A/B -- every frame on two CUs (scan library built with -DGSC_TWO_CU,
# GSC_TWO_CU=1) against one CU per frame, on launches with fewer frames than CUs / 2:
# C5 8-way strong share (452 s = 113 frames), -cs8 and -cs4, and the C4 corpus (76 frames)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V=soundchunks_amd/lib/variants/twocu/libsoundchunks_amd.so
# parity of the two-CU shapes first (a hang ends at the timeout)
GSC_TWO_CU=1 GSC_LIB=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${PTESTS:-scan_reduce_bit_exact or syn8s_48k or syn8s_c2}" > gpurun_out/twocu_test.log 2>&1
rc=$?; tail -2 gpurun_out/twocu_test.log; [ $rc -ne 0 ] && exit $rc
line() { python - "$1" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["frames"], d["ms_per_step"], d["stages_ms"]["gpu_scan_ms"], d["stages_ms"]["gpu_yakmo_ms"], d.get("bit_exact"))
PY
}
for r in 1 2; do
  for cfg in ${CFGS:-c5:452 c5cs4:452 c4d:0}; do
    c=${cfg%%:*}; s=${cfg##*:}
    args="--config $c --steps 2 --warmup 1 --no-cpu-baseline"
    [ "$s" != 0 ] && args="$args --strong --seconds $s"
    timeout -k 10 300 python -u bench.py $args > gpurun_out/tc_one_${c}_$r.log 2>&1 || exit 3
    echo "one-CU $c $s r$r: $(line gpurun_out/tc_one_${c}_$r.log)"
    GSC_TWO_CU=1 GSC_LIB=$V timeout -k 10 300 python -u bench.py $args > gpurun_out/tc_two_${c}_$r.log 2>&1 || exit 3
    echo "two-CU $c $s r$r: $(line gpurun_out/tc_two_${c}_$r.log)"
  done
done
