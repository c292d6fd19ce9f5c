#!/bin/bash
# yakmo phase clocks (stamps library) on the C2 (256 s) and C5 -cs4 (128 s) bench shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in ${CFGS:-c2:256 c5cs4:128}; do
  c=${cfg%%:*}; s=${cfg##*:}
  GSC_LIB=${STLIB:-soundchunks_amd/lib/stamps/libsoundchunks_amd.so} GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config $c --seconds $s --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ystamps_$c.log 2>&1 || exit 3
  echo "$c: $(grep 'yakmo stamps' gpurun_out/ystamps_$c.log | tail -1)"; grep "host timing" gpurun_out/ystamps_$c.log | tail -1
done
