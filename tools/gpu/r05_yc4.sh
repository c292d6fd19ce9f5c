#!/bin/bash
# round 5: yakmo variants on the real-audio corpus (c4: -cs8, D = 16), C2 (256 s) and C5 -cs4 (128 s)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARS:-y0 y2 tree}; do
  [ $v = tree ] && L=soundchunks_amd/lib/libsoundchunks_amd.so || L=soundchunks_amd/lib/variants/$v/libsoundchunks_amd.so
  for cfg in ${CFGS:-c4:0 c4d:0 c2:256 c5cs4:128}; do
    c=${cfg%%:*}; sec=${cfg##*:}; a="--config $c"; [ "$sec" != 0 ] && a="$a --seconds $sec"
    GSC_LIB=$L timeout -k 10 300 python -u bench.py $a --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/yc4_${v}_${c}.log 2>&1 || exit 3
    echo "$v $c: $(tail -1 gpurun_out/yc4_${v}_${c}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stages_ms"]["gpu_yakmo_ms"], d["bit_exact"])')"
  done
done
