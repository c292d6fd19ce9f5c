#!/bin/bash
# round 5: NaN-pass exact DFS A/B on the latency-bound corpus (c4d = the lame_test corpus at the
# encoder defaults, set by 60.wav frame 1), after the parity subset on the in-tree build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${PTESTS:-scan or gsc_matches_golden or corpus or bench or overflow or nan or silence or empty}" > gpurun_out/nan_test.log 2>&1
rc=$?; tail -2 gpurun_out/nan_test.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in ${BASE:-sbase} tree; do
    [ $v = tree ] && L=soundchunks_amd/lib/libsoundchunks_amd.so || L=soundchunks_amd/lib/variants/$v/libsoundchunks_amd.so
    for c in ${CFGS:-c4d c4}; do
      GSC_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/nan_${v}_${c}_$r.log 2>&1 || exit 3
      echo "$v $c r$r: $(tail -1 gpurun_out/nan_${v}_${c}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stages_ms"]["gpu_scan_ms"], d["bit_exact"])')"
    done
  done
done
