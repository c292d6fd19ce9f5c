#!/bin/bash
# scan A/B: parity of the in-tree build (scan / golden / corpus / bench digests), then
# ABAB timings of the in-tree build against variant BASE on C2 (256 s) and C5 -cs4 (128 s),
# then the in-tree stamps library on one C2 and one -cs4 frame
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread \
  -k "${PTESTS:-scan or gsc_matches_golden or corpus_as_one_batch or bench or overflow}" > gpurun_out/ab_test.log 2>&1
rc=$?; tail -2 gpurun_out/ab_test.log; [ $rc -ne 0 ] && exit $rc
lib() { [ "$1" = tree ] && echo soundchunks_amd/lib/libsoundchunks_amd.so || echo soundchunks_amd/lib/variants/$1/libsoundchunks_amd.so; }
for r in 1 2; do
  for v in ${BASE:-base} tree; do
    for cfg in ${CFGS:-c2:256 c5cs4:128}; do
      c=${cfg%%:*}; s=${cfg##*:}
      GSC_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --config $c --seconds $s --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${v}_${c}_$r.log 2>&1 || exit 3
      echo "$v $c $s r$r: $(tail -1 gpurun_out/ab_${v}_${c}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stages_ms"]["gpu_yakmo_ms"], d["stages_ms"]["gpu_scan_ms"], d["bit_exact"])')"
    done
  done
done
[ -n "$NOSTAMPS" ] && exit 0
STCS="8 4" bash tools/gpu/stamps.sh
