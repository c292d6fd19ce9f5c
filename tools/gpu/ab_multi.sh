#!/bin/bash
# scan-kernel A/B over several libraries: parity of the candidate (CAND, a variant name), then two rounds of
# the 256-s C2 bench for every variant in VARIANTS (names under soundchunks_amd/lib/variants, or "tree"),
# then the phase stamps of STAMPS (a variant built with -DGSC_STAMPS) on one C2 frame
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
lib() { [ "$1" = tree ] && echo soundchunks_amd/lib/libsoundchunks_amd.so || echo soundchunks_amd/lib/variants/$1/libsoundchunks_amd.so; }
parity() {
  [ -z "$CAND" ] && return 0
  GSC_LIB=$(lib $CAND) timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "${PTESTS:-scan or gsc_matches_golden or corpus_as_one_batch}" > gpurun_out/abm_test.log 2>&1
  rc=$?; tail -2 gpurun_out/abm_test.log; return $rc
}
[ -z "$PARITY_LAST" ] && { parity || exit 2; }
for r in 1 2; do
  for v in $VARIANTS; do
    GSC_LIB=$(lib $v) GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds ${SECS:-256} --config ${CFG:-c2} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abm_${v}_$r.log 2>&1 || exit 3
    echo "$v.$r: $(grep -E 'host timing' gpurun_out/abm_${v}_$r.log | tail -1 | sed 's/.*reduce (//;s/) .*//')"
  done
done
[ -n "$PARITY_LAST" ] && { parity || exit 2; }
if [ -n "$STAMPS" ]; then
  GSC_LIB=$(lib $STAMPS) GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 ${STCS:-8} 4096 > gpurun_out/abm_stamps.log 2>&1 || exit 4
  grep -A20 "^stamps" gpurun_out/abm_stamps.log; tail -1 gpurun_out/abm_stamps.log
fi
