#!/bin/bash
# round-4 checks: new GPU tests (reference invocations, -pr0, bench bit-exactness, gloo ranks), then scan stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "${TESTS:-refinv or pr0 or bench or gsc_matches_golden}" > gpurun_out/r04_test.log 2>&1
rc=$?; tail -3 gpurun_out/r04_test.log; [ $rc -ne 0 ] && exit $rc
[ -n "$NOSTAMPS" ] && exit 0
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 > gpurun_out/r04_stamps.log 2>&1 || exit 4
grep -A9 "^stamps" gpurun_out/r04_stamps.log; tail -1 gpurun_out/r04_stamps.log
