#!/bin/bash
# scan-kernel A/B: parity, then ABAB 256-s C2 bench against soundchunks_amd/lib/variants/base (a build of
# the previous commit's gsc_scan.hip), then stamps of one C2 frame
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "scan or gsc_matches_golden or corpus_as_one_batch" > gpurun_out/ab_test.log 2>&1
rc=$?; tail -2 gpurun_out/ab_test.log; [ $rc -ne 0 ] && exit $rc
run() {  # name, lib
  GSC_LIB=$2 GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$1.log 2>&1 || return 1
  echo "$1: $(grep -E 'host timing' gpurun_out/ab_$1.log | tail -1 | sed 's/.*reduce (//;s/) .*//')"
}
B=soundchunks_amd/lib/variants/base/libsoundchunks_amd.so
N=soundchunks_amd/lib/libsoundchunks_amd.so
run base1 $B && run new1 $N && run base2 $B && run new2 $N || exit 3
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 > gpurun_out/ab_stamps.log 2>&1 || exit 4
grep -A3 "^stamps" gpurun_out/ab_stamps.log; tail -1 gpurun_out/ab_stamps.log
