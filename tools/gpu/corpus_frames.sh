#!/bin/bash
# parallel NaN-exact tree build + per-wave certificate bounds: parity; corpus stamps; c4; C2 ABAB vs base
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/nan_debug.py quiet_tone_cs4_cpf1024 0 3 > gpurun_out/corpus_dbg.log 2>&1 || exit 2
tail -1 gpurun_out/corpus_dbg.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "silence or quiet or corpus or generic or gsc_matches_golden or scan" > gpurun_out/corpus_test.log 2>&1
rc=$?; tail -2 gpurun_out/corpus_test.log; [ $rc -ne 0 ] && exit $rc
export GSC_SCAN_DEBUG=1
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 tests/golden/lame_test/60.wav 1 > gpurun_out/corpus_60.log 2>&1 || exit 3
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 tests/golden/lame_test/velvet.wav 1 > gpurun_out/corpus_velvet.log 2>&1 || exit 3
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so timeout -k 10 120 python -u tools/scan_stamps.py 100 8 4096 > gpurun_out/corpus_c2.log 2>&1 || exit 3
unset GSC_SCAN_DEBUG
tail -1 gpurun_out/corpus_60.log; tail -1 gpurun_out/corpus_velvet.log; tail -1 gpurun_out/corpus_c2.log
GSC_FRAME_STATS=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/corpus_c4.log 2>&1 || exit 4
grep "^frame" gpurun_out/corpus_c4.log | tail -76 | sort -t+ -k2 -n | tail -4; tail -1 gpurun_out/corpus_c4.log | cut -c1-250
run() {  # name, lib
  GSC_LIB=$2 GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/corpus_$1.log 2>&1 || return 1
  echo "$1: $(grep -E 'host timing' gpurun_out/corpus_$1.log | tail -1 | sed 's/.*reduce (//;s/) .*//')"
}
B=soundchunks_amd/lib/variants/base/libsoundchunks_amd.so
N=soundchunks_amd/lib/libsoundchunks_amd.so
run base1 $B && run new1 $N && run base2 $B && run new2 $N || exit 5
