#!/bin/bash
# padded K (-br goldens), then A/B of the scan changes (256-s C2 bench, 64 frames)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "gsc_matches_golden" > gpurun_out/r03_d_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_d_test.log; [ $rc -ne 0 ] && exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_d_$n.log 2>&1 || return 1
  echo "$n: $(grep -E 'host timing' gpurun_out/r03_d_$n.log | tail -1 | sed 's/.*reduce (//;s/) .*//')"
}
run cur && run cur_full GSC_SCAN_FULL_A1=1 && run vpser GSC_LIB=soundchunks_amd/lib/variants/vpser/libsoundchunks_amd.so \
 && run vser GSC_LIB=soundchunks_amd/lib/variants/vser/libsoundchunks_amd.so \
 && run bothser GSC_LIB=soundchunks_amd/lib/variants/bothser/libsoundchunks_amd.so \
 && run bothser_full GSC_SCAN_FULL_A1=1 GSC_LIB=soundchunks_amd/lib/variants/bothser/libsoundchunks_amd.so || exit 3
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config br128 --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_d_br.log 2>&1 || exit 4
echo "br128: $(grep -E 'host timing' gpurun_out/r03_d_br.log | tail -1)"; tail -1 gpurun_out/r03_d_br.log | cut -c1-300
