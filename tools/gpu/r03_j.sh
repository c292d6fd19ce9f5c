#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/nan_debug.py quiet_tone_cs4_cpf1024 0 4 > gpurun_out/r03_j.log 2>&1 || exit 2
tail -6 gpurun_out/r03_j.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "silence or quiet or corpus or generic or gsc_matches_golden or scan" > gpurun_out/r03_j_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_j_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_j_c4.log 2>&1 || exit 3
grep -E "host timing" gpurun_out/r03_j_c4.log | tail -1; tail -1 gpurun_out/r03_j_c4.log | cut -c1-300
GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_j_c2.log 2>&1 || exit 4
grep -E "host timing" gpurun_out/r03_j_c2.log | tail -1
