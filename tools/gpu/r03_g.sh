#!/bin/bash
# re-entry check: full -m gpu suite, then c2 (default), c3, c4, br128 benches with host stage timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r03_g_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_g_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_g_c2.log 2>&1 || exit 3
grep -E "host timing|prepare \[ms\]" gpurun_out/r03_g_c2.log | tail -2; tail -1 gpurun_out/r03_g_c2.log | cut -c1-400
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_g_c3.log 2>&1 || exit 4
grep -E "host timing" gpurun_out/r03_g_c3.log | tail -1; tail -1 gpurun_out/r03_g_c3.log | cut -c1-400
timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_g_c4.log 2>&1 || exit 5
tail -1 gpurun_out/r03_g_c4.log | cut -c1-400
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config br128 --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_g_br.log 2>&1 || exit 6
grep -E "host timing" gpurun_out/r03_g_br.log | tail -1; tail -1 gpurun_out/r03_g_br.log | cut -c1-400
