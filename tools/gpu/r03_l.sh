#!/bin/bash
# small-K layouts (one / two leaves per lane, up to 8 waves): parity, then br128 / c1 benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "gsc_matches_golden or scan or abi or shard or smoke or corpus_as_one_batch or knnfit" > gpurun_out/r03_l_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_l_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config br128 --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_l_br.log 2>&1 || exit 3
grep -E "host timing" gpurun_out/r03_l_br.log | tail -1
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config c1 --seconds 10 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_l_c1.log 2>&1 || exit 4
grep -E "host timing" gpurun_out/r03_l_c1.log | tail -1
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_l_c2.log 2>&1 || exit 5
grep -E "host timing" gpurun_out/r03_l_c2.log | tail -1
