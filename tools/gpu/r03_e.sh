#!/bin/bash
# round-3 state: parity (goldens, scan, batch/prepare/shard/-py), phase stamps, benches (c2 default, br128, c4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "gsc_matches_golden or scan or corpus_as_one_batch or two_rank_hip or python_reduce or birch or frame_dsp" \
  > gpurun_out/r03_e_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_e_test.log; [ $rc -ne 0 ] && exit $rc
GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 timeout -k 10 120 python -u tools/scan_stamps.py 100 8 > gpurun_out/r03_e_stamps.log 2>&1 || exit 3
tail -1 gpurun_out/r03_e_stamps.log
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_e_c2.log 2>&1 || exit 4
grep -E "host timing|prepare \[ms\]" gpurun_out/r03_e_c2.log | tail -2; tail -1 gpurun_out/r03_e_c2.log | cut -c1-330
GSC_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --config br128 --seconds 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_e_br.log 2>&1 || exit 5
grep -E "host timing" gpurun_out/r03_e_br.log | tail -1
timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_e_c4.log 2>&1 || exit 6
tail -1 gpurun_out/r03_e_c4.log | cut -c1-300
