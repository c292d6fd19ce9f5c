#!/bin/bash
# prepare / batch / shard changes: their GPU tests, then the new bench (c2 default, c4 corpus)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "corpus_as_one_batch or two_rank_hip or gsc_matches_golden or frame_dsp or python_reduce or birch" \
  > gpurun_out/r03_b_test.log 2>&1
rc=$?; tail -3 gpurun_out/r03_b_test.log; [ $rc -ne 0 ] && exit $rc
GSC_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_b_c2.log 2>&1 || exit 3
tail -1 gpurun_out/r03_b_c2.log
timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_b_c4.log 2>&1 || exit 4
tail -1 gpurun_out/r03_b_c4.log
