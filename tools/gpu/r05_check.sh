#!/bin/bash
# round-5 checks: the new GPU tests (default-flag corpus, refinv additions, mstest -py, overflow
# replay twice per stream), then the c4d bench with per-frame scan finish times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "${TESTS:-overflow or corpus_as_one_batch or refinv or python_reduce_file}" > gpurun_out/r05_test.log 2>&1
rc=$?; tail -3 gpurun_out/r05_test.log; [ $rc -ne 0 ] && exit $rc
[ -n "$NOBENCH" ] && exit 0
GSC_FRAME_STATS=1 timeout -k 10 400 python -u bench.py --config c4d --steps 3 --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/c4d.log 2>&1 || exit 4
grep "^frame" gpurun_out/c4d.log | tail -80 | sort -t+ -k2 -n | tail -5; tail -1 gpurun_out/c4d.log | cut -c1-300
