#!/bin/bash
# round-2 GPU check: the whole -m gpu suite, then one default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputests.log 2>&1
rc=$?
tail -40 gpurun_out/gputests.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 > gpurun_out/bench.log 2>&1
rc2=$?
tail -5 gpurun_out/bench.log
exit $((rc + rc2))
