#!/bin/bash
# round-2 profile set + the affected parity subset
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "dsp or yakmo or gsc or knnfit or corpus or hip_encoder or reconstruction or python_reduce or abi" > gpurun_out/gputests_i.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_i.log | tail -20
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/trace.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 &&
GSC_HOST_TIMING=1 timeout -k 10 400 python3 -u bench.py > $O/bench_default.log 2>&1
rc=$?
grep "host timing" $O/bench_default.log | tail -1
tail -1 $O/bench_default.log | cut -c1-600
exit $rc
