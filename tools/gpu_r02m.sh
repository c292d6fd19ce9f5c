#!/bin/bash
# round-2 final profile set: kernel trace + stats, FETCH/WRITE PMC passes, default bench with CPU baseline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/trace.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 &&
GSC_HOST_TIMING=1 timeout -k 10 400 python3 -u bench.py > $O/bench_default.log 2>&1
rc=$?
grep "host timing" $O/bench_default.log | tail -1
tail -1 $O/bench_default.log | cut -c1-400
exit $rc
