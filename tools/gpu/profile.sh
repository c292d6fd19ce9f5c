#!/bin/bash
# round-3 final profile set: kernel trace + FETCH/WRITE PMC passes of the default bench, the default bench with
# its CPU baseline, c4 and br128 with theirs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/trace.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 || exit 4
timeout -k 10 400 python3 -u bench.py > $O/bench_default.log 2>&1 || exit 5
tail -1 $O/bench_default.log | cut -c1-200
GSC_HOST_TIMING=1 timeout -k 10 400 python3 -u bench.py --config c4 --steps 2 > $O/bench_c4.log 2>&1 || exit 6
tail -1 $O/bench_c4.log | cut -c1-200
timeout -k 10 400 python3 -u bench.py --config br128 --steps 2 > $O/bench_br128.log 2>&1 || exit 7
tail -1 $O/bench_br128.log | cut -c1-200
