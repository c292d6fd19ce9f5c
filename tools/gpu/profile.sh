#!/bin/bash
# The round's profile set, each pass its own run: rocprofv3 kernel trace + stats of the default bench
# (C2, 1024 s), FETCH_SIZE and WRITE_SIZE PMC passes (256 s), one SQ pass (64 s); then the default
# bench with its CPU baseline (NODEFAULT=1 skips it).  Copy with: python tools/refresh_profiles.py rNN
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/trace.log 2>&1 || exit 2
tail -1 $O/trace.log | cut -c1-200
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY -d $O/sq -o run -- python3 -u bench.py --seconds 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/sq.log 2>&1 || exit 5
[ -n "$NODEFAULT" ] && exit 0
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || exit 6
tail -1 $O/bench_default.log | cut -c1-300
