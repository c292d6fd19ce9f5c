#!/bin/bash
# one PMC pass of SQ counters over a short C2 bench (instruction mix and waits of the scan kernel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY -d $O/sq -o run -- python3 -u bench.py --seconds 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/sq.log 2>&1 || exit 3
tail -1 $O/sq.log | cut -c1-120
