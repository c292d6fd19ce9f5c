#!/bin/bash
# C5 under strong scaling, measured per rank on one GPU: the fixed 1-hour 48 kHz stereo file
# split 8 / 4 / 2 ways is 452 / 900 / 1800 s per rank (113 / 225 / 450 frames).  Also records the
# box's CPU share (cgroup quota) for the CPU-baseline leg.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/strong
mkdir -p $O
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cgroup v2 cpu.max";
  grep -m1 'model name' /proc/cpuinfo; } > $O/box.txt
cat $O/box.txt
for s in 452 900 1800; do
  timeout -k 10 300 python3 -u bench.py --config ${CFG:-c5} --strong --seconds $s --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/c5_${CFG:-c5}_$s.log 2>&1 || exit 2
  tail -1 $O/c5_${CFG:-c5}_$s.log | cut -c1-220
done
