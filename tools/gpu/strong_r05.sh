#!/bin/bash
# round 5: C5 (-cs8) strong-scaling shares of the 1-hour file, per rank on one GPU
# (bench.py --strong --seconds S = one rank's share of an N-way split); JSON lines in gpurun_out/prof/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/prof
mkdir -p $O
for s in ${SHARES:-1800 900 452}; do
  timeout -k 10 600 python3 -u bench.py --config ${CFG:-c5} --strong --seconds $s --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/strong_${CFG:-c5}_$s.log 2>&1 || exit 3
  tail -1 $O/strong_${CFG:-c5}_$s.log | cut -c1-160
done
