#!/bin/bash
# Strong scaling of the fixed 1-hour C5 file, measured per rank on one GPU:
# bench.py --strong --seconds 3600 --share R/N encodes rank R of N's frame range
# of the whole file's PrepareFrames cut, checked frame by frame against the
# whole-file digests.  SHARES = "R/N ..." (default: every rank of 8 and of 4),
# CFGS = "c5 c5cs4"; JSON lines in gpurun_out/prof/strong_<cfg>_r<R>of<N>.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/prof
mkdir -p $O
SH=${SHARES:-"0/8 1/8 2/8 3/8 4/8 5/8 6/8 7/8 0/4 1/4 2/4 3/4"}
for c in ${CFGS:-c5 c5cs4}; do
  for s in $SH; do
    f=$O/strong_${c}_r${s%/*}of${s#*/}.log
    timeout -k 10 300 python3 -u bench.py --config $c --strong --seconds 3600 --share $s \
      --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > $f 2>&1 || exit 3
    tail -1 $f | cut -c1-140
  done
done
