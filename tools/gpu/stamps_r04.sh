#!/bin/bash
# phase stamps of the batched scan kernel (a -DGSC_STAMPS variant, tools/build_variant.sh NAME -DGSC_STAMPS)
# on one 44.1 kHz stereo frame at -cs8 (the C2 frame, D = 16) and at -cs4 (D = 8), 100 passes each
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/prof
mkdir -p $O
S=soundchunks_amd/lib/variants/${STAMPS:-r4stamps}/libsoundchunks_amd.so
export GSC_SCAN_DEBUG=1
for cs in ${STCS:-8 4}; do
  GSC_LIB=$S timeout -k 10 150 python -u tools/scan_stamps.py 100 $cs 4096 > $O/stamps_cs$cs.log 2>&1 || exit 3
  grep -A20 "^stamps" $O/stamps_cs$cs.log; tail -1 $O/stamps_cs$cs.log
done
