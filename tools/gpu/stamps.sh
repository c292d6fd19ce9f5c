#!/bin/bash
# phase stamps + iteration-kind counters (make -C soundchunks_amd/csrc stamps) on one C2 frame
# (-cs8, D = 16), one -cs4 frame (D = 8), and the C4-default tail frame (60.wav frame 1 at -cs4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/prof
mkdir -p $O
S=${STLIB:-soundchunks_amd/lib/stamps/libsoundchunks_amd.so}
export GSC_SCAN_DEBUG=1
for cs in ${STCS:-8 4}; do
  GSC_LIB=$S timeout -k 10 150 python -u tools/scan_stamps.py 100 $cs 4096 > $O/stamps_cs$cs.log 2>&1 || exit 3
  grep -A24 "^stamps" $O/stamps_cs$cs.log | grep -v "^  w[1-35-7]:"; tail -1 $O/stamps_cs$cs.log
done
[ -n "$NOC4" ] && exit 0
GSC_LIB=$S timeout -k 10 150 python -u tools/scan_stamps.py 100 4 4096 tests/golden/lame_test/60.wav 1 > $O/stamps_60f1.log 2>&1 || exit 3
grep -A24 "^stamps" $O/stamps_60f1.log | grep -v "^  w[1-35-7]:"; tail -1 $O/stamps_60f1.log
