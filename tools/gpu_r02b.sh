#!/bin/bash
# round-2: scan kernel checks (C2 regression, D = 32 two-CU frames), quiet-case diagnosis
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_stages.py quiet_tone_cs8_cpf1024 > gpurun_out/diag_quiet.log 2>&1
cat gpurun_out/diag_quiet.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_scan.py "tests/test_gpu_parity.py::test_gsc_matches_golden" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests3.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gputests3.log | tail -40
exit $rc
