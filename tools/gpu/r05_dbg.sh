cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VS:-tree foldlate}; do
  L=soundchunks_amd/lib/libsoundchunks_amd.so; [ $v != tree ] && L=soundchunks_amd/lib/variants/$v/libsoundchunks_amd.so
  GSC_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_bench.py -x -q --timeout 120 --timeout-method thread -k "${K:-scan_k4096_full or bench_line_is_bit_exact}" > gpurun_out/dbg_$v.log 2>&1; echo "$v rc=$? $(tail -1 gpurun_out/dbg_$v.log)"
done
