# scan kernel compile-flag experiment: short bench per variant library (GSC_LIB)
set -o pipefail
for v in A B C D; do
  GSC_LIB=soundchunks_amd/lib/s$v/libsoundchunks_amd.so timeout -k 10 200 python -u bench.py --seconds 256 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/sv_$v.log 2>&1 || exit 1
done
