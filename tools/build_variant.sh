#!/bin/bash
# A/B build of the scan kernel with extra defines, linked as its own library:
#   tools/build_variant.sh NAME [-src FILE.hip] -DFLAG ...  ->  soundchunks_amd/lib/variants/NAME/libsoundchunks_amd.so
# (select it with GSC_LIB=...; the in-tree build must be current; -src: another
# scan source, e.g. the previous commit's, compiled against the current headers)
set -e
cd "$(dirname "$0")/../soundchunks_amd/csrc"
name=$1; shift
src=gsc_scan.hip
if [ "$1" = "-src" ]; then src=$2; shift 2; fi
out=../lib/variants/$name
mkdir -p $out
/opt/rocm/bin/hipcc -O2 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
  --offload-arch=gfx950 -fno-gpu-rdc -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize -fno-vectorize \
  -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c -o $out/gsc_scan.o $src
objs=$(ls ../lib/*.o | grep -v gsc_scan.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libsoundchunks_amd.so $objs $out/gsc_scan.o -lpthread
echo built $out
