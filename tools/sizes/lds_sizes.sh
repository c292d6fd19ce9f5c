#!/bin/bash
# print the scan kernel's LDS bytes per frame (host build, no GPU needed)
set -e
d=$(mktemp -d)
/opt/rocm/bin/hipcc -std=c++17 --offload-arch=gfx950 -O0 -w -o $d/lds_sizes "$(dirname "$0")/lds_sizes.hip"
$d/lds_sizes
rm -rf $d
