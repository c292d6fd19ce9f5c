"""Code-object resource checks of the batched scan kernel (CPU, no GPU needed).

The scan kernel keeps K x D centroid floats in VGPRs.  If any access to that
register block uses a runtime index, LLVM demotes the whole block to scratch
memory and the kernel runs several times slower while staying bit-exact, so
no parity test notices.  The private segment then exceeds the spill slots by
far more than the small fixed frame.  This test reads the code object's
metadata (llvm-readelf --notes of the gfx950 bundle in gsc_scan.o) and fails
on that signature.
"""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
OBJ = ROOT / "soundchunks_amd" / "lib" / "gsc_scan.o"
LLVM = Path("/opt/rocm/lib/llvm/bin")


def _kernel_notes(tmp_path):
    fatbin = tmp_path / "scan.fatbin"
    dev = tmp_path / "scan_dev.o"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fatbin}", str(OBJ)], check=True,
                   cwd=tmp_path)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fatbin}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True, cwd=tmp_path)
    notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(dev)], check=True, capture_output=True,
                           text=True).stdout
    kernels = []
    cur = {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count" and cur:
            kernels.append(cur)
            cur = {}
        cur[k] = v
    if cur:
        kernels.append(cur)
    return [k for k in kernels if "scan_batch_kernel" in k.get("name", "")]


@pytest.mark.skipif(not OBJ.exists() or not (LLVM / "llvm-readelf").exists() or shutil.which("python3") is None,
                    reason="scan kernel object not built here")
def test_scan_kernel_register_block_not_in_scratch(tmp_path):
    ks = _kernel_notes(tmp_path)
    assert len(ks) >= 10, "expected every batched scan kernel instance"
    for k in ks:
        spills = int(k.get("vgpr_spill_count", 0))
        private = int(k.get("private_segment_fixed_size", 0))
        # spill slots (4 B per VGPR) plus a small fixed frame (up to 204 B
        # seen: D = 32 K = 4096 with the out-of-line exact DFS's call frame);
        # a demoted centroid block adds >= 256 B (K = 256 at D = 8) up to
        # 512 B per lane
        assert private <= 4 * spills + 224, (k["name"], spills, private)
