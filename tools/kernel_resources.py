"""Resource lines of the gfx950 code objects (llvm-readelf --notes of the
offload bundle): python tools/kernel_resources.py soundchunks_amd/lib/gsc_scan.o"""
import sys, subprocess, re, tempfile, os
from pathlib import Path
LLVM=Path("/opt/rocm/lib/llvm/bin")
obj=sys.argv[1]
d=tempfile.mkdtemp()
subprocess.run([str(LLVM/"llvm-objcopy"), f"--dump-section=.hip_fatbin={d}/f", obj],check=True)
subprocess.run([str(LLVM/"clang-offload-bundler"),"--unbundle","--type=o",f"--input={d}/f","--targets=hipv4-amdgcn-amd-amdhsa--gfx950",f"--output={d}/o"],check=True)
notes=subprocess.run([str(LLVM/"llvm-readelf"),"--notes",f"{d}/o"],capture_output=True,text=True).stdout
cur={};ks=[]
for line in notes.splitlines():
    m=re.match(r"\s*-?\s*\.(\w+):\s+(\S+)",line)
    if not m: continue
    k,v=m.groups()
    if k=="agpr_count" and cur: ks.append(cur); cur={}
    cur[k]=v
ks.append(cur)
for k in ks:
    n=k.get("name","")
    if "kernel" in n:
        print(re.sub(r"_ZN3gsc|EEEEEvPNS.*","",n)[:60], "vgpr",k.get("vgpr_count"),"sgpr",k.get("sgpr_count"),"vspill",k.get("vgpr_spill_count"),"sspill",k.get("sgpr_spill_count"),"priv",k.get("private_segment_fixed_size"))
