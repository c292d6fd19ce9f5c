"""Phase stamps of the batched KNNScanReduce kernel on one C2 frame (GPU box).
Build the stamps library first (make -C soundchunks_amd/csrc stamps), then:
    GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 \
        python tools/scan_stamps.py [passes] [cs]
(The batched kernel, scan_batch_kernel, is the only A1 layout: the MFMA one
of round 2 was not kept)"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

import soundchunks_amd as sc  # noqa: E402
from soundchunks_amd.synth import synth_wav  # noqa: E402

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
k = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
argv = [f"-cs{cs}", f"-cpf{k}", "-cbd8"]
# optional: a WAV file and frame index instead of the synthetic C2 frame
wav = Path(sys.argv[4]).read_bytes() if len(sys.argv) > 4 else synth_wav(8.0)
frame = int(sys.argv[5]) if len(sys.argv) > 5 else 0
if len(sys.argv) > 4:
    argv = [f"-cs{cs}", f"-cpf{k}"]
att, feat = sc.frame_dsp(wav, frame, argv)
y = sc.yakmo_seed_means(feat, k)
os.environ["GSC_SCAN_MAX_PASSES"] = str(passes)
t = time.time()
c, cl, it = sc.scan_reduce(feat, y, 3)
dt = time.time() - t
print(f"lib={os.environ.get('GSC_LIB', 'in-tree')} N={feat.shape[0]} D={feat.shape[1]} "
      f"passes={it} wall={dt:.3f}s us/search={dt / (it * feat.shape[0]) * 1e6:.3f} "
      f"crc={int(np.frombuffer(c.tobytes(), np.uint32).sum()) & 0xffffffff:08x}", flush=True)
