"""soundchunks_amd: MI355X-native SoundChunks encode hot path.

Reference: GliGli's SoundChunks encoder (bravesoftdz/soundchunks), whose
per-frame vector quantisation (yakmo k-means++ + KNNScanReduce over ANN's
kd-tree, then the KNNFit nearest-chunk search) runs here as hand-written
gfx950 HIP kernels behind the extern.pas C ABI (include/soundchunks.h).
"""
from .encoder import Encoder, encode_many, frame_dsp, knnfit_assign, parse_options, scan_reduce, set_device, yakmo_seed_means  # noqa: F401
from ._lib import GscError, LIB_PATH, load  # noqa: F401

__all__ = ["Encoder", "encode_many", "frame_dsp", "parse_options", "set_device", "yakmo_seed_means", "scan_reduce", "knnfit_assign", "GscError", "load",
           "LIB_PATH"]
