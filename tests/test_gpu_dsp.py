"""Device DSP (gsc_dsp.hip) against the oracle (pytest -m gpu): the
attenuation divider of FindAttenuationDivider (encoder.lpr:566-605) and the
MakeChunks features (DCT-II + cepstrum, encoder.lpr:258-322, 349-363,
467-485) of single frames, bit for bit.  End-to-end .gsc parity
(test_gpu_parity.py) covers the same kernels inside the full encode.
"""
from __future__ import annotations

import numpy as np
import pytest

from golden.cases import CASES

pytestmark = pytest.mark.gpu

# every golden case except the passthrough one (its frames never reach yakmo,
# but the DSP still runs: keep it, it is the smallest frame shape)
NAMES = sorted(CASES)


@pytest.mark.parametrize("name", NAMES)
def test_frame_dsp_bit_exact(oracle, name):
    import soundchunks_amd as sc

    make, argv = CASES[name]
    wav = make()
    tr = oracle.trace_frame(wav, argv, 0)
    att, feat = sc.frame_dsp(wav, 0, argv)
    assert att == tr["atten_div"]
    assert feat.shape == tr["dataset"].shape
    np.testing.assert_array_equal(feat.view(np.uint32), np.ascontiguousarray(tr["dataset"]).view(np.uint32))


def test_frame_dsp_last_frame(oracle):
    """A ragged last frame (partial chunk zero-padded, partial atten chunk dropped)."""
    import soundchunks_amd as sc

    make, argv = CASES["syn3s_cs8_cpf1000_cbd12"]
    wav = make()
    n = sc.Encoder(argv).frame_count(wav)
    tr = oracle.trace_frame(wav, argv, n - 1)
    att, feat = sc.frame_dsp(wav, n - 1, argv)
    assert att == tr["atten_div"]
    np.testing.assert_array_equal(feat.view(np.uint32), np.ascontiguousarray(tr["dataset"]).view(np.uint32))
