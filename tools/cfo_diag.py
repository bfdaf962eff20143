"""GPU srsran_cfo_correct vs the reference's srsran_vec_apply_cfo: first mismatches (diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import torch  # noqa: E402,F401

import ofdm_np  # noqa: E402
from srsran_4g_amd import ue_dl as U  # noqa: E402

rng = np.random.default_rng(2)
for n in (30720, 1001, 8):
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    ones = np.ones(n, np.complex64)
    for f in (1.6e-5, 0.01, 0.37):
        for name, v in (("ones", ones), ("rand", x)):
            got, want = U.cfo_correct(v, f), ofdm_np.ref_apply_cfo(v, f)
            bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
            print(n, f, name, "mismatch", bad.size, "first", bad[:6].tolist(),
                  "got", got.view(np.float32)[bad[:4]].tolist(), "want", want.view(np.float32)[bad[:4]].tolist(),
                  "maxabs", float(np.abs(got - want).max()))
