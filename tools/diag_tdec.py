"""Per-half-iteration GPU vs oracle diagnostics (prints where decisions first diverge)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import Oracle, make_llrs  # noqa: E402
from srsran_4g_amd import tdec  # noqa: E402

ora = Oracle()
dec = tdec.TurboDecoder()
rng = np.random.default_rng(1)
ok = True
for K in [int(a) for a in sys.argv[1:]] or [6144, 1024, 512, 416, 40, 400]:
    _, llr = make_llrs(K, 2.0, rng, 1, ora)
    x = ora.natural_to_sb(K, llr[0])
    _, tr = ora.tdec_run(K, x, True, 6, trace=True)
    want = np.packbits((tr > 0).astype(np.uint8), axis=-1)
    dec.new_cb(K)
    for n in range(6):
        got = dec.iteration(x)
        nb = int(np.unpackbits(got ^ want[n]).sum())
        print(f"K={K} half-it {n}: {'OK' if nb == 0 else 'MISMATCH bits=%d' % nb}", flush=True)
        if nb:
            ok = False
            d = np.nonzero(np.unpackbits(got) != np.unpackbits(want[n]))[0]
            print("   first diff positions:", d[:12].tolist())
            break
print("ALL OK" if ok else "FAILURES")
