"""Generate tests/golden/tdec_golden.npz from the reference decoder (oracle/_ref).

Run in the build container (where /root/reference exists and oracle/_ref was built
by `make -C oracle`):  python tests/golden/make_golden.py

Each case is one code block: int16 LLRs in natural 3K+12 layout (AWGN in the
convention of turbodecoder_test.c:217-255, or uniform random int16 to exercise
saturation), and the REFERENCE's outputs:
  out_nat_{8,16}  srsran_tdec_run_all with force_not_sb (natural layout)
  out_sb_{8,16}   same input permuted to the rm_turbo sub-block layout
  trace_crc       crc32 of the reference's decoder output after each of 16 half-iterations
The script asserts that the natural and SB runs agree, which pins the
natural->SB permutation helper against the reference's own input extraction.
"""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import Oracle, Reference, make_llrs  # noqa: E402

KS = [40, 48, 104, 200, 400, 408, 512, 528, 800, 816, 1024, 1056, 2048, 2112, 3072, 5824, 6144]


def main():
    ref = Reference()
    ora = Oracle()
    rng = np.random.default_rng(0x5EED)
    cases = {}
    idx = 0
    for K in KS:
        for kind in ("awgn", "rand"):
            if kind == "awgn":
                _, llr = make_llrs(K, 1.0, rng, 1, ref)
                llr = llr[0]
            else:
                llr = rng.integers(-32768, 32768, size=3 * K + 12, dtype=np.int16)
            sb = ora.natural_to_sb(K, llr)
            _, tr = ref.tdec_run(K, llr, False, 16, trace=True)
            o16 = ref.tdec_run(K, llr, False, 16)
            o8 = ref.tdec_run(K, llr, False, 8)
            s8 = ref.tdec_run(K, sb, True, 8)
            s16 = ref.tdec_run(K, sb, True, 16)
            assert np.array_equal(o8, s8) and np.array_equal(o16, s16), K
            crc = np.array([zlib.crc32(row.tobytes()) for row in tr], dtype=np.uint32)
            p = f"c{idx:03d}_"
            cases[p + "K"] = np.array([K], np.int32)
            cases[p + "llr"] = llr
            cases[p + "out_nat_8"] = o8
            cases[p + "out_nat_16"] = o16
            cases[p + "out_sb_8"] = s8
            cases[p + "out_sb_16"] = s16
            cases[p + "trace_crc"] = crc
            idx += 1
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tdec_golden.npz")
    np.savez_compressed(out, ncases=np.array([idx]), **cases)
    print(f"wrote {idx} cases to {out} ({os.path.getsize(out)} bytes)")


if __name__ == "__main__":
    main()
