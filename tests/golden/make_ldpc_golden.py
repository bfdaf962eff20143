"""Generate tests/golden/ldpc_examples.npz from the reference's LDPC golden examples.

Source (data held by the reference's own tests, read as text; run in the build container):
  /root/reference/lib/src/phy/fec/ldpc/test/examplesBG1.dat, examplesBG2.dat
Format there (ldpc_dec_test.c:get_examples): for every lifting size a block "ls<Z>msgs" of 10
messages (liftK characters '0' / '1' / '-' = filler bit) and a block "ls<Z>cwds" of the 10
codewords (liftN - 2*Z characters, the first 2*Z bits punctured).  We keep the first NKEEP
examples per (base graph, lifting size) with bits packed; filler positions are stored as
index lists.

    python tests/golden/make_ldpc_golden.py
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = "/root/reference/lib/src/phy/fec/ldpc/test/examplesBG{}.dat"
OUT = os.path.join(ROOT, "tests", "golden", "ldpc_examples.npz")
NKEEP = 3
BG_SHAPE = {0: (46, 68, 22), 1: (42, 52, 10)}


def parse(path):
    blocks, cur, key = {}, None, None
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if not line:
                continue
            if line.startswith("ls"):
                key = line
                cur = blocks.setdefault(key, [])
            else:
                cur.append(line)
    return blocks


def main():
    arrays = {}
    for bg in (0, 1):
        M, N, K = BG_SHAPE[bg]
        blocks = parse(SRC.format(bg + 1))
        for key in blocks:
            if not key.endswith("msgs"):
                continue
            ls = int(key[2:-4])
            msgs = blocks[key][:NKEEP]
            cwds = blocks[f"ls{ls}cwds"][:NKEEP]
            assert all(len(m) == K * ls for m in msgs) and all(len(c) == (N - 2) * ls for c in cwds)
            m = np.array([[c == "1" for c in s] for s in msgs], np.uint8)
            c = np.array([[ch == "1" for ch in s] for s in cwds], np.uint8)
            mf = {len(s) - len(s.rstrip("-")) for s in msgs}
            assert len(mf) == 1 and all("-" not in s.rstrip("-") for s in msgs)
            cf = [i for i, ch in enumerate(cwds[0]) if ch == "-"]
            assert all([i for i, ch in enumerate(s) if ch == "-"] == cf for s in cwds)
            arrays[f"{bg}_{ls}_msg"] = np.packbits(m, axis=1)
            arrays[f"{bg}_{ls}_cw"] = np.packbits(c, axis=1)
            arrays[f"{bg}_{ls}_fill"] = np.array([mf.pop(), len(cf)], np.int32)
            if cf:
                arrays[f"{bg}_{ls}_cfill"] = np.array(cf, np.int32)
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, os.path.getsize(OUT), "bytes,", sum(k.endswith("_msg") for k in arrays), "lifting cases")


if __name__ == "__main__":
    main()
