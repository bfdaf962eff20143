"""Stage micro-benchmarks on the GPU (developer tool): LLR (demap / descramble / CSI) and MMSE
predecoding on one large item, timed with events on the launch stream."""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from srsran_4g_amd import phch  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


n = 128 * 14400
sym = torch.randn(2 * n, device="cuda") * 0.5
llr = torch.zeros(6 * n, dtype=torch.int16, device="cuda")
csi = torch.rand(n, device="cuda")
mx = torch.ones(1, device="cuda")
for scr in (0, 1):
    for c in (False, True):
        us = timeit(lambda: phch.gpu_llr(3, sym.data_ptr(), n, scr, 12345, llr.data_ptr(), None,
                                         csi.data_ptr() if c else None, mx.data_ptr() if c else None))
        print(f"llr 64QAM n={n} scramble={scr} csi={c}: {us:.1f} us  {n * (8 + 12 + (4 if c else 0)) / us / 1e3:.0f} GB/s")

m = 64 * 14400
y = [torch.randn(2 * m, device="cuda") for _ in range(2)]
h = [[torch.randn(2 * m, device="cuda") for _ in range(2)] for _ in range(2)]
x = [torch.zeros(2 * m, device="cuda") for _ in range(2)]
cs = [torch.zeros(m, device="cuda") for _ in range(2)]
cm = torch.zeros(2, device="cuda")
for withmax in (False, True):
    us = timeit(lambda: phch.predecode_gpu(3, [t.data_ptr() for t in y], [[t.data_ptr() for t in r] for r in h],
                                           [t.data_ptr() for t in x], [t.data_ptr() for t in cs],
                                           cm.data_ptr() if withmax else None, 2, 2, 2, 0, m, 1.0, 0.01))
    print(f"predecode CDD n={m} csi_max={withmax}: {us:.1f} us  {m * (16 + 32 + 16 + 8) / us / 1e3:.0f} GB/s")
