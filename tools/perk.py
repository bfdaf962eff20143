"""Per-K turbo decoder throughput on the GPU (developer tool): 1024 CBs of each size, 8
half-its, SB layout, one launch per K timed with events on the launch stream."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from srsran_4g_amd import tdec  # noqa: E402
from synth import synth as SY  # noqa: E402

rng = np.random.default_rng(1)
Ks = [int(a) for a in sys.argv[1:]] or list(tdec.CB_SIZES)
stream = torch.cuda.current_stream()
tot_ms = 0.0
rows = []
for K in Ks:
    _, llr = SY.make_llrs(K, 4.0, rng, 8)
    sb = SY.natural_to_sb(K, llr)
    host = np.tile(sb, (128, 1))
    d_in = torch.from_numpy(np.ascontiguousarray(host)).cuda()
    d_out = torch.empty((1024, K // 8), dtype=torch.uint8, device="cuda")
    run = lambda: tdec.gpu_run_batch(K, d_in.data_ptr(), d_in.shape[1], True, d_out.data_ptr(), 1024, 8,  # noqa
                                     stream.cuda_stream)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    tot_ms += ms
    rows.append((K, ms, 1024 * K / ms / 1e6))
for K, ms, gb in rows:
    print(f"K={K:5d} {ms:8.3f} ms {gb:8.2f} Gbit/s")
print(f"serial total {tot_ms:.2f} ms")
