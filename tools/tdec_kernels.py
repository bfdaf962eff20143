"""Turbo-decoder kernel micro-benchmark (developer tool, for timing and rocprofv3 --pmc passes): N identical
launches of one 16-sub-block-class decoder on one workload, HIP events on the launch stream.

  python tools/tdec_kernels.py --kernel single|pair|quad --workload k6144|all188|class8|class1 [--K k]
                               [--batch 1024] [--launches 5]

k6144: K = 6144 x batch blocks (srsran_tdec_gpu_run_batch); all188: every K >= 816 x batch blocks in one
fused srsran_tdec_gpu_run_multi call (the 16-sub-block class of the bench's all-188 step); class8: the
same for the 32 sizes of the 8-sub-block class (408 <= K <= 800).  Inputs: AWGN
blocks at Eb/No 4 dB (the bench's), 8 distinct blocks per size tiled.  8 half-iterations."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from srsran_4g_amd import tdec  # noqa: E402
from synth import synth as SY  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kernel", choices=["single", "pair", "quad"], default="single")
    p.add_argument("--workload", choices=["k6144", "all188", "class8", "class1"], default="k6144")
    p.add_argument("--K", type=int, default=0, help="one code block size instead of the workload's")
    p.add_argument("--w8", type=int, default=0, help="srsran_tdec_gpu_set_w8_max_k (8-step-window build up to K)")
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--launches", type=int, default=5)
    p.add_argument("--iters", type=int, default=8)
    p.add_argument("--lib", default="", help="another build of the library (A/B timing)")
    a = p.parse_args()
    if a.lib:
        tdec.LIB_PATH = os.path.abspath(a.lib)
    never = 1 << 30
    pair_min, single_min = {"single": (0, 0), "pair": (0, never), "quad": (never, never)}[a.kernel]
    lib = tdec.load_library()
    lib.srsran_tdec_gpu_set_w8_max_k(a.w8)
    lib.srsran_tdec_gpu_set_pair_threshold(pair_min)
    lib.srsran_tdec_gpu_set_single_threshold(single_min)
    lib.srsran_tdec_gpu_set_generic_single_threshold(single_min)
    nsb = {"class8": 8, "class1": 0}.get(a.workload, 16)  # srsran_tdec_autoimp_get_subblocks: 0 = generic
    Ks = [6144] if a.workload == "k6144" else [k for k in tdec.CB_SIZES if tdec.nof_subblocks(k) == nsb]
    if a.K:
        Ks, nsb = [a.K], tdec.nof_subblocks(a.K)
    rng = np.random.default_rng(5)
    ins, outs = [], []
    for K in Ks:
        _, llr = SY.make_llrs(K, 4.0, rng, 8)
        sb = SY.natural_to_sb(K, llr) if nsb else llr
        ins.append(torch.from_numpy(np.ascontiguousarray(np.tile(sb, (a.batch // 8 + 1, 1))[: a.batch])).cuda())
        outs.append(torch.empty((a.batch, K // 8), dtype=torch.uint8, device="cuda"))
    s = torch.cuda.current_stream()

    def launch():
        if len(Ks) == 1:
            tdec.gpu_run_batch(Ks[0], ins[0].data_ptr(), ins[0].shape[1], True, outs[0].data_ptr(), a.batch, a.iters,
                               s.cuda_stream)
        else:
            tdec.gpu_run_multi(Ks, [t.data_ptr() for t in ins], [t.shape[1] for t in ins], True,
                               [t.data_ptr() for t in outs], [a.batch] * len(Ks), a.iters, s.cuda_stream)

    launch()
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.launches):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch()
        e1.record(s)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    bits = a.batch * sum(Ks)
    print(json.dumps({"lib": os.path.basename(a.lib) if a.lib else "head", "kernel": tdec.last_kernel(), "workload": a.workload, "batch": a.batch, "blocks": a.batch * len(Ks),
                      "ms": [round(x, 4) for x in ms], "gbps": round(bits / (min(ms) * 1e-3) / 1e9, 2)}))


if __name__ == "__main__":
    main()
