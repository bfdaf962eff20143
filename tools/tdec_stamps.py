"""Cycles per trellis step of the single-lane turbo decoder (developer tool).

Loads the diagnostic build srsran_4g_amd/lib/stamps/libsrsran_4g_amd.so (Makefile `stamps`:
tdecs_kernel.hip with -DTDECS_STAMPS), where lane 0 of every wave writes the shader clock (clock64)
at five points of every half-iteration: start, end of the 40-step training, end of phase 1, after the
phase barrier, end of phase 2.  One K x batch launch (8 half-iterations), then per phase the median
over waves of the cycles and of the cycles per trellis step.

  python tools/tdec_stamps.py [--K 6144] [--batch 1024] [--w8 0]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--K", type=int, default=6144)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--iters", type=int, default=8)
    p.add_argument("--w8", type=int, default=0, help="srsran_tdec_gpu_set_w8_max_k")
    p.add_argument("--lib", default="stamps", help="lib/<dir> of the diagnostic build: stamps, stamps_fake")
    a = p.parse_args()
    import ctypes

    import torch

    from srsran_4g_amd import tdec
    from synth import synth as SY
    tdec.LIB_PATH = os.path.join(ROOT, "srsran_4g_amd", "lib", a.lib, "libsrsran_4g_amd.so")
    lib = tdec.load_library()
    lib.srsran_tdec_gpu_debug_set_stamps.argtypes = [ctypes.c_void_p]
    lib.srsran_tdec_gpu_debug_set_stamps.restype = ctypes.c_int
    lib.srsran_tdec_gpu_set_w8_max_k(a.w8)
    lib.srsran_tdec_gpu_set_pair_threshold(0)
    lib.srsran_tdec_gpu_set_single_threshold(0)  # the single-lane kernel at every batch size
    K = a.K
    nsb = tdec.nof_subblocks(K)
    assert nsb in (8, 16), "window classes only"
    W = 8 if K <= a.w8 else 16
    L = K // nsb
    Ma = (L + W - 1) // W
    h = max(1, min((L + W) // (2 * W), L // W))
    rng = np.random.default_rng(3)
    _, llr = SY.make_llrs(K, 4.0, rng, 8)
    sb = SY.natural_to_sb(K, llr)
    d_in = torch.from_numpy(np.ascontiguousarray(np.tile(sb, (a.batch // 8 + 1, 1))[: a.batch])).cuda()
    d_out = torch.empty((a.batch, K // 8), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    def launch():
        tdec.gpu_run_batch(K, d_in.data_ptr(), d_in.shape[1], True, d_out.data_ptr(), a.batch, a.iters, s.cuda_stream)

    launch()
    torch.cuda.synchronize()
    cpw = 64 // nsb
    nwg = (a.batch + cpw - 1) // cpw
    buf = torch.zeros(nwg * 2 * 64, dtype=torch.int64, device="cuda")
    assert lib.srsran_tdec_gpu_debug_set_stamps(buf.data_ptr()) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    launch()
    e1.record(s)
    torch.cuda.synchronize()
    assert lib.srsran_tdec_gpu_debug_set_stamps(None) == 0
    ms = e0.elapsed_time(e1)
    st = buf.cpu().numpy().reshape(nwg, 2, 64)[:, :, : 5 * a.iters].reshape(nwg, 2, a.iters, 5).astype(np.float64)
    span = float(np.median(st[:, :, -1, 4] - st[:, :, 0, 0]))  # one wave's first to last stamp
    # steps per phase and side (crossover schedule, tdecs_kernel.hip map16s)
    steps = {"training": (40, 40), "phase1": (h * W, L - h * W), "phase2": (L - h * W, h * W)}
    out = {"lib": a.lib, "kernel": tdec.last_kernel(), "K": K, "batch": a.batch, "W": W, "L": L, "windows": Ma, "h": h,
           "launch_ms": round(ms, 4), "wave_span_cycles": int(span),
           "clock_ghz_implied": round(span / (ms * 1e6), 3)}
    sides = ("alpha", "beta")
    for name, (k0, k1) in (("training", (0, 1)), ("phase1", (1, 2)), ("barrier_wait", (2, 3)), ("phase2", (3, 4))):
        for w, side in enumerate(sides):
            cyc = np.median(st[:, w, :, k1] - st[:, w, :, k0], axis=0)  # per half-iteration
            ent = {"cycles_per_half_it": [int(c) for c in cyc]}
            if name in steps:
                n = steps[name][w]
                ent["steps"] = n
                ent["cycles_per_step"] = round(float(np.median(cyc) / n), 1)
            out[f"{name}_{side}"] = ent
    gap = np.median(st[:, :, 1:, 0] - st[:, :, :-1, 4], axis=(0, 2))
    out["between_half_its_cycles"] = [int(g) for g in gap]
    half = np.median(st[:, :, :, 4] - st[:, :, :, 0], axis=(0, 2))
    out["half_it_cycles"] = [int(x) for x in half]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
