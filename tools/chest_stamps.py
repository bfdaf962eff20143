"""Where the batch channel estimator's time goes (developer tool).

Loads the diagnostic build srsran_4g_amd/lib/stamps/libsrsran_4g_amd.so (Makefile `stamps`: chest_kernel.hip with
-DCHEST_STAMPS), where thread 0 of every chest_kernel workgroup writes the device wall clock (100 MHz) at its
phase boundaries: 0 start, 1 pilots + RSSI loaded, 2 RSRP / RSSI reduced, 3 CFO sums, 4 noise, 5 smoothing,
6 estimates written, 7 end (after the subframe's finalize).  Runs the C3 UE DL batch (78 subframes) as bench.py
does and prints, per phase, the median duration over workgroups, plus the spread of start and end times.

  python tools/chest_stamps.py [--subframes 78]
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
    p.add_argument("--subframes", type=int, default=78)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    os.environ["SRSRAN_AMD_LIB"] = os.path.join(ROOT, "srsran_4g_amd", "lib", "stamps", "libsrsran_4g_amd.so")
    import ctypes

    import torch

    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    from srsran_4g_amd import ue_dl as U
    from synth import synth as SY

    lib = tdec.load_library()
    lib.srsran_chest_dl_gpu_debug_set_stamps.argtypes = [ctypes.c_void_p]
    lib.srsran_chest_dl_gpu_debug_set_stamps.restype = ctypes.c_int
    tbs, qm, nfft = 75376, 6, 2048
    rng = np.random.default_rng(5)
    pool = []
    for i in range(10):
        tti = i + 1
        pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(2)]
        x, nre = SY.pdsch_subframe(100, 1, 2, tti, 1, 0x1234, tbs, qm, 0, pls, snr_db=30.0, rng=rng, N=nfft)
        pool.append((tti, x, nre))
    nsf = a.subframes
    d_x = torch.from_numpy(np.ascontiguousarray(np.stack([pool[b % 10][1] for b in range(nsf)])).view(np.float32)).cuda()
    U.use_standard_symbol_size(True)
    ue = U.UeDl(U.cell(100, 2, 1), 2)
    sbs = [[S.SoftbufferRx(nof_prb=100) for _ in range(2)] for _ in range(nsf)]
    cfgs = [U.pdsch_cfg(100, pool[b % 10][2], (tbs, tbs), (qm, qm), rnti=0x1234, softbuffers=sbs[b]) for b in range(nsf)]
    d_pl = torch.zeros((nsf, 2, tbs // 8 + 64), dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(2 * nsf, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(2 * nsf, dtype=torch.float32, device="cuda")
    arr = U.UeDl.batch_entries([(pool[b % 10][0], 1, cfgs[b], [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1])
                                for b in range(nsf)])
    nwg = 4 * nsf
    st = torch.zeros(nwg * 16, dtype=torch.int64, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # warm-up without stamps
        assert ue.gpu_decode_batch(arr, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, sp) == 2 * nsf
    torch.cuda.synchronize()
    assert lib.srsran_chest_dl_gpu_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
    phases = {}
    spans = []
    for _ in range(a.reps):
        st.zero_()
        assert ue.gpu_decode_batch(arr, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, sp) == 2 * nsf
        torch.cuda.synchronize()
        t = st.cpu().numpy().reshape(nwg, 16)[:, :8].astype(np.float64) * 10e-3  # 100 MHz ticks -> us
        t0 = t[:, 0].min()
        spans.append({"start_spread_us": float(t[:, 0].max() - t0), "end_us": float(t[:, 7].max() - t0),
                      "median_wg_us": float(np.median(t[:, 7] - t[:, 0]))})
        for k in range(1, 8):
            phases.setdefault(k, []).extend(list(t[:, k] - t[:, k - 1]))
    names = {1: "pilot+rssi loads", 2: "rsrp/rssi reduce", 3: "cfo sums", 4: "noise", 5: "average+smooth",
             6: "interp+store", 7: "finalize/exit"}
    out = {"workgroups": nwg, "phase_median_us": {names[k]: round(float(np.median(v)), 3) for k, v in phases.items()},
           "phase_p90_us": {names[k]: round(float(np.percentile(v, 90)), 3) for k, v in phases.items()},
           "launch": {k: round(float(np.median([s[k] for s in spans])), 3) for k in spans[0]}}
    print(json.dumps(out, indent=1))
    lib.srsran_chest_dl_gpu_debug_set_stamps(ctypes.c_void_p(0))
    ue.free()


if __name__ == "__main__":
    main()
