"""How much turbo-decoder work the DL-SCH early stop wastes at the workgroup level in the C3 chain (developer tool;
VERDICT r05 item 3).  Runs one batch of C3 subframes (100 PRB, CDD 2x2, 64QAM, the bench's subframes) at --snr through
srsran_ue_dl_gpu_decode_batch with the diagnostic build (Makefile `stamps`, tdecs_kernel.hip -DTDECS_STAMPS), whose
DL-SCH decoder writes, per workgroup, the half-iterations each of its 4 blocks needed and the half-iterations the
workgroup ran (the max over them: early stop retires whole workgroups).  Prints the block and workgroup
distributions and the waste: sum over workgroups of (4 x ran - sum needed) / sum ran x 4.

  python tools/chain_stamps.py [--snr 17] [--subframes 78]
"""
import argparse
import collections
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SRSRAN_AMD_LIB", os.path.join(ROOT, "srsran_4g_amd", "lib", "stamps", "libsrsran_4g_amd.so"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--snr", type=float, default=17.0)
    p.add_argument("--subframes", type=int, default=78)
    p.add_argument("--iters", type=int, default=8)
    a = p.parse_args()
    import torch

    import bench as B
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import tdec
    from srsran_4g_amd import ue_dl as U
    from synth import synth as SY

    lib = tdec.load_library()
    lib.srsran_tdec_gpu_debug_set_stamps.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(1)
    pool = []
    for i in range(10):
        pls = [rng.integers(0, 256, B.C3_TBS // 8, dtype=np.uint8) for _ in range(2)]
        x, nre = SY.pdsch_subframe(100, 1, 2, i + 1, 1, 0x1234, B.C3_TBS, B.C3_QM, 0, pls, snr_db=a.snr, rng=rng, N=2048)
        pool.append((i + 1, x, nre))
    nsf = a.subframes
    d_x = torch.from_numpy(np.ascontiguousarray(np.stack([pool[b % 10][1] for b in range(nsf)])).view(np.float32)).cuda()
    U.use_standard_symbol_size(True)
    ue = U.UeDl(U.cell(100, 2, 1), 2)
    ue.cfg.cfg.pdsch.max_nof_iterations = a.iters
    sbs = [[S.SoftbufferRx(nof_prb=100) for _ in range(2)] for _ in range(nsf)]
    cfgs = [U.pdsch_cfg(100, pool[b % 10][2], (B.C3_TBS, B.C3_TBS), (B.C3_QM, B.C3_QM), rnti=0x1234,
                        max_iterations=a.iters, softbuffers=sbs[b]) for b in range(nsf)]
    d_pl = torch.zeros((nsf, 2, B.C3_TBS // 8 + 64), dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(2 * nsf, dtype=torch.int32, device="cuda")
    d_avg = torch.zeros(2 * nsf, dtype=torch.float32, device="cuda")
    arr = U.UeDl.batch_entries([(pool[b % 10][0], 1, cfgs[b], [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1])
                                for b in range(nsf)])
    st = torch.cuda.current_stream().cuda_stream
    assert ue.gpu_decode_batch(arr, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, st) == 2 * nsf
    torch.cuda.synchronize()
    nwg = 4096
    buf = torch.zeros(nwg * 2 * 64, dtype=torch.int64, device="cuda")
    assert lib.srsran_tdec_gpu_debug_set_stamps(buf.data_ptr()) == 0
    assert ue.gpu_decode_batch(arr, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, st) == 2 * nsf
    torch.cuda.synchronize()
    lib.srsran_tdec_gpu_debug_set_stamps(None)
    s = buf.cpu().numpy().reshape(nwg, 2, 64)[:, 0, :]
    ran = s[:, 63]
    need = s[:, 56:60]
    used = ran > 0
    ran, need = ran[used], need[used]
    live = need > 0
    blocks = int(live.sum())
    work_needed = int(need[live].sum())
    work_ran = int((ran[:, None] * live).sum())
    # the DEC1/DEC2 half-iteration clock of a workgroup's stamps: cycles of the group from its first to last stamp
    out = {"snr_db": a.snr, "workgroups": int(used.sum()), "blocks": blocks,
           "block_half_its": dict(sorted(collections.Counter(need[live].tolist()).items())),
           "workgroup_half_its": dict(sorted(collections.Counter(ran.tolist()).items())),
           "mean_needed": round(work_needed / blocks, 3), "mean_ran_per_block": round(work_ran / blocks, 3),
           "waste_frac": round(1 - work_needed / work_ran, 4),
           "tb_ok_fraction": float((d_res.cpu().numpy() == 0).mean()),
           "launch_span_half_its": int(ran.max())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
