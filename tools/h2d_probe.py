"""PCIe-inclusive PDSCH chain timing probe (developer tool): where the time of the double-buffered
H2D + decode loop of bench.py run_pdsch goes.  Prints one JSON line per variant."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from synth import synth as SY  # noqa: E402
from srsran_4g_amd import sch as S  # noqa: E402
from srsran_4g_amd import ue_dl as U  # noqa: E402

C3_TBS, C3_QM = 75376, 6


def main():
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(1)
    cell_id, rnti, nsf, iters = 1, 0x1234, 78, 8
    pool = []
    for i in range(10):
        tti = i + 1
        pls = [rng.integers(0, 256, C3_TBS // 8, dtype=np.uint8) for _ in range(2)]
        x, nre = SY.pdsch_subframe(100, cell_id, 2, tti, 1, rnti, C3_TBS, C3_QM, 0, pls, snr_db=30, rng=rng)
        pool.append((tti, x, nre, pls))
    host = np.stack([pool[b % 10][1] for b in range(nsf)])
    U.use_standard_symbol_size(True)
    ue = U.UeDl(U.cell(100, 2, cell_id), 2)
    ue.cfg.cfg.pdsch.max_nof_iterations = iters
    sbs = [[S.SoftbufferRx(nof_prb=100) for _ in range(2)] for _ in range(nsf)]
    cfgs = [U.pdsch_cfg(100, pool[b % 10][2], (C3_TBS, C3_TBS), (C3_QM, C3_QM), rnti=rnti, max_iterations=iters,
                        softbuffers=sbs[b]) for b in range(nsf)]
    d_pl = torch.zeros((nsf, 2, C3_TBS // 8 + 64), dtype=torch.uint8, device=dev)
    d_res = torch.zeros(2 * nsf, dtype=torch.int32, device=dev)
    d_avg = torch.zeros(2 * nsf, dtype=torch.float32, device=dev)
    arr = U.UeDl.batch_entries([(pool[b % 10][0], 1, cfgs[b], [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1])
                                for b in range(nsf)])
    h_x = torch.from_numpy(np.ascontiguousarray(host).view(np.float32)).pin_memory()
    d_xs = [torch.empty(h_x.shape, dtype=torch.float32, device=dev) for _ in range(2)]
    d_xs[0].copy_(h_x)
    d_xs[1].copy_(h_x)
    stream = torch.cuda.current_stream(dev)
    cs = torch.cuda.Stream(dev)
    print(json.dumps({"compute_stream": int(stream.cuda_stream), "copy_stream": int(cs.cuda_stream)}), flush=True)

    cur = [stream]

    def step(ptr):
        if ue.gpu_decode_batch(arr, ptr, d_res.data_ptr(), d_avg.data_ptr(), 0.0, cur[0].cuda_stream) != 2 * nsf:
            raise RuntimeError("decode failed")

    n = 20
    for _ in range(3):
        step(d_xs[0].data_ptr())
    torch.cuda.synchronize()

    def timeit(name, body):
        torch.cuda.synchronize()
        t_enq = [0.0, 0.0]
        t0 = time.perf_counter()
        body(t_enq)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"variant": name, "ms_per_iter": round((t2 - t0) / n * 1e3, 4),
                          "host_loop_ms_per_iter": round((t1 - t0) / n * 1e3, 4),
                          "copy_enqueue_ms": round(t_enq[0] / n * 1e3, 4), "step_enqueue_ms": round(t_enq[1] / n * 1e3, 4),
                          "sf_per_s": round(nsf * n / (t2 - t0), 1)}), flush=True)

    def steps_only(t):
        for i in range(n):
            a = time.perf_counter()
            step(d_xs[i % 2].data_ptr())
            t[1] += time.perf_counter() - a

    def copies_only(t):
        for i in range(n):
            a = time.perf_counter()
            with torch.cuda.stream(cs):
                d_xs[i % 2].copy_(h_x, non_blocking=True)
            t[0] += time.perf_counter() - a

    def serial(t):
        for i in range(n):
            a = time.perf_counter()
            d_xs[0].copy_(h_x, non_blocking=True)
            b = time.perf_counter()
            step(d_xs[0].data_ptr())
            t[0] += b - a
            t[1] += time.perf_counter() - b

    def overlapped(t):
        copied = [torch.cuda.Event(), torch.cuda.Event()]
        used = [torch.cuda.Event(), torch.cuda.Event()]
        with torch.cuda.stream(cs):
            d_xs[0].copy_(h_x, non_blocking=True)
        copied[0].record(cs)
        for i in range(n):
            b = i % 2
            a = time.perf_counter()
            if i + 1 < n:
                nb = (i + 1) % 2
                if i >= 1:
                    cs.wait_event(used[nb])
                with torch.cuda.stream(cs):
                    d_xs[nb].copy_(h_x, non_blocking=True)
                copied[nb].record(cs)
            c = time.perf_counter()
            cur[0].wait_event(copied[b])
            step(d_xs[b].data_ptr())
            used[b].record(cur[0])
            t[0] += c - a
            t[1] += time.perf_counter() - c

    def overlapped_nowait(t):  # the copies do not wait for the decode that reads the other buffer (timing only)
        copied = [torch.cuda.Event(), torch.cuda.Event()]
        for i in range(n):
            b = i % 2
            a = time.perf_counter()
            with torch.cuda.stream(cs):
                d_xs[b].copy_(h_x, non_blocking=True)
            copied[b].record(cs)
            c = time.perf_counter()
            cur[0].wait_event(copied[b])
            step(d_xs[b].data_ptr())
            t[0] += c - a
            t[1] += time.perf_counter() - c

    for name, body in (("steps_only", steps_only), ("copies_only", copies_only), ("serial_same_stream", serial),
                       ("overlapped", overlapped), ("overlapped_nowait", overlapped_nowait)):
        timeit(name, body)
    cur[0] = torch.cuda.Stream(dev)  # the same loops with the decode on a created stream
    for name, body in (("steps_only_created_stream", steps_only), ("overlapped_created_stream", overlapped)):
        timeit(name, body)

    # bench.py's loop as it runs there: both streams created after the decodes above, events reused,
    # an untimed warm pass; then the same with the copy's wait done on the host instead of the GPU
    cs2 = torch.cuda.Stream(dev, priority=-1)
    ks2 = torch.cuda.Stream(dev)
    cp2 = [torch.cuda.Event(), torch.cuda.Event()]
    us2 = [torch.cuda.Event(), torch.cuda.Event()]

    def bench_loop(m, host_wait):
        with torch.cuda.stream(cs2):
            d_xs[0].copy_(h_x, non_blocking=True)
        cp2[0].record(cs2)
        for i in range(m):
            b = i % 2
            if i + 1 < m:
                nb = (i + 1) % 2
                if i >= 1:
                    if host_wait:
                        us2[nb].synchronize()
                    else:
                        cs2.wait_event(us2[nb])
                with torch.cuda.stream(cs2):
                    d_xs[nb].copy_(h_x, non_blocking=True)
                cp2[nb].record(cs2)
            ks2.wait_event(cp2[b])
            if ue.gpu_decode_batch(arr, d_xs[b].data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0,
                                   ks2.cuda_stream) != 2 * nsf:
                raise RuntimeError("decode failed")
            us2[b].record(ks2)

    for name, hw in (("bench_like", False), ("bench_like_host_wait", True)):
        bench_loop(4, hw)
        torch.cuda.synchronize()
        timeit(name, lambda t, hw=hw: bench_loop(n, hw))


if __name__ == "__main__":
    main()
