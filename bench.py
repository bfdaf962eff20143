#!/usr/bin/env python3
"""Benchmark: turbo-decoded info Mbps on MI355X (BASELINE.json metric, turbo part).

A "step" is one pass of the hot path over one batch of synthetic input:
  workload "all188" (default, BASELINE configs[1]): 1024 code blocks of EACH of the
      188 LTE sizes, 8 half-iterations, rm_turbo sub-block input layout;
  workload "k6144" (BASELINE configs[0] shape on the GPU): 1024 x 6144-bit blocks.
Inputs are AWGN code blocks (turbodecoder_test.c convention) resident in HBM before
the timed region; every launch decodes the full batch (no early stop, no caching).

Multi-GPU: one process per GPU (torch.distributed.run); every rank decodes its own
batch (units partition with no data-path collective, "weak" scaling); the only
collectives are the timing barrier and the max-over-ranks of the elapsed time.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "turbo-decoded info Mbps + PDSCH subframes/s, 20 MHz 64QAM, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algo_bytes(K):
    """Algorithmic HBM bytes per code block: int16 LLRs in + K/8 bytes out."""
    return (3 * K + 12) * 2 + K // 8


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=["all188", "k6144", "dlsch"], default="all188")
    p.add_argument("--subframes", type=int, default=64, help="dlsch: subframes (2 TBs each) per step")
    p.add_argument("--sigma", type=float, default=0.42, help="dlsch: AWGN std on +-1 symbols before LLR scaling")
    p.add_argument("--batch", type=int, default=1024, help="code blocks per size per step")
    p.add_argument("--iters", type=int, default=8, help="half-iterations (srsran nof_iterations)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--pool", type=int, default=8, help="distinct AWGN code blocks per size")
    return p.parse_args()


def make_inputs(ora, Ks, pool, batch, rng, torch, device):
    """Per size: `pool` AWGN code blocks (Eb/No label 4 dB) in SB layout, tiled to `batch` rows on device."""
    from oracle import make_llrs

    data = {}
    for K in Ks:
        _, llr = make_llrs(K, 4.0, rng, pool, ora)
        sb = np.stack([ora.natural_to_sb(K, x) for x in llr])
        reps = (batch + pool - 1) // pool
        host = np.tile(sb, (reps, 1))[:batch]
        d_in = torch.from_numpy(np.ascontiguousarray(host)).to(device)
        d_out = torch.empty((batch, K // 8), dtype=torch.uint8, device=device)
        data[K] = (d_in, d_out, sb)
    return data


def cpu_baseline(Ks, data, iters, budget_s):
    """Reference decoder (oracle/_ref, compiled from /root/reference) on one host core.

    Bounded sample: repeated passes over the pool code blocks of the workload's
    sizes until ~budget_s seconds of CPU work; reports decoded info Mbps."""
    from oracle import Oracle, Reference, ref_available

    kind = "reference" if ref_available() else "port"
    dec = Reference() if kind == "reference" else Oracle()
    bits = 0
    n_cb = 0
    t0 = time.perf_counter()
    passes = 0
    while True:
        for K in Ks:
            sb = data[K][2]
            for x in sb:
                dec.tdec_run(K, x, True, iters)
                bits += K
                n_cb += 1
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {
        "value": round(bits / dt / 1e6, 3),
        "unit": "Mbps",
        "cores": 1,
        "kind": kind,
        "sample": f"{passes} pass(es) over {len(data[Ks[0]][2])} AWGN blocks of each of {len(Ks)} size(s), "
                  f"{n_cb} blocks, {iters} half-its, SB layout, {dt:.1f} s on 1 thread",
    }


# C3 grant (srsran_ra_dl_dci_to_grant probe): 100 PRB, TM3 2 CW, MCS28 64QAM, cfi 1
C3_TBS, C3_QM, C3_BITS = 75376, 6, 86400


def run_dlsch(args, torch, dist, world, rank, device):
    """DL-SCH decode of C3 subframes: per step `subframes` x 2 TBs (TBS 75376, 13 x K=5824 CBs,
    86400 LLRs each), new transmissions, CRC early stop, at most `iters` half-iterations.
    Value = decoded TB info bits / s (PDSCH Mbps at the DL-SCH stage) and subframes/s."""
    from oracle import Oracle
    from srsran_4g_amd import sch as S

    ora = Oracle()
    rng = np.random.default_rng(0x5EED + rank)
    ntb = 2 * args.subframes
    pool = []
    for _ in range(args.pool):
        tb = rng.integers(0, 256, C3_TBS // 8, dtype=np.uint8)
        e = ora.dlsch_encode(C3_TBS, C3_QM, 0, C3_BITS, tb).astype(np.float32) * 2 - 1
        y = e + rng.standard_normal(e.shape).astype(np.float32) * args.sigma
        pool.append(np.trunc(100 * y).astype(np.int16))
    host = np.stack([pool[i % args.pool] for i in range(ntb)])
    d_e = torch.from_numpy(host).to(device)
    d_data = torch.zeros((ntb, C3_TBS // 8 + 64), dtype=torch.uint8, device=device)
    d_res = torch.zeros(ntb, dtype=torch.int32, device=device)
    d_avg = torch.zeros(ntb, dtype=torch.float32, device=device)
    q = S.Sch()
    q.set_max_noi(args.iters)
    sbs = [S.SoftbufferRx(nof_prb=100) for _ in range(ntb)]
    entries = [(C3_TBS, C3_QM, 0, C3_BITS, d_e[i].data_ptr(), d_data[i].data_ptr(), sbs[i], 1) for i in range(ntb)]
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream

    def step():
        if q.decode_batch(entries, d_res.data_ptr(), d_avg.data_ptr(), sp) != 0:
            raise RuntimeError("srsran_dlsch_gpu_decode_batch failed")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = d_res.cpu().numpy()
    avg = d_avg.cpu().numpy()
    bits_per_step = ntb * C3_TBS
    value = world * bits_per_step * args.steps / elapsed / 1e6

    # whole-batch launch time on the stream (rm + turbo + TB kernels), outside the timed region
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    step()
    e1.record(stream)
    torch.cuda.synchronize()
    batch_ms = e0.elapsed_time(e1)
    # algorithmic bytes per TB: E LLRs in + soft buffer write (new data) and turbo read per
    # half-iteration is on-chip after the first read -> count E*2 + C*(3K+12)*2*2 + TBS/8 out
    algo = C3_BITS * 2 + 13 * (3 * 5824 + 12) * 2 * 2 + C3_TBS // 8
    achieved = ntb * algo / (batch_ms * 1e-3) / 1e9
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mbps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": f"synthetic: DL-SCH TBs (TBS {C3_TBS}, 64QAM bits as +-1, AWGN sigma {args.sigma}, LLR=trunc(100y)), "
                f"{args.pool} distinct TBs tiled to the batch, HBM-resident",
        "config": {
            "workload": f"dlsch C3 grant: {args.subframes} subframes x 2 TBs ({C3_TBS} bits, C=13 K=5824, "
                        f"E={C3_BITS}), new transmissions, CRC early stop, max {args.iters} half-its",
            "tbs_per_step_per_gpu": ntb,
            "subframes_per_s": round(world * args.subframes * args.steps / elapsed, 1),
            "tb_ok_fraction": round(float((res == 0).mean()), 4),
            "avg_half_iterations": round(float(avg.mean()), 3),
            "parallelism": f"tb-sharded x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "rm_rx_kernel + tdec_kernel<16,ES> + tb_kernel (whole batch)",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": None,
            "avg_launch_ms": round(batch_ms, 4),
            "algo_bytes_per_launch": int(ntb * algo),
        },
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from oracle import Reference, ref_available
        kind = "reference" if ref_available() else "port"
        dec = Reference() if kind == "reference" else ora
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            dec.dlsch_decode(C3_TBS, C3_QM, 0, pool[n % args.pool], args.iters)
            n += 1
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": round(n * C3_TBS / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": kind,
                                  "sample": f"{n} TBs of the same pool decoded (decode_tb loop over the reference's "
                                            f"rm_turbo/turbo/CRC code), {dt:.1f} s on 1 thread"}
    elif rank == 0:
        result["cpu_baseline"] = None
    for sb in sbs:
        sb.free()
    q.free()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from oracle import Oracle
    from srsran_4g_amd import tdec

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl", init_method="env://")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if not tdec.gpu_available():
        raise RuntimeError("bench: HIP device not visible to libsrsran_4g_amd")
    if args.workload == "dlsch":
        return run_dlsch(args, torch, dist, world, rank, device)

    Ks = list(tdec.CB_SIZES) if args.workload == "all188" else [6144]
    ora = Oracle()
    rng = np.random.default_rng(0x5EED + rank)
    data = make_inputs(ora, Ks, args.pool, args.batch, rng, torch, device)
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream

    groups = (list(Ks), [data[K][0].data_ptr() for K in Ks], [data[K][0].shape[1] for K in Ks],
              [data[K][1].data_ptr() for K in Ks], [args.batch] * len(Ks))

    def step(events=None):
        if events is None and len(Ks) > 1:
            # one multi-size call: groups fan out over internal streams, joined back into `stream`
            tdec.gpu_run_multi(groups[0], groups[1], groups[2], True, groups[3], groups[4], args.iters, sp)
            return
        for K in Ks:
            d_in, d_out, _ = data[K]
            if events is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            tdec.gpu_run_batch(K, d_in.data_ptr(), d_in.shape[1], True, d_out.data_ptr(), args.batch, args.iters, sp)
            if events is not None:
                e1.record(stream)
                events.append((K, e0, e1))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- timed region: exactly `steps` steps, barrier + sync on both sides ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    bits_per_step = args.batch * sum(Ks)
    value = world * bits_per_step * args.steps / elapsed / 1e6

    # ---- per-launch kernel durations (HIP events on the launch stream), outside the timed region ----
    events = []
    for _ in range(max(1, min(args.steps, 3))):
        step(events)
    torch.cuda.synchronize()
    per_kernel = {}
    for K, e0, e1 in events:
        name = tdec.load_library().srsran_tdec_gpu_kernel_name(K).decode()
        ms = e0.elapsed_time(e1)
        d = per_kernel.setdefault(name, {"launches": 0, "ms": 0.0, "bytes": 0, "bits": 0})
        d["launches"] += 1
        d["ms"] += ms
        d["bytes"] += args.batch * algo_bytes(K)
        d["bits"] += args.batch * K
    dom = max(per_kernel, key=lambda n: per_kernel[n]["ms"])
    dk = per_kernel[dom]
    avg_ms = dk["ms"] / dk["launches"]
    bytes_per_launch = dk["bytes"] / dk["launches"]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            traffic = json.load(open(tf)).get(args.workload, {}).get(dom)
        except Exception:
            traffic = None

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mbps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic: AWGN turbo code blocks (Eb/No label 4 dB, turbodecoder_test.c convention), "
                f"{args.pool} distinct blocks per size tiled to the batch, HBM-resident",
        "config": {
            "workload": ("tdec all 188 LTE CB sizes x %d CBs, %d half-its, rm_turbo SB layout" % (args.batch, args.iters))
            if args.workload == "all188" else ("tdec K=6144 x %d CBs, %d half-its, rm_turbo SB layout" % (args.batch, args.iters)),
            "cbs_per_size": args.batch,
            "cb_sizes": len(Ks),
            "half_iterations": args.iters,
            "info_bits_per_step_per_gpu": bits_per_step,
            "parallelism": f"cb-sharded x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "avg_launch_ms": round(avg_ms, 4),
            "algo_bytes_per_launch": int(bytes_per_launch),
        },
        "per_kernel_mbps": {n: round(d["bits"] / (d["ms"] * 1e-3) / 1e6, 1) for n, d in per_kernel.items()},
    }
    if args.workload == "all188":
        k = [e for e in events if e[0] == 6144]
        if k:
            ms = np.mean([e0.elapsed_time(e1) for _, e0, e1 in k])
            result["k6144_mbps"] = round(args.batch * 6144 / (ms * 1e-3) / 1e6, 1)

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(Ks if args.workload == "k6144" else Ks, data, args.iters,
                                              args.cpu_seconds)
    elif rank == 0:
        result["cpu_baseline"] = None

    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
