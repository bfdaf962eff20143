#!/usr/bin/env python3
"""Benchmark: turbo-decoded info Mbps on MI355X (BASELINE.json metric, turbo part).

A "step" is one pass of the hot path over one batch of synthetic input:
  workload "all188" (default, BASELINE configs[1]): 1024 code blocks of EACH of the
      188 LTE sizes, 8 half-iterations, rm_turbo sub-block input layout;
  workload "k6144" (BASELINE configs[0] shape on the GPU): 1024 x 6144-bit blocks;
  workload "dlsch": srsran_dlsch_decode of C3 transport blocks (rate dematch + turbo + CRC);
  workload "ulsch": the same TBs as PUSCH data through srsran_ulsch_gpu_decode_batch (channel
      de-interleaver + decode_tb; SURVEY 8f rank 1, data part);
  workload "pusch": the eNB PUSCH chain from the received subframe grid -- DMRS channel estimation,
      equalisation + SC-FDMA inverse DFT, demap/descramble, UL-SCH decode;
  workload "dlenc": the eNB DL-SCH transmit side: TB CRC, segmentation, turbo
      encoding and rate matching of C3 transport blocks through srsran_dlsch_gpu_encode_batch;
  workload "pdsch" (BASELINE configs[2], C3): the whole UE DL chain from time-domain samples --
      OFDM, CRS channel estimation, MMSE predecoding, demap/descramble/CSI, DL-SCH decode;
  workload "ldpc" (BASELINE configs[4]): NR LDPC decode (srsran_ldpc_decoder, 8-bit layered
      min-sum, AVX2 arithmetic) of a batch of BG1 / Z=384 codewords, 10 iterations;
  workload "nrsch" (configs[4] with its callers): srsran_dlsch_nr_decode of full-carrier NR TBs
      (273 PRB, 256QAM, R 948/1024: LDPC rate de-matching + LDPC with CRC early stop + TB CRC).
Inputs come from the synthetic eNB transmitter (synth/, not the oracle) and are resident in
HBM before the timed region; every step decodes the full batch (no caching).

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
# VALU ceilings (MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, a wave64 VALU instruction issues over 2 cycles,
# 2.4 GHz): wave-instruction issue rate, and packed-int16 lane operations (v_pk_*_i16: 2 per lane)
VALU_ISSUE_PEAK = 256 * 4 * 0.5 * 2.4e9          # 1.229e12 wave-instructions / s
# the same measured on this hardware for the decoder's instruction forms (tools/valu_issue.hip,
# profiles/r03_valu_issue.jsonl: v_pk_add_i16 clamp / v_perm_b32 at 3.45-3.5 cycles a SIMD with two
# waves, 5.0-5.1 cycles for one wave alone)
VALU_ISSUE_MEASURED = 256 * 4 / 3.5 * 2.4e9       # 7.02e11 wave-instructions / s, two waves a SIMD
VALU_PK16_PEAK = 256 * 4 * 32 * 2 * 2.4e9        # 1.573e14 int16 operations / s
TDEC_OPS_PER_BIT_HALF_IT = 86                    # max-log-MAP alpha + beta + LLR, turbodecoder_win.h


def pmc_entry(workload, kernel):
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return json.load(open(tf)).get(workload, {}).get(kernel)
    except Exception:
        return None


def pmc_traffic(workload, kernel, units):
    """HBM bytes per launch of `kernel` from profiles/pmc_traffic.json, scaled to `units` code blocks."""
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        e = json.load(open(tf)).get(workload, {}).get(kernel)
    except Exception:
        return None
    if not e:
        return None
    return int(round(e["bytes"] * units / e["units"]))


def trace_traffic(roof, workload):
    """roofline.traffic_source: the PMC summary the traffic figure of roof["kernel"] comes from"""
    if not isinstance(roof, dict) or "traffic" not in roof:
        return
    e = pmc_entry(workload, roof.get("kernel"))
    roof["traffic_source"] = e.get("source") if e and roof.get("traffic") is not None else None


def emit_line(result, workload):
    trace_traffic(result.get("roofline"), workload)
    for key in ("pdsch", "pusch"):
        sub = result.get(key)
        if isinstance(sub, dict):
            trace_traffic(sub.get("roofline"), key)
            for k, fe in (sub.get("front_end_roofline") or {}).items():
                fe.setdefault("kernel", k)
                trace_traffic(fe, key)
    for k, fe in (result.get("front_end_roofline") or {}).items():
        fe.setdefault("kernel", k)
        trace_traffic(fe, workload)
    print(json.dumps(result), flush=True)


def shard(rank):
    """Per-rank unit of work (independent carriers / CB batches, no data-path collective):
    rank r decodes its own carrier (cell id 1 + r) from its own seeded synthetic inputs."""
    return {"cell_id": 1 + rank, "seed": 0x5EED + rank}


def timed_region(step, steps, warmup, world, dist, sync, device):
    """Warm up, then time exactly `steps` steps bracketed by barrier + device sync on both sides;
    returns the MAX elapsed seconds over ranks (one all_reduce of a scalar, the only collective)."""
    import gc

    import torch

    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    # the harness's Python garbage collector stays out of the timed steps (a collection pause of the calling
    # thread is a property of this script, not of the library, which a C caller such as srsUE does not have)
    gc_was = gc.isenabled()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if gc_was:
        gc.enable()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def timed_region_n(run_n, steps, warmup, world, dist, sync, device):
    """timed_region for callers that run their steps themselves (run_n(n): n steps, e.g. several host threads each
    taking n batches): the same warm-up, barriers, device syncs and max over ranks"""
    import gc

    import torch

    run_n(warmup)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    gc_was = gc.isenabled()
    gc.disable()
    t0 = time.perf_counter()
    run_n(steps)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if gc_was:
        gc.enable()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def step_spread(step, n, torch, stream, host_phases=None, stream_of=None):
    """Per-step spread of `n` back-to-back steps (after the timed region, the same launch pattern): the
    GPU time between HIP events recorded after every step, the host time of every enqueue call, and -- when
    `host_phases` (srsran_4g_amd.prof) is given -- the library's host phases of the slowest call.  With
    `stream_of` (the stream the step just enqueued went to: several workers taking the steps in turn) each event
    goes on that step's stream, so an interval is the time between two consecutive steps' completions (in
    completion order: steps on different streams can finish out of order) -- what the timed region's rate is made
    of.  -> {"gpu_ms": min/median/max, "host_ms": min/median/max, ...}"""
    import gc

    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    host, phases = [], []
    gc_was = gc.isenabled()
    gc.disable()
    # untimed steps first (two, or one a worker), so that the first timed interval starts with work queued behind
    # it (an event recorded on an idle stream would time the host's first enqueue as GPU time)
    for _ in range(2 if stream_of is None else 3):
        step()
    ev[0].record(stream if stream_of is None else stream_of())
    for i in range(n):
        if host_phases is not None:
            host_phases.host_enable(True)
        t = time.perf_counter()
        step()
        host.append((time.perf_counter() - t) * 1e3)
        if host_phases is not None:
            phases.append({k: round(us, 1) for k, (us, _) in host_phases.host_read().items()})
            host_phases.host_enable(False)
        ev[i + 1].record(stream if stream_of is None else stream_of())
    torch.cuda.synchronize()
    if gc_was:
        gc.enable()
    if stream_of is None:
        gpu = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    else:
        # the workers' steps can complete out of order (a step on one stream before the previous one on another):
        # the intervals between consecutive completions, in completion order
        t = sorted([0.0] + [ev[0].elapsed_time(ev[i + 1]) for i in range(n)])
        gpu = [t[i + 1] - t[i] for i in range(n)]

    def mmm(v):
        return {"min": round(min(v), 4), "median": round(float(np.median(v)), 4), "max": round(max(v), 4)}
    out = {"steps": n, "gpu_ms": mmm(gpu), "host_ms": mmm(host),
           "max_over_median": round(max(gpu) / float(np.median(gpu)), 3)}
    if phases:
        out["host_phases_us_slowest_call"] = phases[int(np.argmax(host))]
    return out


def algo_bytes(K):
    """Algorithmic HBM bytes per code block: int16 LLRs in + K/8 bytes out."""
    return (3 * K + 12) * 2 + K // 8


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs of this node, one rank each (default: WORLD_SIZE under a launcher, else 1); without a "
                        "launcher N > 1 starts the N ranks itself")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=["all188", "k6144", "dlsch", "ulsch", "pusch", "dlenc", "pdsch", "dlloop", "ldpc",
                                          "nrsch"],
                   default="all188")
    p.add_argument("--snr", type=float, default=30.0, help="pdsch: AWGN SNR (dB) of the synthetic subframes")
    p.add_argument("--nfft", type=int, default=2048, choices=[2048, 1536],
                   help="pdsch: OFDM size of the 100-PRB carrier (2048: standard rate, C3; 1536: the reference default)")
    p.add_argument("--subframes", type=int, default=78,
                   help="dlsch / pdsch: subframes (2 TBs each) per step; 78 x 26 CBs = two full turbo-decoder rounds")
    p.add_argument("--sigma", type=float, default=0.42, help="dlsch: AWGN std on +-1 symbols before LLR scaling")
    p.add_argument("--batch", type=int, default=1024, help="code blocks per size per step")
    p.add_argument("--iters", type=int, default=8, help="half-iterations (srsran nof_iterations)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--pool", type=int, default=8, help="distinct AWGN code blocks per size")
    p.add_argument("--bg", type=int, default=1, choices=[1, 2], help="ldpc: base graph")
    p.add_argument("--ls", type=int, default=384, help="ldpc: lifting size")
    p.add_argument("--codewords", type=int, default=4096, help="ldpc: codewords per step")
    p.add_argument("--ldpc-iters", type=int, default=10, help="ldpc: iterations (srsran max_nof_iter)")
    p.add_argument("--ldpc-snr", type=float, default=1.5, help="ldpc: BPSK Es/N0 (dB) of the synthetic codewords")
    p.add_argument("--nr-tbs", type=int, default=64, help="nrsch: transport blocks per step")
    p.add_argument("--nr-snr", type=float, default=12.0, help="nrsch: Es/N0 (dB) of the bits as +-1 before int8 LLRs")
    p.add_argument("--pdsch-probe", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--pusch-workers", type=int, default=2,
                   help="pusch: PUSCH objects on host threads of their own, each taking every timed step's batch "
                        "(srsENB's PHY workers, enb.conf nof_phy_threads); a step = one batch on each.  Default 2: "
                        "1 / 2 / 3 / 4 workers 253 k / 447 k / 425 k / 437 k UE-subframes/s (r06ao, r06au: the GPU is "
                        "the bound from two)")
    p.add_argument("--pdsch-workers", type=int, default=4,
                   help="pdsch: UE DL objects, each on its own stream, taking the timed batches in turn (srsUE's PHY "
                        "workers, phy.nof_phy_threads, srsue/src/main.cc:313-314: srsUE's default 3).  Default 4: with "
                        "a hardware queue a worker, 439 k against 424 k subframes/s for 3 (r06bb, alternated in one "
                        "process); 6 workers 415 k (r06ba)")
    p.add_argument("--worker-queues", choices=("own", "shared"), default="own",
                   help="pdsch: the workers' streams from srsran_gpu_worker_stream_create, a hardware queue each "
                        "(own), or ordinary streams on HIP's shared hardware queues (shared)")
    p.add_argument("--pdsch-steps", type=int, default=20,
                   help="all188: timed steps of the C3 PDSCH chain reported in the same line (0 = skip)")
    p.add_argument("--pdsch-cpu-seconds", type=float, default=4.0, help="all188: CPU baseline budget of the PDSCH part")
    p.add_argument("--pdsch-low-snr", type=float, default=17.0,
                   help="all188: SNR (dB) of a second, shorter PDSCH chain run at the operating point where the "
                        "turbo decoder needs ~5 half-iterations and ~10%% of TBs fail (0 = skip)")
    p.add_argument("--tdec16", choices=["auto", "single", "pair", "quad"], default="auto",
                   help="decoder of the 16-sub-block class: the library's choice by batch size, or forced")
    p.add_argument("--h2d-priority", type=int, default=0, choices=[0, -1],
                   help="pdsch: priority of the PCIe-loop copy stream (-1: high)")
    p.add_argument("--w8-max-k", type=int, default=-1,
                   help="srsran_tdec_gpu_set_w8_max_k (-1: the library default)")
    p.add_argument("--w8-fused-max-k", type=int, default=-1,
                   help="srsran_tdec_gpu_set_w8_fused_max_k (-1: the library default)")
    p.add_argument("--generic-single-min-cb", type=int, default=-1,
                   help="srsran_tdec_gpu_set_generic_single_threshold (-1: the library default, the quad decoder)")
    p.add_argument("--cpu-worker", type=int, default=None, help=argparse.SUPPRESS)
    p.add_argument("--dry-run", action="store_true",
                   help="launch path only (no GPU): ranks, devices and shards on a gloo group, one line")
    return p.parse_args()


def make_inputs(Ks, pool, batch, rng, torch, device):
    """Per size: `pool` AWGN code blocks (Eb/No label 4 dB) in SB layout, tiled to `batch` rows on device."""
    from synth import synth as SY

    data = {}
    for K in Ks:
        _, llr = SY.make_llrs(K, 4.0, rng, pool)
        sb = SY.natural_to_sb(K, llr)
        reps = (batch + pool - 1) // pool
        host = np.tile(sb, (reps, 1))[:batch]
        d_in = torch.from_numpy(np.ascontiguousarray(host)).to(device)
        d_out = torch.empty((batch, K // 8), dtype=torch.uint8, device=device)
        data[K] = (d_in, d_out, sb)
    return data


def cpu_threads():
    """Host threads of this job's CPU share: OMP_NUM_THREADS where the pool sets it (16 on the GPU
    box, whose nproc counts the whole machine), else the affinity mask."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, min(n or len(os.sched_getaffinity(0)), 16))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _tdec_decoder():
    from oracle import Oracle, Reference, ref_available
    kind = "reference" if ref_available() else "port"
    return kind, (Reference() if kind == "reference" else Oracle())


def cpu_worker(args):
    """--cpu-worker SEED: one host process of the all-cores CPU baseline (no torch, no GPU): decodes
    its own AWGN pool of every workload size with the reference decoder for --cpu-seconds."""
    from synth import synth as SY
    from srsran_4g_amd.tdec import CB_SIZES

    if args.workload == "pdsch":
        return pdsch_cpu_worker(args)
    Ks = list(CB_SIZES) if args.workload == "all188" else [6144]
    rng = np.random.default_rng(args.cpu_worker)
    pool = {K: SY.natural_to_sb(K, SY.make_llrs(K, 4.0, rng, args.pool)[1]) for K in Ks}
    _, dec = _tdec_decoder()
    bits = n_cb = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        for K in Ks:
            for x in pool[K]:
                dec.tdec_run(K, x, True, args.iters)
                bits += K
                n_cb += 1
    print(json.dumps({"bits": bits, "blocks": n_cb, "dt": time.perf_counter() - t0}), flush=True)


def bench_8bit(torch, device, n, K=6144, iters=8, reps=3):
    """The 8-bit LLR decoder (srsran_tdec_gpu_run_batch_8bit, the reference's AVX2 8-bit window decoder
    restated) on the C1 shape: n x K = 6144 int8 code blocks (SB layout, 32 sub-blocks), 8 half-its.
    Random LLRs: the decoder runs every half-iteration whatever the values (no early stop)."""
    from srsran_4g_amd import tdec
    L = 3 * (K + 32) + 12
    g = torch.Generator(device=device).manual_seed(8)
    x = torch.randint(-100, 100, (n, L), dtype=torch.int8, device=device, generator=g)
    out = torch.zeros((n, K // 8), dtype=torch.uint8, device=device)
    st = torch.cuda.current_stream()
    tdec.gpu_run_batch_8bit(K, x.data_ptr(), L, True, out.data_ptr(), n, iters, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        tdec.gpu_run_batch_8bit(K, x.data_ptr(), L, True, out.data_ptr(), n, iters, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"workload": f"K={K} x {n}, {iters} half-its, int8 LLRs (srsran_tdec_gpu_run_batch_8bit)",
            "kernel": tdec.last_kernel(), "ms_per_launch": round(ms, 4),
            "mbps": round(n * K / (ms * 1e-3) / 1e6, 1)}


def c1_cpu_leg(data, iters, budget_s, gpu_mbps, gpu_mbps_16=None):
    """BASELINE configs[0] (C1: K = 6144 code blocks, 8 half-its) on the host, beside the GPU's K = 6144 rate of the
    same line: the reference decoder (oracle/_ref) on one thread for ~budget_s/2 s over the pool blocks, and one
    process per core of this job's share for ~budget_s/2 s (cpu_worker, K = 6144 only).  The whole host is not this
    job's to use (nproc counts every hardware thread of the machine): its figure is the one-thread rate times nproc,
    a linear extrapolation and an upper bound."""
    import subprocess

    kind, dec = _tdec_decoder()
    pool = data[6144][2]
    half = budget_s / 2
    bits = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < half:
        for x in pool:
            dec.tdec_run(6144, x, True, iters)
            bits += 6144
    one = bits / (time.perf_counter() - t0) / 1e6
    bits16 = 0  # 16 half-iterations on one thread, a quarter of the budget
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s / 4:
        for x in pool:
            dec.tdec_run(6144, x, True, 16)
            bits16 += 6144
    one16 = bits16 / (time.perf_counter() - t0) / 1e6
    n = cpu_threads()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", str(2000 + i),
                               "--cpu-seconds", str(half), "--iters", str(iters), "--workload", "k6144"],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env, cwd=ROOT) for i in range(n)]
    agg_bits, agg_dt, ok = 0, 0.0, 0
    for p in procs:
        try:
            out, _ = p.communicate(timeout=half + 120)
            r = json.loads(out.decode().strip().splitlines()[-1])
            agg_bits, agg_dt, ok = agg_bits + r["bits"], max(agg_dt, r["dt"]), ok + 1
        except Exception:
            p.kill()
    share = agg_bits / agg_dt / 1e6 if ok else None
    host = one * (os.cpu_count() or 1)
    return {
        "workload": f"K=6144, {iters} half-its, SB layout (BASELINE configs[0])",
        "kind": kind, "cpu_model": cpu_model(), "unit": "Mbps",
        "gpu_k6144_mbps": gpu_mbps,
        "cpu_1thread_mbps": round(one, 2),
        "cpu_share_mbps": round(share, 2) if share else None, "cpu_share_processes": ok,
        "cpu_host_estimate_mbps": round(host, 1), "nproc": os.cpu_count(),
        "gpu_over_1thread": round(gpu_mbps / one, 1) if gpu_mbps else None,
        "gpu_over_share": round(gpu_mbps / share, 2) if gpu_mbps and share else None,
        "gpu_over_host_estimate": round(gpu_mbps / host, 2) if gpu_mbps else None,
        "gpu_k6144_mbps_16_half_its": gpu_mbps_16,
        "cpu_1thread_mbps_16_half_its": round(one16, 2),
        "gpu_over_1thread_16_half_its": round(gpu_mbps_16 / one16, 1) if gpu_mbps_16 else None,
        "gpu_over_share_16_half_its_est": round(gpu_mbps_16 / (share * one16 / one), 2) if gpu_mbps_16 and share else None,
        "sample": f"1 thread {half:.0f} s over {len(pool)} pool blocks; {ok} processes x {half:.0f} s over their own "
                  f"pools; host = 1 thread x nproc (linear extrapolation, SMT threads counted: an upper bound); "
                  f"16 half-its: 1 thread {budget_s / 4:.0f} s, the share scaled by the 1-thread 16 / 8 ratio",
    }


def cpu_baseline(Ks, data, iters, budget_s, workload):
    """Reference decoder (oracle/_ref, compiled from /root/reference) on the host cores of this job.

    Bounded samples: (1) one thread in this process, repeated passes over the pool code blocks of
    the workload's sizes for ~budget_s/2 s; (2) the all-cores aggregate: one child process per core (started
    as children, no exec of this GPU process), each decoding its own pool for ~budget_s/2 s.
    `value` is the aggregate; decoded info Mbps."""
    import subprocess

    kind, dec = _tdec_decoder()
    bits = n_cb = passes = 0
    half = budget_s / 2
    t0 = time.perf_counter()
    while True:
        for K in Ks:
            sb = data[K][2]
            for i, x in enumerate(sb):
                dec.tdec_run(K, x, True, iters)
                bits += K
                n_cb += 1
        passes += 1
        if time.perf_counter() - t0 >= half:
            break
    dt = time.perf_counter() - t0
    one = bits / dt / 1e6
    n = cpu_threads()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", str(1000 + i),
                               "--cpu-seconds", str(half), "--iters", str(iters), "--workload", workload],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env, cwd=ROOT) for i in range(n)]
    agg_bits, agg_dt, ok = 0, 0.0, 0
    for p in procs:
        try:
            out, _ = p.communicate(timeout=half + 120)
            r = json.loads(out.decode().strip().splitlines()[-1])
            agg_bits += r["bits"]
            agg_dt = max(agg_dt, r["dt"])
            ok += 1
        except Exception:
            p.kill()
    agg = agg_bits / agg_dt / 1e6 if ok else None
    res = {
        "value": round(agg, 3) if agg else round(one, 3),
        "unit": "Mbps",
        "cores": ok if agg else 1,
        "kind": kind,
        "cpu_model": cpu_model(),
        "nproc": os.cpu_count(),
        "value_1thread": round(one, 3),
        "sample": f"all-cores: {ok} processes x {half:.0f} s, each over its own {len(data[Ks[0]][2])} AWGN blocks of "
                  f"each of {len(Ks)} size(s); 1 thread: {passes} pass(es), {n_cb} blocks, {dt:.1f} s; "
                  f"{iters} half-its, SB layout",
    }
    return res


def ref_outputs(Ks, data, iters):
    """The reference decoder's output for every distinct pool block of every size (the timed batch
    tiles these blocks), for the post-timing check of the GPU batch."""
    _, dec = _tdec_decoder()
    return {K: np.stack([dec.tdec_run(K, x, True, iters) for x in data[K][2]]) for K in Ks}


# C3 grant (srsran_ra_dl_dci_to_grant probe): 100 PRB, TM3 2 CW, MCS28 64QAM, cfi 1
C3_TBS, C3_QM, C3_BITS = 75376, 6, 86400
UL_NSYMB = 12  # ulsch workload: N_symb^PUSCH of a normal-CP subframe without SRS


def run_dlsch(args, torch, dist, world, rank, device):
    """DL-SCH decode of C3 subframes: per step `subframes` x 2 TBs (TBS 75376, 13 x K=5824 CBs,
    86400 LLRs each), new transmissions, CRC early stop, at most `iters` half-iterations.
    Value = decoded TB info bits / s (PDSCH Mbps at the DL-SCH stage) and subframes/s."""
    from synth import synth as SY
    from srsran_4g_amd import sch as S

    rng = np.random.default_rng(shard(rank)["seed"])
    ntb = 2 * args.subframes
    pool = []
    for _ in range(args.pool):
        tb = rng.integers(0, 256, C3_TBS // 8, dtype=np.uint8)
        e = SY.dlsch_encode(C3_TBS, C3_QM, 0, C3_BITS, tb).astype(np.float32) * 2 - 1
        y = e + rng.standard_normal(e.shape).astype(np.float32) * args.sigma
        pool.append(np.trunc(100 * y).astype(np.int16))
    uplink = args.workload == "ulsch"  # the same grant as a PUSCH: 100 PRB x 12 SC-FDMA symbols x 64QAM
    if uplink:
        from synth.ulsch_tx import ulsch_interleave
        host = np.stack([ulsch_interleave(pool[i % args.pool], C3_QM, UL_NSYMB) for i in range(ntb)])
    else:
        host = np.stack([pool[i % args.pool] for i in range(ntb)])
    d_e = torch.from_numpy(host).to(device)
    d_g = torch.zeros_like(d_e) if uplink else None
    d_data = torch.zeros((ntb, C3_TBS // 8 + 64), dtype=torch.uint8, device=device)
    d_res = torch.zeros(ntb, dtype=torch.int32, device=device)
    d_avg = torch.zeros(ntb, dtype=torch.float32, device=device)
    q = S.Sch()
    q.set_max_noi(args.iters)
    sbs = [S.SoftbufferRx(nof_prb=100) for _ in range(ntb)]
    if uplink:
        entries = [(C3_TBS, C3_QM, 0, C3_BITS, UL_NSYMB, d_e[i].data_ptr(), d_g[i].data_ptr(), d_data[i].data_ptr(),
                    sbs[i], 1) for i in range(ntb)]
    else:
        entries = [(C3_TBS, C3_QM, 0, C3_BITS, d_e[i].data_ptr(), d_data[i].data_ptr(), sbs[i], 1) for i in range(ntb)]
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream

    def step():
        if uplink:
            if q.ulsch_decode_batch(entries, d_res.data_ptr(), d_avg.data_ptr(), sp) != 0:
                raise RuntimeError("srsran_ulsch_gpu_decode_batch failed")
        elif q.decode_batch(entries, d_res.data_ptr(), d_avg.data_ptr(), sp) != 0:
            raise RuntimeError("srsran_dlsch_gpu_decode_batch failed")

    elapsed = timed_region(step, args.steps, args.warmup, world, dist, torch.cuda.synchronize, device)
    res = d_res.cpu().numpy()
    avg = d_avg.cpu().numpy()
    bits_per_step = ntb * C3_TBS
    value = world * bits_per_step * args.steps / elapsed / 1e6

    # per-stage kernel durations (library HIP events on the launch stream), outside the timed region
    from srsran_4g_amd import prof
    prof.enable(True)
    nrep = max(1, min(args.steps, 3))
    for _ in range(nrep):
        step()
    torch.cuda.synchronize()
    stages = prof.read()
    prof.enable(False)
    sb_ = stage_bytes(0, 0, ntb)
    per_stage = {}
    for name, (ms, n) in stages.items():
        lps = n / nrep
        per_stage[name] = {"ms_per_step": round(ms / nrep, 4), "launches_per_step": lps,
                           "avg_launch_ms": round(ms / n, 4),
                           "GBps": round(sb_.get(name, 0) / lps / (ms / n * 1e-3) / 1e9, 1)}
    dom = max(per_stage, key=lambda k: per_stage[k]["ms_per_step"])
    d = per_stage[dom]
    bytes_per_launch = sb_[dom] / d["launches_per_step"]
    achieved = bytes_per_launch / (d["avg_launch_ms"] * 1e-3) / 1e9
    if dom == "tdec_kernel":  # the turbo stage's kernel as it ran (srsran_tdec_gpu_last_kernel)
        from srsran_4g_amd import tdec as TD
        dom = TD.last_kernel()
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
            "workload": (f"ulsch: {ntb} PUSCH TBs (100 PRB x {UL_NSYMB} symbols, 64QAM: {C3_TBS} bits, C=13 K=5824, "
                         f"E={C3_BITS}; channel de-interleaver + decode_tb, no UCI)" if uplink else
                         f"dlsch C3 grant: {args.subframes} subframes x 2 TBs ({C3_TBS} bits, C=13 K=5824, "
                         f"E={C3_BITS})") + f", new transmissions, CRC early stop, max {args.iters} half-its",
            "tbs_per_step_per_gpu": ntb,
            "subframes_per_s": round(world * args.subframes * args.steps / elapsed, 1),
            "tb_ok_fraction": round(float((res == 0).mean()), 4),
            "avg_half_iterations": round(float(avg.mean()), 3),
            "parallelism": f"tb-sharded x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": pmc_traffic(args.workload, dom, ntb * 13),
            "avg_launch_ms": d["avg_launch_ms"],
            "algo_bytes_per_launch": int(bytes_per_launch),
        },
        "stages": per_stage,
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from oracle import Oracle, Reference, ref_available
        kind = "reference" if ref_available() else "port"
        dec = Reference() if kind == "reference" else Oracle()
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            dec.dlsch_decode(C3_TBS, C3_QM, 0, pool[n % args.pool], args.iters)
            n += 1
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": round(n * C3_TBS / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": kind,
                                  "sample": f"{n} TBs of the same pool decoded (decode_tb loop over the reference's "
                                            f"rm_turbo/turbo/CRC code), {dt:.1f} s on 1 thread"
                                            + ("; the UL channel de-interleaver (a permutation; sch.c is not "
                                               "buildable here) is not in the CPU timing" if uplink else "")}
    elif rank == 0:
        result["cpu_baseline"] = None
    for sb in sbs:
        sb.free()
    q.free()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit_line(result, args.workload)


C3_NRE = {0: 13992, 5: 14256}  # PDSCH REs of the C3 grant per subframe index (others: 14400)
SF_LEN = 30720                  # 20 MHz, N = 2048 (standard sampling rate)


def stage_bytes(nsf, nre_sum, ntb, sf_len=SF_LEN):
    """Algorithmic HBM bytes per launch of each stage kernel for nsf C3 subframes (2 rx, 2 ports):
    the inputs each kernel must read once and the outputs it must write once."""
    nrx, ports, nre_row = 2, 2, 1200
    K, C = 5824, 13
    return {
        "ofdm_rx_kernel": nsf * nrx * (sf_len + 14 * nre_row) * 8,
        "chest_kernel": nsf * ports * nrx * (4 * nre_row * 8 + nre_row * 8),
        "predecode_batch_kernel": nre_sum * (nrx * 8 + 4 + 2 * 8 + 2 * 4) + nsf * ports * nrx * nre_row * 8,
        "llr_batch_kernel": nre_sum * 2 * (8 + 4 + 6 * 2),
        "rm_rx_lds_kernel": ntb * (C3_BITS * 2 + C * (3 * (K + 32) + 12) * 2),
        "tdec_kernel": ntb * C * ((3 * (K + 32) + 12) * 2 + K // 8),
        "tb_kernel": ntb * (C * K // 8 + C3_TBS // 8),
    }


def pusch_stage_bytes(nue, M, nsymb, ncell_re):
    """Algorithmic HBM bytes per launch of the PUSCH kernels for nue UEs of M subcarriers: the chest
    reads 2M pilots + 2M DMRS values and writes the 2 x 7-symbol estimate rows; the equaliser reads
    the data REs and their estimates and writes the de-precoded symbols (all complex float)."""
    K, C = 5824, 13
    return {
        "chest_ul_kernel": nue * (4 * M * 8 + 14 * M * 8),
        "pusch_eq_idft_kernel": nue * 3 * nsymb * M * 8,
        "llr_batch_kernel": nue * nsymb * M * (8 + 6 * 2),
        "rm_rx_lds_kernel": nue * (C3_BITS * 2 + C * (3 * (K + 32) + 12) * 2),
        "tdec_kernel": nue * C * ((3 * (K + 32) + 12) * 2 + K // 8),
        "tb_kernel": nue * (C * K // 8 + C3_TBS // 8),
    }


def run_pusch(args, torch, dist, world, rank, device, steps=None, warmup=None, cpu_seconds=None, emit=True):
    """eNB PUSCH receive: per step `subframes` UEs, each a 100-PRB 64QAM PUSCH (TBS 75376, 12
    SC-FDMA symbols, normal CP) in its own received subframe grid (device-resident), through
    srsran_pusch_gpu_decode_batch: DMRS estimation, MMSE equalisation + 1200-point inverse DFT,
    demap/descramble, channel de-interleaver, rate de-matching, turbo decoding with CRC early stop.
    Value = decoded UL info Mbps; also UE-subframes/s.  emit=False: return the result (the default
    all188 line embeds a summary) instead of printing it."""
    import ctypes

    from synth import pusch_tx as PT
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    cpu_seconds = args.cpu_seconds if cpu_seconds is None else cpu_seconds
    from srsran_4g_amd import prof
    from srsran_4g_amd import pusch as P
    from srsran_4g_amd import sch as S
    from srsran_4g_amd.ue_dl import cell as make_cell

    rng = np.random.default_rng(shard(rank)["seed"])
    cell_id = shard(rank)["cell_id"]
    cell = make_cell(100, 1, cell_id)
    dm = P.srsran_refsignal_dmrs_pusch_cfg_t()
    dm.cyclic_shift, dm.delta_ss, dm.group_hopping_en = 1, 3, True
    rnti, L = 0x46, 100
    pool = []
    for i in range(args.pool):
        tti = i % 10
        g, pl = PT.subframe(cell, dm, 100, L, 0, C3_TBS, C3_QM, tti, rnti, rng, snr_db=args.snr)
        pool.append((tti, g, pl))
    nue = args.subframes
    host = np.stack([pool[b % args.pool][1] for b in range(nue)])
    d_grid = torch.from_numpy(np.ascontiguousarray(host).view(np.float32)).to(device)
    per_grid = host[0].size * 8

    def make_worker():
        """one eNB PHY worker's objects: its PUSCH and UL estimator objects, soft buffers and batch entries (over
        the shared, read-only device grids)"""
        ch = P.ChestUl(cell, dm)
        pu = P.Pusch(cell)
        sbs = [S.SoftbufferRx(nof_prb=100) for _ in range(nue)]
        cfgs, sfs = [], []
        for b in range(nue):
            cfg = S.srsran_pusch_cfg_t()
            cfg.rnti = rnti
            g = cfg.grant
            g.L_prb, g.nof_symb, g.nof_re = L, UL_NSYMB, L * 12 * UL_NSYMB
            g.tb.mod, g.tb.tbs, g.tb.rv, g.tb.nof_bits, g.tb.enabled = S.MOD_FROM_QM[C3_QM], C3_TBS, 0, C3_BITS, True
            cfg.enable_64qam = True
            cfg.max_nof_iterations = args.iters
            cfg.softbuffers.rx = ctypes.pointer(sbs[b].s)
            sf = P.srsran_ul_sf_cfg_t()
            sf.tti = pool[b % args.pool][0]
            cfgs.append(cfg)
            sfs.append(sf)
        arr = (P.srsran_pusch_gpu_ue_t * nue)()
        res = (P.srsran_pusch_res_t * nue)()
        cres = (P.srsran_chest_ul_res_t * nue)()
        datas = np.zeros((nue, C3_TBS // 8 + 64), np.uint8)
        for b in range(nue):
            arr[b].chest = ctypes.pointer(ch.q)
            arr[b].sf = ctypes.pointer(sfs[b])
            arr[b].cfg = ctypes.pointer(cfgs[b])
            arr[b].d_sf_symbols = d_grid.data_ptr() + b * per_grid
            arr[b].new_data = 1
            res[b].data = datas[b].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        return dict(ch=ch, pu=pu, sbs=sbs, cfgs=cfgs, sfs=sfs, arr=arr, res=res, cres=cres, datas=datas)

    # srsENB decodes uplink subframes on several PHY workers at once (enb.conf nof_phy_threads, default 3): `nwork`
    # host threads, each with its own objects, each taking `steps` batches -- one worker's host work (descriptors,
    # UCI, the synchronous result copy) overlaps another's GPU work.  A step = one batch on every worker.
    nwork = max(1, int(getattr(args, "pusch_workers", 1)))
    workers = [make_worker() for _ in range(nwork)]
    w0 = workers[0]
    pu, arr, res, cres, datas = w0["pu"], w0["arr"], w0["res"], w0["cres"], w0["datas"]
    L_ = P.lib()

    def batch(w):  # new transmissions: new_data = 1 (the soft buffers are reset in the decode launch)
        if L_.srsran_pusch_gpu_decode_batch(ctypes.byref(w["pu"].q), nue, w["arr"], w["cres"], w["res"]) != 0:
            raise RuntimeError("srsran_pusch_gpu_decode_batch failed")

    def step():
        batch(w0)

    def run_n(n):
        if nwork == 1:
            for _ in range(n):
                batch(w0)
            return
        import threading
        errs = []

        def loop(w):
            try:
                for _ in range(n):
                    batch(w)
            except Exception as e:  # surfaced on the main thread below
                errs.append(e)
        ths = [threading.Thread(target=loop, args=(w,)) for w in workers]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]

    elapsed = timed_region_n(run_n, steps, warmup, world, dist, torch.cuda.synchronize, device)
    ok = np.array([bool(w["res"][b].crc) and np.array_equal(w["datas"][b][:C3_TBS // 8], pool[b % args.pool][2])
                   for w in workers for b in range(nue)])
    avg = np.array([w["res"][b].avg_iterations_block for w in workers for b in range(nue)])
    value = world * nwork * nue * C3_TBS * steps / elapsed / 1e6

    prof.enable(True)
    nrep = max(1, min(steps, 3))
    for _ in range(nrep):
        step()
    torch.cuda.synchronize()
    stages = prof.read()
    prof.enable(False)
    sb_ = pusch_stage_bytes(nue, 12 * L, UL_NSYMB, 1200)
    per_stage = {}
    for name, (ms, n) in stages.items():
        lps = n / nrep
        per_stage[name] = {"ms_per_step": round(ms / nrep, 4), "launches_per_step": lps,
                           "avg_launch_ms": round(ms / n, 4),
                           "GBps": round(sb_.get(name, 0) / lps / (ms / n * 1e-3) / 1e9, 1)}
    dom = max(per_stage, key=lambda k: per_stage[k]["ms_per_step"])
    d = per_stage[dom]
    bytes_per_launch = sb_.get(dom, 0) / d["launches_per_step"]
    achieved = bytes_per_launch / (d["avg_launch_ms"] * 1e-3) / 1e9
    fe = [k for k in ("chest_ul_kernel", "pusch_eq_idft_kernel") if k in per_stage]
    if dom == "tdec_kernel":  # the turbo stage's kernel as it ran (srsran_tdec_gpu_last_kernel)
        from srsran_4g_amd import tdec as TD
        dom = TD.last_kernel()
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mbps",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 front end, int16 LLRs",
        "data": f"synthetic: {args.pool} distinct PUSCH subframes (3-tap frequency-selective channel, AWGN "
                f"{args.snr} dB) tiled to the batch, HBM-resident grids",
        "config": {
            "workload": f"pusch: {nue} UEs x (100 PRB, 64QAM, TBS {C3_TBS}, 12 SC-FDMA symbols, normal CP) per batch, "
                        f"{nwork} worker(s) a batch each per step, "
                        f"srsran_pusch_gpu_decode_batch, max {args.iters} half-its, CRC early stop, no UCI",
            "ue_subframes_per_s": round(world * nwork * nue * steps / elapsed, 1),
            "tb_ok_fraction": round(float(ok.mean()), 4),
            "avg_half_iterations": round(float(avg.mean()), 3),
            "parallelism": f"ue-sharded x{world}",
            "batch_workers": nwork,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": pmc_traffic("pusch", dom, nue),
            "avg_launch_ms": d["avg_launch_ms"],
            "algo_bytes_per_launch": int(bytes_per_launch),
        },
        "front_end_roofline": {k: {"GBps": per_stage[k]["GBps"], "frac": round(per_stage[k]["GBps"] / HBM_PEAK_GBS, 4),
                                   "avg_launch_ms": per_stage[k]["avg_launch_ms"],
                                   "algo_bytes_per_launch": sb_.get(k, 0),
                                   "traffic": pmc_traffic("pusch", k, nue)} for k in fe},
        "stages": per_stage,
    }
    if rank == 0 and world == 1 and cpu_seconds > 0:
        result["cpu_baseline"] = pusch_cpu_baseline(pool, cell_id, dm, rnti, args, cpu_seconds)
    elif rank == 0:
        result["cpu_baseline"] = None
    for w in workers:
        for sb in w["sbs"]:
            sb.free()
        w["pu"].free()
        w["ch"].free()
    if not emit:
        return result
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit_line(result, args.workload)


def pusch_cpu_baseline(pool, cell_id, dm, rnti, args, budget_s):
    """The PUSCH chain on one host thread: the oracle's numpy estimator / equaliser / inverse FFT (FFTW
    and chest_ul.c are not buildable here) + the reference's compiled demapper, descrambler and
    decode_tb, over the same pool, for about args.cpu_seconds."""
    import pusch as OP  # oracle/pusch.py

    from srsran_4g_amd import pusch as P
    from srsran_4g_amd.ue_dl import cell as make_cell
    from oracle import Reference
    po = OP.PuschOracle()
    ref = Reference()
    cell = make_cell(100, 1, cell_id)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        tti, grid, _ = pool[n % len(pool)]
        _, r = P.dmrs(cell, dm, 100, tti % 10, 0)
        est = po.chest(grid, 100, 0, 100, (0, 0), (0, 0), r)
        dsym = po.symbols(grid, est["ce"], est["noise"], 0, False, 100, (0, 0))
        q = po.llrs(dsym, 3, rnti, tti, cell_id)
        g = po.ora.ulsch_deinterleave(q, C3_QM, UL_NSYMB)
        ref.dlsch_decode(C3_TBS, C3_QM, 0, g, args.iters)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * C3_TBS / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": "reference",
            "ue_subframes_per_s": round(n / dt, 2),
            "sample": f"{n} PUSCH subframes, {dt:.1f} s on 1 thread: reference-compiled demapper / descrambler / "
                      f"decode_tb, oracle numpy estimator + equaliser + FFT (FFTW and chest_ul.c absent), "
                      f"oracle UL de-interleaver"}


def run_dlenc(args, torch, dist, world, rank, device):
    """DL-SCH encode of C3 transport blocks: per step `subframes` x 2 TBs (TBS 75376, 13 x K=5824
    CBs, 86400 e bits each, rv 0) through srsran_dlsch_gpu_encode_batch.  Value = encoded info Mbps."""
    import ctypes

    from srsran_4g_amd import sch as S

    rng = np.random.default_rng(shard(rank)["seed"])
    ntb = 2 * args.subframes
    host = rng.integers(0, 256, (ntb, C3_TBS // 8), dtype=np.uint8)
    d_in = torch.from_numpy(host).to(device)
    d_out = torch.zeros((ntb, C3_BITS // 8), dtype=torch.uint8, device=device)
    q = S.Sch()
    arr = (S.srsran_dlsch_gpu_enc_t * ntb)()
    for i in range(ntb):
        arr[i].tbs, arr[i].Qm, arr[i].rv, arr[i].nof_e_bits = C3_TBS, C3_QM, 0, C3_BITS
        arr[i].d_data, arr[i].d_e_bits = d_in[i].data_ptr(), d_out[i].data_ptr()
    sp = torch.cuda.current_stream(device).cuda_stream
    L = S.lib()

    def step():
        if L.srsran_dlsch_gpu_encode_batch(ctypes.byref(q.q), ntb, arr, sp) != 0:
            raise RuntimeError("srsran_dlsch_gpu_encode_batch failed")

    elapsed = timed_region(step, args.steps, args.warmup, world, dist, torch.cuda.synchronize, device)
    value = world * ntb * C3_TBS * args.steps / elapsed / 1e6
    # output check against the oracle encoder on a few TBs (outside the timed region)
    from oracle import Oracle
    ora = Oracle()
    out = d_out.cpu().numpy()
    chk = [int(np.array_equal(out[i], np.packbits(ora.dlsch_encode(C3_TBS, C3_QM, 0, C3_BITS, host[i]))))
           for i in range(0, ntb, max(1, ntb // 8))]
    algo = ntb * (C3_TBS // 8 + C3_BITS // 8 + C3_BITS)  # payload in, packed e out, unpacked scratch once
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mbps", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8 bits",
        "data": "synthetic: random C3 transport blocks, HBM-resident",
        "config": {"workload": f"dlenc: {ntb} TBs x (TBS {C3_TBS}, C=13 K=5824, E={C3_BITS}, 64QAM, rv 0) per step: "
                               "TB CRC24A + CB CRC24B + turbo encode + rate matching + packing",
                   "tbs_per_step_per_gpu": ntb, "output_check": {"tbs": len(chk), "equal_to_oracle": sum(chk)},
                   "parallelism": f"tb-sharded x{world}"},
        "roofline": {"bound": "hbm", "kernel": "whole batch (3 launches)",
                     "achieved": round(algo / (elapsed / args.steps) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(algo / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 5), "traffic": None,
                     "algo_bytes_per_launch": algo},
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            ora.dlsch_encode(C3_TBS, C3_QM, 0, C3_BITS, host[n % ntb])
            n += 1
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": round(n * C3_TBS / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": "port",
                                  "sample": f"{n} TBs through the oracle's C encoder (bit-serial turbo encoder, "
                                            f"table rate matching), {dt:.1f} s on 1 thread"}
    elif rank == 0:
        result["cpu_baseline"] = None
    q.free()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit_line(result, args.workload)


def run_dlloop(args, torch, dist, world, rank, device):
    """Device-resident C3 loopback: per step the GPU eNB transmitter
    (srsran_enb_dl_gpu_tx_batch: DL-SCH encode, CRS, scrambling, 64QAM, CDD 2x2, OFDM) produces
    `subframes` C3 subframes, a static 2x2 channel [[1, 1], [1, -1]] with AWGN is applied on the GPU
    (torch), and the GPU UE DL chain (srsran_ue_dl_gpu_decode_batch) decodes them -- no host data in
    the loop.  Value = loop subframes/s; the transmitter alone is timed with HIP events."""
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import ue_dl as U
    from synth import synth as SY

    cell_id, rnti, nsf = shard(rank)["cell_id"], 0x1234, args.subframes
    U.use_standard_symbol_size(True)
    cell = U.cell(100, 2, cell_id)
    enb = E.EnbDl(cell)
    ue = U.UeDl(cell, 2)
    ue.cfg.cfg.pdsch.max_nof_iterations = args.iters
    gen = torch.Generator(device=device)
    gen.manual_seed(shard(rank)["seed"])
    d_tx_pl = torch.randint(0, 256, (nsf, 2, C3_TBS // 8), dtype=torch.uint8, device=device, generator=gen)
    ttis = [b % 10 + 1 for b in range(nsf)]
    nres = [int(SY.pdsch_mask(100, 2, cell_id, 1, t % 10).sum()) for t in ttis]
    tx_cfgs = [U.pdsch_cfg(100, nres[b], (C3_TBS, C3_TBS), (C3_QM, C3_QM), rnti=rnti) for b in range(nsf)]
    sbs = [[S.SoftbufferRx(nof_prb=100) for _ in range(2)] for _ in range(nsf)]
    rx_cfgs = [U.pdsch_cfg(100, nres[b], (C3_TBS, C3_TBS), (C3_QM, C3_QM), rnti=rnti, max_iterations=args.iters,
                           softbuffers=sbs[b]) for b in range(nsf)]
    tx_sfs = [(ttis[b], 1, tx_cfgs[b], [d_tx_pl[b, 0].data_ptr(), d_tx_pl[b, 1].data_ptr()]) for b in range(nsf)]
    sf_len = 30720  # SRSRAN_SF_LEN_PRB(100) at N = 2048: 1 ms at 30.72 Msps
    d_tx = torch.zeros((nsf, 2, sf_len), dtype=torch.complex64, device=device)
    d_x = torch.zeros((nsf, 2, sf_len), dtype=torch.complex64, device=device)
    H = torch.tensor([[1, 1], [1, -1]], dtype=torch.complex64, device=device)
    d_pl = torch.zeros((nsf, 2, C3_TBS // 8 + 64), dtype=torch.uint8, device=device)
    d_res = torch.zeros(2 * nsf, dtype=torch.int32, device=device)
    d_avg = torch.zeros(2 * nsf, dtype=torch.float32, device=device)
    arr = U.UeDl.batch_entries([(ttis[b], 1, rx_cfgs[b], [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1])
                                for b in range(nsf)])
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream
    if enb.tx_batch(tx_sfs, d_tx.data_ptr(), 0.0, sp) != 0:
        raise RuntimeError("srsran_enb_dl_gpu_tx_batch failed")
    rx0 = torch.matmul(H, d_tx)
    sigma = float(torch.sqrt(torch.mean(torch.abs(rx0) ** 2) / 10 ** (args.snr / 10) / 2))
    noise = torch.zeros((nsf, 2, sf_len, 2), dtype=torch.float32, device=device)

    def step():
        if enb.tx_batch(tx_sfs, d_tx.data_ptr(), 0.0, sp) != 0:
            raise RuntimeError("srsran_enb_dl_gpu_tx_batch failed")
        noise.normal_(0.0, sigma, generator=gen)
        # H = [[1, 1], [1, -1]] elementwise (a batched 2 x 2 GEMM of this shape is ~0.2 ms in rocBLAS)
        torch.add(d_tx[:, 0], d_tx[:, 1], out=d_x[:, 0])
        torch.sub(d_tx[:, 0], d_tx[:, 1], out=d_x[:, 1])
        d_x.add_(torch.view_as_complex(noise))
        if ue.gpu_decode_batch(arr, d_x.data_ptr(), d_res.data_ptr(), d_avg.data_ptr(), 0.0, sp) != 2 * nsf:
            raise RuntimeError("srsran_ue_dl_gpu_decode_batch failed")

    elapsed = timed_region(step, args.steps, args.warmup, world, dist, torch.cuda.synchronize, device)
    ok = float((d_res == 0).float().mean().item())
    match = bool(torch.equal(d_pl[:, :, : C3_TBS // 8], d_tx_pl))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        enb.tx_batch(tx_sfs, d_tx.data_ptr(), 0.0, sp)
    e1.record(stream)
    torch.cuda.synchronize()
    tx_ms = e0.elapsed_time(e1) / args.steps
    value = world * nsf * args.steps / elapsed
    result = {
        "metric": "PDSCH loopback subframes/s (GPU eNB TX -> channel -> GPU UE RX), C3",
        "value": round(value, 1),
        "unit": "subframes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic, device-resident: random payloads encoded and transmitted on the GPU every step",
        "config": {"workload": "dlloop C3: %d subframes x (2 TBs x 75376 bits, 64QAM, CDD 2x2, 100 PRB, CFI 1), "
                               "channel [[1,1],[1,-1]] + AWGN %.0f dB, max %d half-its" % (nsf, args.snr, args.iters),
                   "parallelism": f"carrier-sharded x{world}"},
        "mbps": round(value * 2 * C3_TBS / 1e6, 1),
        "tx_subframes_per_s": round(nsf / (tx_ms * 1e-3), 1),
        "tx_ms_per_step": round(tx_ms, 4),
        "tb_ok_fraction": ok,
        "payloads_equal": match,
    }
    if rank == 0:
        emit_line(result, args.workload)
    enb.free()
    ue.free()
    return result


def pdsch_probe(step, steps, torch, device, prof):
    """--pdsch-probe (diagnostic, stderr): where the host waits in back-to-back batch calls -- per-call host
    time and library host phases, on torch's current stream and on a created stream, after a short and a long
    warm-up, with and without an event recorded between calls"""
    import gc
    import sys

    def loop(on, n, events):
        torch.cuda.synchronize()
        gc.disable()
        per, phases = [], []
        t0 = time.perf_counter()
        for _ in range(n):
            prof.host_enable(True)
            t = time.perf_counter()
            step(None, on)
            per.append(round((time.perf_counter() - t) * 1e6, 1))
            phases.append({k: round(us, 1) for k, (us, _) in prof.host_read().items()})
            prof.host_enable(False)
            if events:
                torch.cuda.Event().record(on if on is not None else torch.cuda.current_stream(device))
        torch.cuda.synchronize()
        total = (time.perf_counter() - t0) / n * 1e3
        gc.enable()
        return {"ms_per_step": round(total, 4), "host_us": per, "phases_first3": phases[:3],
                "phases_last": phases[-1]}

    created = torch.cuda.Stream(device)
    for name, on, ev in (("current", None, False), ("current_ev", None, True), ("created", created, False),
                         ("current_again", None, False)):
        r = loop(on, max(steps, 20), ev)
        print(json.dumps({"probe": name, **r}), file=sys.stderr, flush=True)


def run_pdsch(args, torch, dist, world, rank, device, steps=None, warmup=None, cpu_seconds=None, emit=True):
    """UE DL chain on C3 subframes: per step `subframes` subframes of 2 rx x 30720 cf32 samples
    -> 2 TBs each (TBS 75376, 64QAM, TM3 CDD 2x2, CFI 1), new transmissions, at most `iters`
    half-iterations with CRC early stop.  Value = decoded PDSCH info Mbps; also subframes/s.
    emit=False: return the result (the default all188 line embeds it) instead of printing it."""
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    cpu_seconds = args.cpu_seconds if cpu_seconds is None else cpu_seconds
    from synth import synth as SY
    from srsran_4g_amd import prof
    from srsran_4g_amd import sch as S
    from srsran_4g_amd import ue_dl as U

    rng = np.random.default_rng(shard(rank)["seed"])
    cell_id = shard(rank)["cell_id"]  # C4: an independent carrier per GPU
    rnti = 0x1234
    pool = []
    for i in range(10):  # one subframe of each index (tti 1..10 -> sf 1..9, 0)
        tti = i + 1
        pls = [rng.integers(0, 256, C3_TBS // 8, dtype=np.uint8) for _ in range(2)]
        x, nre = SY.pdsch_subframe(100, cell_id, 2, tti, 1, rnti, C3_TBS, C3_QM, 0, pls, snr_db=args.snr, rng=rng,
                                   N=args.nfft)
        pool.append((tti, x, nre, pls))
    nsf = args.subframes
    host = np.stack([pool[b % 10][1] for b in range(nsf)])
    d_x = torch.from_numpy(np.ascontiguousarray(host).view(np.float32)).to(device)
    # C3 is quoted at N = 2048 (standard rates, as srsUE runs); --nfft 1536 is the reference's default rate
    U.use_standard_symbol_size(args.nfft == 2048)
    sf_len = 15 * args.nfft
    ue = U.UeDl(U.cell(100, 2, cell_id), 2)
    ue.cfg.cfg.pdsch.max_nof_iterations = args.iters
    sbs = [[S.SoftbufferRx(nof_prb=100) for _ in range(2)] for _ in range(nsf)]
    cfgs = [U.pdsch_cfg(100, pool[b % 10][2], (C3_TBS, C3_TBS), (C3_QM, C3_QM), rnti=rnti,
                        max_iterations=args.iters, softbuffers=sbs[b]) for b in range(nsf)]
    d_pl = torch.zeros((nsf, 2, C3_TBS // 8 + 64), dtype=torch.uint8, device=device)
    d_res = torch.zeros(2 * nsf, dtype=torch.int32, device=device)
    d_avg = torch.zeros(2 * nsf, dtype=torch.float32, device=device)
    arr = U.UeDl.batch_entries([(pool[b % 10][0], 1, cfgs[b], [d_pl[b, 0].data_ptr(), d_pl[b, 1].data_ptr()], [1, 1])
                                for b in range(nsf)])
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream

    def step(x_ptr=None, on=None):
        if ue.gpu_decode_batch(arr, d_x.data_ptr() if x_ptr is None else x_ptr, d_res.data_ptr(), d_avg.data_ptr(),
                               0.0, sp if on is None else on.cuda_stream) != 2 * nsf:
            raise RuntimeError("srsran_ue_dl_gpu_decode_batch failed")

    # the timed batches go to `workers` UE DL objects in turn, each on its own stream (srsUE decodes subframes on
    # several PHY workers at once): one batch's front end can run beside the previous one's decoder tail.  Worker 0
    # is the object above; the secondary measurements below (PCIe, spread, stages, host) use it alone.
    nwork = max(1, int(getattr(args, "pdsch_workers", 1)))
    # the workers' streams: each on a hardware queue of its own (srsran_gpu_worker_stream_create) -- on HIP's shared
    # queues two workers' batches can land on one queue and run one after the other, depending on the streams created
    # and freed before (tools/r06aw_pdsch_queues.py: 402-431 k shared, 441-442 k own)
    own_streams = []

    def worker_stream():
        if getattr(args, "worker_queues", "own") == "shared":
            return torch.cuda.Stream(device)
        own_streams.append(U.WorkerStream(device))
        return own_streams[-1].stream
    workers = [(ue, arr, d_pl, d_res, d_avg, stream if nwork == 1 else worker_stream())]
    extra_sbs = []
    for _ in range(1, nwork):
        ue_w = U.UeDl(U.cell(100, 2, cell_id), 2)
        ue_w.cfg.cfg.pdsch.max_nof_iterations = args.iters
        sbs_w = [[S.SoftbufferRx(nof_prb=100) for _ in range(2)] for _ in range(nsf)]
        extra_sbs.append(sbs_w)
        cfgs_w = [U.pdsch_cfg(100, pool[b % 10][2], (C3_TBS, C3_TBS), (C3_QM, C3_QM), rnti=rnti,
                              max_iterations=args.iters, softbuffers=sbs_w[b]) for b in range(nsf)]
        pl_w = torch.zeros((nsf, 2, C3_TBS // 8 + 64), dtype=torch.uint8, device=device)
        res_w = torch.zeros(2 * nsf, dtype=torch.int32, device=device)
        avg_w = torch.zeros(2 * nsf, dtype=torch.float32, device=device)
        arr_w = U.UeDl.batch_entries([(pool[b % 10][0], 1, cfgs_w[b], [pl_w[b, 0].data_ptr(), pl_w[b, 1].data_ptr()],
                                       [1, 1]) for b in range(nsf)])
        workers.append((ue_w, arr_w, pl_w, res_w, avg_w, worker_stream(), cfgs_w))
    turn = [0]

    def step_workers():
        w = workers[turn[0] % nwork]
        turn[0] += 1
        if w[0].gpu_decode_batch(w[1], d_x.data_ptr(), w[3].data_ptr(), w[4].data_ptr(), 0.0, w[5].cuda_stream) != 2 * nsf:
            raise RuntimeError("srsran_ue_dl_gpu_decode_batch failed")

    def last_worker_stream():  # the stream of the step step_workers() enqueued last
        return workers[(turn[0] - 1) % nwork][5]

    # every worker's first batch (its ring, scratch and descriptor growth) before the timed region, whatever
    # the warm-up count: a worker first used inside the timed steps would time its allocations
    for w in workers[1:]:
        if w[0].gpu_decode_batch(w[1], d_x.data_ptr(), w[3].data_ptr(), w[4].data_ptr(), 0.0, w[5].cuda_stream) != 2 * nsf:
            raise RuntimeError("srsran_ue_dl_gpu_decode_batch failed")
    torch.cuda.synchronize()
    elapsed = timed_region(step_workers, steps, warmup, world, dist, torch.cuda.synchronize, device)
    if getattr(args, "pdsch_probe", False):
        pdsch_probe(step, steps, torch, device, prof)
    # PCIe-inclusive rate (never `value`): every step's time samples start in pinned host memory.
    # Two device sample buffers: step i+1's H2D runs on a copy stream while step i decodes
    # (phy_dl_test.c:658-671 feeds one subframe at a time; here the copy hides under the batch).
    # Both on created (non-default) streams: on the legacy NULL stream the waits below serialise the loop
    # (tools/h2d_probe.py: 1.74 ms per step there against 0.72 ms with the copy alone).
    h_x = torch.from_numpy(np.ascontiguousarray(host).view(np.float32)).pin_memory()
    d_xs = [d_x, torch.empty_like(d_x)]
    cs = torch.cuda.Stream(device, priority=args.h2d_priority)
    ks = torch.cuda.Stream(device)
    copied = [torch.cuda.Event(), torch.cuda.Event()]
    used = [torch.cuda.Event(), torch.cuda.Event()]
    n_h2d = max(steps, 20)

    def h2d_loop(n, h_src, bufs, stepf):
        with torch.cuda.stream(cs):
            bufs[0].copy_(h_src, non_blocking=True)
        copied[0].record(cs)
        for i in range(n):
            b = i % 2
            if i + 1 < n:
                nb = (i + 1) % 2
                if i >= 1:
                    # step i-1 is done with that buffer: waited on the host (a GPU-side wait of the copy
                    # stream on the decode stream serialises the two on this runtime: tools/h2d_probe.py
                    # bench_like 1.04 ms against bench_like_host_wait 0.81 ms a step, r03r)
                    used[nb].synchronize()
                with torch.cuda.stream(cs):
                    bufs[nb].copy_(h_src, non_blocking=True)
                copied[nb].record(cs)
            ks.wait_event(copied[b])
            stepf(bufs[b].data_ptr(), ks)
            used[b].record(ks)

    def h2d_rates(h_src, bufs, stepf):
        # the copy alone first (the PCIe bound of the same bytes; also maps the pinned samples for the GPU)
        for timed in (False, True):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(n_h2d if timed else 4):
                with torch.cuda.stream(cs):
                    bufs[1].copy_(h_src, non_blocking=True)
            torch.cuda.synchronize()
            c_s = (time.perf_counter() - t1) / n_h2d
        h2d_loop(4, h_src, bufs, stepf)  # untimed: the first work on freshly created streams pays their queue set-up
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        h2d_loop(n_h2d, h_src, bufs, stepf)
        torch.cuda.synchronize()
        return c_s, (time.perf_counter() - t1) / n_h2d

    copy_s, h2d_s = h2d_rates(h_x, d_xs, step)
    del d_xs[1]
    # the same with the radio's int16 I/Q samples (srsran_ue_dl_gpu_decode_batch_sc16: converted x scale in the OFDM
    # load): half the bytes over PCIe.  The samples quantised to 14 bits of their peak.
    sc16_scale = float(np.float32(np.abs(host.view(np.float32)).max() / (1 << 14)))
    hq = np.empty(host.shape + (2,), np.int16)
    hq[..., 0] = np.clip(np.rint(host.real / sc16_scale), -32768, 32767)
    hq[..., 1] = np.clip(np.rint(host.imag / sc16_scale), -32768, 32767)
    h_q = torch.from_numpy(hq).pin_memory()
    d_qs = [torch.empty(hq.shape, dtype=torch.int16, device=device) for _ in range(2)]

    def step16(x_ptr, on):
        if ue.gpu_decode_batch_sc16(arr, x_ptr, sc16_scale, d_res.data_ptr(), d_avg.data_ptr(), 0.0,
                                    on.cuda_stream) != 2 * nsf:
            raise RuntimeError("srsran_ue_dl_gpu_decode_batch_sc16 failed")
    d_res.fill_(7)
    copy16_s, h2d16_s = h2d_rates(h_q, d_qs, step16)
    ok16 = int((d_res.cpu().numpy() == 0).sum())
    del d_qs
    # per-step spread of the timed configuration (the workers taking the steps in turn: events on each step's own
    # stream, intervals between consecutive completions; host phases per call), and of worker 0 alone
    spread = step_spread(step_workers, max(steps, 10), torch, stream, prof, stream_of=last_worker_stream)
    spread_one = step_spread(step, max(steps, 10), torch, stream) if nwork > 1 else None
    # host cost of one step (the API builds descriptors and launches asynchronously), each call on an idle GPU:
    # in a free-running loop the host runs ahead until a ring slot's wait blocks it, and the call time is then
    # the GPU's step time, not the host's work
    import gc
    gc.disable()
    host_calls = []
    prof.host_enable(True)
    prof.host_read()
    for _ in range(max(steps, 10)):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        host_calls.append((time.perf_counter() - t1) * 1e3)
    host_phases = {k: round(us / n, 1) for k, (us, n) in prof.host_read().items()}
    prof.host_enable(False)
    gc.enable()
    torch.cuda.synchronize()
    host_ms = float(np.median(host_calls))
    res = d_res.cpu().numpy()
    avg = d_avg.cpu().numpy()
    pl = d_pl.cpu().numpy()
    ok = sum(int(np.array_equal(pl[b, q, : C3_TBS // 8], pool[b % 10][3][q])) for b in range(nsf) for q in range(2))
    for w in workers[1:]:  # every worker decoded the same subframes
        plw = w[2].cpu().numpy()
        ok_w = sum(int(np.array_equal(plw[b, q, : C3_TBS // 8], pool[b % 10][3][q])) for b in range(nsf) for q in range(2))
        if ok_w != ok or not np.array_equal(w[3].cpu().numpy(), res):
            raise RuntimeError("bench: PDSCH workers disagree")
    value = world * nsf * 2 * C3_TBS * steps / elapsed / 1e6

    # per-stage kernel durations from HIP events on the launch streams (library-side), same batch
    prof.enable(True)
    nrep = max(1, min(steps, 3))
    for _ in range(nrep):
        step()
    torch.cuda.synchronize()
    stages = prof.read()
    prof.enable(False)
    nre_sum = sum(pool[b % 10][2] for b in range(nsf))
    sb = stage_bytes(nsf, nre_sum, 2 * nsf, sf_len)
    per_stage = {}
    for name, (ms, n) in stages.items():
        avg_ms = ms / n
        launches_per_step = n / nrep
        byts = sb.get(name, 0) / launches_per_step
        per_stage[name] = {"ms_per_step": round(ms / nrep, 4), "launches_per_step": launches_per_step,
                           "avg_launch_ms": round(avg_ms, 4), "GBps": round(byts / (avg_ms * 1e-3) / 1e9, 1)}
    dom = max(per_stage, key=lambda k: per_stage[k]["ms_per_step"])
    d = per_stage[dom]
    bytes_per_launch = sb[dom] / d["launches_per_step"]
    achieved = bytes_per_launch / (d["avg_launch_ms"] * 1e-3) / 1e9
    from srsran_4g_amd import tdec as TD
    # the turbo stage's kernel as it ran (srsran_tdec_gpu_last_kernel), e.g. tdec16s_kernel<true>
    dom_name = TD.last_kernel() if dom == "tdec_kernel" else dom
    traffic = pmc_traffic("pdsch", dom_name, nsf * 26)
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mbps",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32+int16",
        "data": f"synthetic: eNB-side TX (synth/: DL-SCH encode, scrambling, 64QAM, CDD, CRS, OFDM) through "
                f"[[1,1],[1,-1]] + AWGN {args.snr} dB; 10 distinct subframes (indices 0-9) tiled, HBM-resident",
        "config": {
            "workload": f"pdsch C3: {nsf} subframes x (2 rx x {sf_len} cf32 samples -> OFDM {args.nfft} -> CRS chest -> "
                        f"MMSE CDD 2x2 -> 64QAM LLR -> 2 TBs x {C3_TBS} bits), CFI 1, max {args.iters} half-its",
            "subframes_per_step_per_gpu": nsf,
            "subframes_per_s": round(world * nsf * steps / elapsed, 1),
            "subframes_per_s_h2d_inclusive": round(world * nsf / h2d_s, 1),
            "h2d_copy_only_subframes_per_s": round(world * nsf / copy_s, 1),
            "h2d_gbps": round(host.nbytes / copy_s / 1e9, 2),
            "subframes_per_s_h2d_sc16_inclusive": round(world * nsf / h2d16_s, 1),
            "h2d_sc16_copy_only_subframes_per_s": round(world * nsf / copy16_s, 1),
            "sc16_tb_ok_fraction": round(ok16 / (2 * nsf), 4),
            "tb_ok_fraction": round(ok / (2 * nsf), 4),
            "avg_half_iterations": round(float(avg.mean()), 3),
            "cell_id": cell_id,
            "parallelism": f"carrier-per-gpu x{world}",
            "batch_workers": nwork,
            "worker_queues": getattr(args, "worker_queues", "own") if nwork > 1 else None,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom_name,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "avg_launch_ms": d["avg_launch_ms"],
            "algo_bytes_per_launch": int(bytes_per_launch),
        },
        "stages": per_stage,
        "step_spread": spread,
        "step_spread_one_worker": spread_one,
        "host_enqueue_ms_per_step": round(host_ms, 4),
        "host_enqueue_note": "median of per-call times, each call issued on an idle GPU (no ring waits)",
        "host_phases_us_per_call": host_phases,
        "chain_bytes_per_sf": 2 * sf_len * 8 + 2 * C3_TBS // 8,
    }
    if (res != 0).any():
        result["config"]["tb_fail"] = int((res != 0).sum())
    if rank == 0 and world == 1 and cpu_seconds > 0:
        result["cpu_baseline"] = pdsch_cpu_baseline(pool, args, cpu_seconds)
    elif rank == 0:
        result["cpu_baseline"] = None
    ue.free()
    for pair in sbs:
        for s_ in pair:
            s_.free()
    for w in workers[1:]:
        w[0].free()
    for sbs_w in extra_sbs:
        for pair in sbs_w:
            for s_ in pair:
                s_.free()
    for ws in own_streams:
        ws.free()
    if not emit:
        return result
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit_line(result, args.workload)
    return result


def _pdsch_cpu_chain():
    """(decode one subframe -> None, kind): the reference's compiled PDSCH pieces (oracle/_ref: predecoding,
    demod_soft, sequence, DL-SCH decode_tb over rm_turbo/turbodecoder/crc) with the oracle's C channel estimator and
    numpy's FFT (FFTW is not in the image)"""
    import pdsch_chain as PC
    from oracle import Oracle, Reference, ref_available

    ora = Oracle()
    ref = Reference() if ref_available() else None

    class Hybrid:
        def __getattr__(self, name):
            if ref is not None and name in ("predecode", "demod_s", "sequence_apply_s", "dlsch_decode"):
                return getattr(ref, name)
            return getattr(ora, name)

    h = Hybrid()

    def decode(tti, x, iters, cell_id=1):
        g, ce, st = PC.fft_estimate(ora, x, 100, cell_id, 2, tti)
        PC.pdsch_decode(h, g, ce, st["noise"], 100, cell_id, 2, tti, 1, 0x1234, [C3_TBS, C3_TBS], [C3_QM, C3_QM],
                        [0, 0], max_iterations=iters)
    return decode, "reference" if ref is not None else "port"


def pdsch_cpu_worker(args):
    """--cpu-worker SEED --workload pdsch: one host process of the PDSCH CPU leg's job-share run (no torch, no GPU):
    its own C3 subframes (4, synthetic, --snr / --nfft of the line), decoded in turn for --cpu-seconds."""
    from synth import synth as SY

    rng = np.random.default_rng(args.cpu_worker)
    pool = []
    for i in range(4):
        pls = [rng.integers(0, 256, C3_TBS // 8, dtype=np.uint8) for _ in range(2)]
        x, _ = SY.pdsch_subframe(100, 1, 2, i + 1, 1, 0x1234, C3_TBS, C3_QM, 0, pls, snr_db=args.snr, rng=rng,
                                 N=args.nfft)
        pool.append((i + 1, x))
    decode, _ = _pdsch_cpu_chain()
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        tti, x = pool[n % len(pool)]
        decode(tti, x, args.iters)
        n += 1
    print(json.dumps({"subframes": n, "dt": time.perf_counter() - t0}), flush=True)


def pdsch_cpu_baseline(pool, args, budget_s):
    """The PDSCH chain on the host, over the same subframes (_pdsch_cpu_chain): one thread for budget_s, then one
    process per core of this job's share (the tdec leg's 16 on the GPU box, cpu_threads()) for budget_s, each over its
    own subframes -- the same core share as the turbo decoder's cpu_share figure."""
    import subprocess

    decode, kind = _pdsch_cpu_chain()
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        tti, x, nre, _ = pool[n % len(pool)]
        decode(tti, x, args.iters)
        n += 1
    dt = time.perf_counter() - t0
    nproc = cpu_threads()
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", str(3000 + i),
                               "--cpu-seconds", str(budget_s), "--iters", str(args.iters), "--workload", "pdsch",
                               "--snr", str(args.snr), "--nfft", str(args.nfft)],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env, cwd=ROOT)
             for i in range(nproc)]
    agg, agg_dt, ok = 0, 0.0, 0
    for p in procs:
        try:
            out, _ = p.communicate(timeout=budget_s + 180)
            r = json.loads(out.decode().strip().splitlines()[-1])
            agg, agg_dt, ok = agg + r["subframes"], max(agg_dt, r["dt"]), ok + 1
        except Exception:
            p.kill()
    share = agg / agg_dt if ok else None
    return {"value": round(n * 2 * C3_TBS / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": kind,
            "subframes_per_s": round(n / dt, 2),
            "share_subframes_per_s": round(share, 2) if share else None, "share_processes": ok,
            "share_mbps": round(share * 2 * C3_TBS / 1e6, 3) if share else None,
            "cpu_model": cpu_model(),
            "sample": f"{n} C3 subframes, {dt:.1f} s on 1 thread; then {ok} processes x {budget_s:.0f} s over their own "
                      f"4 subframes: reference-compiled predecoding / demod / descrambling / DL-SCH; oracle C channel "
                      f"estimator; numpy FFT (FFTW absent)" if kind == "reference"
                      else f"{n} C3 subframes, {dt:.1f} s on 1 thread (oracle C port + numpy FFT); {ok} processes"}


def run_ldpc(args, torch, dist, world, rank, device):
    """NR LDPC decode (BASELINE configs[4]): per step `codewords` BG/Z codewords (int8 LLRs of
    noisy BPSK codewords from synth/ldpc_tx.py), `ldpc-iters` iterations, no early stop (the
    reference test's decode_c), packed message bits out.  Value = decoded info bits / s."""
    from synth import ldpc_tx
    from srsran_4g_amd import ldpc as G

    bg = args.bg - 1
    M, N, K = G.BG_SHAPE[bg]
    ls = args.ls
    liftK, n = K * ls, (N - 2) * ls
    rng = np.random.default_rng(shard(rank)["seed"])
    pool = []
    pcm = G.compact_pcm(bg, ls)
    for _ in range(args.pool):
        cw = ldpc_tx.encode(bg, ls, rng.integers(0, 2, liftK).astype(np.uint8), pcm)[2 * ls:]
        pool.append(ldpc_tx.bpsk_awgn_int8(cw, rng, args.ldpc_snr))
    ncw = args.codewords
    host = np.stack([pool[i % args.pool] for i in range(ncw)])
    d_in = torch.from_numpy(host).to(device)
    d_out = torch.zeros((ncw, liftK // 8), dtype=torch.uint8, device=device)
    dec = G.LdpcDecoder(bg, ls, G.DEC_C_AVX2, scaling=0.8, max_nof_iter=args.ldpc_iters)
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream

    def step():
        if dec.gpu_decode_batch(d_in.data_ptr(), n, ncw, d_out.data_ptr(), liftK // 8, packed=True, stream=sp) != 0:
            raise RuntimeError("srsran_ldpc_decoder_gpu_decode_batch failed")

    elapsed = timed_region(step, args.steps, args.warmup, world, dist, torch.cuda.synchronize, device)
    value = world * ncw * liftK * args.steps / elapsed / 1e6
    ms = []
    for _ in range(max(1, min(args.steps, 3))):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step()
        e1.record(stream)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    avg_ms = float(np.mean(ms))
    bytes_per_launch = ncw * (n + liftK // 8)  # int8 LLRs in + packed message out (SURVEY 8d style)
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    cs = 384 if ls > 256 else 256 if ls > 128 else 128 if ls > 64 else 64 if ls > 32 else 32 if ls > 16 else 16
    # ldpc_kernel.hip dispatch: full-length codewords use every layer (46 for BG1, 42 for BG2)
    dom = f"ldpc_kernel_pk<{bg}, {cs}, {46 if bg == 0 else 42}>" if ls > 16 else f"ldpc_kernel<{bg}, {cs}, signed char>"
    # decode quality on the pool (the reference's ldpc_chain_test reports BER the same way)
    out = d_out.cpu().numpy()
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
        "dtype": "int8",
        "data": f"synthetic: BPSK AWGN (Es/N0 {args.ldpc_snr} dB) LDPC codewords from synth/ldpc_tx.py, int8 LLRs, "
                f"{args.pool} distinct codewords tiled to the batch, HBM-resident",
        "config": {
            "workload": f"ldpc BG{args.bg} Z={ls}: {ncw} codewords x {liftK} info bits, {args.ldpc_iters} iterations "
                        "(no early stop), SRSRAN_LDPC_DECODER_C_AVX2 arithmetic, scaling 0.8, packed output",
            "codewords_per_step_per_gpu": ncw,
            "parallelism": f"cw-sharded x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": pmc_traffic(args.workload, dom, ncw),
            "avg_launch_ms": round(avg_ms, 4),
            "algo_bytes_per_launch": int(bytes_per_launch),
        },
        "decoded_pool_bits_set": int(np.unpackbits(out[:1]).sum()),
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from ldpc import RefLdpc, ref_available, OracleLdpc, DEC_C_AVX2
        kind = "reference" if ref_available() else "port"
        nd = 0
        t0 = time.perf_counter()
        pool2d = np.stack(pool)
        if kind == "reference":
            ref = RefLdpc()
            while time.perf_counter() - t0 < args.cpu_seconds:
                ref.decode_many(DEC_C_AVX2, bg, ls, pool2d, scaling=0.8, max_iter=args.ldpc_iters)
                nd += len(pool)
        else:
            ora = OracleLdpc()
            while time.perf_counter() - t0 < args.cpu_seconds:
                ora.decode_c(bg, ls, pool[nd % args.pool], scaling=0.8, max_iter=args.ldpc_iters)
                nd += 1
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": round(nd * liftK / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": kind,
                                  "sample": f"{nd} codewords (passes over the {args.pool}-codeword pool) through one "
                                            f"srsran_ldpc_decoder_t (C_AVX2, {args.ldpc_iters} iterations), "
                                            f"{dt:.1f} s on 1 thread"}
    elif rank == 0:
        result["cpu_baseline"] = None
    dec.free()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit_line(result, args.workload)


NR_PRB, NR_QM, NR_R = 273, 8, 948.0 / 1024.0  # 100 MHz @ 30 kHz, MCS 27 of the 256QAM table (38.214 5.1.3.1-2)
NR_NRE = 12 * 12 * NR_PRB                      # 12 PDSCH symbols (2 DMRS symbols of 14), 1 layer


def run_nrsch(args, torch, dist, world, rank, device):
    """NR DL-SCH receive: per step `nr-tbs` new transmissions (rv 0) of one full-carrier TB shape,
    through srsran_sch_nr_gpu_decode_batch (rate de-matching into the soft buffers, LDPC decode
    with per-CB CRC early stop, max `ldpc-iters` iterations, TB assembly + CRC).  Value = decoded
    TB bits / s."""
    from srsran_4g_amd import prof
    from srsran_4g_amd import sch_nr as S
    from synth.nr_tx import NrCodeblocks, aligned_tbs, bpsk_llrs

    tbs = aligned_tbs(NR_NRE, NR_R, NR_QM, 1)
    G = NR_NRE * NR_QM
    t = S.tb_info(tbs, NR_R, NR_QM, G, 1, nof_prb=NR_PRB, mcs256=True)
    rng = np.random.default_rng(shard(rank)["seed"])
    pool, pays = [], []
    for _ in range(args.pool):
        pl = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        pool.append(bpsk_llrs(rng, NrCodeblocks(t, pl).rate_match(0), args.nr_snr))
        pays.append(pl)
    ntb = args.nr_tbs
    d_e = torch.from_numpy(np.stack([pool[i % args.pool] for i in range(ntb)])).to(device)
    d_p = torch.zeros((ntb, tbs // 8 + 8), dtype=torch.uint8, device=device)
    d_crc = torch.zeros(ntb, dtype=torch.uint8, device=device)
    d_avg = torch.zeros(ntb, dtype=torch.float32, device=device)
    q = S.SchNr(nof_prb=NR_PRB, scaling=0.8, max_nof_iter=args.ldpc_iters)
    sbs = [S.SoftbufferRx(max_cb=t.C, max_cb_size=S.MAX_CB_SIZE) for _ in range(ntb)]
    cfg = S.make_cfg(mcs256=True)
    tbd = [S.make_tb(tbs, NR_R, NR_QM, G, 1, 0, sb) for sb in sbs]
    arr = (S.srsran_sch_nr_gpu_tb_t * ntb)()
    for i in range(ntb):
        arr[i].sch_cfg = S.ctypes.pointer(cfg)
        arr[i].tb = S.ctypes.pointer(tbd[i])
        arr[i].d_e_bits, arr[i].d_payload, arr[i].new_data = d_e[i].data_ptr(), d_p[i].data_ptr(), 1
    L = S.lib()
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream

    def step():
        if L.srsran_sch_nr_gpu_decode_batch(S.ctypes.byref(q.q), ntb, arr, d_crc.data_ptr(), d_avg.data_ptr(), sp):
            raise RuntimeError("srsran_sch_nr_gpu_decode_batch failed")

    elapsed = timed_region(step, args.steps, args.warmup, world, dist, torch.cuda.synchronize, device)
    value = world * ntb * tbs * args.steps / elapsed / 1e6
    crc = d_crc.cpu().numpy()
    avg = d_avg.cpu().numpy()
    out = d_p.cpu().numpy()
    payload_ok = all(np.array_equal(out[i, :tbs // 8], pays[i % args.pool]) for i in range(ntb) if crc[i])

    prof.enable(True)
    nrep = max(1, min(args.steps, 3))
    for _ in range(nrep):
        step()
    torch.cuda.synchronize()
    stages = prof.read()
    prof.enable(False)
    ncb = ntb * t.C
    E = G // t.C
    Ncb = t.Z * (66 if t.bg == 0 else 50)
    cb_bytes = (t.Kp - t.L_cb) // 8
    # algorithmic bytes per launch (SURVEY 8d style): LLRs in, soft buffers / payloads out
    algo = {"nr_rm_kernel": ncb * (E + Ncb + cb_bytes),       # E LLRs in, whole circular buffer + cleared payload out
            "ldpc_kernel": ncb * (min(E, Ncb) + cb_bytes),      # soft bits covered by the transmission in, payload out
            "nr_tb_kernel": ntb * 2 * (tbs // 8)}               # block payloads in, TB payload out
    per_stage = {}
    for name, (ms, n) in stages.items():
        lps = n / nrep
        per_stage[name] = {"ms_per_step": round(ms / nrep, 4), "launches_per_step": lps,
                           "avg_launch_ms": round(ms / n, 4),
                           "GBps": round(algo.get(name, 0) / (ms / n * 1e-3) / 1e9, 1)}
    dom = max(per_stage, key=lambda k: per_stage[k]["ms_per_step"])
    d = per_stage[dom]
    achieved = algo[dom] / (d["avg_launch_ms"] * 1e-3) / 1e9
    # ldpc_kernel.hip dispatch for Z = 384: rv-0 blocks above R ~0.6 need <= 8 layers
    bg_cs = f"ldpc_kernel_pk<{t.bg}, 384, 8>"
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
        "dtype": "int8",
        "data": f"synthetic: NR DL-SCH TBs from synth/nr_tx.py (bits as +-1, AWGN Es/N0 {args.nr_snr} dB, int8 "
                f"LLRs = clip(round(10 y))), {args.pool} distinct TBs tiled to the batch, HBM-resident",
        "config": {
            "workload": f"nrsch: {ntb} TBs x {tbs} bits (273 PRB, 256QAM, R 948/1024, 1 layer, G={G}; BG{t.bg + 1} "
                        f"Z={t.Z}, C={t.C}), new transmissions (rv 0), CRC early stop, max {args.ldpc_iters} "
                        "iterations, C_AVX2 arithmetic, scaling 0.8",
            "tbs_per_step_per_gpu": ntb,
            "tb_ok_fraction": round(float((crc == 1).mean()), 4),
            "payload_ok": bool(payload_ok),
            "avg_iterations": round(float(avg.mean()), 3),
            "parallelism": f"tb-sharded x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": bg_cs if dom == "ldpc_kernel" else dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": pmc_traffic(args.workload, bg_cs if dom == "ldpc_kernel" else dom, ncb),
            "avg_launch_ms": d["avg_launch_ms"],
            "algo_bytes_per_launch": int(algo[dom]),
        },
        "stages": per_stage,
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from nr_sch import OracleNr, RefNr, RefNrRx, new_state, ref_available, oracle_nr_tb_info_t
        kind = "reference" if ref_available() else "port"
        n = 0
        t0 = time.perf_counter()
        if kind == "reference":
            ref = RefNr()
            rx, sb = RefNrRx(ref, NR_PRB, 0.8, args.ldpc_iters), ref.softbuffer()
            while time.perf_counter() - t0 < args.cpu_seconds:
                sb.reset()  # new transmission
                rx.decode(sb, tbs, NR_R, NR_QM, G, 1, 0, pool[n % args.pool], mcs256=True)
                n += 1
            dt = time.perf_counter() - t0
            rx.free()
            sb.free()
        else:
            ora = OracleNr()
            ot = oracle_nr_tb_info_t()
            for k, v in t.as_dict().items():
                setattr(ot, k, v)
            while time.perf_counter() - t0 < args.cpu_seconds:
                ora.decode(ot, 0, pool[n % args.pool], new_state(t.C), max_iter=args.ldpc_iters)
                n += 1
            dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": round(n * tbs / dt / 1e6, 3), "unit": "Mbps", "cores": 1, "kind": kind,
                                  "sample": f"{n} TBs of the same pool (soft buffer reset per TB) through one "
                                            f"srsran_sch_nr_t receiver (srsran_dlsch_nr_decode), {dt:.1f} s on 1 thread"}
    elif rank == 0:
        result["cpu_baseline"] = None
    for sb in sbs:
        sb.free()
    q.free()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit_line(result, args.workload)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_local_ranks(n):
    """--gpus N > 1 with no launcher around us: start N rank processes of this script as CHILDREN (one per
    GPU, RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), before this process touches the
    GPU -- nothing is exec'd.  Rank 0 prints the line; returns the worst exit status (a failed rank stops
    the others)."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:  # a rank failed: the others would wait at the next barrier forever
                    q.terminate()
        time.sleep(0.05)
    return rc


def dry_run(args):
    """--dry-run: the launch path without a GPU (tests/test_dist_cpu.py): every rank joins a gloo group,
    maps LOCAL_RANK to its device index and takes its shard; rank 0 prints one line with them all."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    me = dict(rank=rank, local_rank=local, device=f"cuda:{local}", **shard(rank))
    ranks = [me]
    if world > 1:
        dist.init_process_group(backend="gloo", init_method="env://")
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "dry_run": True, "ranks": ranks}), flush=True)
    return 0


def main():
    args = parse()
    if args.cpu_worker is not None:
        return cpu_worker(args)
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0 and (args.gpus or 1) > 1:
        return launch_local_ranks(args.gpus)
    if world and args.gpus is not None and world != args.gpus:
        print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    world = world or 1
    if args.dry_run:
        return dry_run(args)
    import torch
    import torch.distributed as dist

    from srsran_4g_amd import tdec

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl", init_method="env://")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if not tdec.gpu_available():
        raise RuntimeError("bench: HIP device not visible to libsrsran_4g_amd")
    if args.tdec16 != "auto":  # srsran_tdec_gpu_set_pair_threshold / _class_single_threshold(16, .)
        never = 1 << 30
        pair_min, single_min = {"single": (0, 0), "pair": (0, never), "quad": (never, never)}[args.tdec16]
        tdec.load_library().srsran_tdec_gpu_set_pair_threshold(pair_min)
        tdec.load_library().srsran_tdec_gpu_set_class_single_threshold(16, single_min)
    if args.w8_max_k >= 0:
        tdec.load_library().srsran_tdec_gpu_set_w8_max_k(args.w8_max_k)
    if args.w8_fused_max_k >= 0:
        tdec.load_library().srsran_tdec_gpu_set_w8_fused_max_k(args.w8_fused_max_k)
    if args.generic_single_min_cb >= 0:
        tdec.load_library().srsran_tdec_gpu_set_generic_single_threshold(args.generic_single_min_cb)
    if args.workload in ("dlsch", "ulsch"):
        return run_dlsch(args, torch, dist, world, rank, device)
    if args.workload == "pusch":
        return run_pusch(args, torch, dist, world, rank, device)
    if args.workload == "dlenc":
        return run_dlenc(args, torch, dist, world, rank, device)
    if args.workload == "dlloop":
        return run_dlloop(args, torch, dist, world, rank, device)
    if args.workload == "pdsch":
        return run_pdsch(args, torch, dist, world, rank, device)
    if args.workload == "ldpc":
        return run_ldpc(args, torch, dist, world, rank, device)
    if args.workload == "nrsch":
        return run_nrsch(args, torch, dist, world, rank, device)

    Ks = list(tdec.CB_SIZES) if args.workload == "all188" else [6144]
    rng = np.random.default_rng(shard(rank)["seed"])
    data = make_inputs(Ks, args.pool, args.batch, rng, torch, device)
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

    # ---- timed region: exactly `steps` steps, barrier + sync on both sides, max over ranks ----
    elapsed = timed_region(step, args.steps, args.warmup, world, dist, torch.cuda.synchronize, device)

    bits_per_step = args.batch * sum(Ks)
    value = world * bits_per_step * args.steps / elapsed / 1e6
    spread = step_spread(step, max(args.steps, 5), torch, stream)

    # ---- per-launch kernel durations (HIP events on the launch stream), outside the timed region ----
    events = []
    for _ in range(max(1, min(args.steps, 3))):
        step(events)
    torch.cuda.synchronize()
    per_kernel = {}
    for K, e0, e1 in events:
        name = tdec.load_library().srsran_tdec_gpu_kernel_name_batch(K, args.batch).decode()
        ms = e0.elapsed_time(e1)
        d = per_kernel.setdefault(name, {"launches": 0, "ms": 0.0, "bytes": 0, "bits": 0})
        d["launches"] += 1
        d["ms"] += ms
        d["bytes"] += args.batch * algo_bytes(K)
        d["bits"] += args.batch * K
    if len(Ks) > 1:
        # the timed step runs one fused launch per decoder class; its dominant part is the
        # 16-sub-block class (every K >= 816 of the batch: the single-lane decoder, its sizes up to
        # srsran_tdec_gpu_get_w8_fused_max_k as a second concurrent launch on 8-step windows), timed
        # here alone with events on the launch stream
        k16 = [i for i, K in enumerate(Ks) if tdec.nof_subblocks(K) == 16]
        sel = [[groups[j][i] for i in k16] for j in range(5)]
        ms16 = []
        for _ in range(max(1, min(args.steps, 3))):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            tdec.gpu_run_multi(sel[0], sel[1], sel[2], True, sel[3], sel[4], args.iters, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            ms16.append(e0.elapsed_time(e1))
        dom = tdec.last_kernel()  # the 16-class launch just timed (srsran_tdec_gpu_last_kernel)
        cut = tdec.load_library().srsran_tdec_gpu_get_w8_fused_max_k()
        if dom == "tdec16sw8_multi_kernel" and any(Ks[i] > cut for i in k16):
            # the class cut at srsran_tdec_gpu_get_w8_fused_max_k: two concurrent launches, timed together
            dom = "tdec16s_multi_kernel+tdec16sw8_multi_kernel"
        avg_ms = float(np.mean(ms16))
        bytes_per_launch = sum(args.batch * algo_bytes(Ks[i]) for i in k16)
        dom_units = args.batch * len(k16)
        traffic = pmc_traffic(args.workload, dom, dom_units)
    else:
        dk = per_kernel[max(per_kernel, key=lambda n: per_kernel[n]["ms"])]
        dom = tdec.last_kernel()  # the kernel as it ran and as rocprofv3 names it, e.g. tdec16s_kernel<false>
        avg_ms = dk["ms"] / dk["launches"]
        bytes_per_launch = dk["bytes"] / dk["launches"]
        dom_units = args.batch
        k16 = [0]
        traffic = pmc_traffic(args.workload, dom, dom_units)
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    # VALU view of the same launch (the binding ceiling of the turbo decoder):
    #  * valu_issue_frac: VALU wave-instructions per launch (rocprofv3 SQ_INSTS_VALU, committed in
    #    profiles/pmc_traffic.json, scaled to this batch) / (launch time x issue peak)
    #  * valu_alg_frac: SURVEY 8d's 86 packed-int16 ops per bit and half-iteration / the pk-int16 peak
    dom_bits = sum(args.batch * Ks[i] for i in k16) if len(Ks) > 1 else args.batch * Ks[0]
    ent = pmc_entry(args.workload, dom)
    valu_insts = ent["valu_insts"] * dom_units / ent["units"] if ent and "valu_insts" in ent else None
    valu = {
        "valu_issue_frac": round(valu_insts / (avg_ms * 1e-3) / VALU_ISSUE_PEAK, 4) if valu_insts else None,
        "valu_insts_per_launch": int(valu_insts) if valu_insts else None,
        "valu_alg_frac": round(TDEC_OPS_PER_BIT_HALF_IT * dom_bits * args.iters / (avg_ms * 1e-3) / VALU_PK16_PEAK, 4),
        "valu_issue_peak": VALU_ISSUE_PEAK,
        "valu_issue_frac_measured_rate": round(valu_insts / (avg_ms * 1e-3) / VALU_ISSUE_MEASURED, 4)
        if valu_insts else None,
        "valu_issue_measured_rate": round(VALU_ISSUE_MEASURED),
        "valu_pk16_peak": VALU_PK16_PEAK,
    }

    # 16 half-iterations (SURVEY 8d "also 16"): the same batch, events on the launch stream
    ms_16 = []
    for _ in range(2):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if len(Ks) > 1:
            tdec.gpu_run_multi(groups[0], groups[1], groups[2], True, groups[3], groups[4], 16, sp)
        else:
            tdec.gpu_run_batch(Ks[0], groups[1][0], groups[2][0], True, groups[3][0], args.batch, 16, sp)
        e1.record(stream)
        torch.cuda.synchronize()
        ms_16.append(e0.elapsed_time(e1))
    mbps_16 = world * bits_per_step / (min(ms_16) * 1e-3) / 1e6

    # output check: re-run the timed batch and compare every decoded block with the reference
    # decoder's output for its pool block (oracle/_ref, or the port where /root/reference is absent)
    step()
    torch.cuda.synchronize()
    want = ref_outputs(Ks, data, args.iters)
    bad = 0
    for K in Ks:
        got = data[K][1].cpu().numpy()
        exp = want[K][np.arange(args.batch) % args.pool]
        bad += int((got != exp).any(axis=1).sum())

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
            "tdec16": args.tdec16,
        },
        "roofline": dict({
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "avg_launch_ms": round(avg_ms, 4),
            "algo_bytes_per_launch": int(bytes_per_launch),
        }, **valu),
        "step_spread": spread,
        "per_kernel_mbps": {n: round(d["bits"] / (d["ms"] * 1e-3) / 1e6, 1) for n, d in per_kernel.items()},
        "mbps_16_half_its": round(mbps_16, 1),
        "output_check": {"blocks": args.batch * len(Ks), "mismatched": bad,
                         "against": "reference decoder (oracle/_ref) on each pool block"},
    }
    if args.workload == "all188":
        k = [e for e in events if e[0] == 6144]
        if k:
            ms = np.mean([e0.elapsed_time(e1) for _, e0, e1 in k])
            result["k6144_mbps"] = round(args.batch * 6144 / (ms * 1e-3) / 1e6, 1)
        if 6144 in data:  # C1 at 16 half-iterations too: BASELINE's "8 iter" may mean full iterations
            d_in, d_out, _ = data[6144]
            ms16 = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                tdec.gpu_run_batch(6144, d_in.data_ptr(), d_in.shape[1], True, d_out.data_ptr(), args.batch, 16, sp)
                e1.record(stream)
                torch.cuda.synchronize()
                ms16.append(e0.elapsed_time(e1))
            result["k6144_mbps_16_half_its"] = round(args.batch * 6144 / (min(ms16) * 1e-3) / 1e6, 1)
        result["tdec_8bit"] = bench_8bit(torch, device, args.batch)

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(Ks, data, args.iters, args.cpu_seconds, args.workload)
        if args.workload == "all188" and 6144 in data:
            result["c1_cpu"] = c1_cpu_leg(data, args.iters, min(args.cpu_seconds, 8.0), result.get("k6144_mbps"),
                                          result.get("k6144_mbps_16_half_its"))
    elif rank == 0:
        result["cpu_baseline"] = None

    if args.workload == "all188" and args.pdsch_steps > 0:
        # the PDSCH half of the metric (BASELINE configs[2], C3): the whole UE DL chain, same line
        del data
        torch.cuda.empty_cache()
        pd = run_pdsch(args, torch, dist, world, rank, device, steps=args.pdsch_steps, warmup=3,
                       cpu_seconds=args.pdsch_cpu_seconds if args.cpu_seconds > 0 else 0, emit=False)
        result["pdsch_subframes_per_s"] = pd["config"]["subframes_per_s"]
        result["pdsch"] = {
            "workload": pd["config"]["workload"],
            "subframes_per_s": pd["config"]["subframes_per_s"],
            "subframes_per_s_h2d_inclusive": pd["config"]["subframes_per_s_h2d_inclusive"],
            "h2d_copy_only_subframes_per_s": pd["config"]["h2d_copy_only_subframes_per_s"],
            "subframes_per_s_h2d_sc16_inclusive": pd["config"]["subframes_per_s_h2d_sc16_inclusive"],
            "h2d_sc16_copy_only_subframes_per_s": pd["config"]["h2d_sc16_copy_only_subframes_per_s"],
            "mbps": pd["value"],
            "ms_per_step": pd["ms_per_step"],
            "steps": pd["steps"],
            "tb_ok_fraction": pd["config"]["tb_ok_fraction"],
            "avg_half_iterations": pd["config"]["avg_half_iterations"],
            "roofline": pd["roofline"],
            "stages": pd["stages"],
            "host_enqueue_ms_per_step": pd["host_enqueue_ms_per_step"],
            "step_spread": pd["step_spread"],
            "host_phases_us_per_call": pd["host_phases_us_per_call"],
            "chain_bytes_per_sf": pd["chain_bytes_per_sf"],
            "batch_workers": pd["config"]["batch_workers"],
            "chain_roofline_frac": round(pd["config"]["subframes_per_s"] * pd["chain_bytes_per_sf"]
                                         / (world * HBM_PEAK_GBS * 1e9), 5),
            "cpu_baseline": pd.get("cpu_baseline"),
        }
        if args.pdsch_low_snr > 0:
            # the same chain where the turbo decoder works for its result: several half-iterations a TB
            import copy
            a2 = copy.copy(args)
            a2.snr = args.pdsch_low_snr
            pl = run_pdsch(a2, torch, dist, world, rank, device, steps=args.pdsch_steps, warmup=2, cpu_seconds=0,
                           emit=False)
            result["pdsch_low_snr"] = {
                "snr_db": args.pdsch_low_snr,
                "subframes_per_s": pl["config"]["subframes_per_s"],
                "mbps": pl["value"],
                "ms_per_step": pl["ms_per_step"],
                "avg_half_iterations": pl["config"]["avg_half_iterations"],
                "tb_ok_fraction": pl["config"]["tb_ok_fraction"],
                "turbo_kernel": pl["roofline"]["kernel"],
                "turbo_ms_per_step": pl["stages"].get("tdec_kernel", {}).get("ms_per_step"),
                "batch_workers": pl["config"]["batch_workers"],
            }
        # the uplink counterpart: the eNB PUSCH chain, summary only
        pu = run_pusch(args, torch, dist, world, rank, device, steps=args.pdsch_steps, warmup=2,
                       cpu_seconds=2.0 if args.cpu_seconds > 0 else 0, emit=False)
        result["pusch"] = {
            "workload": pu["config"]["workload"],
            "ue_subframes_per_s": pu["config"]["ue_subframes_per_s"],
            "mbps": pu["value"],
            "ms_per_step": pu["ms_per_step"],
            "tb_ok_fraction": pu["config"]["tb_ok_fraction"],
            "front_end_roofline": pu["front_end_roofline"],
            "batch_workers": pu["config"]["batch_workers"],
            "cpu_baseline": pu.get("cpu_baseline"),
        }

    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit_line(result, args.workload)


if __name__ == "__main__":
    rc = main()
    sys.exit(rc if isinstance(rc, int) else 0)  # the workload runners return their result dict
