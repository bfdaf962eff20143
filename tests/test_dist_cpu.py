"""Multi-process path of bench.py on CPU (gloo, world size 2): every rank times the same region
between barriers and reports the MAX over ranks; ranks own disjoint carriers (no
data-path collective) -- here each rank decodes its own synthetic C3 carrier with the CPU oracle
chain, the stand-in for its GPU."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import time

    import torch.distributed as dist

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle import Oracle
    import pdsch_chain as PC
    from synth import synth as S

    sh = bench.shard(rank)
    rng = np.random.default_rng(sh["seed"])
    tbs = 75376
    pls = [rng.integers(0, 256, tbs // 8, dtype=np.uint8) for _ in range(2)]
    x, nre = S.pdsch_subframe(100, sh["cell_id"], 2, 1, 1, 0x1234, tbs, 6, 0, pls, snr_db=30.0, rng=rng)
    ora = Oracle()
    decoded = []

    def step():
        time.sleep(0.02 * (rank + 1))
        g, ce, st = PC.fft_estimate(ora, x, 100, sh["cell_id"], 2, 1)
        res = PC.pdsch_decode(ora, g, ce, st["noise"], 100, sh["cell_id"], 2, 1, 1, 0x1234, [tbs, tbs], [6, 6],
                              [0, 0])
        decoded.append(all(r["ret"] == 0 and np.array_equal(r["data"][: tbs // 8], p) for r, p in zip(res, pls)))

    t0 = time.perf_counter()
    elapsed = bench.timed_region(step, 3, 1, world, dist, lambda: None, "cpu")
    local = time.perf_counter() - t0
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump({"elapsed": elapsed, "local": local, "cell": sh["cell_id"], "ok": all(decoded),
                   "n": len(decoded)}, f)
    dist.destroy_process_group()


def test_bench_timed_region_gloo_world2(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [json.load(open(tmp_path / f"r{i}.json")) for i in range(2)]
    assert r[0]["elapsed"] == pytest.approx(r[1]["elapsed"])  # max over ranks, identical everywhere
    assert r[0]["elapsed"] >= 3 * 0.04                          # at least the slower rank's 3 steps
    assert r[0]["cell"] != r[1]["cell"]                         # disjoint carriers
    assert all(x["ok"] and x["n"] == 4 for x in r)              # warmup + 3 timed steps, all decoded


def _run_bench(args, env_extra=None, timeout=180):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_gpus_spawns_ranks(n):
    """bench.py --gpus N with no launcher starts N rank processes itself (children, before any GPU call):
    one JSON line from rank 0 with n_gpus N, LOCAL_RANK r -> device cuda:r, disjoint cells and seeds"""
    p = _run_bench(["--gpus", str(n), "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == n
    assert [r["rank"] for r in d["ranks"]] == list(range(n))
    assert [r["device"] for r in d["ranks"]] == [f"cuda:{r}" for r in range(n)]
    assert len({r["cell_id"] for r in d["ranks"]}) == n and len({r["seed"] for r in d["ranks"]}) == n


def test_bench_torchrun_launcher_8_ranks():
    """the driver's own N = 8 launch line (torch.distributed.run, one process per GPU, rendezvous on
    127.0.0.1), as a dry run: 8 ranks, LOCAL_RANK r -> cuda:r, disjoint carriers (the C4 layout)"""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 8
    assert sorted(r["rank"] for r in d["ranks"]) == list(range(8))
    assert all(r["device"] == f"cuda:{r['local_rank']}" for r in d["ranks"])
    assert len({r["cell_id"] for r in d["ranks"]}) == 8 and len({r["seed"] for r in d["ranks"]}) == 8


def test_bench_world_size_disagreeing_with_gpus_fails():
    """under a launcher, WORLD_SIZE must equal --gpus when --gpus is given"""
    p = _run_bench(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_bench_single_rank_under_launcher_env():
    """WORLD_SIZE=1 (a launcher with one process) and no --gpus: one rank, no spawn"""
    p = _run_bench(["--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["ranks"][0]["device"] == "cuda:0"
