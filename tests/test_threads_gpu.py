"""One process, several host threads, each owning its own srsran_tdec_t / srsran_sch_t (and so its own
HIP stream), decoding concurrently -- the "one host thread per carrier / per GPU" layout SURVEY
§8b/§8e allows next to one process per GPU.  Checks the process-wide device-table caches (QPP tables,
rate de-matching tables, CRC shift tables: built lazily, guarded by a mutex and keyed by device) under
concurrent first use, and every decode bit-exact against the oracle.  With two or more GPUs visible
the threads are spread over devices (each thread selects its device first), so a table built on one
device is never handed to a kernel on another."""
import threading

import numpy as np
import pytest
import torch

from oracle import Oracle, make_llrs

pytestmark = pytest.mark.gpu

NTHREADS = 4


def _run_threads(fn):
    errors = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors.append((i, repr(e)))

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(NTHREADS)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a decoding thread hung"
    assert not errors, errors


def test_tdec_threads_bit_exact():
    from srsran_4g_amd import tdec
    ora = Oracle()
    ndev = torch.cuda.device_count()
    rng = np.random.default_rng(31)
    # sizes of all three decoder classes, a different set per thread, some shared between threads
    sizes = [(6144, 2016, 416), (5056, 2016, 40), (1024, 800, 104), (6144, 3392, 408)]
    cases = []
    for i in range(NTHREADS):
        per = []
        for K in sizes[i]:
            _, llr = make_llrs(K, 2.0, rng, 6, ora)
            if tdec.nof_subblocks(K):
                llr = np.stack([ora.natural_to_sb(K, x) for x in llr])
            per.append((K, llr, ora.run_batch(K, llr, tdec.nof_subblocks(K) > 0, 8)))
        cases.append(per)

    def work(i):
        torch.cuda.set_device(i % ndev)
        dec = tdec.TurboDecoder()
        for _ in range(3):
            for K, llr, want in cases[i]:
                got = dec.run_all_batch(llr, 8, K)
                assert np.array_equal(got, want), (i, K)
        dec.free()

    _run_threads(work)


def test_dlsch_threads_bit_exact():
    from srsran_4g_amd import sch
    ora = Oracle()
    ndev = torch.cuda.device_count()
    rng = np.random.default_rng(32)
    grants = [(75376, 6, 0, 86400), (36696, 6, 0, 43200), (18336, 4, 0, 27600), (30576, 4, 2, 36000)]
    cases = []
    for i in range(NTHREADS):
        tbs, Qm, rv, G = grants[i]
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        e = ora.dlsch_encode(tbs, Qm, rv, G, tb, 0).astype(np.float32) * 2 - 1
        e = e + rng.standard_normal(e.shape).astype(np.float32) * 0.5
        llr = np.trunc(100 * e).astype(np.int16)
        oret, odata, _, oavg, _ = ora.dlsch_decode(tbs, Qm, rv, llr, 8, None)
        cases.append((tbs, Qm, rv, llr, oret, odata, oavg))

    def work(i):
        torch.cuda.set_device(i % ndev)
        q = sch.Sch()
        q.set_max_noi(8)
        tbs, Qm, rv, llr, oret, odata, oavg = cases[i]
        for _ in range(3):
            sb = sch.SoftbufferRx(nof_prb=100)
            ret, data, avg = q.decode(sb, tbs, Qm, rv, llr)
            assert ret == oret, i
            assert np.array_equal(data[: len(odata)], odata), i
            assert avg == pytest.approx(oavg, abs=0), i
            sb.free()
        q.free()

    _run_threads(work)
