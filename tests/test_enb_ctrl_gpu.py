"""eNB control channels transmitted on the GPU (srsran_enb_dl_gpu_tx_batch with srsran_enb_dl_gpu_ctrl_t:
ctrl_tx_kernel) against the reference's own transmitter code (oracle/_ref, ref_enb_ctrl_harness.c):
PSS / SSS (subframes 0 and 5), PBCH with the MIB of SFN tti / 10 (subframe 0, every SFN mod 4 quarter),
PCFICH and the PDCCH messages of srsran_pdcch_encode, on 1 / 2 / 4 ports, normal and extended CP, cell
sizes 6..100 PRB, every CFI, several subframes of one batch, DCIs of every aggregation level and a later
DCI overwriting CCEs of an earlier one.  The control REs of the GPU grids (srsran_enb_dl_gpu_sf_symbols,
minus the CRS of a batch without control channels) equal the reference grids."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pdcch as OP  # noqa: E402  (oracle/pdcch.py)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from srsran_4g_amd import tdec
    if not tdec.gpu_available():
        pytest.skip("no HIP device")
    if not OP.ref_available():
        pytest.fail("oracle/_ref/libsrsref.so missing: build it with `make -C oracle` (never skipped on a GPU box)")
    import torch
    return torch, OP.Ref()


def _msgs(rng, nof_cce, spec):
    """spec: list of (L, ncce or None) -> [(bits, L, ncce, rnti)]"""
    out = []
    for L, ncce in spec:
        n = 1 << L
        if ncce is None:
            ncce = int(rng.integers(0, nof_cce // n)) * n
        bits = rng.integers(0, 2, int(rng.integers(20, 58)), dtype=np.uint8)
        out.append((bits, L, ncce, int(rng.integers(1, 0xFFF4))))
    return out


def _run(torch, ref, nprb, ports, cell_id, cp, subframes, phich_res=2):
    """subframes: list of (tti, cfi, put_base, msgs).  GPU grids (control only) vs reference grids."""
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import pdcch as PD
    from srsran_4g_amd import ue_dl as U
    from srsran_4g_amd.sch import _memcpy_d2h
    U.use_standard_symbol_size(True)
    cell = PD.cell(nprb, ports, cell_id, phich_len=0, phich_res=phich_res, cp=cp)
    enb = E.EnbDl(cell)
    nsymb = 7 if cp == 0 else 6
    nre = 12 * nprb
    N = {6: 128, 15: 256, 25: 512, 50: 1024, 75: 1536, 100: 2048}[nprb]
    sf_len = 15 * N  # SRSRAN_SF_LEN: 1 ms for either CP
    d_out = torch.zeros((len(subframes), ports, sf_len, 2), dtype=torch.float32, device="cuda")

    def grids(with_ctrl):
        sfs = []
        for tti, cfi, put_base, msgs in subframes:
            ctrl = None
            if with_ctrl:
                ms = []
                for bits, L, ncce, rnti in msgs:
                    m = PD.srsran_dci_msg_t()
                    m.payload[:len(bits)] = [int(b) for b in bits]
                    m.nof_bits, m.rnti = len(bits), rnti
                    m.location.L, m.location.ncce = L, ncce
                    ms.append(m)
                ctrl = (put_base, ms)
            sfs.append((tti, cfi, None, [], ctrl))
        assert enb.tx_batch(sfs, d_out.data_ptr(), 1.0) == 0
        torch.cuda.synchronize()
        ptr = enb.sf_symbols()
        assert ptr
        n = len(subframes) * ports * 2 * nsymb * nre
        host = torch.empty(2 * n, dtype=torch.float32)
        _memcpy_d2h(host, ptr, n * 8)
        host = host.numpy().view(np.complex64)
        return host.reshape(len(subframes), ports, 2 * nsymb, nre)

    crs_only = grids(False)
    got = grids(True) - crs_only
    enb.free()
    for i, (tti, cfi, put_base, msgs) in enumerate(subframes):
        want = ref.enb_ctrl_tx(nprb, ports, cell_id, tti, cfi, msgs, put_base=put_base, cp=cp, phich_res=phich_res)
        want = want[:, :2 * nsymb, :]
        err = np.abs(got[i] - want)
        assert err.max() < 1e-6, (i, tti, float(err.max()), np.argwhere(err > 1e-6)[:5].tolist())
        assert np.count_nonzero(np.abs(want) > 0) > 0


CELLS = [  # (nof_prb, ports, cell_id, cp)
    (6, 1, 0, 0),
    (15, 2, 101, 0),
    (25, 2, 37, 0),
    (50, 4, 250, 0),
    (100, 2, 503, 0),
    (100, 1, 77, 0),
    (25, 2, 38, 1),
    (75, 4, 2, 1),
]


@pytest.mark.parametrize("cell", CELLS, ids=[f"{c[0]}prb_{c[1]}p_id{c[2]}_{'ext' if c[3] else 'norm'}" for c in CELLS])
def test_put_base_and_pdcch_match_reference(env, cell):
    torch, ref = env
    nprb, ports, cell_id, cp = cell
    rng = np.random.default_rng(nprb * 7 + cell_id)
    from srsran_4g_amd import pdcch as PD
    regs = PD.Regs(PD.cell(nprb, ports, cell_id, cp=cp))
    subframes = []
    for k, tti in enumerate((0, 10, 25, 3, 35, 1020, 5, 9)):  # subframes 0 (all 4 SFN quarters), 5, others
        cfi = 1 + k % 3
        nof_cce = regs.q.pdcch_nregs[cfi - 1] // 9
        spec = [(L, None) for L in range(4) if (1 << L) <= nof_cce][: 1 + k % 4]
        subframes.append((tti, cfi, True, _msgs(rng, nof_cce, spec)))
    regs.free()
    _run(torch, ref, nprb, ports, cell_id, cp, subframes)


def test_overlapping_dci_later_wins(env):
    """two messages sharing CCEs: the later one's symbols on the shared CCEs, the earlier one's elsewhere"""
    torch, ref = env
    rng = np.random.default_rng(9)
    msgs = _msgs(rng, 20, [(2, 4), (1, 6), (0, 4), (3, 0)])
    _run(torch, ref, 25, 2, 11, 0, [(7, 3, True, msgs), (8, 2, False, msgs[:2])])


def test_pdcch_only_and_phich_resources(env):
    torch, ref = env
    rng = np.random.default_rng(12)
    for res in (0, 1, 3):
        from srsran_4g_amd import pdcch as PD
        regs = PD.Regs(PD.cell(50, 2, 19, phich_res=res))
        nof_cce = regs.q.pdcch_nregs[1] // 9
        regs.free()
        _run(torch, ref, 50, 2, 19, 0, [(4, 2, False, _msgs(rng, nof_cce, [(0, None), (2, None)]))], phich_res=res)


def test_illegal_dci_location_refused(env):
    torch, _ = env
    from srsran_4g_amd import enb_dl as E
    from srsran_4g_amd import pdcch as PD
    cell = PD.cell(6, 1, 1)
    enb = E.EnbDl(cell)
    m = PD.srsran_dci_msg_t()
    m.nof_bits, m.rnti = 27, 0x46
    m.location.L, m.location.ncce = 3, 8  # past the CCEs of a 6-PRB cell
    d_out = torch.zeros((1, 1, 15 * 128, 2), dtype=torch.float32, device="cuda")
    assert enb.tx_batch([(1, 1, None, [], (False, [m]))], d_out.data_ptr(), 1.0) != 0
    enb.free()
