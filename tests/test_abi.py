"""C-ABI boundary checks (CPU only, no kernel launches).

* the in-tree library loads and exports every function declared in include/*.h
* the header compiles as C99 and a C caller links against the library
* the host-side AUTO dispatch equals the reference's (turbodecoder.c:381-424)
* without a HIP device the product fails loudly (no CPU fallback)
"""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from srsran_4g_amd import tdec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_functions():
    names = set()
    for f in os.listdir(INCLUDE):
        if f.endswith(".h"):
            src = open(os.path.join(INCLUDE, f)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            for m in re.finditer(r"^\s*[A-Za-z_][\w\s\*]*?\b(srsran_\w+|create_compact_pcm)\s*\(", src, flags=re.M):
                names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = tdec.load_library()
    names = declared_functions()
    assert len(names) >= 16
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_header_is_c_and_links():
    src = r'''
#include "srsran_tdec.h"
#include "srsran_sch.h"
#include "srsran_phch.h"
#include "srsran_ldpc.h"
#include "srsran_sch_nr.h"
#include <stdio.h>
int main(void) {
  srsran_tdec_t q;
  srsran_sch_t sch;
  srsran_cbsegm_t s;
  printf("%u %zu\n", srsran_tdec_autoimp_get_subblocks(6144), sizeof(srsran_ldpc_decoder_t));
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(srsran_carrier_nr_t), sizeof(srsran_sch_cfg_t), sizeof(srsran_sch_tb_t),
         sizeof(srsran_sch_tb_res_nr_t), sizeof(srsran_sch_nr_args_t), sizeof(srsran_sch_nr_tb_info_t),
         sizeof(srsran_sch_nr_gpu_tb_t));
  if (srsran_cbsegm_ldpc_bg1(&s, 100000) || s.C != 12 || s.Z != 384) return 3;
  if (srsran_sch_nr_select_basegraph(200, 0.9) != BG2) return 4;
  if (0) { srsran_sch_nr_t nr; srsran_sch_nr_args_t na = {0}; srsran_sch_nr_init_rx(&nr, &na);
           srsran_dlsch_nr_decode(&nr, 0, 0, 0, 0); srsran_sch_nr_gpu_decode_batch(&nr, 0, 0, 0, 0, 0);
           srsran_sch_nr_free(&nr); }
  uint16_t pcm[BG1M * BG1Nfull];
  int8_t   pos[BG1M][MAX_CNCT];
  if (create_compact_pcm(pcm, pos, BG1, 384) || pos[4][2] != 26 || pos[4][3] != -1) return 2;
  if (0) { srsran_ldpc_decoder_t d; srsran_ldpc_decoder_args_t a = {0}; srsran_ldpc_decoder_init(&d, &a);
           srsran_ldpc_decoder_decode_c(&d, 0, 0, 0); srsran_ldpc_decoder_free(&d); }
  if (srsran_cbsegm(&s, 75376) || s.C != 13 || s.K1 != 5824) return 1;
  if (0) { srsran_tdec_init(&q, 6144); srsran_tdec_run_all(&q, 0, 0, 8, 6144); srsran_tdec_free(&q); }
  if (0) { srsran_sch_init(&sch); srsran_dlsch_decode(&sch, 0, 0, 0); srsran_sch_free(&sch); }
  if (0) { cf_t x[4]; short l[24]; srsran_demod_soft_demodulate_s(SRSRAN_MOD_64QAM, x, l, 4); }
  return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "caller.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "caller")
        libdir = os.path.dirname(tdec.LIB_PATH)
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", INCLUDE, c, "-L", libdir,
                        "-lsrsran_4g_amd", "-Wl,-rpath," + libdir, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
        from srsran_4g_amd import ldpc
        from srsran_4g_amd import sch_nr as N
        lines = out.split("\n")
        assert lines[0].split() == ["16", str(ctypes.sizeof(ldpc.srsran_ldpc_decoder_t))]
        assert [int(x) for x in lines[1].split()] == [ctypes.sizeof(t) for t in (
            N.srsran_carrier_nr_t, N.srsran_sch_cfg_t, N.srsran_sch_tb_t, N.srsran_sch_tb_res_nr_t,
            N.srsran_sch_nr_args_t, N.srsran_sch_nr_tb_info_t, N.srsran_sch_nr_gpu_tb_t)]


def ref_subblocks(K):
    if K % 16 == 0 and K > 800:
        return 16
    if K % 8 == 0 and K > 400:
        return 8
    return 0


def ref_subblocks_8bit(K):
    if K % 32 == 0 and K > 2048:
        return 32
    return ref_subblocks(K)


def test_auto_dispatch_matches_reference():
    lib = tdec.load_library()
    for K in tdec.CB_SIZES:
        assert lib.srsran_tdec_autoimp_get_subblocks(K) == ref_subblocks(K)
        assert lib.srsran_tdec_autoimp_get_subblocks_8bit(K) == ref_subblocks_8bit(K)


def test_struct_layout():
    assert ctypes.sizeof(tdec.srsran_tdec_t) == 32


@pytest.mark.skipif(tdec.gpu_available(), reason="a HIP device is present")
def test_fails_loudly_without_gpu():
    with pytest.raises(RuntimeError):
        tdec.TurboDecoder()


def test_ldpc_compact_pcm_matches_oracle():
    """create_compact_pcm (host table code of the product) == the oracle's 38.212 tables."""
    from ldpc import LIFT_SIZES, OracleLdpc
    from srsran_4g_amd import ldpc

    ora = OracleLdpc()
    for bg in (0, 1):
        for ls in LIFT_SIZES:
            p, q = ldpc.compact_pcm(bg, ls)
            p0, q0 = ora.pcm(bg, ls)
            assert np.array_equal(p, p0) and np.array_equal(q, q0), (bg, ls)
    with pytest.raises(ValueError):
        ldpc.compact_pcm(0, 17)


@pytest.mark.skipif(tdec.gpu_available(), reason="a HIP device is present")
def test_ldpc_fails_loudly_without_gpu():
    from srsran_4g_amd import ldpc

    with pytest.raises(RuntimeError):
        ldpc.LdpcDecoder(0, 384)


@pytest.mark.skipif(tdec.gpu_available(), reason="a HIP device is present")
def test_nr_sch_fails_loudly_without_gpu():
    from srsran_4g_amd import sch_nr

    with pytest.raises(RuntimeError):
        sch_nr.SchNr()


def test_library_exports_only_the_c_abi():
    """libsrsran_4g_amd.so exports the srsran_* C entry points and nothing else (exports.map): no C++
    helper or kernel symbol can collide with srsRAN's own when the library is linked into it."""
    import subprocess
    so = tdec.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    syms = [ln.split()[-1] for ln in out.splitlines() if ln.strip()]
    bad = [s for s in syms if not s.startswith("srsran_") and s != "create_compact_pcm"]  # base_graph.h:113
    assert syms and not bad, bad[:20]
