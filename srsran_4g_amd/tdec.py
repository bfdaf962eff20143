"""Python mirror of the srsran_tdec_* C API (include/srsran_tdec.h).

The product is the C-ABI shared library ``srsran_4g_amd/lib/libsrsran_4g_amd.so``
(HIP kernels for gfx950).  This module only binds it with ctypes so tests and
bench.py can drive it the way the reference's own C tests drive
lib/src/phy/fec/turbo/turbodecoder.c (turbodecoder_test.c:115-312).  There is no
Python or CPU fallback: if the library or a HIP device is missing, calls raise.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRSRAN_AMD_LIB") or os.path.join(HERE, "lib", "libsrsran_4g_amd.so")  # env override: developer A/B builds only

SRSRAN_SUCCESS = 0
SRSRAN_ERROR = -1
SRSRAN_ERROR_INVALID_INPUTS = -2
SRSRAN_TCOD_MAX_LEN_CB = 6144

# turbodecoder_impl.h:26-36
SRSRAN_TDEC_AUTO = 0
SRSRAN_TDEC_GENERIC = 1
SRSRAN_TDEC_SSE = 2
SRSRAN_TDEC_SSE_WINDOW = 3
SRSRAN_TDEC_NEON_WINDOW = 4
SRSRAN_TDEC_AVX_WINDOW = 5
SRSRAN_TDEC_SSE8_WINDOW = 6
SRSRAN_TDEC_AVX8_WINDOW = 7

CB_SIZES = (
    [40 + 8 * i for i in range(60)]
    + [528 + 16 * i for i in range(32)]
    + [1056 + 32 * i for i in range(32)]
    + [2112 + 64 * i for i in range(64)]
)


class srsran_tdec_t(ctypes.Structure):
    """Layout of srsran_tdec_t in include/srsran_tdec.h."""

    _fields_ = [
        ("max_long_cb", ctypes.c_uint32),
        ("force_not_sb", ctypes.c_bool),
        ("dec_type", ctypes.c_int),
        ("current_long_cb", ctypes.c_uint32),
        ("current_cbidx", ctypes.c_int),
        ("n_iter", ctypes.c_int),
        ("gpu", ctypes.c_void_p),
    ]


_i16p = ctypes.POINTER(ctypes.c_int16)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_lib = None


def load_library():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C srsran_4g_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER(srsran_tdec_t)
    u32 = ctypes.c_uint32
    sig = {
        "srsran_tdec_init": ([P, u32], ctypes.c_int),
        "srsran_tdec_init_manual": ([P, u32, ctypes.c_int], ctypes.c_int),
        "srsran_tdec_free": ([P], None),
        "srsran_tdec_force_not_sb": ([P], None),
        "srsran_tdec_new_cb": ([P, u32], ctypes.c_int),
        "srsran_tdec_get_nof_iterations": ([P], ctypes.c_int),
        "srsran_tdec_autoimp_get_subblocks": ([u32], u32),
        "srsran_tdec_autoimp_get_subblocks_8bit": ([u32], u32),
        "srsran_tdec_iteration": ([P, _i16p, _u8p], None),
        "srsran_tdec_run_all": ([P, _i16p, _u8p, u32, u32], ctypes.c_int),
        "srsran_tdec_iteration_8bit": ([P, ctypes.POINTER(ctypes.c_int8), _u8p], None),
        "srsran_tdec_run_all_8bit": ([P, ctypes.POINTER(ctypes.c_int8), _u8p, u32, u32], ctypes.c_int),
        "srsran_tdec_run_all_batch": ([P, _i16p, u32, _u8p, u32, u32, u32], ctypes.c_int),
        "srsran_tdec_gpu_run_batch": ([u32, ctypes.c_void_p, u32, ctypes.c_int, ctypes.c_void_p, u32, u32,
                                       ctypes.c_void_p], ctypes.c_int),
        "srsran_tdec_gpu_run_batch_8bit": ([u32, ctypes.c_void_p, u32, ctypes.c_int, ctypes.c_void_p, u32, u32,
                                            ctypes.c_void_p], ctypes.c_int),
        "srsran_tdec_gpu_run_multi": ([u32, ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(u32),
                                       ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(u32), u32,
                                       ctypes.c_void_p], ctypes.c_int),
        "srsran_tdec_gpu_available": ([], ctypes.c_int),
        "srsran_tdec_gpu_kernel_name": ([u32], ctypes.c_char_p),
        "srsran_tdec_gpu_kernel_name_batch": ([u32, u32], ctypes.c_char_p),
        "srsran_tdec_gpu_last_kernel": ([], ctypes.c_char_p),
        "srsran_tdec_gpu_set_pair_threshold": ([u32], None),
        "srsran_tdec_gpu_get_pair_threshold": ([], u32),
        "srsran_tdec_gpu_set_single_threshold": ([u32], None),
        "srsran_tdec_gpu_get_single_threshold": ([], u32),
        "srsran_tdec_gpu_set_class_single_threshold": ([u32, u32], None),
        "srsran_tdec_gpu_get_class_single_threshold": ([u32], u32),
        "srsran_tdec_gpu_set_generic_single_threshold": ([u32], None),
        "srsran_tdec_gpu_set_w8_max_k": ([u32], None),
        "srsran_tdec_gpu_get_w8_max_k": ([], u32),
        "srsran_tdec_gpu_set_w8_fused_max_k": ([u32], None),
        "srsran_tdec_gpu_get_w8_fused_max_k": ([], u32),
        "srsran_tdec_gpu_get_generic_single_threshold": ([], u32),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    _lib = lib
    return lib


def last_kernel():
    """Name of the last turbo-decoder kernel this thread launched (srsran_tdec_gpu_last_kernel)."""
    return load_library().srsran_tdec_gpu_last_kernel().decode()


class pair_threshold:
    """Context manager: blocks per launch from which the lane-pair decoder runs
    (srsran_tdec_gpu_set_pair_threshold), restored on exit."""

    def __init__(self, nof_cb):
        self.n = nof_cb

    def __enter__(self):
        lib = load_library()
        self.old = lib.srsran_tdec_gpu_get_pair_threshold()
        lib.srsran_tdec_gpu_set_pair_threshold(self.n)
        return self

    def __exit__(self, *exc):
        load_library().srsran_tdec_gpu_set_pair_threshold(self.old)


class w8_max_k(pair_threshold):
    """block sizes up to which the single-lane decoders run their 8-step-window build
    (srsran_tdec_gpu_set_w8_max_k)"""

    def __enter__(self):
        lib = load_library()
        self.old = lib.srsran_tdec_gpu_get_w8_max_k()
        lib.srsran_tdec_gpu_set_w8_max_k(self.n)
        return self

    def __exit__(self, *exc):
        load_library().srsran_tdec_gpu_set_w8_max_k(self.old)


class w8_fused_max_k(pair_threshold):
    """the 16-sub-block class's cut in fused multi-size launches: sizes up to it on 8-step windows
    (srsran_tdec_gpu_set_w8_fused_max_k)"""

    def __enter__(self):
        lib = load_library()
        self.old = lib.srsran_tdec_gpu_get_w8_fused_max_k()
        lib.srsran_tdec_gpu_set_w8_fused_max_k(self.n)
        return self

    def __exit__(self, *exc):
        load_library().srsran_tdec_gpu_set_w8_fused_max_k(self.old)


class class_single_threshold:
    """Context manager: blocks per launch from which the single-lane decoders of the given classes
    (16, 8, 0 = generic) run (srsran_tdec_gpu_set_class_single_threshold), each restored on exit."""
    classes = (16, 8)

    def __init__(self, nof_cb, classes=None):
        self.n = nof_cb
        if classes is not None:
            self.classes = tuple(classes)

    def __enter__(self):
        lib = load_library()
        self.old = {c: lib.srsran_tdec_gpu_get_class_single_threshold(c) for c in self.classes}
        for c in self.classes:
            lib.srsran_tdec_gpu_set_class_single_threshold(c, self.n)
        return self

    def __exit__(self, *exc):
        lib = load_library()
        for c, n in self.old.items():
            lib.srsran_tdec_gpu_set_class_single_threshold(c, n)


class single_threshold(class_single_threshold):
    """the 16- and 8-sub-block classes (srsran_tdec_gpu_set_single_threshold)"""
    classes = (16, 8)


class generic_single_threshold(class_single_threshold):
    """the generic class (srsran_tdec_gpu_set_generic_single_threshold)"""
    classes = (0,)


def nof_subblocks(K):
    return load_library().srsran_tdec_autoimp_get_subblocks(K)


def input_len(K, layout_sb):
    return 3 * (K + 32) + 12 if (layout_sb and nof_subblocks(K)) else 3 * K + 12


def gpu_available():
    return bool(load_library().srsran_tdec_gpu_available())


class TurboDecoder:
    """srsran_tdec_t object: init / new_cb / iteration / run_all / free."""

    def __init__(self, max_long_cb=SRSRAN_TCOD_MAX_LEN_CB, dec_type=SRSRAN_TDEC_AUTO):
        self.lib = load_library()
        self.h = srsran_tdec_t()
        rc = self.lib.srsran_tdec_init_manual(ctypes.byref(self.h), max_long_cb, dec_type)
        if rc != SRSRAN_SUCCESS:
            raise RuntimeError(f"srsran_tdec_init_manual failed ({rc}); is a HIP device visible?")

    def free(self):
        if self.h.gpu:
            self.lib.srsran_tdec_free(ctypes.byref(self.h))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def force_not_sb(self):
        self.lib.srsran_tdec_force_not_sb(ctypes.byref(self.h))

    @property
    def layout_sb(self):
        return not self.h.force_not_sb

    def new_cb(self, K):
        return self.lib.srsran_tdec_new_cb(ctypes.byref(self.h), K)

    def get_nof_iterations(self):
        return self.lib.srsran_tdec_get_nof_iterations(ctypes.byref(self.h))

    def iteration(self, llr):
        """One half-iteration + hard decision (srsran_tdec_iteration)."""
        llr = np.ascontiguousarray(llr, dtype=np.int16)
        K = self.h.current_long_cb
        out = np.zeros(K // 8, dtype=np.uint8)
        n0 = self.h.n_iter
        self.lib.srsran_tdec_iteration(ctypes.byref(self.h), llr.ctypes.data_as(_i16p), out.ctypes.data_as(_u8p))
        if self.h.n_iter != n0 + 1:
            raise RuntimeError("srsran_tdec_iteration failed")
        return out

    def run_all(self, llr, nof_iterations, K):
        llr = np.ascontiguousarray(llr, dtype=np.int16)
        out = np.zeros(K // 8, dtype=np.uint8)
        rc = self.lib.srsran_tdec_run_all(ctypes.byref(self.h), llr.ctypes.data_as(_i16p),
                                          out.ctypes.data_as(_u8p), nof_iterations, K)
        if rc != SRSRAN_SUCCESS:
            raise RuntimeError(f"srsran_tdec_run_all failed ({rc})")
        return out

    def run_all_8bit(self, llr, nof_iterations, K):
        """srsran_tdec_run_all_8bit: int8 LLRs."""
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        out = np.zeros(K // 8, dtype=np.uint8)
        rc = self.lib.srsran_tdec_run_all_8bit(ctypes.byref(self.h), llr.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
                                               out.ctypes.data_as(_u8p), nof_iterations, K)
        if rc != SRSRAN_SUCCESS:
            raise RuntimeError(f"srsran_tdec_run_all_8bit failed ({rc})")
        return out

    def iteration_8bit(self, llr):
        """One more half-iteration + hard decision (srsran_tdec_iteration_8bit)."""
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        K = self.h.current_long_cb
        out = np.zeros(K // 8, dtype=np.uint8)
        n0 = self.h.n_iter
        self.lib.srsran_tdec_iteration_8bit(ctypes.byref(self.h), llr.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
                                            out.ctypes.data_as(_u8p))
        if self.h.n_iter != n0 + 1:
            raise RuntimeError("srsran_tdec_iteration_8bit failed")
        return out

    def run_all_batch(self, llr2d, nof_iterations, K):
        llr2d = np.ascontiguousarray(llr2d, dtype=np.int16)
        n = llr2d.shape[0]
        out = np.zeros((n, K // 8), dtype=np.uint8)
        rc = self.lib.srsran_tdec_run_all_batch(ctypes.byref(self.h), llr2d.ctypes.data_as(_i16p), llr2d.shape[1],
                                                out.ctypes.data_as(_u8p), n, nof_iterations, K)
        if rc != SRSRAN_SUCCESS:
            raise RuntimeError(f"srsran_tdec_run_all_batch failed ({rc})")
        return out


def gpu_run_batch(K, d_in, in_stride, layout_sb, d_out, nof_cb, nof_iterations, stream=None):
    """Device-resident batch decode (pointers are device addresses, async on stream)."""
    rc = load_library().srsran_tdec_gpu_run_batch(K, d_in, in_stride, int(bool(layout_sb)), d_out, nof_cb,
                                                  nof_iterations, stream)
    if rc != SRSRAN_SUCCESS:
        raise RuntimeError(f"srsran_tdec_gpu_run_batch failed ({rc})")


def gpu_run_batch_8bit(K, d_in, in_stride, layout_sb, d_out, nof_cb, nof_iterations, stream=None):
    """Device-resident batch decode of int8 code blocks (srsran_tdec_gpu_run_batch_8bit)."""
    rc = load_library().srsran_tdec_gpu_run_batch_8bit(K, d_in, in_stride, int(bool(layout_sb)), d_out, nof_cb,
                                                       nof_iterations, stream)
    if rc != SRSRAN_SUCCESS:
        raise RuntimeError(f"srsran_tdec_gpu_run_batch_8bit failed ({rc})")


def gpu_run_multi(Ks, d_ins, strides, layout_sb, d_outs, ncbs, nof_iterations, stream=None):
    """Device-resident multi-size batch (srsran_tdec_gpu_run_multi): one group per code-block size."""
    n = len(Ks)
    u32 = ctypes.c_uint32
    vp = ctypes.c_void_p
    rc = load_library().srsran_tdec_gpu_run_multi(
        n, (u32 * n)(*Ks), (vp * n)(*d_ins), (u32 * n)(*strides), int(bool(layout_sb)), (vp * n)(*d_outs),
        (u32 * n)(*ncbs), nof_iterations, stream)
    if rc != SRSRAN_SUCCESS:
        raise RuntimeError(f"srsran_tdec_gpu_run_multi failed ({rc})")
