"""Per-stage HIP-event kernel timing of the GPU pipeline (include/srsran_amd_prof.h)."""
import ctypes

from .tdec import load_library

NOF_STAGES = 12
NOF_HOST_PHASES = 8
_bound = False


def _lib():
    global _bound
    L = load_library()
    if not _bound:
        L.srsran_amd_timing_enable.argtypes = [ctypes.c_int]
        L.srsran_amd_timing_enable.restype = None
        L.srsran_amd_timing_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.srsran_amd_timing_read.restype = ctypes.c_int
        L.srsran_amd_stage_name.argtypes = [ctypes.c_int]
        L.srsran_amd_stage_name.restype = ctypes.c_char_p
        L.srsran_amd_host_timing_enable.argtypes = [ctypes.c_int]
        L.srsran_amd_host_timing_enable.restype = None
        L.srsran_amd_host_timing_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.srsran_amd_host_timing_read.restype = ctypes.c_int
        L.srsran_amd_host_phase_name.argtypes = [ctypes.c_int]
        L.srsran_amd_host_phase_name.restype = ctypes.c_char_p
        _bound = True
    return L


def enable(on=True):
    _lib().srsran_amd_timing_enable(1 if on else 0)


def read():
    """-> {kernel name: (total ms, launches)} for the stages that launched, and clears them"""
    ms = (ctypes.c_float * NOF_STAGES)()
    n = (ctypes.c_uint32 * NOF_STAGES)()
    _lib().srsran_amd_timing_read(ms, n)
    return {_lib().srsran_amd_stage_name(i).decode(): (float(ms[i]), int(n[i])) for i in range(NOF_STAGES) if n[i]}


def host_enable(on=True):
    """host-side phase timers of the batch APIs (wall clock of the calling thread)"""
    _lib().srsran_amd_host_timing_enable(1 if on else 0)


def host_read():
    """-> {phase name: (total us, calls)} for the phases that ran, and clears them"""
    us = (ctypes.c_double * NOF_HOST_PHASES)()
    n = (ctypes.c_uint32 * NOF_HOST_PHASES)()
    _lib().srsran_amd_host_timing_read(us, n)
    return {_lib().srsran_amd_host_phase_name(i).decode(): (float(us[i]), int(n[i]))
            for i in range(NOF_HOST_PHASES) if n[i]}
