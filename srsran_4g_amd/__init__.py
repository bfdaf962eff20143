"""srsran_4g_amd: MI355X-native LTE downlink receive hot path (turbo decoder first).

The product is the C-ABI library built from srsran_4g_amd/csrc (HIP for gfx950),
declared in include/srsran_tdec.h.  ``srsran_4g_amd.tdec`` binds it for Python.
"""
from . import tdec  # noqa: F401
from . import sch  # noqa: F401
from . import phch  # noqa: F401
from . import ue_dl  # noqa: F401
from . import prof  # noqa: F401
