import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's): whichever
# loads first serves the whole process.  Import torch before the decoder library
# so tests that mix torch device buffers with libsrsran_4g_amd share one runtime.
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


import pytest  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _reset_symbol_size():
    """srsran_use_standard_symbol_size is process-global: every module ends with the library default
    (3/4 sampling rates, phy_common.c:31-35), whatever its tests selected, so no result depends on
    module order."""
    yield
    mod = sys.modules.get("srsran_4g_amd.ue_dl")
    if mod is not None:
        try:
            mod.use_standard_symbol_size(False)
        except Exception:  # library not loadable: nothing was changed
            pass
