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
