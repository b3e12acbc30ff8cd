import os
import subprocess
import sys

import pytest

try:  # one HIP runtime per process: let torch-ROCm load it first (see huygens_amd/_lib.py)
    import torch  # noqa: F401
except Exception:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X) and libhuygens_hip.so")
    # the oracle is test infrastructure: build it on demand (gcc, seconds)
    so = os.path.join(ROOT, "oracle", "_build", "libhz_oracle.so")
    odir = os.path.join(ROOT, "oracle")
    newest = max(os.path.getmtime(os.path.join(odir, f)) for f in os.listdir(odir) if f.endswith((".c", ".h")))
    if not os.path.exists(so) or os.path.getmtime(so) < newest:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session")
def gpu_lib():
    """The HIP library, with a device check; GPU tests fail loudly without it."""
    from huygens_amd import load
    lib = load()
    assert lib.hz_device_count() > 0, "no GPU visible to libhuygens_hip"
    return lib
