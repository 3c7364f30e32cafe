import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-flac_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device and libflacgpu.so")


@pytest.fixture
def diag_build():
    """Skip unless libflacgpu.so is a diagnostic build (`make -C zig-flac_amd diag`, then
    FLACGPU_LIB=zig-flac_amd/build_diag/libflacgpu.so): the measured-slower alternatives (k_ana1,
    the fused kernel, the overlapped schedule) and the diagnostic knobs exist only there."""
    import flacgpu

    if not flacgpu.diag_build():
        pytest.skip("diagnostic build only (make -C zig-flac_amd diag; FLACGPU_LIB=.../build_diag/libflacgpu.so)")
