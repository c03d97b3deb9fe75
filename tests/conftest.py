"""Shared test setup: import paths, the `gpu` marker, the device context fixture."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path[:0] = [str(ROOT / "mapping-private_amd"), str(ROOT / "oracle")]

THR = (147, 146, 148)  # color_voxel_recognition/demos/param/color_threshold.txt


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


@pytest.fixture(scope="session")
def ctx():
    """One HIP context for the GPU tests.  A missing library is an error, not a skip."""
    import c3hlac
    from c3hlac import _capi
    _capi.load()  # raises loudly when libc3hlac_mi355x.so is absent
    try:
        c = c3hlac.Context(0)
    except _capi.C3HError as e:
        if os.environ.get("C3H_REQUIRE_GPU"):
            raise
        pytest.skip("no HIP device: %s" % e)
    yield c
    c.close()


def load_golden(name):
    with np.load(GOLDEN / (name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


GOLDEN_CASES = ["cfg0_parity_64", "cfg1_parity_24", "kinect_40_offsets", "kinect_32_whole"]
