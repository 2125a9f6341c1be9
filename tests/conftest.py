import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libqpd.so on cuda:0)")


def golden_files(pattern="*.npz"):
    """Decoder fixtures.  The default pattern gives the LUT and SC decoders'
    fixtures; the LUT-generator (lutgen_*.npz) and float-domain (float_*.npz)
    fixtures and the code-construction pin (codes_*.npz) have their own tests
    and are returned only when asked for."""
    own = ("lutgen_", "float_", "codes_")
    return sorted(p for p in glob.glob(os.path.join(GOLDEN_DIR, pattern))
                  if pattern.startswith(own) or not os.path.basename(p).startswith(own))


def load_golden(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def golden_packed(g):
    from quantized_decoder_polar_codes_amd.lut import PackedLUT

    return PackedLUT(N=int(g["N"]), v=int(g["v"]), lut_f=g["lut_f"], f_base=g["f_base"], f_step=int(g["f_step"]),
                     lut_g=g["lut_g"], g_base=g["g_base"], g_step=int(g["g_step"]),
                     vcl=np.ascontiguousarray(g["vcl"]))


@pytest.fixture(scope="session")
def native_lib():
    from quantized_decoder_polar_codes_amd import build

    build.build_native()
    from quantized_decoder_polar_codes_amd import _lib

    return _lib.load()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.lib()
    return oracle
