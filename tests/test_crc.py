"""CRC-aided decoding pieces that run without a GPU: the register form of the
reference's CRC::encoding (the one the kernels and the Monte-Carlo generator
use) against the reference's bit-array division as restated in the oracle,
and the oracle's CA decoders against the golden fixtures (expected outputs
from the reference CASCLLUT / CAFastSCLLUT compiled from their own sources)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

from conftest import golden_files, golden_packed, load_golden  # noqa: E402


def crc_register(info, crc_n, loc):
    """The MSB-first register form used on the device (qpd_common.hpp:
    ca_winner, qpd_mc.hip): coefficient j >= 1 -> register bit crc_n - j."""
    q = 0
    for j in loc:
        if j >= 1:
            q |= 1 << (crc_n - j)
    top, mask = 1 << (crc_n - 1), (1 << crc_n) - 1
    out = []
    for row in np.atleast_2d(info):
        r = 0
        for b in row:
            fb = int(b) ^ (1 if r & top else 0)
            r = ((r << 1) & mask) ^ (q if fb else 0)
        out.append([(r >> (crc_n - 1 - j)) & 1 for j in range(crc_n)])
    return np.array(out, dtype=np.uint8)


@pytest.mark.parametrize("crc_n,loc", [
    (24, O.CRC24_LOC),
    (11, (11, 10, 9, 5, 0)),   # 5G CRC11
    (6, (6, 5, 0)),            # 5G CRC6
    (8, (7, 3, 1)),            # no leading / trailing coefficient: the leading one only clears the bit
    (32, (32, 26, 23, 22, 16, 12, 11, 10, 8, 7, 5, 4, 2, 1, 0)),
])
def test_crc_register_form_equals_reference_division(crc_n, loc):
    rng = np.random.default_rng(crc_n)
    for A in (1, 7, 40, 200):
        info = rng.integers(0, 2, size=(20, A), dtype=np.uint8)
        assert np.array_equal(crc_register(info, crc_n, loc), O.crc_encode(info, crc_n, loc))


CA_FILES = golden_files("ca_*.npz")


def test_ca_fixtures_exist():
    assert len(CA_FILES) >= 4


def test_ca_fixtures_exercise_the_crc():
    # the fixtures are only a pin if the CRC changes the chosen path on some frames
    seen = 0
    for path in CA_FILES:
        g = load_golden(path)
        plain = O.decode_lut(str(g["kind"])[3:], golden_packed(g), int(g["K"]), int(g["L"]), g["frozen"],
                             g["symbols"].astype(np.int32), g["node_type"])[:, : int(g["A"])]
        seen += int((plain != g["expected"]).any(1).sum())
    assert seen > 0
