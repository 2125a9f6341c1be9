"""codes.construct_pw / codes.identify_nodes against the reference's own
PolarCodeConstructor.PW and NodeIdentifier.run (CodeConstruction.py:65-84,
IdentifyNodes.py:13-150), run by tests/golden/make_code_golden.py for 49
codes N = 16..1024 and both use_new_node settings."""
import os

import numpy as np
import pytest

from quantized_decoder_polar_codes_amd import codes as C

Z = np.load(os.path.join(os.path.dirname(__file__), "golden", "codes_pw_nodes.npz"))
CASES = [tuple(int(x) for x in c) for c in Z["cases"]]


@pytest.mark.parametrize("N,K", CASES)
def test_pw_and_node_labels_match_reference(N, K):
    _, msgbits, fmask, mmask = C.construct_pw(N, K)
    assert np.array_equal(fmask, Z[f"frozen_{N}_{K}"])
    assert np.array_equal(mmask, 1 - Z[f"frozen_{N}_{K}"])
    for new in (0, 1):
        got = C.identify_nodes(N, msgbits, use_new_node=bool(new))
        assert np.array_equal(got.astype(np.int8), Z[f"nodes{new}_{N}_{K}"]), f"use_new_node={bool(new)}"
