"""The CPU oracle (oracle/qpd_oracle.cpp) is pinned against the reference:
(1) the committed golden vectors, produced by the reference decoders compiled
from /root/reference (tests/golden/make_golden.py), and (2) when that build is
present, the reference itself on fresh random tie-heavy tables."""
import os

import numpy as np
import pytest

from conftest import golden_files, golden_packed, load_golden


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_matches_golden(path, oracle_mod):
    g = load_golden(path)
    N, K, L = int(g["N"]), int(g["K"]), int(g["L"])
    if str(g["kind"]) == "SC":
        got = oracle_mod.decode_sc_float(N, K, g["frozen"], g["llr"])
    elif str(g["kind"]).startswith("CA-"):
        got = oracle_mod.decode_lut_ca(str(g["kind"]), golden_packed(g), K, int(g["A"]), L, g["frozen"],
                                       g["symbols"].astype(np.int32), node_type=g["node_type"])
    else:
        got = oracle_mod.decode_lut(str(g["kind"]), golden_packed(g), K, L, g["frozen"],
                                    g["symbols"].astype(np.int32), node_type=g["node_type"])
    assert got.shape == g["expected"].shape
    bad = np.flatnonzero((got != g["expected"]).any(1))
    assert bad.size == 0, f"{bad.size} frames differ, first {bad[:5]}"


def _ref_decoder(R, kind, N, K, L, fm, mm, nt, fs, gs, vcl):
    if kind == "SC-LUT":
        return R.SCLUTDecoder(N, K, fm, mm, fs, gs, vcl)
    if kind == "SCL-LUT":
        return R.SCLLUTDecoder(N, K, L, fm, mm, fs, gs, vcl)
    if kind == "FastSC-LUT":
        return R.FastSCLUTDecoder(N, K, fm, mm, nt, fs, gs, vcl)
    return R.FastSCLLUTDecoder(N, K, L, fm, mm, nt, fs, gs, vcl)


CASES = [(4, 2, 2), (16, 8, 4), (32, 13, 3), (128, 32, 8), (128, 64, 8), (256, 100, 5), (1024, 512, 8)]


@pytest.mark.parametrize("N,K,L", CASES)
@pytest.mark.parametrize("kind", ["SC-LUT", "SCL-LUT", "FastSC-LUT", "FastSCL-LUT"])
def test_oracle_vs_reference_random(N, K, L, kind, oracle_mod):
    R = oracle_mod.reference_module()
    if R is None:
        pytest.skip("reference build (oracle/_ref) not present")
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    seed = N * 31 + L + len(kind)
    p = LU.random_luts(N, 16, seed=seed, distinct_mags=3, per_element=(N == 32))
    fs, gs, vcl = LU.unpack_to_reference(p)
    _, mb, fm, mm = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb).astype(np.int32)
    B = 12 if N == 1024 else 60
    sym = np.random.default_rng(seed).integers(0, 16, size=(B, N), dtype=np.int32)
    d = _ref_decoder(R, kind, N, K, L, fm.tolist(), mm.tolist(), nt.tolist(), fs, gs, vcl)
    ref = np.stack([d.decode(s) for s in sym])
    got = oracle_mod.decode_lut(kind, p, K, L, fm, sym, node_type=nt)
    assert (ref == got).all()
