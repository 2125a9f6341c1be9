"""MinDistortion LUT generator (lutgen.py / csrc/qpd_lutgen.cpp) against the
reference's own Python generator code (fixtures: tests/golden/make_lutgen_golden.py).
Host code only -- runs without a GPU."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN_DIR

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def G(native_lib):
    from quantized_decoder_polar_codes_amd import lutgen

    return lutgen


def _z(name):
    return np.load(os.path.join(GOLDEN_DIR, name), allow_pickle=False)


def test_optls_matches_reference_python_twin(G):
    z = _z("lutgen_optls.npz")
    for i in range(int(z["n_cases"])):
        d, q, K = z[f"q{i}_density"], z[f"q{i}_quanta"], int(z[f"q{i}_K"])
        od, oq, lut, dist = G.optls_quantizer(d, q, K, sum_order="numpy")
        assert np.array_equal(lut, z[f"q{i}_out_lut"]), i
        assert np.array_equal(od, z[f"q{i}_out_density"]), i
        assert np.array_equal(oq, z[f"q{i}_out_quanta"]), i
        # the C++-order mode: same partition on these inputs, sums agree to rounding
        od2, oq2, lut2, dist2 = G.optls_quantizer(d, q, K, sum_order="cpp")
        assert np.array_equal(lut2, lut), i
        assert np.allclose(oq2, oq, rtol=1e-12, atol=1e-14) and np.allclose(od2, od, rtol=1e-12, atol=1e-16)
        assert dist >= 0 and abs(dist2 - dist) <= 1e-9 * max(1.0, dist)


def test_optls_properties(G):
    rng = np.random.default_rng(1)
    q = np.sort(rng.normal(size=40))
    d = rng.random(40)
    od, oq, lut, dist = G.optls_quantizer(d, q, 40)  # K == M: identity, zero distortion
    assert np.array_equal(lut, np.arange(40)) and dist < 1e-20 and np.allclose(oq, q)
    od, oq, lut, dist = G.optls_quantizer(d, q, 1)  # one group: the weighted mean
    assert (lut == 0).all() and np.isclose(oq[0], (d * q).sum() / d.sum())
    od, oq, lut, dist = G.optls_quantizer(d, q, 6)
    assert (np.diff(lut) >= 0).all() and np.isclose(od.sum(), d.sum())  # contiguous groups of sorted quanta
    perm = rng.permutation(40)  # input order does not change the partition of values
    od2, oq2, lut2, _ = G.optls_quantizer(d[perm], q[perm], 6)
    assert np.array_equal(lut2, lut[perm])
    with pytest.raises(ValueError):
        G.optls_quantizer(d, q, 41)


@pytest.mark.parametrize("name", ["lutgen_n8_v8_snr2.npz", "lutgen_n16_v16_snr3.npz", "lutgen_n32_v16_snr3.npz"])
def test_design_matches_reference_generator(G, name):
    path = os.path.join(GOLDEN_DIR, name)
    if not os.path.exists(path):
        pytest.skip("fixture not generated")
    z = _z(name)
    N, v, snr = int(z["N"]), int(z["v"]), float(z["design_snr_db"])
    d = G.design(N, v, snr, sum_order="numpy")
    assert np.array_equal(d.channel_quanta, z["channel_quanta"]) and np.array_equal(d.channel_density,
                                                                                     z["channel_density"])
    assert np.array_equal(d.lut_f, z["lut_f"])
    assert np.array_equal(d.lut_g, z["lut_g"])
    assert np.array_equal(d.llr_quanta, z["llr_quanta"])
    assert np.array_equal(d.llr_density, z["llr_density"])


def test_cpp_order_agrees_with_numpy_order(G):
    a = G.design(128, 16, 3.0, sum_order="cpp")
    b = G.design(128, 16, 3.0, sum_order="numpy")
    same = np.mean(a.lut_f == b.lut_f), np.mean(a.lut_g == b.lut_g)
    assert min(same) > 0.99, same
    assert np.allclose(a.llr_quanta, b.llr_quanta, rtol=1e-6)


def test_design_formats_and_threads(G, tmp_path):
    from quantized_decoder_polar_codes_amd import lut as LU

    a = G.design(64, 16, 2.0, threads=1)
    b = G.design(64, 16, 2.0, threads=7)
    assert np.array_equal(a.lut_f, b.lut_f) and np.array_equal(a.lut_g, b.lut_g)
    assert np.array_equal(a.llr_quanta, b.llr_quanta)
    p = a.packed()
    assert p.N == 64 and p.v == 16 and p.f_step == 0
    fs, gs = a.reference_dicts()
    assert len(fs[0]) == 32 and len(fs[62]) == 1 and np.array_equal(fs[5][0], a.lut_f[5])
    p2 = LU.pack_luts(64, fs, gs, a.llr_quanta.tolist())  # the reference's dict format packs to the same tables
    assert np.array_equal(p2.lut_f[p2.f_base], p.lut_f[p.f_base])
    G.save_npz(str(tmp_path / "d.npz"), a)
    c = G.load_npz(str(tmp_path / "d.npz"))
    assert np.array_equal(c.lut_g, a.lut_g) and np.array_equal(c.llr_quanta, a.llr_quanta)
    files = G.write_reference_pickles(str(tmp_path / "LUT"), a)
    assert [os.path.basename(f) for f in files] == ["LUT_F_SNRdB=2.pkl", "LUT_G_SNRdB=2.pkl", "LLRQuanta_SNRdB=2.pkl",
                                                    "LLRDensity_SNRdB=2.pkl"]


def test_designed_tables_decode_well(G, oracle_mod):
    """Decoding with generated tables (CPU oracle): far better than uncoded at 3 dB."""
    from quantized_decoder_polar_codes_amd import codes as C

    N, K, L = 128, 64, 8
    d = G.design(N, 16, 3.0)
    _, mb, fm, mm = C.construct_pw(N, K)
    rng = np.random.default_rng(0)
    sigma = np.sqrt(1 / (2 * (K / N) * 10 ** (3.0 / 10)))
    cd, cq, edges, clut = G.channel_quantizer(sigma, 128, 16)
    msg = rng.integers(0, 2, size=(300, K), dtype=np.uint8)
    x = C.polar_encode(msg, mb, N)
    llr = ((1.0 - 2.0 * x) + rng.normal(0, sigma, size=x.shape)) * 2 / sigma ** 2
    sym = C.quantize_channel(llr, edges, clut, 16)
    out = oracle_mod.decode_lut("SCL-LUT", d.packed(), K, L, fm, sym)
    assert (out != msg).any(1).mean() < 0.1
