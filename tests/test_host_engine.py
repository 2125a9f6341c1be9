"""The host engine (csrc/qpd_host.hpp) -- the C++ decoder libqpd.so runs the
few frames of a per-frame ``decode()`` call on (qpd_decode_host; the
reference drivers call decode once per frame, mainQuantizedDecoder_LLRDomain.py:178)
-- checked bit-exact on CPU, built with g++ into a test harness
(tests/native/host_engine_harness.cpp) from the same sources and fed the
same configuration the Python classes hand to qpd_create:

* every decoder golden vector of the reference (LUT and plain float
  domains; the re-quantized float kinds stay on the GPU);
* the oracle on seeded random inputs across N, K, L (1..32), every LUT kind,
  tie-heavy and per-element tables, and the CRC-aided kinds.
The same engine behind the C-ABI on the GPU box: tests/test_gpu_host_engine.py.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, assert_frames_equal, golden_files, golden_packed, load_golden

CSRC = os.path.join(ROOT, "quantized_decoder_polar_codes_amd", "csrc")
BUILD = os.path.join(ROOT, "tests", "_build")


@pytest.fixture(scope="module")
def harness():
    os.makedirs(BUILD, exist_ok=True)
    so = os.path.join(BUILD, "host_engine_harness.so")
    src = os.path.join(ROOT, "tests", "native", "host_engine_harness.cpp")
    deps = [src] + [os.path.join(CSRC, f) for f in ("qpd_host.hpp", "qpd_schedule.hpp", "qpd_types.hpp", "stl_sort.hpp")]
    if not os.path.exists(so) or any(os.path.getmtime(d) > os.path.getmtime(so) for d in deps):
        subprocess.run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
                        src, "-o", so + ".tmp"], check=True)
        os.replace(so + ".tmp", so)
    L = ctypes.CDLL(so)
    L.hh_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.hh_decode.restype = ctypes.c_int
    return L


def run(harness, dec, x):
    x = np.ascontiguousarray(x, dtype=np.float64 if dec._float_input else np.int32)
    out = np.zeros((len(x), dec.out_bits), dtype=np.uint8)
    rc = harness.hh_decode(ctypes.byref(dec._cfg), x.ctypes.data, len(x), out.ctypes.data)
    if rc:
        raise ValueError(f"host engine flag {rc}")
    return out


def _code(N, K):
    from quantized_decoder_polar_codes_amd import codes as C

    _, mb, fm, mm = C.construct_pw(N, K)
    return mb, fm, C.identify_nodes(N, mb).astype(np.int32)


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: os.path.basename(p)[:-4])
def test_host_engine_matches_golden(path, harness):
    from quantized_decoder_polar_codes_amd import decoders as D

    g = load_golden(path)
    N, K, L = int(g["N"]), int(g["K"]), int(g["L"])
    if str(g["kind"]) == "SC":
        dec = D.SCDecoder(N, K, g["frozen"], 1 - g["frozen"], create=False)
        got = run(harness, dec, g["llr"])
    else:
        kw = {"A": int(g["A"])} if str(g["kind"]).startswith("CA-") else {}
        dec = D.from_packed(str(g["kind"]), golden_packed(g), K, g["frozen"], L=L, node_type=g["node_type"],
                            create=False, **kw)
        got = run(harness, dec, g["symbols"])
    assert_frames_equal(got, g["expected"], None, f"host-golden-{os.path.basename(path)[:-4]}")


@pytest.mark.parametrize("path", golden_files("float_*.npz"), ids=lambda p: os.path.basename(p)[:-4])
def test_host_engine_matches_float_golden(path, harness):
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    g = load_golden(path)
    kind = str(g["kind"])
    if kind not in ("SC", "SCL", "CA-SCL", "FastSC", "FastSCL"):
        pytest.skip("re-quantized float kinds run on the GPU only")
    N, K, L = int(g["N"]), int(g["K"]), int(g["L"])
    kw = dict(A=int(g["A"]), crc_n=int(g["crc_n"]), crc_loc=g["crc_loc"]) if kind == "CA-SCL" else {}
    dec = from_quant(kind, N, K, g["frozen"], L=L, node_type=g["node_type"], create=False, **kw)
    assert_frames_equal(run(harness, dec, g["llr"]), g["expected"], None, f"host-float-golden-{kind}")


CASES = [(2, 1, 2), (8, 4, 3), (16, 8, 4), (32, 16, 8), (64, 20, 5), (128, 64, 8), (128, 32, 12), (256, 128, 7),
         (256, 200, 16), (512, 256, 8), (128, 64, 32), (1024, 512, 8)]


@pytest.mark.parametrize("tables", ["ties", "continuous", "perelem"])
@pytest.mark.parametrize("N,K,L", CASES)
@pytest.mark.parametrize("kind", ["SC-LUT", "SCL-LUT", "FastSC-LUT", "FastSCL-LUT"])
def test_host_engine_matches_oracle(kind, N, K, L, tables, harness, oracle_mod):
    from quantized_decoder_polar_codes_amd import decoders as D
    from quantized_decoder_polar_codes_amd import lut as LU

    seed = 7000 + N + 3 * L + len(tables)
    if tables == "continuous":
        p = LU.random_luts(N, 16, seed=seed, distinct_mags=None)
    else:
        p = LU.random_luts(N, 16, seed=seed, distinct_mags=3, per_element=tables == "perelem")
    mb, fm, nt = _code(N, K)
    if kind.startswith("Fast") and 0 <= nt[0] <= 3:
        pytest.skip("root labelled special: undefined in the reference")
    B = 6 if N >= 1024 and "SCL" in kind else 40
    sym = np.random.default_rng(seed).integers(0, 16, size=(B, N), dtype=np.int32)
    want = oracle_mod.decode_lut(kind, p, K, L, fm, sym, node_type=nt)
    dec = D.from_packed(kind, p, K, fm, L=L, node_type=nt, create=False)
    assert_frames_equal(run(harness, dec, sym), want, None, f"host-oracle-{kind}-{N}-{K}-{L}-{tables}")


@pytest.mark.parametrize("N,A,crc_n,L", [(64, 20, 24, 4), (128, 40, 24, 8), (256, 100, 11, 8), (128, 40, 24, 16)])
@pytest.mark.parametrize("kind", ["CA-SCL-LUT", "CA-FastSCL-LUT"])
def test_host_engine_ca_matches_oracle(kind, N, A, crc_n, L, harness, oracle_mod):
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import decoders as D
    from quantized_decoder_polar_codes_amd import lut as LU

    loc = oracle_mod.CRC24_LOC if crc_n == 24 else (11, 10, 9, 5, 0)
    K = A + crc_n
    mb, fm, nt = _code(N, K)
    if kind == "CA-FastSCL-LUT" and 0 <= nt[0] <= 2:
        pytest.skip("root labelled special")
    p = LU.minsum_uniform_luts(N)
    rng = np.random.default_rng(N + A + L)
    msg = rng.integers(0, 2, size=(60, A), dtype=np.uint8)
    u = np.concatenate([msg, oracle_mod.crc_encode(msg, crc_n, loc)[:, : K - A]], axis=1)
    x = C.polar_encode(u, mb, N)
    sigma = np.sqrt(1 / (2 * (K / N) * 10 ** (1.0 / 10)))
    llr = ((1.0 - 2.0 * x) + rng.normal(0, sigma, size=(60, N))) * 2 / sigma ** 2
    sym = np.clip(np.rint(llr / 0.5 + 7.5), 0, 15).astype(np.int32)
    want = oracle_mod.decode_lut_ca(kind, p, K, A, L, fm, sym, node_type=nt, crc_n=crc_n, crc_loc=loc)
    dec = D.from_packed(kind, p, K, fm, L=L, node_type=nt, A=A, crc_n=crc_n, crc_loc=loc, create=False)
    assert_frames_equal(run(harness, dec, sym), want, None, f"host-ca-{kind}-{N}-{A}-{L}")


def test_host_engine_reports_out_of_range_symbol(harness):
    from quantized_decoder_polar_codes_amd import decoders as D
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K = 64, 32
    mb, fm, nt = _code(N, K)
    dec = D.from_packed("SC-LUT", LU.random_luts(N, 16, seed=1), K, fm, create=False)
    sym = np.zeros((2, N), dtype=np.int32)
    sym[1, 5] = 16
    with pytest.raises(ValueError):
        run(harness, dec, sym)


def test_host_engine_reports_nan_path_metric(harness):
    """A NaN path metric reaching a list sort (undefined in the reference's
    std::sort) is flagged, as the GPU engine flags it; SC has no sort."""
    from quantized_decoder_polar_codes_amd import decoders as D

    N, K = 64, 32
    mb, fm, nt = _code(N, K)
    llr = np.ones((2, N))
    llr[1, 0] = np.nan
    scl = D.SCLDecoder(N, K, 4, fm, 1 - fm, create=False)
    with pytest.raises(ValueError):
        run(harness, scl, llr)
    assert run(harness, scl, llr[:1]).shape == (1, K)
    sc = D.SCDecoder(N, K, fm, 1 - fm, create=False)
    assert run(harness, sc, llr).shape == (2, K)
