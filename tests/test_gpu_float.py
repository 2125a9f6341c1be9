"""GPU parity of the float-domain decoders: SCL, CA-SCL,
FastSC, FastSCL and the uniform / Lloyd re-quantized SC and SCL decoders,
through the C-ABI (qpd_decode_f64) in libqpd.so's generic engine.

* golden vectors made by the reference decoders (tests/golden/float_*.npz) --
  bit-exact;
* the CPU oracle (itself pinned to the reference, test_float_oracle.py) on
  seeded AWGN and tie-heavy integer LLRs across N, K, L -- bit-exact;
* size-independent properties at N=1024: noiseless codewords decode to their
  messages; results do not depend on batch composition;
* the reference's per-frame class API (shape (1, N) input);
* inputs the reference cannot decode defined-ly are reported (ValueError).
"""
import os

import numpy as np
import pytest

from conftest import assert_engine, golden_files, load_golden
from test_float_oracle import CRC11, CRC24, FLOAT_KINDS, float_inputs, golden_quant, quant_for

pytestmark = pytest.mark.gpu

# Both engines behind the host-buffer calls, chosen explicitly (qpd_set_host_engine):
# the kernels, and the host engine that serves per-frame calls (not the re-quantized kinds).
ENGINES = ["gpu", pytest.param("host", marks=pytest.mark.host_engine)]


@pytest.fixture(scope="module")
def qpd(native_lib):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import quantized_decoder_polar_codes_amd as Q

    return Q


def _code(N, K):
    from quantized_decoder_polar_codes_amd import codes as C

    _, mb, fm, mm = C.construct_pw(N, K)
    return mb, fm, C.identify_nodes(N, mb).astype(np.int32)


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("path", golden_files("float_*.npz"), ids=lambda p: os.path.basename(p)[:-4])
def test_gpu_float_matches_golden(path, engine, qpd):
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    g = load_golden(path)
    kind = str(g["kind"])
    if engine == "host" and kind.endswith(("Uniform", "Lloyd")):
        pytest.skip("the host engine does not decode the re-quantized kinds (test_gpu_host_engine.py)")
    N, K, L = int(g["N"]), int(g["K"]), int(g["L"])
    kw = {}
    if kind == "CA-SCL":
        kw = dict(A=int(g["A"]), crc_n=int(g["crc_n"]), crc_loc=g["crc_loc"])
    dec = from_quant(kind, N, K, g["frozen"], L=L, node_type=g["node_type"], quant=golden_quant(g), **kw)
    dec.set_host_engine("cpu" if engine == "host" else "gpu")
    got = dec.decode_batch(g["llr"])
    assert_engine(dec, engine)
    assert got.shape == g["expected"].shape
    bad = np.flatnonzero((got != g["expected"]).any(1))
    assert bad.size == 0, f"{bad.size}/{len(got)} frames differ, first {bad[:5]}"


CASES = [(2, 1, 2), (4, 2, 2), (8, 4, 3), (16, 8, 4), (32, 16, 8), (64, 20, 5), (128, 64, 8), (256, 128, 7),
         (512, 256, 8), (1024, 512, 8), (1024, 512, 1),
         (64, 40, 16), (128, 64, 32), (128, 70, 13)]  # L > 8: introsort replay of 2L > 16 candidates


@pytest.mark.parametrize("style", ["awgn", "ties"])
@pytest.mark.parametrize("N,K,L", CASES)
@pytest.mark.parametrize("kind", ["SC"] + FLOAT_KINDS)
def test_gpu_float_matches_oracle(kind, N, K, L, style, qpd, oracle_mod):
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    if kind == "CA-SCL" and K < 16:
        pytest.skip("needs K >= A + crc_n")
    mb, fm, nt = _code(N, K)
    q = quant_for(kind, N)
    B = 96 if N >= 512 else 256
    llr = float_inputs(N, B, seed=N * 13 + L + len(kind) + (7 if style == "ties" else 0), style=style)
    kw, okw = {}, {}
    if kind == "CA-SCL":
        crc_n, loc = (24, CRC24) if K >= 64 else (11, CRC11)
        A = K - crc_n - (5 if N == 512 else 0)
        kw = dict(A=A, crc_n=crc_n, crc_loc=loc)
        okw = dict(A=A, crc_n=crc_n, crc_loc=loc)
    special_root = (kind == "FastSC" and 0 <= nt[0] <= 3) or (kind == "FastSCL" and 0 <= nt[0] <= 2)
    if special_root:  # undefined behaviour in the reference: both sides refuse
        with pytest.raises(RuntimeError):
            oracle_mod.decode_float(kind, N, K, fm, llr, L=L, node_type=nt, quant=q, **okw)
        with pytest.raises(ValueError):
            from_quant(kind, N, K, fm, L=L, node_type=nt, quant=q, **kw)
        return
    dec = from_quant(kind, N, K, fm, L=L, node_type=nt, quant=q, **kw)
    got = dec.decode_batch(llr)
    want = oracle_mod.decode_float(kind, N, K, fm, llr, L=L, node_type=nt, quant=q, **okw)
    assert got.shape == want.shape
    bad = np.flatnonzero((got != want).any(1))
    assert bad.size == 0, f"{bad.size}/{B} frames differ, first {bad[:5]}"


def test_gpu_float_dropin_api(qpd, oracle_mod):
    """The reference's ctor signatures and per-frame decode(llr) with a (1, N) array."""
    from PolarDecoder.Decoder.CASCLDecoder import CASCLDecoder
    from PolarDecoder.Decoder.FastSCDecoder import FastSCDecoder
    from PolarDecoder.Decoder.FastSCLDecoder import FastSCLDecoder
    from PolarDecoder.Decoder.SCLDecoder import SCLDecoder
    from PolarDecoder.Decoder.SCLLloydQuantizedDecoder import SCLLloydQuantizedDecoder
    from PolarDecoder.Decoder.SCLUniformQuantizedDecoder import SCLUniformQuantizedDecoder
    from PolarDecoder.Decoder.SCLloydQuantizedDecoder import SCLloydQuantizedDecoder
    from PolarDecoder.Decoder.SCUniformQuantizedDecoder import SCUniformQuantizedDecoder
    from test_float_oracle import lloyd_lists

    N, K, L = 128, 64, 8
    mb, fm, nt = _code(N, K)
    fz, mm = fm.tolist(), (1 - fm).tolist()
    uq, lq = quant_for("SC-Uniform", N), quant_for("SC-Lloyd", N)
    lists = lloyd_lists(lq)
    decs = {
        "SCL": SCLDecoder(N, K, L, fz, mm),
        "CA-SCL": CASCLDecoder(N, K, 40, L, fz, mm, 24, list(CRC24)),
        "FastSC": FastSCDecoder(N, K, fz, mm, nt.tolist()),
        "FastSCL": FastSCLDecoder(N=N, K=K, L=L, frozen_bits=fz, message_bits=mm, node_type=nt.tolist()),
        "SC-Uniform": SCUniformQuantizedDecoder(N, K, fz, mm, uq.r_f.tolist(), uq.r_g.tolist(), uq.v),
        "SCL-Uniform": SCLUniformQuantizedDecoder(N, K, L, fz, mm, decoder_r_f=uq.r_f.tolist(),
                                                  decoder_r_g=uq.r_g.tolist(), v=uq.v),
        "SC-Lloyd": SCLloydQuantizedDecoder(N, K, fz, mm, *lists, lq.v),
        "SCL-Lloyd": SCLLloydQuantizedDecoder(N, K, L, fz, mm, *lists, v=lq.v),
    }
    llr = float_inputs(N, 6, seed=5, style="awgn")
    for kind, d in decs.items():
        q = uq if "Uniform" in kind else lq if "Lloyd" in kind else None
        okw = dict(A=40, crc_n=24, crc_loc=CRC24) if kind == "CA-SCL" else {}
        want = oracle_mod.decode_float(kind, N, K, fm, llr, L=L, node_type=nt, quant=q, **okw)
        for b in range(len(llr)):
            got = d.decode(llr[b][None])  # the drivers pass shape (1, N)
            assert got.dtype == np.uint8 and got.shape == (want.shape[1],), kind
            assert np.array_equal(got, want[b]), f"{kind} frame {b}"


@pytest.mark.parametrize("kind", ["SC", "SCL", "FastSC", "FastSCL", "SCL-Uniform", "SCL-Lloyd"])
def test_gpu_float_full_size_noiseless(kind, qpd):
    """N=1024 K=512: 2^14 noiseless BPSK frames decode to their messages."""
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    N, K, L = 1024, 512, 8
    mb, fm, nt = _code(N, K)
    B = 1 << 14
    msg = np.random.default_rng(3).integers(0, 2, size=(B, K), dtype=np.uint8)
    x = C.polar_encode(msg, mb, N)
    llr = (1.0 - 2.0 * x) * 4.0
    dec = from_quant(kind, N, K, fm, L=L, node_type=nt, quant=quant_for(kind, N, sigma=0.7))
    got = dec.decode_batch(llr)
    assert np.array_equal(got, msg)


def test_gpu_float_batch_invariance(qpd):
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    N, K, L = 256, 128, 8
    mb, fm, nt = _code(N, K)
    llr = float_inputs(N, 3000, seed=11, style="awgn")
    dec = from_quant("FastSCL", N, K, fm, L=L, node_type=nt, max_waves=7)
    full = dec.decode_batch(llr)
    parts = np.concatenate([dec.decode_batch(llr[i:i + 977]) for i in range(0, 3000, 977)])
    assert np.array_equal(full, parts)
    rev = dec.decode_batch(llr[::-1].copy())[::-1]
    assert np.array_equal(full, rev)


def test_gpu_float_torch_device_path(qpd):
    import torch

    from quantized_decoder_polar_codes_amd.decoders import from_quant

    N, K, L = 128, 64, 4
    mb, fm, nt = _code(N, K)
    llr = float_inputs(N, 500, seed=2, style="awgn")
    dec = from_quant("SCL-Uniform", N, K, fm, L=L, quant=quant_for("SCL-Uniform", N))
    host = dec.decode_batch(llr)
    dev = dec.decode_batch(torch.from_numpy(llr).cuda())
    torch.cuda.synchronize()
    assert dev.is_cuda and np.array_equal(dev.cpu().numpy(), host)


def test_gpu_lloyd_index_outside_reconstruction_is_reported(qpd):
    """Boundaries whose first entry is finite: x <= boundary[0] makes the
    reference read reconstruct[-1] (utils.cpp:23, UB); reported here."""
    from quantized_decoder_polar_codes_amd import quant as QT
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    N, K = 64, 32
    mb, fm, nt = _code(N, K)
    b = np.tile([-1.0, -0.5, 0.0, 0.5, np.inf], (N - 1, 1))  # finite first boundary
    r = np.tile(np.linspace(-1, 1, 4), (N - 1, 1))
    q = QT.pack_lloyd(N, b, b, r, r, 4)
    dec = from_quant("SC-Lloyd", N, K, fm, quant=q)
    with pytest.raises(ValueError, match="Lloyd"):
        dec.decode_batch(np.full((4, N), -5.0))
    ok = dec.decode_batch(np.full((4, N), 0.3))  # every value stays above boundary[0]: fine
    assert ok.shape == (4, K)


@pytest.mark.parametrize("engine", ENGINES)
def test_gpu_nan_path_metric_is_reported(engine, qpd):
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    mode = "cpu" if engine == "host" else "gpu"
    N, K = 64, 32
    mb, fm, nt = _code(N, K)
    llr = np.ones((2, N))
    llr[1, 0] = np.nan
    dec = from_quant("SCL", N, K, fm, L=4)
    dec.set_host_engine(mode)
    with pytest.raises(ValueError, match="NaN"):
        dec.decode_batch(llr)
    assert_engine(dec, engine)
    assert dec.decode_batch(np.ones((2, N))).shape == (2, K)  # flag cleared
    sc = from_quant("SC", N, K, fm)  # SC has no sort: NaN flows through as in the reference
    sc.set_host_engine(mode)
    assert sc.decode_batch(llr).shape == (2, K)
    assert_engine(sc, engine)
