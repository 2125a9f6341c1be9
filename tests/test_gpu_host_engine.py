"""The host engine behind the C-ABI (qpd_decode_host, qpd_set_host_engine):
the reference drivers' per-frame ``decode()`` runs on it (a GPU call costs
~0.1 ms before decoding anything; the reference's SC-LUT call ~10 us,
SCLUTDecoder.cpp:21-124).  Through a real device decoder:

* golden vectors: host engine (mode "cpu") = GPU kernels (mode "gpu") =
  the reference's bits;
* AUTO sends the few frames of a per-frame call to the host engine and
  batches to the GPU, and both give the same bits;
* the re-quantized float kinds refuse the host engine.
The engine's own parity across N, K, L, kinds and tables: tests/test_host_engine.py (CPU).
"""
import os

import numpy as np
import pytest

from conftest import assert_engine, assert_frames_equal, golden_files, golden_packed, load_golden

pytestmark = [pytest.mark.gpu, pytest.mark.host_engine]  # engines chosen per call here


@pytest.fixture(scope="module")
def qpd(native_lib):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import quantized_decoder_polar_codes_amd as Q

    return Q


def _dec(g, qpd):
    N, K, L = int(g["N"]), int(g["K"]), int(g["L"])
    if str(g["kind"]) == "SC":
        return qpd.SCDecoder(N, K, g["frozen"], 1 - g["frozen"]), g["llr"]
    kw = {"A": int(g["A"])} if str(g["kind"]).startswith("CA-") else {}
    return (qpd.from_packed(str(g["kind"]), golden_packed(g), K, g["frozen"], L=L, node_type=g["node_type"], **kw),
            g["symbols"].astype(np.int32))


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: os.path.basename(p)[:-4])
def test_host_engine_and_gpu_match_golden(path, qpd):
    g = load_golden(path)
    dec, x = _dec(g, qpd)
    name = os.path.basename(path)[:-4]
    dec.set_host_engine("cpu")
    host = dec.decode_batch(x)
    assert_frames_equal(host, g["expected"], dec, f"host-engine-{name}", engine="host")
    dec.set_host_engine("gpu")
    gpu = dec.decode_batch(x)
    assert_frames_equal(gpu, g["expected"], dec, f"gpu-{name}", engine="gpu")


@pytest.mark.parametrize("kind,N,K,L", [("SC-LUT", 128, 32, 1), ("SCL-LUT", 1024, 512, 8), ("FastSCL-LUT", 1024, 512, 8),
                                        ("FastSC-LUT", 1024, 512, 1), ("CA-SCL-LUT", 128, 64, 8)])
def test_auto_dispatch_per_frame_and_batch(kind, N, K, L, qpd, oracle_mod):
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    _, mb, fm, mm = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb).astype(np.int32)
    p = LU.random_luts(N, 16, seed=N + L, distinct_mags=3)
    kw = {"A": K - 24} if kind.startswith("CA-") else {}
    dec = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt, **kw)
    hm = dec.info()["host_max_frames"]
    assert hm >= 1  # a per-frame call runs on the host engine
    sym = np.random.default_rng(5).integers(0, 16, size=(max(64, 2 * hm + 3), N), dtype=np.int32)
    one = np.stack([dec.decode(s) for s in sym[:6]])  # host engine
    assert_engine(dec, "host")
    batch = dec.decode_batch(sym)  # GPU (larger than host_max_frames)
    assert_frames_equal(one, batch[:6], dec, f"auto-{kind}", engine="gpu")
    if kind.startswith("CA-"):
        want = oracle_mod.decode_lut_ca(kind, p, K, K - 24, L, fm, sym[:6], node_type=nt)
    else:
        want = oracle_mod.decode_lut(kind, p, K, L, fm, sym[:6], node_type=nt)
    assert_frames_equal(one, want, None, f"auto-oracle-{kind}")


def test_requantized_kinds_stay_on_gpu(qpd):
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import quant as QU
    from quantized_decoder_polar_codes_amd.decoders import from_quant

    N, K = 64, 32
    _, mb, fm, mm = C.construct_pw(N, K)
    dec = from_quant("SC-Uniform", N, K, fm, quant=QU.ga_uniform(N, 0.8))
    assert dec.info()["host_max_frames"] == 0
    with pytest.raises(ValueError):
        dec.set_host_engine("cpu")


def test_gpu_parity_check_refuses_a_host_served_case(qpd, oracle_mod):
    """The kernels-only guard of the GPU parity tests (conftest: assert_frames_equal
    checks qpd_info.last_engine): bits from the host engine, however correct, do
    not pass as a GPU result."""
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 128, 64, 4
    _, mb, fm, mm = C.construct_pw(N, K)
    p = LU.random_luts(N, 16, seed=11, distinct_mags=3)
    dec = qpd.from_packed("SCL-LUT", p, K, fm, L=L)
    sym = np.random.default_rng(2).integers(0, 16, size=(3, N), dtype=np.int32)
    want = oracle_mod.decode_lut("SCL-LUT", p, K, L, fm, sym)
    dec.set_host_engine("cpu")
    got = dec.decode_batch(sym)
    assert dec.info()["last_engine"] == 2  # QPD_RAN_HOST
    assert_frames_equal(got, want, dec, "host-served", engine="host")
    with pytest.raises(AssertionError, match="host engine"):
        assert_frames_equal(got, want, dec, "host-served-as-gpu")  # default: the GPU kernels
    dec.set_host_engine("gpu")
    assert_frames_equal(dec.decode_batch(sym), want, dec, "gpu-served")
    assert dec.info()["last_engine"] == 1  # QPD_RAN_GPU
