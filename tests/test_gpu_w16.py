"""SCL-LUT with 9 <= L <= 16 on the fast engine (lane groups of 16: qpd_fast.hip
keep_all16 / select_survivors16, W16 instantiations).

mink (SCLLUTDecoder.cpp:8-21) sorts 2L > 16 candidates there, so libstdc++ runs
its introsort, which is not stable: with tied path metrics the survivors' order
depends on the partitions.  The kernel ranks by counting
when the first L ranks hold no tie and replays the introsort otherwise; both
must give the reference's bits:
* against the CPU oracle (the reference's own std::sort) on tie-heavy random
  tables (3 distinct magnitudes: ties at nearly every fork), exact-zero quanta,
  MinDistortion bench tables on AWGN frames, L = 9 / 12 / 16;
* against the generic engine (pinned by the L = 12 / 16 reference goldens) on
  2^14 bench frames at L = 16;
* noiseless codewords at N = 1024, L = 16 decode to their messages (2^16 frames).
"""
import dataclasses

import numpy as np
import pytest

from conftest import assert_frames_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qpd(native_lib):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import quantized_decoder_polar_codes_amd as Q

    return Q


def _code(N, K):
    from quantized_decoder_polar_codes_amd import codes as C

    _, mb, fm, mm = C.construct_pw(N, K)
    return fm, C.identify_nodes(N, mb).astype(np.int32)


@pytest.mark.parametrize("N,K,L,mags", [(64, 32, 16, 3), (128, 64, 16, 2), (256, 128, 12, 3), (256, 100, 9, 3),
                                        (512, 256, 16, None), (1024, 512, 16, 3), (1024, 512, 13, 3)])
def test_w16_random_tables_vs_oracle(N, K, L, mags, qpd, oracle_mod):
    from quantized_decoder_polar_codes_amd import lut as LU

    p = LU.random_luts(N, 16, seed=N + L, distinct_mags=mags)
    fm, nt = _code(N, K)
    B = 40 if N >= 1024 else 160
    rng = np.random.default_rng(N * L)
    sym = rng.integers(0, 16, size=(B, N), dtype=np.int32)
    sym[: B // 4] = np.clip(sym[: B // 4] // 2 + 8, 0, 15)  # confident runs: long identity stretches
    sym[B // 4: B // 2] = 7  # all-equal symbols: every fork a tie
    dec = qpd.from_packed("SCL-LUT", p, K, fm, L=L, engine="fast")
    assert dec.info()["engine"] == 2 and dec.info()["lanes_per_frame"] == 16
    want = oracle_mod.decode_lut("SCL-LUT", p, K, L, fm, sym, node_type=nt)
    redo = lambda rows: qpd.from_packed("SCL-LUT", p, K, fm, L=L, engine="fast").decode_batch(sym[rows])  # noqa: E731
    assert_frames_equal(dec.decode_batch(sym), want, dec, f"w16-{N}-{K}-{L}-{mags}", redo, sym)


def test_w16_zero_quanta_ties(qpd, oracle_mod):
    """Exact-zero leaf quanta: keep and flip of a path tie (kf == pm), the
    selection's own pair included."""
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 256, 128, 16
    p = LU.random_luts(N, 16, seed=77, distinct_mags=3)
    vcl = p.vcl.copy()
    vcl[vcl.shape[0] - 2][:, ::3] = 0.0  # leaf row n-1: a third of the symbols decide with |dm| = 0
    p = dataclasses.replace(p, vcl=vcl)
    fm, nt = _code(N, K)
    sym = np.random.default_rng(3).integers(0, 16, size=(128, N), dtype=np.int32)
    dec = qpd.from_packed("SCL-LUT", p, K, fm, L=L, engine="fast")
    want = oracle_mod.decode_lut("SCL-LUT", p, K, L, fm, sym, node_type=nt)
    assert_frames_equal(dec.decode_batch(sym), want, dec, "w16-zero-quanta")


def test_w16_bench_workload_vs_oracle_and_generic(qpd, oracle_mod):
    """The bench workload (MinDistortion tables, AWGN at 2 dB) at L = 16: the
    oracle on 96 frames, the generic engine on 2^14."""
    import bench

    wl = bench.workload(1024, 512, 16, "SCL-LUT", 1 << 14, 2.0)
    assert wl.dec.info()["engine"] == 2
    got = wl.dec.decode_batch(wl.sym).cpu().numpy()
    sym = wl.sym.cpu().numpy()
    want = oracle_mod.decode_lut("SCL-LUT", wl.packed, 512, 16, wl.fm, sym[:96], node_type=wl.nt)
    assert_frames_equal(got[:96], want, wl.dec, "w16-bench-oracle")
    gen = qpd.from_packed("SCL-LUT", wl.packed, 512, wl.fm, L=16, engine="generic")
    ref = gen.decode_batch(wl.sym).cpu().numpy()
    bad = np.flatnonzero((got != ref).any(1))
    assert bad.size == 0, f"{bad.size} of {len(got)} frames differ from the generic engine: {bad[:10]}"
    # the errors are the code's, not the kernel's: the list beats L = 8 on the same frames
    wl8 = qpd.from_packed("SCL-LUT", wl.packed, 512, wl.fm, L=8)
    e16 = (got != wl.msg.cpu().numpy()).any(1).sum()
    e8 = (wl8.decode_batch(wl.sym).cpu().numpy() != wl.msg.cpu().numpy()).any(1).sum()
    assert e16 <= e8


def test_w16_noiseless_roundtrip(qpd):
    import torch

    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 1024, 512, 16
    _, mb, fm, mm = C.construct_pw(N, K)
    rng = np.random.default_rng(11)
    msg = rng.integers(0, 2, size=(1 << 16, K), dtype=np.uint8)
    u = C.polar_encode(msg, mb, N)
    sym = np.where(u == 0, 15, 0).astype(np.int32)  # confident symbols of the right sign
    d = qpd.from_packed("SCL-LUT", LU.minsum_uniform_luts(N), K, fm, L=L)
    assert d.info()["engine"] == 2
    got = d.decode_batch(torch.from_numpy(sym).cuda()).cpu().numpy()
    assert np.array_equal(got, msg)
