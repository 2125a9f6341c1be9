"""FastSCL-LUT height-3 subtrees with special nodes in registers (BOTX:
qpd_capi.hip bot3_mixed, qpd_fast.hip botx_op / bx_spec).  A subtree whose
size-4 / size-2 nodes are R0 / R1 / REP nodes (FastSCLLUTDecoder.cpp:83-213)
runs as one op; its bits must equal the interpreted schedule's
(QPD_NO_BOTX=1) and the oracle's, for every mix of node types (random
information sets at N = 64 produce all of them), tie-heavy tables whose
special nodes share one quanta row each, the bench code, and the CRC-aided
kind.
"""
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


def _random_code(N, seed):
    from quantized_decoder_polar_codes_amd import codes as C

    rng = np.random.default_rng(seed)
    while True:
        mb = np.flatnonzero(rng.random(N) < rng.uniform(0.3, 0.7))
        nt = C.identify_nodes(N, mb).astype(np.int32)
        if len(mb) and not 0 <= nt[0] <= 2:  # (a special root is refused by both sides)
            fm = np.ones(N, dtype=np.int64)
            fm[mb] = 0
            return fm, nt, len(mb)


def _pair(qpd, monkeypatch, kind, p, K, fm, L, nt, **kw):
    monkeypatch.delenv("QPD_NO_BOTX", raising=False)
    a = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt, engine="fast", **kw)
    monkeypatch.setenv("QPD_NO_BOTX", "1")
    b = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt, engine="fast", **kw)
    monkeypatch.delenv("QPD_NO_BOTX")
    return a, b


@pytest.mark.parametrize("N", [64, 128, 256])
@pytest.mark.parametrize("seed", range(6))
def test_botx_random_codes(N, seed, qpd, oracle_mod, monkeypatch):
    from quantized_decoder_polar_codes_amd import lut as LU

    fm, nt, K = _random_code(N, 100 * N + seed)
    p = LU.random_luts(N, 16, seed=seed, distinct_mags=3, node_rows=True)
    rng = np.random.default_rng(seed)
    sym = rng.integers(0, 16, size=(300, N), dtype=np.int32)
    sym[:100] = np.clip(sym[:100] // 2 + 8, 0, 15)  # confident runs: long identity stretches
    a, b = _pair(qpd, monkeypatch, "FastSCL-LUT", p, K, fm, 8, nt)
    want = oracle_mod.decode_lut("FastSCL-LUT", p, K, 8, fm, sym, node_type=nt)
    ga = a.decode_batch(sym)
    assert_frames_equal(ga, want, a, f"botx-{N}-{seed}")
    assert_frames_equal(b.decode_batch(sym), want, b, f"nobotx-{N}-{seed}")


@pytest.mark.parametrize("N", [64, 256])
@pytest.mark.parametrize("seed", range(4))
def test_special_folds_random_codes(N, seed, qpd, oracle_mod, monkeypatch):
    """Size-8 special nodes that take their parent's f / g and combine
    (MF_SFG / MF_SGG / MF_SCOMB) = the unfolded schedule (QPD_NO_SFOLD=1) = the
    oracle, on codes with every mix of size-8 special and BOT3 siblings."""
    from quantized_decoder_polar_codes_amd import lut as LU

    fm, nt, K = _random_code(N, 300 * N + seed)
    p = LU.random_luts(N, 16, seed=seed + 50, distinct_mags=3, node_rows=True)
    sym = np.random.default_rng(seed).integers(0, 16, size=(300, N), dtype=np.int32)
    monkeypatch.delenv("QPD_NO_SFOLD", raising=False)
    a = qpd.from_packed("FastSCL-LUT", p, K, fm, L=8, node_type=nt, engine="fast")
    monkeypatch.setenv("QPD_NO_SFOLD", "1")
    b = qpd.from_packed("FastSCL-LUT", p, K, fm, L=8, node_type=nt, engine="fast")
    monkeypatch.delenv("QPD_NO_SFOLD")
    want = oracle_mod.decode_lut("FastSCL-LUT", p, K, 8, fm, sym, node_type=nt)
    assert_frames_equal(a.decode_batch(sym), want, a, f"sfold-{N}-{seed}")
    assert_frames_equal(b.decode_batch(sym), want, b, f"nosfold-{N}-{seed}")


@pytest.mark.parametrize("N,K,mags", [(1024, 512, 2), (1024, 512, 3), (1024, 480, 2), (1024, 560, 4), (512, 300, 2)])
def test_r1_masked_partition_argsort(N, K, mags, qpd, oracle_mod):
    """R1 nodes of 17..32 elements with one quanta row (MF_R1_RK): the introsort's
    partitions replayed in the LDS tail by partition_prefix_masked (>= / <= pivot
    masks, only the swaps touch LDS), then the first m outputs as the m smallest
    (rank, position) entries by packed 16-bit min trees (r1_prep), on tie-heavy
    tables (2-4 magnitudes: the partitions meet many equal keys) = the oracle."""
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    _, mb, fm, _ = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb).astype(np.int32)
    sizes = [N >> d for d in range(int(np.log2(N))) for node in range(1 << d)
             if nt[(1 << d) + node - 1] == 1]
    assert any(16 < t <= 32 for t in sizes)
    p = LU.random_luts(N, 16, seed=N + K + mags, distinct_mags=mags, node_rows=True)
    sym = np.random.default_rng(K).integers(0, 16, size=(128, N), dtype=np.int32)
    want = oracle_mod.decode_lut("FastSCL-LUT", p, K, 8, fm, sym, node_type=nt)
    dec = qpd.from_packed("FastSCL-LUT", p, K, fm, L=8, node_type=nt, engine="fast")
    assert_frames_equal(dec.decode_batch(sym), want, dec, f"r1-masked-{N}-{K}-{mags}")


def test_special_folds_engage(qpd, monkeypatch):
    """The bench code's 13 size-16 nodes with one size-8 special child lose their F / G / COMB ops
    (39; a few more of the depth n-5 combines then fold into right BOT3s, MF_BC2)."""
    import bench

    wl = bench.workload(1024, 512, 8, "FastSCL-LUT", 0, 2.0)
    monkeypatch.setenv("QPD_NO_SFOLD", "1")
    b = qpd.from_packed("FastSCL-LUT", wl.packed, 512, wl.fm, L=8, node_type=wl.nt)
    monkeypatch.delenv("QPD_NO_SFOLD")
    assert wl.dec.info()["num_ops"] <= b.info()["num_ops"] - 39


def test_botx_engages_on_random_codes(qpd, monkeypatch):
    """The random codes above do take the fused op (fewer ops than unfused)."""
    from quantized_decoder_polar_codes_amd import lut as LU

    fewer = 0
    for seed in range(6):
        fm, nt, K = _random_code(64, 6400 + seed)
        p = LU.random_luts(64, 16, seed=seed, distinct_mags=3, node_rows=True)
        a, b = _pair(qpd, monkeypatch, "FastSCL-LUT", p, K, fm, 8, nt)
        fewer += a.info()["num_ops"] < b.info()["num_ops"]
    assert fewer >= 4


def test_botx_needs_one_quanta_row(qpd, oracle_mod, monkeypatch):
    """Per-element quanta rows: no BOTX (same op count), bits still the oracle's."""
    from quantized_decoder_polar_codes_amd import lut as LU

    fm, nt, K = _random_code(128, 77)
    p = LU.random_luts(128, 16, seed=77, distinct_mags=3)
    monkeypatch.setenv("QPD_NO_SFOLD", "1")  # (the special-node folds need no quanta row)
    a, b = _pair(qpd, monkeypatch, "FastSCL-LUT", p, K, fm, 8, nt)
    assert a.info()["num_ops"] == b.info()["num_ops"]
    sym = np.random.default_rng(77).integers(0, 16, size=(200, 128), dtype=np.int32)
    want = oracle_mod.decode_lut("FastSCL-LUT", p, K, 8, fm, sym, node_type=nt)
    assert_frames_equal(a.decode_batch(sym), want, a, "botx-perelem")


@pytest.mark.parametrize("ebn0", [1.0, 2.5])
def test_botx_bench_code(ebn0, qpd, oracle_mod, monkeypatch):
    """The bench code (5G PW N=1024 K=512: 20 mixed subtrees) with designed tables."""
    import bench

    wl = bench.workload(1024, 512, 8, "FastSCL-LUT", 512, ebn0)
    sym = wl.sym.cpu().numpy() if hasattr(wl.sym, "cpu") else np.asarray(wl.sym)
    p = wl.packed
    a, b = _pair(qpd, monkeypatch, "FastSCL-LUT", p, 512, wl.fm, 8, wl.nt)
    assert a.info()["num_ops"] < b.info()["num_ops"]
    want = oracle_mod.decode_lut("FastSCL-LUT", p, 512, 8, wl.fm, sym[:96], node_type=wl.nt)
    assert_frames_equal(a.decode_batch(sym[:96]), want, a, f"botx-bench-{ebn0}")
    assert np.array_equal(a.decode_batch(sym), b.decode_batch(sym))


@pytest.mark.parametrize("seed", range(3))
def test_botx_ca(seed, qpd, oracle_mod, monkeypatch):
    from quantized_decoder_polar_codes_amd import lut as LU

    N = 256
    fm, nt, K = _random_code(N, 900 + seed)
    A = K - 24 if K > 40 else K - 8
    p = LU.random_luts(N, 16, seed=seed, distinct_mags=3, node_rows=True)
    sym = np.random.default_rng(seed).integers(0, 16, size=(200, N), dtype=np.int32)
    a, b = _pair(qpd, monkeypatch, "CA-FastSCL-LUT", p, K, fm, 8, nt, A=A, crc_n=24, crc_loc=oracle_mod.CRC24_LOC)
    want = oracle_mod.decode_lut_ca("CA-FastSCL-LUT", p, K, A, 8, fm, sym, node_type=nt)
    assert_frames_equal(a.decode_batch(sym), want, a, f"botx-ca-{seed}")
    assert_frames_equal(b.decode_batch(sym), want, b, f"nobotx-ca-{seed}")


def test_bench_codes_run_the_lean_kernels(qpd, oracle_mod):
    """The bench workloads decode on the kernels the bench measures: one pointer
    word per path, and for FastSCL-LUT the lean special-node instantiation (no R1L);
    tables whose R0 / REP nodes read per-position quanta take the general one
    (qpd_info.fast_variant), with the same bits as the oracle."""
    import bench
    from quantized_decoder_polar_codes_amd import lut as LU

    for kind in ("SCL-LUT", "FastSCL-LUT"):
        wl = bench.workload(1024, 512, 8, kind, 64, 2.0)
        assert wl.dec.info()["fast_variant"] == 1, (kind, wl.dec.info()["fast_variant"])
    p = LU.random_luts(1024, 16, seed=5, distinct_mags=3)  # quanta per position: no one-row nodes
    dec = qpd.from_packed("FastSCL-LUT", p, 512, wl.fm, L=8, node_type=wl.nt, engine="fast")
    assert dec.info()["fast_variant"] & 2
    sym = np.random.default_rng(5).integers(0, 16, size=(64, 1024), dtype=np.int32)
    want = oracle_mod.decode_lut("FastSCL-LUT", p, 512, 8, wl.fm, sym, node_type=wl.nt)
    assert_frames_equal(dec.decode_batch(sym), want, dec, "fscl-general-variant")


@pytest.mark.parametrize("kind,env", [("FastSCL-LUT", "QPD_NO_R1RK"), ("SCL-LUT", "QPD_NO_PW1")])
def test_lean_kernel_equals_general_at_scale(kind, env, qpd, monkeypatch):
    """2^18 bench frames -- more than the oracle decodes in a test -- give the same
    bits on the bench kernel (fast_variant 1) and on the general instantiation
    (FastSCL-LUT without op-record ranks: R1L; SCL-LUT with two pointer words), a
    size-independent check of the lean kernel at the bench's scale."""
    import bench

    wl = bench.workload(1024, 512, 8, kind, 1 << 18, 2.0)
    assert wl.dec.info()["fast_variant"] == 1
    monkeypatch.setenv(env, "1")
    gen = qpd.from_packed(kind, wl.packed, 512, wl.fm, L=8, node_type=wl.nt, engine="fast")
    monkeypatch.delenv(env)
    assert gen.info()["fast_variant"] != 1
    a = wl.dec.decode_batch(wl.sym)
    b = gen.decode_batch(wl.sym)
    import torch

    assert torch.equal(a, b) if hasattr(a, "cpu") else np.array_equal(a, b)
