"""GPU parity of the fast engine's schedule variants against the oracle:

* root pre-pass (pre-mode): the root f and both root g variants computed once
  per frame by root_pre_kernel, S[1] of the root's left child read from that
  row, the root g built by nibble selects -- on, off (QPD_NO_PRE) and with the
  batch cut into small pre-pass chunks (QPD_PRE_CHUNK); out-of-range channel
  symbols are still reported (the pre-pass reads the channel now);
* fused BOT3 ops (the depth n-4 node's f / g and combine folded into its
  BOT3 children) -- on and off (QPD_NO_BFUSE), with their rows in LDS or in
  the global slab;
* N up to 4096 (R1 nodes above 32 elements: the untrimmed layout)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KINDS = ["SC-LUT", "SCL-LUT", "FastSC-LUT", "FastSCL-LUT"]
MODES = [{"QPD_NO_PRE": "1", "QPD_NO_BFUSE": "1"}, {}, {"QPD_PRE_CHUNK": "7"}, {"QPD_NO_BFUSE": "1"}]
ENV = ("QPD_NO_PRE", "QPD_PRE_CHUNK", "QPD_NO_BFUSE", "QPD_LDS_BUDGET")


@pytest.fixture(scope="module")
def qpd(native_lib):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import quantized_decoder_polar_codes_amd as Q

    return Q


def _node_type(N, K):
    from quantized_decoder_polar_codes_amd import codes as C

    if N <= 1024:
        _, mb, fm, mm = C.construct_pw(N, K)
    else:  # beyond the 5G sequence: BEC(1/2) Bhattacharyya construction, the N-K worst frozen
        z = np.array([0.5])
        while z.size < N:
            z = np.stack([2 * z - z * z, z * z], axis=1).reshape(-1)
        fm = np.zeros(N, dtype=np.int64)
        fm[np.argsort(-z, kind="stable")[: N - K]] = 1
        mb = np.flatnonzero(fm == 0)
    return fm, C.identify_nodes(N, mb).astype(np.int32)


def _set_env(monkeypatch, env):
    for k in ENV:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("N,K,L", [(16, 8, 4), (32, 12, 8), (64, 40, 3), (128, 64, 8), (1024, 512, 8), (2048, 1024, 8),
                                   (4096, 1400, 4)])
@pytest.mark.parametrize("kind", KINDS)
def test_schedule_modes_match_oracle(N, K, L, kind, qpd, oracle_mod, monkeypatch):
    from quantized_decoder_polar_codes_amd import lut as LU

    p = LU.random_luts(N, 16, seed=3 * N + K, distinct_mags=3)
    fm, nt = _node_type(N, K)
    if (kind == "FastSC-LUT" and 0 <= nt[0] <= 3) or (kind == "FastSCL-LUT" and 0 <= nt[0] <= 2):
        pytest.skip("special root: rejected on both sides (test_gpu_parity)")
    B = (40 if N <= 1024 else 12) if "SCL" in kind else (150 if N <= 1024 else 40)
    sym = np.random.default_rng(N + K + L).integers(0, 16, size=(B, N), dtype=np.int32)
    want = oracle_mod.decode_lut(kind, p, K, L, fm, sym, node_type=nt)
    for env in MODES:
        _set_env(monkeypatch, env)
        d = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt, engine="fast")
        got = d.decode_batch(sym)
        bad = np.flatnonzero((got != want).any(1))
        assert bad.size == 0, (env, bad[:5])
        wrong = sym.copy()
        wrong[B // 2, N // 2 + 1] = 16  # a symbol of the root's second half
        with pytest.raises(ValueError):
            d.decode_batch(wrong)
        assert (d.decode_batch(sym[:9]) == want[:9]).all()  # flag cleared


def test_fused_bot3_lds_sweep(qpd, oracle_mod, monkeypatch):
    """Fused BOT3 ops with their rows in LDS or in the global slab (the drains
    placed for the fused reads of S[n-4] / U[n-3])."""
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 256, 128, 8
    p = LU.random_luts(N, 16, seed=91, distinct_mags=3)
    fm, nt = _node_type(N, K)
    sym = np.random.default_rng(92).integers(0, 16, size=(96, N), dtype=np.int32)
    for kind in ("SCL-LUT", "FastSCL-LUT"):
        want = oracle_mod.decode_lut(kind, p, K, L, fm, sym, node_type=nt)
        for budget in (256, 2048, 4096, 65536):
            _set_env(monkeypatch, {"QPD_LDS_BUDGET": str(budget)})
            d = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt, engine="fast")
            assert (d.decode_batch(sym) == want).all(), (kind, budget)


def test_root_prepass_torch_batches(qpd, oracle_mod, monkeypatch):
    """Device-buffer path, batches that grow the pre-pass buffer and batches
    split over several chunks, same bits as the oracle."""
    import torch

    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 256, 128, 8
    p = LU.random_luts(N, 16, seed=71, distinct_mags=3)
    fm, nt = _node_type(N, K)
    sym = np.random.default_rng(72).integers(0, 16, size=(700, N), dtype=np.int32)
    want = oracle_mod.decode_lut("SCL-LUT", p, K, L, fm, sym, node_type=nt)
    _set_env(monkeypatch, {"QPD_PRE_CHUNK": "256"})
    d = qpd.from_packed("SCL-LUT", p, K, fm, L=L, node_type=nt, engine="fast")
    t = torch.from_numpy(sym).cuda()
    for lo, hi in ((0, 5), (0, 256), (0, 700), (13, 600)):
        got = d.decode_batch(t[lo:hi])
        torch.cuda.synchronize()
        assert (got.cpu().numpy() == want[lo:hi]).all(), (lo, hi)
