"""Folded ops of the SCL-LUT schedule (qpd_capi.hip: fuse_descent, fold_combine;
qpd_fast.hip: ff_op, the MF_BC2 end of bot3_op).  An F / G op that also runs
its left child's f from registers, and a right BOT3 that also runs its
grandparent's combine, must give the bits of the unfolded schedule
(QPD_NO_FF=1 QPD_NO_BC2=1) and the oracle's, whatever row spaces the layout
puts the folded rows in (LDS budgets), with one or two frame sets per wave in
the decode and prefix kernels, and for the CRC-aided kind.
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


def _code(N, K):
    from quantized_decoder_polar_codes_amd import codes as C

    _, mb, fm, _ = C.construct_pw(N, K)
    return fm, C.identify_nodes(N, mb).astype(np.int32)


def _make(qpd, monkeypatch, kind, p, K, fm, L, folds, env=(), **kw):
    for k in ("QPD_NO_FF", "QPD_NO_BC2", "QPD_LDS_BUDGET", "QPD_SETS", "QPD_PFX_SETS"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env:
        monkeypatch.setenv(k, v)
    if not folds:
        monkeypatch.setenv("QPD_NO_FF", "1")
        monkeypatch.setenv("QPD_NO_BC2", "1")
    return qpd.from_packed(kind, p, K, fm, L=L, **kw)


ENVS = {
    "default": (),
    "lds-budget-6k": (("QPD_LDS_BUDGET", "6144"),),    # shallower LDS: folded rows in the slab
    "lds-budget-14k": (("QPD_LDS_BUDGET", "14336"),),  # depth 4 in LDS: child rows in LDS
    "one-set": (("QPD_SETS", "1"),),                   # no descent folds in the decode kernel
    "prefix-one-set": (("QPD_PFX_SETS", "1"),),
}


@pytest.mark.parametrize("env", list(ENVS))
@pytest.mark.parametrize("N,K,L", [(1024, 512, 8), (512, 300, 8), (1024, 700, 4), (256, 100, 8)])
def test_folds_equal_unfolded(N, K, L, env, qpd, monkeypatch):
    import torch

    from quantized_decoder_polar_codes_amd import lut as LU

    fm, _ = _code(N, K)
    p = LU.minsum_uniform_luts(N)
    rng = np.random.default_rng(N + K + L)
    sym = rng.integers(0, 16, size=(2053, N), dtype=np.int32)
    sym[:1024] = np.clip(sym[:1024] // 2 + 8, 0, 15)  # a biased half: long runs of confident symbols
    a = _make(qpd, monkeypatch, "SCL-LUT", p, K, fm, L, True, ENVS[env])
    b = _make(qpd, monkeypatch, "SCL-LUT", p, K, fm, L, False, ENVS[env])
    assert a.info()["num_ops"] < b.info()["num_ops"]  # something was folded
    st = torch.from_numpy(sym).cuda()
    ga, gb = a.decode_batch(st).cpu().numpy(), b.decode_batch(st).cpu().numpy()
    assert np.array_equal(ga, gb), np.flatnonzero((ga != gb).any(1))[:10]


@pytest.mark.parametrize("env", ["default", "lds-budget-6k", "lds-budget-14k"])
@pytest.mark.parametrize("kind", ["SCL-LUT", "CA-SCL-LUT"])
def test_folds_match_oracle(kind, env, qpd, oracle_mod, monkeypatch):
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 1024, 512, 8
    fm, nt = _code(N, K)
    p = LU.random_luts(N, 16, seed=811, distinct_mags=3)
    sym = np.random.default_rng(17).integers(0, 16, size=(40, N), dtype=np.int32)
    if kind.startswith("CA-"):
        dec = _make(qpd, monkeypatch, kind, p, K, fm, L, True, ENVS[env], A=K - 24)
        want = oracle_mod.decode_lut_ca(kind, p, K, K - 24, L, fm, sym, node_type=nt)
    else:
        dec = _make(qpd, monkeypatch, kind, p, K, fm, L, True, ENVS[env])
        want = oracle_mod.decode_lut(kind, p, K, L, fm, sym, node_type=nt)
    assert_frames_equal(dec.decode_batch(sym), want, dec, f"folds-{kind}-{env}")
