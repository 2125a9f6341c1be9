"""Host-side pieces that need no GPU: code construction, node labels, channel
quantization, LUT packing/validation, and the C-ABI library surface."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from quantized_decoder_polar_codes_amd import codes as C
from quantized_decoder_polar_codes_amd import lut as LU


def test_reliability_sequence_is_permutation():
    q = C.reliability_sequence()
    assert sorted(q.tolist()) == list(range(1024))
    assert q[:7].tolist() == [0, 1, 2, 4, 8, 16, 32]


@pytest.mark.parametrize("N,K", [(128, 32), (1024, 512), (64, 0), (64, 64)])
def test_construct_pw(N, K):
    fb, mb, fm, mm = C.construct_pw(N, K)
    assert fm.sum() == N - K and mm.sum() == K and (fm + mm == 1).all()
    q = C.reliability_sequence()
    q = q[q < N]
    assert set(fb.tolist()) == set(q[: N - K].tolist())  # least reliable frozen
    assert (np.diff(fb) > 0).all() if len(fb) > 1 else True


@pytest.mark.parametrize("N,K,census", [(1024, 512, (14, 15, 28, 26)), (128, 32, (2, 1, 7, 3))])
def test_identify_nodes_census(N, K, census):
    # node counts measured on the reference NodeIdentifier
    _, mb, _, _ = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb)
    n = int(np.log2(N))
    inner = nt[: N - 1]
    assert tuple(int((inner == t).sum()) for t in range(4)) == census
    assert nt.shape == (2 * N - 1,)
    assert n > 0


def test_identify_nodes_descendants_unlabelled():
    N, K = 256, 100
    _, mb, _, _ = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb)
    for p in range(N - 1):
        if nt[p] >= 0:
            for child in (2 * p + 1, 2 * p + 2):
                assert nt[child] == -1


def test_polar_transform_involution_and_linearity():
    rng = np.random.default_rng(0)
    u = rng.integers(0, 2, size=(5, 64), dtype=np.uint8)
    w = rng.integers(0, 2, size=(5, 64), dtype=np.uint8)
    assert (C.polar_transform(C.polar_transform(u)) == u).all()
    assert (C.polar_transform(u ^ w) == (C.polar_transform(u) ^ C.polar_transform(w))).all()


def test_quantize_channel_matches_driver_loop():
    rng = np.random.default_rng(1)
    edges = np.linspace(-10, 10, 129)
    lut = rng.integers(0, 16, size=128)
    llr = np.concatenate([rng.normal(0, 6, size=500), edges[:5], [-10.0, 10.0, -11, 11]])
    a = C.quantize_channel(llr, edges, lut, 16)
    b = C.quantize_channel_scalar(llr, edges, lut, 16)
    assert (a == b).all()


def test_pack_nested_lists_dedup_roundtrip():
    p = LU.random_luts(16, 4, seed=3)
    fs, gs, vcl = LU.unpack_to_reference(p)
    q = LU.pack_luts(16, fs, gs, vcl)
    assert q.deduplicated and q.f_step == 0
    assert (q.lut_f == p.lut_f).all() and (q.lut_g == p.lut_g).all() and (q.vcl == p.vcl).all()
    qd = LU.pack_luts(16, {k: fs[k] for k in range(15)}, {k: gs[k] for k in range(15)}, vcl)
    assert (qd.lut_f == p.lut_f).all()


def test_pack_per_element_tables():
    p = LU.random_luts(16, 4, seed=4, per_element=True)
    fs, gs, vcl = LU.unpack_to_reference(p)
    q = LU.pack_luts(16, fs, gs, vcl)
    assert not q.deduplicated and q.f_step == 1
    for node in range(15):
        depth = (node + 1).bit_length() - 1
        for j in range(16 >> (depth + 1)):
            assert (q.lut_f[q.f_base[node] + j] == np.asarray(fs[node][j])).all()
            assert (q.lut_g[q.g_base[node] + j] == np.asarray(gs[node][j])).all()


def test_pack_validation_errors():
    p = LU.random_luts(8, 4, seed=5)
    fs, gs, vcl = LU.unpack_to_reference(p)
    with pytest.raises(ValueError):
        LU.pack_luts(8, fs[:-1], gs, vcl)  # missing node
    bad = [list(e) for e in fs]
    bad[3] = [[[9] * 4] * 4]
    with pytest.raises(ValueError):
        LU.pack_luts(8, bad, gs, vcl)  # entry >= v
    v2 = np.array(vcl)
    v2[1, 2, 3] = np.nan
    with pytest.raises(ValueError):
        LU.pack_luts(8, fs, gs, v2)  # non-finite quanta
    with pytest.raises(ValueError):
        LU.pack_luts(8, fs, gs, np.array(vcl)[:, :4])  # wrong N


# ---------------------------------------------------------------------------
# C-ABI library surface (no device calls)
# ---------------------------------------------------------------------------

def _header_functions():
    txt = open(os.path.join(ROOT, "include", "qpd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)  # drop comments
    return sorted(set(re.findall(r"\b(qpd_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(native_lib):
    from quantized_decoder_polar_codes_amd import _lib

    declared = _header_functions()
    assert set(declared) == set(_lib.EXPORTED)
    for name in declared:
        assert hasattr(native_lib, name), name
    txt = open(os.path.join(ROOT, "include", "qpd.h")).read()
    ver = int(re.search(r"#define QPD_ABI_VERSION (\d+)", txt).group(1))
    assert native_lib.qpd_abi_version() == ver == _lib.ABI_VERSION


def _cfg(kind=2, N=8, K=4, L=4, frozen=None, over=None):
    from quantized_decoder_polar_codes_amd import _lib

    p = LU.random_luts(N, 4, seed=6)
    keep = [p]
    fz = np.zeros(N, dtype=np.int32) if frozen is None else np.asarray(frozen, dtype=np.int32)
    if frozen is None:
        fz[: N - K] = 1
    keep.append(fz)
    c = _lib.QpdConfig()
    c.kind, c.N, c.K, c.L, c.v = kind, N, K, L, 4
    c.frozen_bits = fz.ctypes.data
    c.lut_f, c.lut_f_count, c.f_base, c.f_step = p.lut_f.ctypes.data, p.lut_f.shape[0], p.f_base.ctypes.data, 0
    c.lut_g, c.lut_g_count, c.g_base, c.g_step = p.lut_g.ctypes.data, p.lut_g.shape[0], p.g_base.ctypes.data, 0
    c.vcl, c.vcl_rows, c.device = p.vcl.ctypes.data, p.vcl.shape[0], -1
    for k, v in (over or {}).items():
        setattr(c, k, v)
    return c, keep


@pytest.mark.parametrize("over,code", [
    ({"L": 33}, -2),           # L > 32 not supported
    ({"L": 0}, -2),
    ({"N": 12}, -1),           # not a power of two
    ({"K": 3}, -1),            # K != number of information bits
    ({"v": 300}, -1),
    ({"f_step": 2}, -1),
    ({"vcl_rows": 1}, -1),
    ({"kind": 9}, -1),
])
def test_create_rejects_bad_config(native_lib, over, code):
    c, keep = _cfg(over=over)
    h = ctypes.c_void_p()
    rc = native_lib.qpd_create(ctypes.byref(c), ctypes.byref(h))
    assert rc == code
    assert native_lib.qpd_last_error()


@pytest.mark.parametrize("over", [
    {"A": 0, "crc_n": 24},               # A outside [1, K]
    {"A": 5, "crc_n": 24},
    {"A": 2, "crc_n": 0},                # crc_n outside [1, 32]
    {"A": 2, "crc_n": 33},
    {"A": 1, "crc_n": 2},                # K - A > crc_n (reference reads past its check code)
    {"A": 2, "crc_n": 24, "crc_loc_count": 1},  # crc_loc count without pointer
])
def test_create_rejects_bad_crc_config(native_lib, over):
    from quantized_decoder_polar_codes_amd import _lib

    for kind in (_lib.QPD_CASCL_LUT, _lib.QPD_CAFASTSCL_LUT):
        c, keep = _cfg(kind=kind, over=over)
        nt = -np.ones(15, dtype=np.int32)
        c.node_type = nt.ctypes.data
        h = ctypes.c_void_p()
        assert native_lib.qpd_create(ctypes.byref(c), ctypes.byref(h)) == -1
        assert native_lib.qpd_last_error()


def test_create_rejects_crc_loc_out_of_range(native_lib):
    from quantized_decoder_polar_codes_amd import _lib

    loc = np.array([24, 25, 0], dtype=np.int32)
    c, keep = _cfg(kind=_lib.QPD_CASCL_LUT, over={"A": 2, "crc_n": 24, "crc_loc": loc.ctypes.data,
                                                  "crc_loc_count": 3})
    h = ctypes.c_void_p()
    assert native_lib.qpd_create(ctypes.byref(c), ctypes.byref(h)) == -1


def test_create_rejects_special_root(native_lib):
    c, keep = _cfg(kind=4)
    nt = -np.ones(15, dtype=np.int32)
    nt[0] = 1
    c.node_type = nt.ctypes.data
    h = ctypes.c_void_p()
    assert native_lib.qpd_create(ctypes.byref(c), ctypes.byref(h)) == -2
    c.node_type = None
    assert native_lib.qpd_create(ctypes.byref(c), ctypes.byref(h)) == -1  # node_type required


def test_frozen_mask_values_validated(native_lib):
    fz = np.array([1, 1, 2, 0, 0, 0, 0, 1], dtype=np.int32)
    c, keep = _cfg(frozen=fz, K=4)
    h = ctypes.c_void_p()
    assert native_lib.qpd_create(ctypes.byref(c), ctypes.byref(h)) == -1
