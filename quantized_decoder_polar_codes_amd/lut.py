"""LUT ingestion: the reference's nested-list / pickle-dict table format ->
the packed device format of the C-ABI (include/qpd.h).

Reference format (built by
mainQuantizedDecoder_LLRDomain.py:87-95 from QLLRDensityEvolution_MinDistortion.py:
116-124):

* ``LUT_f``: N-1 entries indexed by node_posi = 2^depth + node - 1; entry p holds
  ``N >> (depth+1)`` tables ``int[v][v]`` (index [a][b], a = first-half symbol).
* ``LUT_g``: same with ``int[2][v][v]`` (index [u_left][a][b]).
* ``virtual_channel_llr``: float64 ``[rows][N][v]`` (rows = n+1 for the LLR-domain
  generators, n for the probability-domain ones).

Packed format: ``lut_f uint8[T_f][v][v]``, ``lut_g uint8[T_g][2][v][v]`` and per
node ``f_base/g_base int32[N-1]``; element j of node p uses table
``base[p] + j*step``.  Every reference generator writes identical copies per
node, so ``step`` is normally 0 (one table per node, 786 KB at N=1024 v=16);
tables that differ per element are kept whole with ``step`` = 1.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class PackedLUT:
    N: int
    v: int
    lut_f: np.ndarray  # uint8 [T_f, v, v]
    f_base: np.ndarray  # int32 [N-1]
    f_step: int
    lut_g: np.ndarray  # uint8 [T_g, 2, v, v]
    g_base: np.ndarray  # int32 [N-1]
    g_step: int
    vcl: np.ndarray  # float64 [rows, N, v], C-contiguous
    # True when the reference's per-node table copies were all identical.
    deduplicated: bool = True

    @property
    def vcl_rows(self) -> int:
        return int(self.vcl.shape[0])


def _log2(N: int) -> int:
    n = int(N).bit_length() - 1
    if N < 2 or (1 << n) != N:
        raise ValueError(f"N must be a power of two >= 2, got {N}")
    return n


def _entries(tables, N: int, what: str):
    """Return the N-1 per-node entries of a reference LUT container in node_posi order."""
    if isinstance(tables, dict):
        keys = sorted(tables.keys())
        if keys != list(range(N - 1)):
            raise ValueError(f"{what}: dict keys must be node_posi 0..{N - 2}")
        return [tables[k] for k in keys]
    if isinstance(tables, np.ndarray) and tables.dtype != object:
        if tables.shape[0] != N - 1:
            raise ValueError(f"{what}: first dimension must be N-1={N - 1}, got {tables.shape[0]}")
        return [tables[k] for k in range(N - 1)]
    entries = list(tables)
    if len(entries) != N - 1:
        raise ValueError(f"{what}: expected N-1={N - 1} node entries, got {len(entries)}")
    return entries


def _pack(tables, N: int, inner: tuple, what: str):
    """Pack one table family; ``inner`` is (v, v) for f or (2, v, v) for g."""
    n = _log2(N)
    entries = _entries(tables, N, what)
    per_node = []
    dedup = True
    v = None
    for p, e in enumerate(entries):
        depth = (p + 1).bit_length() - 1
        need = N >> (depth + 1)
        arr = np.asarray(e)
        if arr.ndim == len(inner):  # already one table per node
            arr = arr[None]
        if arr.ndim != len(inner) + 1:
            raise ValueError(f"{what}[{p}]: expected {len(inner) + 1}-d nested tables, got shape {arr.shape}")
        if v is None:
            v = arr.shape[-1]
        exp = tuple(v if s == "v" else s for s in inner)
        if arr.shape[1:] != exp:
            raise ValueError(f"{what}[{p}]: table shape {arr.shape[1:]} != {exp}")
        if arr.shape[0] != 1 and arr.shape[0] < need:
            raise ValueError(f"{what}[{p}]: node at depth {depth} needs {need} element tables, got {arr.shape[0]}")
        if arr.shape[0] > 1 and not (arr[:need] == arr[0]).all():
            dedup = False
        per_node.append(arr if arr.shape[0] == 1 else arr[:need])
    assert n >= 1
    return per_node, dedup, v


def _to_u8(arr: np.ndarray, v: int, what: str) -> np.ndarray:
    a = np.asarray(arr)
    if a.size and (a.min() < 0 or a.max() >= v):
        raise ValueError(f"{what}: table entries must lie in [0, {v}), found [{a.min()}, {a.max()}]")
    return a.astype(np.uint8)


def pack_luts(N: int, LUT_f, LUT_g, virtual_channel_llr) -> PackedLUT:
    """Convert reference-format tables to :class:`PackedLUT`, validating shapes and
    ranges (the reference performs no checks; out-of-range symbols are UB there)."""
    pf, df, vf = _pack(LUT_f, N, ("v", "v"), "LUT_f")
    pg, dg, vg = _pack(LUT_g, N, (2, "v", "v"), "LUT_g")
    if vf != vg:
        raise ValueError(f"LUT_f alphabet {vf} != LUT_g alphabet {vg}")
    v = int(vf)
    if v < 2 or v > 256:
        raise ValueError(f"alphabet size v={v} outside [2, 256]")
    vcl = np.ascontiguousarray(np.asarray(virtual_channel_llr, dtype=np.float64))
    if vcl.ndim != 3 or vcl.shape[1] != N or vcl.shape[2] != v:
        raise ValueError(f"virtual_channel_llr must be [rows][N={N}][v={v}], got {vcl.shape}")
    n = _log2(N)
    if vcl.shape[0] < n:
        raise ValueError(f"virtual_channel_llr needs at least n={n} rows (decoder reads rows 0..n-1)")
    if not np.isfinite(vcl[:n]).all():
        raise ValueError("virtual_channel_llr rows 0..n-1 must be finite (a non-finite quanta "
                         "makes the reference's path-metric sort ill-defined)")
    dedup = df and dg
    if dedup:
        lut_f = np.stack([_to_u8(t[0], v, "LUT_f") for t in pf])
        lut_g = np.stack([_to_u8(t[0], v, "LUT_g") for t in pg])
        f_base = np.arange(N - 1, dtype=np.int32)
        g_base = f_base.copy()
        f_step = g_step = 0
    else:
        # Expand every node to its full per-element table list.
        def expand(per_node):
            out, base, pos = [], np.zeros(N - 1, dtype=np.int32), 0
            for p, t in enumerate(per_node):
                depth = (p + 1).bit_length() - 1
                need = N >> (depth + 1)
                if t.shape[0] == 1:
                    t = np.repeat(t, need, axis=0)
                base[p] = pos
                out.append(t)
                pos += need
            return np.concatenate(out), base

        lf, f_base = expand(pf)
        lg, g_base = expand(pg)
        lut_f, lut_g = _to_u8(lf, v, "LUT_f"), _to_u8(lg, v, "LUT_g")
        f_step = g_step = 1
    return PackedLUT(N=N, v=v, lut_f=np.ascontiguousarray(lut_f), f_base=f_base, f_step=f_step,
                     lut_g=np.ascontiguousarray(lut_g), g_base=g_base, g_step=g_step, vcl=vcl,
                     deduplicated=dedup)


def unpack_to_reference(p: PackedLUT):
    """Packed -> the reference's nested-list format (one copy per element), for
    feeding the same tables to the reference decoder in tests."""
    N = p.N
    fs, gs = [], []
    for node in range(N - 1):
        depth = (node + 1).bit_length() - 1
        need = N >> (depth + 1)
        fs.append([p.lut_f[p.f_base[node] + j * p.f_step].astype(np.int32).tolist() for j in range(need)])
        gs.append([p.lut_g[p.g_base[node] + j * p.g_step].astype(np.int32).tolist() for j in range(need)])
    return fs, gs, p.vcl.tolist()


# ---------------------------------------------------------------------------
# Synthetic tables (pure-throughput runs and parity stress).
# ---------------------------------------------------------------------------

def minsum_uniform_luts(N: int, v: int = 16, delta: float = 0.5, rows: int | None = None) -> PackedLUT:
    """Saturating min-sum LUTs on a uniform symmetric alphabet
    q_s = (s - (v-1)/2) * delta.  f = Q(sign*sign*min), g = Q((1-2u)a + b); Q
    rounds to the nearest quantum and saturates.  vcl rows are the quanta."""
    n = _log2(N)
    q = (np.arange(v) - (v - 1) / 2.0) * delta

    def Q(x):
        return np.clip(np.rint(x / delta + (v - 1) / 2.0), 0, v - 1).astype(np.uint8)

    a = q[:, None]
    b = q[None, :]
    f = Q(np.sign(a) * np.sign(b) * np.minimum(np.abs(a), np.abs(b)))
    g = np.stack([Q(a + b), Q(-a + b)])
    lut_f = np.repeat(f[None], N - 1, axis=0)
    lut_g = np.repeat(g[None], N - 1, axis=0)
    rows = n + 1 if rows is None else rows
    vcl = np.broadcast_to(q, (rows, N, v)).copy()
    base = np.arange(N - 1, dtype=np.int32)
    return PackedLUT(N=N, v=v, lut_f=lut_f, f_base=base, f_step=0, lut_g=lut_g, g_base=base.copy(),
                     g_step=0, vcl=vcl)


def random_luts(N: int, v: int = 16, seed: int = 0, distinct_mags: int | None = 4,
                per_element: bool = False, rows: int | None = None, node_rows: bool = False) -> PackedLUT:
    """Random tables (every entry uniform in [0, v)) and random vcl drawn from
    ``distinct_mags`` magnitudes with random signs -- a tie-heavy stress input for
    the path-metric sort (hazard H1).  ``distinct_mags=None`` draws continuous
    values.  ``per_element`` makes every element of every node use its own table.
    ``node_rows``: the elements of each node share one quanta row, as the
    MinDistortion generator makes them (row r is read by the special nodes of
    depth r + 1, so its positions are grouped by those nodes)."""
    n = _log2(N)
    rng = np.random.default_rng(seed)
    rows = n + 1 if rows is None else rows
    if per_element:
        T = n * N // 2
        lut_f = rng.integers(0, v, size=(T, v, v), dtype=np.uint8)
        lut_g = rng.integers(0, v, size=(T, 2, v, v), dtype=np.uint8)
        base = np.zeros(N - 1, dtype=np.int32)
        pos = 0
        for p in range(N - 1):
            depth = (p + 1).bit_length() - 1
            base[p] = pos
            pos += N >> (depth + 1)
        f_base, g_base, step = base, base.copy(), 1
    else:
        lut_f = rng.integers(0, v, size=(N - 1, v, v), dtype=np.uint8)
        lut_g = rng.integers(0, v, size=(N - 1, 2, v, v), dtype=np.uint8)
        f_base = np.arange(N - 1, dtype=np.int32)
        g_base, step = f_base.copy(), 0
    if distinct_mags:
        mags = rng.choice(np.array([0.25, 0.5, 1.0, 1.5, 2.0, 3.0, 4.5, 6.0])[:max(1, distinct_mags)],
                          size=(rows, N, v))
        # include exact zeros occasionally: exercises `<= 0` vs `< 0` (H4)
        zero = rng.random((rows, N, v)) < 0.05
        vcl = np.where(zero, 0.0, mags * rng.choice([-1.0, 1.0], size=(rows, N, v)))
    else:
        vcl = rng.normal(0, 3, size=(rows, N, v))
    if node_rows:  # one row per node of depth r + 1: copy each group's first row
        for r in range(rows):
            g = max(1, N >> (r + 1))
            vcl[r] = np.repeat(vcl[r, ::g], g, axis=0)[:N]
    return PackedLUT(N=N, v=v, lut_f=lut_f, f_base=f_base, f_step=step, lut_g=lut_g, g_base=g_base,
                     g_step=step, vcl=np.ascontiguousarray(vcl), deduplicated=not per_element)
