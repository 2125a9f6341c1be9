"""Diagnostic: LDS bank conflicts of the f / g byte-table lookups (lut_lds in
qpd_fast.hip) under alternative table layouts, simulated on the bench workload.

The host engine records every f / g element lookup (u, a, b) of the tree depths
the GPU's F / G ops look up from the byte tables (1 <= d <= n-4); lookups are
grouped as one ds_read_u8 issues them: one element of one op for the 32 lanes
of a half-wave (4 frames x 8 paths; paths with the same inputs read the same
byte).  Per group the LDS needs max over banks of the distinct dwords in that
bank cycles ((byte >> 2) mod 32 banks, MI355X_MICROARCH.md §LDS, ds_read_b32
banking); conflict cycles = that - 1.  CPU only.
usage: python tools/bank_sim.py [frames]"""
import collections
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mc_ref import frames as ref_frames  # noqa: E402
from quantized_decoder_polar_codes_amd import codes as C, decoders as D, lutgen as LG, montecarlo as MC  # noqa: E402

SRC = r'''
#include <cstdio>
#include <cstdint>
#include <vector>
struct Rec { int32_t op, e, path; uint16_t idx; uint8_t isg; };
static std::vector<Rec> *g_rec = nullptr;
static int g_op = 0, g_lo = 1, g_hi = 6;
#define QPD_HOST_FG_ELEMS(op, isg, path, a, uu) do { \
    if ((op).d >= g_lo && (op).d <= g_hi) { const int ct = (op).ct; \
        for (int e = 0; e < ct; ++e) g_rec->push_back(Rec{(op).posi * 2 + ((isg) ? 1 : 0), e, path, \
            (uint16_t)((((isg) ? (uu)[e] : 0) << 8) | ((a)[e] << 4) | (a)[ct + e]), (uint8_t)((isg) ? 1 : 0)}); } } while (0)
#include "qpd_host.hpp"
extern "C" long bs_run(const qpd_config *c, const int32_t *in, int64_t B, int lo, int hi, int32_t *out, long cap) {
    std::unique_ptr<qpd_host::Plan> p = qpd_host::make_plan(c);
    qpd_host::Engine<uint8_t> e(*p);
    std::vector<uint8_t> o(p->out_k);
    std::vector<Rec> v;
    g_rec = &v; g_lo = lo; g_hi = hi;
    long n = 0;
    for (int64_t b = 0; b < B; ++b) {
        v.clear();
        e.decode(in + b * p->N, o.data());
        for (const Rec &r : v) {
            if (n + 5 > cap) return -1;
            out[n++] = (int32_t)b; out[n++] = r.op; out[n++] = r.e; out[n++] = r.path; out[n++] = r.idx | (r.isg << 16);
        }
    }
    return n / 5;
}
'''


def run(F, n_lo=1, n_hi=6, L=8):
    so, cpp = "/tmp/bank_sim.so", "/tmp/bank_sim.cpp"
    open(cpp, "w").write(SRC)
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", f"{ROOT}/include", "-I",
                    f"{ROOT}/quantized_decoder_polar_codes_amd/csrc", cpp, "-o", so], check=True)
    lib = ctypes.CDLL(so)
    N, K = 1024, 512
    _, mb, fm, mm = C.construct_pw(N, K)
    d = LG.design(N, 16, 3.0)
    sigma = MC.sigma_for(2.0, K / N)
    _, _, edges, clut = LG.channel_quantizer(sigma, 128, 16)
    _, sym, _ = ref_frames(N, K, mb, 1234, 0, F, sigma, edges, clut, 16)
    dec = D.from_packed("SCL-LUT", d.packed(), K, fm, L=L, create=False)
    sym = np.ascontiguousarray(sym, dtype=np.int32)
    cap = 5 * F * 8 * 7 * 1024 * 2
    out = np.zeros(cap, np.int32)
    n = lib.bs_run(ctypes.byref(dec._cfg), sym.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(F), n_lo, n_hi,
                   out.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(cap))
    return out[: 5 * n].reshape(n, 5)


# layouts: byte address of (u, a, b) in the staged table (f: u = 0)
def lay_cur(u, a, b):
    return (u << 8) | (a << 4) | b


def lay_xor(u, a, b):  # low nibble b ^ a (X ^= (X >> 4) & 0x0F0F0F0F on the SWAR words)
    return (u << 8) | (a << 4) | (b ^ a)


def lay_swap(u, a, b):
    return (u << 8) | (b << 4) | a


def lay_xor_u(u, a, b):  # and the u half shifted by 16 banks
    return (u << 8) | (a << 4) | ((b ^ a) ^ (u << 3) if True else 0)


LAYOUTS = {"current a<<4|b": lay_cur, "a<<4|(b^a)": lay_xor, "b<<4|a": lay_swap, "a<<4|(b^a^8u)": lay_xor_u}


def conflicts(rec, layout, frames_per_group=4):
    fr, op, e, path, x = rec.T
    u, ab = (x >> 8) & 1, x & 255
    addr = layout(u, ab >> 4, ab & 15)
    grp = fr // frames_per_group
    key = (grp.astype(np.int64) << 40) | (op.astype(np.int64) << 12) | e
    dw = addr >> 2
    bank = dw & 31
    groups = collections.defaultdict(lambda: collections.defaultdict(set))
    for k, b, w in zip(key.tolist(), bank.tolist(), dw.tolist()):
        groups[k][b].add(w)
    cyc = extra = 0
    for g in groups.values():
        m = max(len(s) for s in g.values())
        cyc += m
        extra += m - 1
    return len(groups), cyc, extra


if __name__ == "__main__":
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    rec = run(F)
    isg = (rec[:, 4] >> 16) & 1
    print(f"bench workload, {F} frames: {len(rec)} lookups recorded (depths 1-6; f {np.sum(isg == 0)}, g {np.sum(isg == 1)})")
    for name, lay in LAYOUTS.items():
        for sel, nm in ((isg == 0, "f"), (isg == 1, "g"), (np.ones_like(isg, bool), "all")):
            ng, cyc, extra = conflicts(rec[sel], lay)
            print(f"  {name:16s} {nm:3s}: groups {ng:7d}  cycles {cyc:8d}  conflict cycles {extra:7d} ({extra / cyc:.3f})")


def search_g(rec):
    """g layouts (u << 8) | (idx ^ (u * M)): the u = 1 half XOR-swizzled by a constant M (a multiple of 8:
    the kernel's per-word index bytes XOR u_byte * M, stage_tab moves its 8-byte chunks)."""
    isg = (rec[:, 4] >> 16) & 1
    g = rec[isg == 1]
    res = []
    for M in range(0, 256, 8):
        ng, cyc, extra = conflicts(g, lambda u, a, b, M=M: (u << 8) | (((a << 4) | b) ^ (u * M)))
        res.append((extra / cyc, M, extra, cyc))
    return sorted(res)


def search_f(rec):
    """f layouts (a << 4) | (b ^ ((a >> s) & m)) -- X ^= (X >> (4 + s)) & (m * 0x01010101) on the SWAR words."""
    isg = (rec[:, 4] >> 16) & 1
    f = rec[isg == 0]
    res = []
    for s in range(4):
        for m in range(0, 16):
            ng, cyc, extra = conflicts(f, lambda u, a, b, s=s, m=m: (a << 4) | (b ^ ((a >> s) & m)))
            res.append((extra / cyc, s, m, extra, cyc))
    return sorted(res)
