// qpd_fast.hip -- the fast gfx950 LUT decode kernel (dedicated tables, v <= 16).
//
// Same algorithm, schedule and list management as the generic kernel
// (qpd_generic.hip: one lane per list path, G = pow2 >= L lanes per frame,
// per-depth 4-bit slot pointers instead of deep copies), laid out for the
// CDNA4 memory hierarchy:
//
//  * Symbols are 4-bit nibbles, 8 per dword.  Per tree depth d the path's
//    buffers are S[d] (symbols of the active depth-d node, N>>d nibbles),
//    U[d] (partial sums of the finished left child, N>>d bits) and R[d]
//    (partial sums of a finished right child, consumed by the next combine).
//  * Deep levels (d >= lds_from) -- where almost all ops and all the latency-
//    bound small ops live -- sit in LDS, laid out [row][64 lanes] so a wave's
//    row access hits 64 distinct banks; a cross-lane (pointer) read stays in
//    the same row.  Within one wave LDS instructions complete in order, so no
//    barrier is needed between an op and the next one that reads its results.
//  * Shallow levels (a few large ops per frame) sit in a per-wave global
//    scratch slab with the same row layout; ops that write it end with a
//    vmcnt drain before the next cross-lane read.
//  * The f/g tables of the current node are held in ONE VGPR per lane (f:
//    256 nibbles = 32 dwords, g: 512 nibbles = 64 dwords) and read with
//    ds_bpermute (no LDS storage, no bank conflicts); the next op's table and
//    leaf quanta row are prefetched while the current op runs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qpd_common.hpp"
#include "stl_sort.hpp"

namespace qpd {

struct FastPlan {
    int32_t N, n, K, L, v, gs, fpw, nops, max_r1;
    int32_t lds_rows, glb_rows, lds_from;
    // per-depth buffer rows; depth d lives in LDS iff d >= lds_from
    int32_t S_row[kMaxDepth + 1], U_row[kMaxDepth + 1], R_row[kMaxDepth + 1];
    int32_t H_row, K_row, I_row;  // R1 scratch (global)
    const uint32_t *f_tab;        // [N-1][32] nibble-packed f tables
    const uint32_t *g_tab;        // [N-1][64] nibble-packed g tables (u=0: dwords 0..31)
    const double *vcl;            // [rows][N][v]
    const Op *ops;
    const int32_t *info_pos;
    uint32_t *scratch;            // [waves][glb_rows][64]
    int32_t *err;
};

// Row access in either space.  `in_lds` is wave-uniform.
struct Mem {
    uint32_t *lds;
    uint32_t *glb;
    __device__ __forceinline__ uint32_t ld(bool in_lds, int row, int lane) const {
        return in_lds ? lds[row * 64 + lane] : glb[(size_t)row * 64 + lane];
    }
    __device__ __forceinline__ void st(bool in_lds, int row, int lane, uint32_t v) const {
        if (in_lds)
            lds[row * 64 + lane] = v;
        else
            glb[(size_t)row * 64 + lane] = v;
    }
};

__device__ __forceinline__ uint32_t bperm(uint32_t table, uint32_t dword) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(dword << 2), (int)table);
}

// 4-bit LUT lookup from the table register: entry idx lives in dword idx>>3.
__device__ __forceinline__ uint32_t lut4(uint32_t table, uint32_t idx) {
    return (bperm(table, idx >> 3) >> ((idx & 7u) << 2)) & 15u;
}

// Channel symbols: int32 input, range-checked (UB in the reference).
__device__ __forceinline__ uint32_t chan_sym(const int32_t *y, int e, int v, int32_t *err) {
    int s = y[e];
    if ((unsigned)s >= (unsigned)v) {
        atomicOr(err, 1);
        s = 0;
    }
    return (uint32_t)s;
}

// 8 consecutive channel symbols packed as nibbles.
__device__ __forceinline__ uint32_t chan_word(const int32_t *y, int e0, int cnt, int v, int32_t *err) {
    uint32_t w = 0;
    for (int i = 0; i < cnt; ++i) w |= chan_sym(y, e0 + i, v, err) << (4 * i);
    return w;
}

// Symbol e of the active node at depth d of the path whose slot is `src`.
__device__ __forceinline__ uint32_t node_sym4(const FastPlan &P, const Mem &M, const int32_t *y, int d, int src,
                                              int e) {
    if (d == 0) return chan_sym(y, e, P.v, P.err);
    const uint32_t w = M.ld(d >= P.lds_from, P.S_row[d] + (e >> 3), src);
    return (w >> ((e & 7) << 2)) & 15u;
}

__device__ __forceinline__ double vcl_at4(const FastPlan &P, int row, int pos, int sym) {
    return P.vcl[((size_t)row * P.N + pos) * P.v + sym];
}

// Write word w of a finished node's partial sums: left child -> own U[d],
// right child (or root) -> own R[d].
__device__ __forceinline__ void put_node(const FastPlan &P, const Mem &M, int d, bool to_r, int w, uint32_t word,
                                         int lane) {
    const bool l = d >= P.lds_from;
    M.st(l, (to_r ? P.R_row[d] : P.U_row[d]) + w, lane, word);
}

// f / g op: compute the left (f) or right (g) child symbols at depth d+1 of
// the active node at depth d (SCLLUTDecoder.cpp:83-89 / :157-164).
template <bool ISG>
__device__ __forceinline__ void fg_op(const FastPlan &P, const Mem &M, const int32_t *y, int d, int src, int usrc,
                                      uint32_t T, int lane) {
    const int ctemp = P.N >> (d + 1);
    const bool sl = d >= P.lds_from, dl = (d + 1) >= P.lds_from, ul = (d + 1) >= P.lds_from;
    const int so = P.S_row[d], to = P.S_row[d + 1], uo = P.U_row[d + 1];
    if (ctemp >= 8) {
        const int nwo = ctemp >> 3;
        for (int w = 0; w < nwo; ++w) {
            uint32_t A, B;
            if (d == 0) {
                A = chan_word(y, 8 * w, 8, P.v, P.err);
                B = chan_word(y, ctemp + 8 * w, 8, P.v, P.err);
            } else {
                A = M.ld(sl, so + w, src);
                B = M.ld(sl, so + nwo + w, src);
            }
            uint32_t ub = 0;
            if (ISG) ub = (M.ld(ul, uo + (w >> 2), usrc) >> ((w & 3) << 3)) << 8;
            uint32_t out = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t idx = (((A >> (4 * i)) & 15u) << 4) | ((B >> (4 * i)) & 15u);
                if (ISG) idx |= (ub >> i) & 256u;
                out |= lut4(T, idx) << (4 * i);
            }
            M.st(dl, to + w, lane, out);
        }
    } else {  // ctemp in {2, 4}: the whole depth-d node (a then b) is one word
        const uint32_t W = (d == 0) ? chan_word(y, 0, 2 * ctemp, P.v, P.err) : M.ld(sl, so, src);
        uint32_t ub = ISG ? M.ld(ul, uo, usrc) : 0u;
        uint32_t out = 0;
        for (int i = 0; i < ctemp; ++i) {
            uint32_t idx = (((W >> (4 * i)) & 15u) << 4) | ((W >> (4 * (i + ctemp))) & 15u);
            if (ISG) idx |= ((ub >> i) & 1u) << 8;
            out |= lut4(T, idx) << (4 * i);
        }
        M.st(dl, to, lane, out);
    }
}

// Per-lane argsort arrays (global scratch) for the R1 node.
struct FastSortSeq {
    uint32_t *glb;
    int io, ko, lane;
    __device__ int get(int p) { return (int)glb[(size_t)(io + p) * 64 + lane]; }
    __device__ void set(int p, int e) { glb[(size_t)(io + p) * 64 + lane] = (uint32_t)e; }
    __device__ double key(int e) { return ((double *)(glb + (size_t)(ko + 2 * e) * 64))[lane]; }
    __device__ bool less(int a, int b) { return key(a) < key(b); }
};

// Prefetch of the per-op operands held in registers.
struct Pre {
    uint32_t T;  // f or g table dword of this lane
    double V;    // leaf: vcl row entry of this lane (lanes < v)
};

__device__ __forceinline__ Pre fetch_pre(const FastPlan &P, const Op &op, int lane) {
    Pre p;
    p.T = 0;
    p.V = 0;
    const int posi = (1 << op.d) + op.node - 1;
    if (op.type == OP_F || op.type == OP_LEAF_L) {
        p.T = P.f_tab[(size_t)posi * 32 + (lane & 31)];
    } else if (op.type == OP_G || op.type == OP_LEAF_R) {
        p.T = P.g_tab[(size_t)posi * 64 + lane];
    }
    if (op.type == OP_LEAF_L || op.type == OP_LEAF_R) {
        const int k = 2 * op.node + (op.type == OP_LEAF_R);
        const int s = lane < P.v ? lane : 0;
        p.V = P.vcl[((size_t)(P.n - 1) * P.N + k) * P.v + s];
    }
    return p;
}

template <int KIND>
__global__ __launch_bounds__(64) void lut_fast_kernel(FastPlan P, const int32_t *__restrict__ in, int64_t B,
                                                      uint8_t *__restrict__ out) {
    constexpr bool kList = (KIND == K_SCL_LUT || KIND == K_FASTSCL_LUT);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
    int *sel = (int *)lds_dyn;  // 64 ints of survivor-selection scratch
    Mem M;
    M.lds = lds_dyn + 64;
    M.glb = P.scratch + (size_t)blockIdx.x * P.glb_rows * 64;
    const int lane = threadIdx.x;
    const int gs = P.gs;
    const int gl = lane & (gs - 1);
    const int gbase = lane & ~(gs - 1);
    const int L = kList ? P.L : 1;
    const int N = P.N, n = P.n;
    const int64_t ngroups = (B + P.fpw - 1) / P.fpw;
    const double kInf = __builtin_huge_val();

    uint64_t self = 0;
    for (int d = 0; d < kMaxDepth; ++d) self |= (uint64_t)gl << (4 * d);

    for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        int64_t frame = grp * P.fpw + lane / gs;
        const bool frame_ok = frame < B;
        if (!frame_ok) frame = B - 1;
        const int32_t *y = in + frame * (int64_t)N;
        double pm = (gl == 0) ? 0.0 : kInf;
        uint64_t ps = self, pu = self;

        Op nxt = P.ops[0];
        Pre pre = fetch_pre(P, nxt, lane);
        for (int oi = 0; oi < P.nops; ++oi) {
            const Op op = nxt;
            const Pre cur = pre;
            if (oi + 1 < P.nops) {
                nxt = P.ops[oi + 1];
                pre = fetch_pre(P, nxt, lane);
            }
            const int d = op.d, node = op.node;
            bool touched_glb = d < P.lds_from;
            switch (op.type) {
                case OP_F:
                    fg_op<false>(P, M, y, d, gbase + ptr_get(ps, d), 0, cur.T, lane);
                    ps = ptr_set(ps, d + 1, gl);
                    touched_glb = (d + 1) < P.lds_from;
                    break;
                case OP_G:
                    fg_op<true>(P, M, y, d, gbase + ptr_get(ps, d), gbase + ptr_get(pu, d + 1), cur.T, lane);
                    ps = ptr_set(ps, d + 1, gl);
                    touched_glb = (d + 1) < P.lds_from;
                    break;
                case OP_LEAF_L:
                case OP_LEAF_R: {
                    const bool right = op.type == OP_LEAF_R;
                    const bool frozen = op.aux != 0;
                    const int src = gbase + ptr_get(ps, d);
                    uint32_t dec = 0;
                    if (kList || !frozen) {
                        uint32_t a, b;
                        if (d == 0) {
                            a = chan_sym(y, 0, P.v, P.err);
                            b = chan_sym(y, 1, P.v, P.err);
                        } else {
                            const uint32_t W = M.ld(d >= P.lds_from, P.S_row[d], src);
                            a = W & 15u;
                            b = (W >> 4) & 15u;
                        }
                        uint32_t idx = (a << 4) | b;
                        if (right) idx |= (M.ld(n >= P.lds_from, P.U_row[n], gbase + ptr_get(pu, n)) & 1u) << 8;
                        const int s = (int)lut4(cur.T, idx);
                        const double dm = shfld(cur.V, s);  // vcl[n-1][k][s] (H3)
                        if (!kList) {
                            dec = dm <= 0;  // H4
                        } else if (frozen) {
                            pm += fabs(dm) * (double)(dm < 0);
                        } else {
                            const double kf = pm + fabs(dm);
                            const Sel sl = select_survivors(pm, kf, gl, gbase, L, sel);
                            const int p = gbase + sl.parent;
                            const uint32_t hd = dm < 0;
                            dec = (uint32_t)__shfl((int)hd, p) ^ (sl.upper ? 1u : 0u);
                            pm = pick(sl.upper, shfld(kf, p), shfld(pm, p));
                            ps = shfl64(ps, p);
                            pu = shfl64(pu, p);
                        }
                    }
                    const bool l = n >= P.lds_from;
                    if (right) {
                        M.st(l, P.R_row[n], lane, dec);
                    } else {
                        M.st(l, P.U_row[n], lane, dec);
                        pu = ptr_set(pu, n, gl);
                    }
                    touched_glb = !l;
                    break;
                }
                case OP_COMB: {
                    const int ctemp = N >> (d + 1);
                    const int usrc = gbase + ptr_get(pu, d + 1);
                    const bool to_r = (d == 0) || (node & 1);
                    const bool cl = (d + 1) >= P.lds_from;
                    if (ctemp < 32) {
                        const uint32_t m = (1u << ctemp) - 1u;
                        const uint32_t ul = M.ld(cl, P.U_row[d + 1], usrc) & m;
                        const uint32_t r = M.ld(cl, P.R_row[d + 1], lane) & m;
                        put_node(P, M, d, to_r, 0, (ul ^ r) | (r << ctemp), lane);
                    } else {
                        const int cw = ctemp >> 5;
                        for (int w = 0; w < cw; ++w) {
                            const uint32_t ul = M.ld(cl, P.U_row[d + 1] + w, usrc);
                            const uint32_t r = M.ld(cl, P.R_row[d + 1] + w, lane);
                            put_node(P, M, d, to_r, w, ul ^ r, lane);
                            put_node(P, M, d, to_r, cw + w, r, lane);
                        }
                    }
                    if (!to_r) pu = ptr_set(pu, d, gl);
                    touched_glb = d < P.lds_from || (d + 1) < P.lds_from;
                    break;
                }
                default: {  // special nodes, FastSCLUT.cpp:46-107 / FastSCLLUTDecoder.cpp:82-213
                    const int temp = N >> d;
                    const int src = gbase + ptr_get(ps, d);
                    const bool to_r = (node & 1);
                    const int base_pos = temp * node;
                    const int nwo = (temp + 31) >> 5;
                    if (op.type == OP_R0) {
                        if (kList) {
                            for (int j = 0; j < temp; ++j) {
                                const double l = vcl_at4(P, d - 1, base_pos + j, (int)node_sym4(P, M, y, d, src, j));
                                pm += (double)(float)(l < 0) * fabs(l);
                            }
                        }
                        for (int w = 0; w < nwo; ++w) put_node(P, M, d, to_r, w, 0u, lane);
                    } else if (op.type == OP_REP) {
                        uint32_t fill = 0;
                        if (!kList) {
                            double S = 0;
                            for (int j = 0; j < temp; ++j)
                                S += vcl_at4(P, d - 1, base_pos + j, (int)node_sym4(P, M, y, d, src, j));
                            fill = S <= 0 ? 0xffffffffu : 0u;
                        } else {
                            double kk = pm, kf = pm;
                            for (int j = 0; j < temp; ++j) {
                                const double l = vcl_at4(P, d - 1, base_pos + j, (int)node_sym4(P, M, y, d, src, j));
                                kk += (double)(l < 0) * fabs(l);
                                kf += (double)(l >= 0) * fabs(l);
                            }
                            const Sel sl = select_survivors(kk, kf, gl, gbase, L, sel);
                            const int p = gbase + sl.parent;
                            pm = pick(sl.upper, shfld(kf, p), shfld(kk, p));
                            ps = shfl64(ps, p);
                            pu = shfl64(pu, p);
                            fill = sl.upper ? 0xffffffffu : 0u;
                        }
                        const uint32_t m = temp < 32 ? ((1u << temp) - 1u) : 0xffffffffu;
                        for (int w = 0; w < nwo; ++w) put_node(P, M, d, to_r, w, fill & m, lane);
                    } else if (op.type == OP_SPC) {  // FastSC only
                        uint32_t parity = 0;
                        double best = 0;
                        int bi = 0;
                        uint32_t bw = 0;  // word holding the first-min position
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = 0;
                            for (int i = 0; i < 32 && 32 * w + i < temp; ++i) {
                                const int j = 32 * w + i;
                                const double l = vcl_at4(P, d - 1, base_pos + j, (int)node_sym4(P, M, y, d, src, j));
                                const uint32_t h = l <= 0;
                                word |= h << i;
                                parity ^= h;
                                const double a = fabs(l);
                                if (j == 0 || a < best) {  // first minimum (H6)
                                    best = a;
                                    bi = j;
                                }
                            }
                            put_node(P, M, d, to_r, w, word, lane);
                        }
                        if (parity) {
                            const bool l = d >= P.lds_from;
                            const int row = (to_r ? P.R_row[d] : P.U_row[d]) + (bi >> 5);
                            bw = M.ld(l, row, lane) ^ (1u << (bi & 31));
                            M.st(l, row, lane, bw);
                        }
                    } else if (!kList) {  // OP_R1, FastSC: `<= 0`
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = 0;
                            for (int i = 0; i < 32 && 32 * w + i < temp; ++i) {
                                const int j = 32 * w + i;
                                const double l = vcl_at4(P, d - 1, base_pos + j, (int)node_sym4(P, M, y, d, src, j));
                                word |= (uint32_t)(l <= 0) << i;
                            }
                            put_node(P, M, d, to_r, w, word, lane);
                        }
                    } else if constexpr (KIND == K_FASTSCL_LUT) {  // OP_R1, FastSCL: :99-166
                        const int m = (L - 1) < temp ? (L - 1) : temp;
                        uint32_t *g = M.glb;
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = 0;
                            for (int i = 0; i < 32 && 32 * w + i < temp; ++i) {
                                const int j = 32 * w + i;
                                const double l = vcl_at4(P, d - 1, base_pos + j, (int)node_sym4(P, M, y, d, src, j));
                                word |= (uint32_t)(l < 0) << i;
                                ((double *)(g + (size_t)(P.K_row + 2 * j) * 64))[lane] = fabs(l);
                            }
                            g[(size_t)(P.H_row + w) * 64 + lane] = word;
                        }
                        int ord[kMaxM];
                        double ms[kMaxM];
                        int flip[kMaxM];
#pragma unroll
                        for (int q = 0; q < kMaxM; ++q) {
                            ord[q] = 0;
                            ms[q] = 0;
                            flip[q] = -1;
                        }
                        FastSortSeq seq{g, P.I_row, P.K_row, lane};
                        if (temp <= stl::kThreshold) {
                            uint32_t taken = 0;
#pragma unroll
                            for (int q = 0; q < kMaxM; ++q) {
                                if (q < m) {
                                    int bj = -1;
                                    double bk = 0;
                                    for (int j = 0; j < temp; ++j) {
                                        if (taken & (1u << j)) continue;
                                        const double kj = seq.key(j);
                                        if (bj < 0 || kj < bk) {
                                            bj = j;
                                            bk = kj;
                                        }
                                    }
                                    taken |= 1u << bj;
                                    ord[q] = bj;
                                    ms[q] = bk;
                                }
                            }
                        } else {
                            for (int p = 0; p < temp; ++p) seq.set(p, p);
                            stl::sort(seq, 0, temp);
#pragma unroll
                            for (int q = 0; q < kMaxM; ++q) {
                                if (q < m) {
                                    ord[q] = seq.get(q);
                                    ms[q] = seq.key(ord[q]);
                                }
                            }
                        }
                        wave_sync();  // H rows visible to the whole wave
                        int origin = gl;
#pragma unroll
                        for (int layer = 0; layer < kMaxM; ++layer) {
                            if (layer < m) {
                                const double kf = pm + ms[layer];
                                const Sel sl = select_survivors(pm, kf, gl, gbase, L, sel);
                                const int p = gbase + sl.parent;
                                const int pos_old = ord[layer];  // H2
                                pm = pick(sl.upper, shfld(kf, p), shfld(pm, p));
                                ps = shfl64(ps, p);
                                pu = shfl64(pu, p);
                                origin = __shfl(origin, p);
#pragma unroll
                                for (int q = 0; q < kMaxM; ++q) {
                                    ord[q] = __shfl(ord[q], p);
                                    ms[q] = shfld(ms[q], p);
                                    if (q < layer) flip[q] = __shfl(flip[q], p);
                                }
                                flip[layer] = sl.upper ? pos_old : -1;
                            }
                        }
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = g[(size_t)(P.H_row + w) * 64 + gbase + origin];
#pragma unroll
                            for (int q = 0; q < kMaxM; ++q)
                                if (q < m && flip[q] >= 0 && (flip[q] >> 5) == w) word ^= 1u << (flip[q] & 31);
                            if (temp < 32) word &= (1u << temp) - 1u;
                            put_node(P, M, d, to_r, w, word, lane);
                        }
                        touched_glb = true;
                    }
                    if (!to_r) pu = ptr_set(pu, d, gl);
                    break;
                }
            }
            if (touched_glb) wave_sync();  // drain global writes before any cross-lane read
        }

        // Root partial sums -> u = x F^{(x)n} (FastSCLUT.cpp:186-198), R[0] rows.
        const bool rl = 0 >= P.lds_from;
        const int r0 = P.R_row[0];
        const int nwr = (N + 31) >> 5;
        for (int w = 0; w < nwr; ++w) {
            uint32_t x = M.ld(rl, r0 + w, lane);
            if (N < 32) x &= (1u << N) - 1u;
            x ^= (x >> 1) & 0x55555555u;
            x ^= (x >> 2) & 0x33333333u;
            x ^= (x >> 4) & 0x0f0f0f0fu;
            x ^= (x >> 8) & 0x00ff00ffu;
            x ^= (x >> 16) & 0x0000ffffu;
            M.st(rl, r0 + w, lane, x);
        }
        for (int mw = 1; mw < nwr; mw *= 2)
            for (int i = 0; i < nwr; i += 2 * mw)
                for (int j = 0; j < mw; ++j)
                    M.st(rl, r0 + i + j, lane, M.ld(rl, r0 + i + j, lane) ^ M.ld(rl, r0 + i + mw + j, lane));
        wave_sync();
        int best = 0;
        if (kList) {
            double bpm = shfld(pm, gbase);
            for (int j = 1; j < L; ++j) {
                const double pj = shfld(pm, gbase + j);
                if (pj < bpm) {
                    bpm = pj;
                    best = j;
                }
            }
        }
        if (frame_ok) {
            for (int t = gl; t < P.K; t += gs) {
                const int pos = P.info_pos[t];
                out[frame * P.K + t] = (uint8_t)((M.ld(rl, r0 + (pos >> 5), gbase + best) >> (pos & 31)) & 1u);
            }
        }
        wave_sync();
    }
}

}  // namespace qpd
