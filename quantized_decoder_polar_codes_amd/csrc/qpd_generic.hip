#pragma once
// qpd_generic.hip -- generic gfx950 engine: every decoder of the reference,
// LUT symbols or fp64 LLRs, any table layout.
//
// Work mapping: one 64-lane wavefront per workgroup; a frame
// owns a group of G = pow2 >= L consecutive lanes, one lane per list path, so
// a wave decodes 64/G frames at once (8 at L=8, 64 for SC).  Every frame runs
// the SAME static traversal schedule (host-compiled op list, qpd_capi.hip), so
// control flow is wave-uniform; only data differs between lanes.
//
// List management without the reference's per-fork deep copies
// (src/SCLLUTDecoder.cpp:135-144): each path keeps, per
// tree depth, a 4-bit pointer to the lane whose scratch slot holds its data
// (Balatsoukas-Stimming pointer memory).  A path always writes its own slot;
// a fork copies two 64-bit pointer words from the parent lane instead of
// ~450 KB of state.  Path metrics are fp64, accumulated in exactly the
// reference's order (hazard H5); survivor selection reproduces libstdc++
// std::sort tie order (H1) -- insertion sort (stable) for 2L <= 16 via exact
// ranks, full introsort replay (stl_sort.hpp) for the R1 argsort.
//
// Symbol domains (template parameter DOM, qpd_common.hpp):
//   DOM_LUT      int symbols (one byte per element in scratch), f/g by the
//                per-node tables, node LLR = vcl[row][pos][sym] (H3)
//   DOM_FLOAT    fp64 LLRs (two dwords per element), min-sum f/g
//                (utils.cpp:26-36), node LLR = the value itself
//   DOM_UNIFORM  DOM_FLOAT + uniform re-quantization Q after every f/g
//                (utils.cpp:8-10, q_f/q_g :38-48)
//   DOM_LLOYD    DOM_FLOAT + Lloyd bisect after every f/g (utils.cpp:12-24,
//                non_uniform_q_f/g :50-60)
// The decoder families (KIND) are the reference's SC / SCL / FastSC / FastSCL
// classes, so every one of its 15 decoders is one (KIND, DOM) instantiation
// plus the CRC-aided epilogue.
//
// Per-lane state lives in a per-wave scratch slab laid out [row][64 lanes]
// (one dword per lane per row), so a row access by the wave is one fully
// coalesced 256-B transaction; cross-lane reads stay inside that line.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "qpd_common.hpp"
#include "stl_sort.hpp"

namespace qpd {

struct DevPlan {
    int32_t N, n, K, L, v, gs, fpw, nops;
    int32_t f_step, g_step, max_r1;
    int32_t rows_per_wave;
    int32_t out_k;         // output bits per frame: K, or A (CRC-aided kinds)
    int32_t ca_A, crc_n;   // crc_n > 0: CRC-aided output (ca_winner)
    int32_t ca_chk;        // bits compared after the A info bits
    uint32_t crc_q;
    double pm_init;        // initial metric of paths 1..L-1 (DOUBLE_INF of the class)
    const uint32_t *info_mask;  // [N/32] information-position mask
    // scratch row offsets: S[d] (values of the active node at depth d: bytes
    // for LUT symbols, two rows per element for fp64), U[d] (partial sums of
    // the finished left child at depth d, bits), R (right-chain partial sums,
    // own lane), H (R1 hard decisions), I / Kd (R1 argsort index / key arrays).
    int32_t So[kMaxDepth + 1], Uo[kMaxDepth + 1], Ro, Ho, Io, Ko;
    const uint8_t *lut_f;
    const int32_t *f_base;
    const uint8_t *lut_g;
    const int32_t *g_base;
    const double *vcl;
    // re-quantizers of the float domains (indexed by node_posi; Lloyd table t
    // = 0 (f) / 1 (g) of node p at offset/length [t*(N-1) + p])
    const double *r_f, *r_g;
    const double *q_bnd, *q_rec;
    const int32_t *bnd_off, *bnd_len, *rec_off, *rec_len;
    const Op *ops;
    const int32_t *info_pos;
    uint32_t *scratch;
    int32_t *err;
    uint32_t *task_ctr;  // task queue: groups taken (never reset; see wave_take)
    uint32_t task_base;  // per launch: the counter's value when this launch's takes begin
};

__device__ __forceinline__ double vcl_at(const DevPlan &P, int row, int pos, int sym) {
    return P.vcl[((size_t)row * P.N + pos) * P.v + sym];
}


// Channel symbol read with range check (the reference has none: UB there).
__device__ __forceinline__ int in_sym(const DevPlan &P, const int32_t *y, int e) {
    int s = y[e];
    if ((unsigned)s >= (unsigned)P.v) {
        atomicOr(P.err, ERR_SYMBOL);
        s = 0;
    }
    return s;
}


// Value e of the active node at depth d, for the path whose slot is `src`.
template <int DOM, class In>
__device__ __forceinline__ auto node_val(const DevPlan &P, uint32_t *wsc, const In *y, int d, int src, int e) {
    if constexpr (DOM == DOM_LUT) {
        if (d == 0) return in_sym(P, y, e);
        uint32_t w = row_ptr(wsc, P.So[d] + (e >> 2))[src];
        return (int)((w >> (8 * (e & 3))) & 255u);
    } else {
        if (d == 0) return (double)y[e];
        return ((const double *)row_ptr(wsc, P.So[d] + 2 * e))[src];
    }
}

__device__ __forceinline__ void set_fval(const DevPlan &P, uint32_t *wsc, int d, int e, int lane, double x) {
    ((double *)row_ptr(wsc, P.So[d] + 2 * e))[lane] = x;
}


// ---------------------------------------------------------------------------
// fp64 f/g of the float domains, written as the reference writes them and with
// contraction off so that each product and sum rounds exactly as in its
// scalar C++ (every product involved is by +-1, 0/1 or 0.5, so FMA would not
// change a result either; this keeps it true by construction).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int sgn(double x) { return x < 0 ? -1 : (x > 0); }  // utils.h:13
__device__ __forceinline__ double std_min(double a, double b) { return (b < a) ? b : a; }

// Q(x, r, M), utils.cpp:8-10
__device__ __forceinline__ double q_uniform(double x, double r, double M) {
#pragma clang fp contract(off)
    return fabs(x) > M ? (double)sgn(x) * (M - 0.5 * r) : (floor(x / r) + 0.5) * r;
}

// bisect, utils.cpp:12-24: reconstruct[lo - 1] with lo = the first index whose
// boundary is not below x (the same probe sequence, so unsorted lists agree
// too).  lo - 1 outside the reconstruction list reads out of bounds in the
// reference (UB): flagged, and 0 is used.
__device__ __forceinline__ double q_lloyd(const DevPlan &P, double x, int t, int posi) {
    const int k = t * (P.N - 1) + posi;
    const double *b = P.q_bnd + P.bnd_off[k];
    int lo = 0, hi = P.bnd_len[k];
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if (b[mid] < x)
            lo = mid + 1;
        else
            hi = mid;
    }
    if (lo - 1 < 0 || lo - 1 >= P.rec_len[k]) {
        atomicOr(P.err, ERR_LLOYD);
        return 0.0;
    }
    return P.q_rec[P.rec_off[k] + lo - 1];
}

template <int DOM>
__device__ __forceinline__ double fd_f(const DevPlan &P, int posi, double a, double b) {
#pragma clang fp contract(off)
    const double x = (double)(sgn(a) * sgn(b)) * std_min(fabs(a), fabs(b));  // utils.cpp:28
    if constexpr (DOM == DOM_UNIFORM) {
        const double r = P.r_f[posi];
        return q_uniform(x, r, ((double)(P.v / 2) - 0.5) * r);  // SCUniformQuantizedDecoder.cpp:55-57
    } else if constexpr (DOM == DOM_LLOYD) {
        return q_lloyd(P, x, 0, posi);
    } else {
        return x;
    }
}

template <int DOM>
__device__ __forceinline__ double fd_g(const DevPlan &P, int posi, int u, double a, double b) {
#pragma clang fp contract(off)
    const double x = (double)(1 - 2 * u) * a + b;  // utils.cpp:34
    if constexpr (DOM == DOM_UNIFORM) {
        const double r = P.r_g[posi];
        return q_uniform(x, r, (double)(P.v / 2 - 1) * r);  // SCUniformQuantizedDecoder.cpp:71-73
    } else if constexpr (DOM == DOM_LLOYD) {
        return q_lloyd(P, x, 1, posi);
    } else {
        return x;
    }
}


// LLR of a node element: the LUT domain reads vcl[row][pos][sym] (H3), the
// float domains hold the LLR itself.
template <int DOM, class T>
__device__ __forceinline__ double node_llr(const DevPlan &P, int row, int pos, T s) {
    if constexpr (DOM == DOM_LUT)
        return vcl_at(P, row, pos, s);
    else
        return s;
}


// Write the finished node's partial sums (nbits bits, in `words`) either to the
// path's own U[d] slot (left child) or to the own R chain (right child / root).
__device__ __forceinline__ void store_node_word(const DevPlan &P, uint32_t *wsc, int d, bool to_r, int w,
                                                uint32_t word, int lane) {
    if (to_r)
        row_ptr(wsc, P.Ro + w)[lane] = word;
    else
        row_ptr(wsc, P.Uo[d] + w)[lane] = word;
}

// Per-lane argsort arrays for the R1 node (stl_sort.hpp Seq interface).
struct LaneSortSeq {
    uint32_t *wsc;
    int io, ko, lane;
    __device__ int get(int p) { return (int)row_ptr(wsc, io + p)[lane]; }
    __device__ void set(int p, int e) { row_ptr(wsc, io + p)[lane] = (uint32_t)e; }
    __device__ double key(int e) { return ((double *)row_ptr(wsc, ko + 2 * e))[lane]; }
    __device__ bool less(int a, int b) { return key(a) < key(b); }
};

// List pointer words (pointer memory): per tree depth, the lane-in-group whose
// slot holds the path's data.  4-bit fields in 64 bits for lane groups of up
// to 16 lanes (L <= 8 instantiations), 5-bit fields in 128 bits for groups of
// 32 (the wide instantiations, L <= 32).
template <int ML>
struct PtrW {
    using T = uint64_t;
    static constexpr int B = 4;
};
template <>
struct PtrW<kMaxLWide> {
    using T = unsigned __int128;
    static constexpr int B = 5;
};

template <int ML>
__device__ __forceinline__ int gp_get(typename PtrW<ML>::T p, int d) {
    return (int)(p >> (PtrW<ML>::B * d)) & ((1 << PtrW<ML>::B) - 1);
}

template <int ML>
__device__ __forceinline__ typename PtrW<ML>::T gp_set(typename PtrW<ML>::T p, int d, int v) {
    using T = typename PtrW<ML>::T;
    const T m = (T)((1u << PtrW<ML>::B) - 1u) << (PtrW<ML>::B * d);
    return (p & ~m) | ((T)(unsigned)v << (PtrW<ML>::B * d));
}

template <int ML>
__device__ __forceinline__ typename PtrW<ML>::T gp_shfl(typename PtrW<ML>::T x, int src) {
    if constexpr (ML == kMaxLWide) {
        const uint64_t lo = shfl64((uint64_t)x, src), hi = shfl64((uint64_t)(x >> 64), src);
        return ((unsigned __int128)hi << 64) | lo;
    } else {
        return shfl64(x, src);
    }
}

// Index arrays sorted in LDS by their keys (stl_sort.hpp Seq interface).
struct LdsSortSeq {
    int *idx;
    const double *key;
    __device__ int get(int p) { return idx[p]; }
    __device__ void set(int p, int e) { idx[p] = e; }
    __device__ bool less(int a, int b) { return key[a] < key[b]; }
};

// LDS of the list selection: ranks (sel) and, for 2L > 16, the candidate
// keys and index array the group's lane 0 sorts.
struct ListLds {
    int sel[64];
    int idx[128];
    double key[128];
};

// Survivor selection, mink (src/SCLLUTDecoder.cpp:8-21): 2L <= 16 by stable
// ranks (insertion sort); 2L > 16 (wide instantiations) by replaying
// libstdc++'s introsort of the 2L candidates [PML_0..L-1, PML_i + |DM_i|] on
// lane 0 of each group and taking the first L (H1).
template <int ML>
__device__ __forceinline__ Sel gselect(double kk, double kf, int gl, int gbase, int L, ListLds &sh) {
    if constexpr (ML == kMaxLWide) {
        if (2 * L > stl::kThreshold) {
            double *key = sh.key + 2 * gbase;
            int *idx = sh.idx + 2 * gbase;
            if (gl < L) {
                key[gl] = kk;
                key[L + gl] = kf;
            }
            lds_order();
            if (gl == 0) {
                LdsSortSeq seq{idx, key};
                for (int p = 0; p < 2 * L; ++p) idx[p] = p;
                if (2 * L <= 2 * stl::kThreshold + 1)
                    stl::sort_small_prefix(seq, 0, 2 * L, L);
                else
                    stl::sort(seq, 0, 2 * L);
                for (int i = 0; i < L; ++i) sh.sel[gbase + i] = idx[i];
            }
            lds_order();
            const int c = gl < L ? sh.sel[gbase + gl] : gl;
            lds_order();
            Sel s;
            s.upper = c >= L;
            s.parent = s.upper ? c - L : c;
            return s;
        }
    }
    return select_survivors(kk, kf, gl, gbase, L, sh.sel);
}

// Position of this path in argsort(PML) (the CA epilogue, CASCLLUTDecoder.cpp:264):
// stable for L <= 16, the introsort replay above that.
template <int ML>
__device__ __forceinline__ int grank(double pm, int gl, int gbase, int L, ListLds &sh) {
    if constexpr (ML == kMaxLWide) {
        if (L > stl::kThreshold) {
            double *key = sh.key + 2 * gbase;
            int *idx = sh.idx + 2 * gbase;
            if (gl < L) key[gl] = pm;
            lds_order();
            if (gl == 0) {
                LdsSortSeq seq{idx, key};
                for (int p = 0; p < L; ++p) idx[p] = p;
                stl::sort_small(seq, 0, L);
                for (int i = 0; i < L; ++i) sh.sel[gbase + idx[i]] = i;
            }
            lds_order();
            const int r = gl < L ? sh.sel[gbase + gl] : 0;
            lds_order();
            return r;
        }
    }
    return stable_rank(pm, gl, gbase, L);
}

// A NaN path metric would reach std::sort (UB in the reference): flag it.
template <int DOM>
__device__ __forceinline__ void check_keys(const DevPlan &P, double a, double b) {
    if constexpr (DOM != DOM_LUT) {
        if (a != a || b != b) atomicOr(P.err, ERR_NAN_PM);
    }
}

// ---------------------------------------------------------------------------
// The decoders.  KIND = family (SC / SCL / FastSC / FastSCL), DOM = domain.
// ---------------------------------------------------------------------------
template <int KIND, int DOM, int ML>
__global__ __launch_bounds__(64) void generic_decode_kernel(DevPlan P,
                                                            const std::conditional_t<DOM == DOM_LUT, int32_t, double>
                                                                *__restrict__ in,
                                                            int64_t B, uint8_t *__restrict__ out) {
    constexpr bool kList = (KIND == K_SCL_LUT || KIND == K_FASTSCL_LUT);
    constexpr bool kLut = DOM == DOM_LUT;
    using In = std::conditional_t<kLut, int32_t, double>;
    __shared__ ListLds sh;
    using PT = typename PtrW<ML>::T;
    constexpr int MM = ML - 1;  // R1 layers kept in registers: min(L - 1, temp)
    const int lane = threadIdx.x;
    const int gs = P.gs;
    const int gl = lane & (gs - 1);
    const int gbase = lane & ~(gs - 1);
    const int L = kList ? P.L : 1;
    const int N = P.N, n = P.n, v = P.v;
    const int vv = v * v;
    uint32_t *wsc = P.scratch + (size_t)blockIdx.x * P.rows_per_wave * 64;
    const int64_t ngroups = (B + P.fpw - 1) / P.fpw;

    PT self = 0;
    for (int d = 0; d <= kMaxDepth && PtrW<ML>::B * (d + 1) <= (int)(8 * sizeof(PT)); ++d) self = gp_set<ML>(self, d, gl);

    // groups: the first blockIdx.x, then the next untaken one (qpd_common.hpp)
    for (int64_t grp = blockIdx.x; grp < ngroups;
         grp = QPD_DYN ? (int64_t)gridDim.x + wave_take(P.task_ctr, P.task_base) : grp + gridDim.x) {
        int64_t frame = grp * P.fpw + lane / gs;
        const bool frame_ok = frame < B;
        if (!frame_ok) frame = B - 1;
        const In *y = in + frame * (int64_t)N;
        double pm = (gl == 0) ? 0.0 : P.pm_init;
        PT ps = self, pu = self;

        for (int oi = 0; oi < P.nops; ++oi) {
            const Op op = P.ops[oi];
            const int d = op.d, node = op.node;
            const int posi = (1 << d) + node - 1;
            switch (op.type) {
                case OP_F:
                case OP_G: {
                    const bool isg = op.type == OP_G;
                    const int ctemp = N >> (d + 1);
                    const int src = gbase + gp_get<ML>(ps, d);
                    const int usrc = gbase + gp_get<ML>(pu, d + 1);
                    if constexpr (kLut) {
                        const uint8_t *T = isg ? P.lut_g : P.lut_f;
                        const int tsz = isg ? 2 * vv : vv;
                        const int tb = isg ? P.g_base[posi] : P.f_base[posi];
                        const int ts = isg ? P.g_step : P.f_step;
                        const int nw = (ctemp + 3) >> 2;
                        for (int w = 0; w < nw; ++w) {
                            uint32_t ub = 0;
                            if (isg) ub = row_ptr(wsc, P.Uo[d + 1] + ((4 * w) >> 5))[usrc] >> ((4 * w) & 31);
                            uint32_t res = 0;
                            const int ne = ctemp < 4 ? ctemp : 4;
                            for (int i = 0; i < ne; ++i) {
                                const int e = 4 * w + i;
                                const int a = node_val<DOM>(P, wsc, y, d, src, e);
                                const int b = node_val<DOM>(P, wsc, y, d, src, e + ctemp);
                                const int u = (ub >> i) & 1;
                                const size_t t = (size_t)(tb + e * ts);
                                const uint32_t val = T[t * tsz + u * vv + a * v + b];
                                res |= val << (8 * i);
                            }
                            row_ptr(wsc, P.So[d + 1] + w)[lane] = res;
                        }
                    } else {
                        for (int e = 0; e < ctemp; ++e) {
                            const double a = node_val<DOM>(P, wsc, y, d, src, e);
                            const double b = node_val<DOM>(P, wsc, y, d, src, e + ctemp);
                            double r;
                            if (isg) {
                                const int u = (row_ptr(wsc, P.Uo[d + 1] + (e >> 5))[usrc] >> (e & 31)) & 1;
                                r = fd_g<DOM>(P, posi, u, a, b);
                            } else {
                                r = fd_f<DOM>(P, posi, a, b);
                            }
                            set_fval(P, wsc, d + 1, e, lane, r);
                        }
                    }
                    ps = gp_set<ML>(ps, d + 1, gl);
                    break;
                }
                case OP_LEAF_L:
                case OP_LEAF_R: {
                    const bool right = op.type == OP_LEAF_R;
                    const int k = 2 * node + (right ? 1 : 0);
                    const bool frozen = op.aux != 0;
                    const int src = gbase + gp_get<ML>(ps, d);
                    uint32_t dec = 0;
                    if (!kList && frozen) {
                        dec = 0;  // SCLUTDecoder.cpp:60-61 / SCDecoder.cpp:25-26: frozen leaves are 0
                    } else {
                        const auto a = node_val<DOM>(P, wsc, y, d, src, 0);
                        const auto b = node_val<DOM>(P, wsc, y, d, src, 1);
                        double dm;
                        if constexpr (kLut) {
                            int s;
                            if (right) {
                                const int u = row_ptr(wsc, P.Uo[n])[gbase + gp_get<ML>(pu, n)] & 1;
                                s = P.lut_g[(size_t)P.g_base[posi] * 2 * vv + u * vv + a * v + b];
                            } else {
                                s = P.lut_f[(size_t)P.f_base[posi] * vv + a * v + b];
                            }
                            dm = vcl_at(P, n - 1, k, s);  // H3: row n-1
                        } else {
                            if (right) {
                                const int u = row_ptr(wsc, P.Uo[n])[gbase + gp_get<ML>(pu, n)] & 1;
                                dm = fd_g<DOM>(P, posi, u, a, b);
                            } else {
                                dm = fd_f<DOM>(P, posi, a, b);
                            }
                        }
                        if (!kList) {
                            dec = dm <= 0;  // H4: SC family `<= 0`
                        } else if (frozen) {
#pragma clang fp contract(off)
                            pm += fabs(dm) * (double)(dm < 0);  // :100-104
                        } else {
                            const double kf = pm + fabs(dm);
                            check_keys<DOM>(P, pm, kf);
                            const Sel sl = gselect<ML>(pm, kf, gl, gbase, L, sh);
                            const int p = gbase + sl.parent;
                            const uint32_t hd = dm < 0;  // H4: SCL family `< 0`
                            dec = (uint32_t)__shfl((int)hd, p) ^ (sl.upper ? 1u : 0u);
                            pm = pick(sl.upper, shfld(kf, p), shfld(pm, p));
                            ps = gp_shfl<ML>(ps, p);
                            pu = gp_shfl<ML>(pu, p);
                        }
                    }
                    if (right) {
                        row_ptr(wsc, P.Ro)[lane] = dec;
                    } else {
                        row_ptr(wsc, P.Uo[n])[lane] = dec;
                        pu = gp_set<ML>(pu, n, gl);
                    }
                    break;
                }
                case OP_COMB: {
                    const int ctemp = N >> (d + 1);
                    const int usrc = gbase + gp_get<ML>(pu, d + 1);
                    const bool to_r = (d == 0) || (node & 1);
                    if (ctemp < 32) {
                        const uint32_t m = (1u << ctemp) - 1u;
                        const uint32_t ul = row_ptr(wsc, P.Uo[d + 1])[usrc] & m;
                        const uint32_t r = row_ptr(wsc, P.Ro)[lane] & m;
                        store_node_word(P, wsc, d, to_r, 0, (ul ^ r) | (r << ctemp), lane);
                    } else {
                        const int cw = ctemp >> 5;
                        for (int w = 0; w < cw; ++w) {
                            const uint32_t ul = row_ptr(wsc, P.Uo[d + 1] + w)[usrc];
                            const uint32_t r = row_ptr(wsc, P.Ro + w)[lane];
                            store_node_word(P, wsc, d, to_r, cw + w, r, lane);
                            store_node_word(P, wsc, d, to_r, w, ul ^ r, lane);
                        }
                    }
                    if (!to_r) pu = gp_set<ML>(pu, d, gl);
                    break;
                }
                default: {  // special nodes, FastSCLUT.cpp:46-107 / FastSCLLUTDecoder.cpp:82-213,
                            // FastSCDecoder.cpp:45-106 / FastSCLDecoder.cpp:122-251
                    const int temp = N >> d;
                    const int src = gbase + gp_get<ML>(ps, d);
                    const bool to_r = (node & 1);
                    const int base_pos = temp * node;
                    const int nwo = (temp + 31) >> 5;
                    // LLR of element j: vcl row depth-1 (H3) or the value itself
                    auto lval = [&](int j) {
                        return node_llr<DOM>(P, d - 1, base_pos + j, node_val<DOM>(P, wsc, y, d, src, j));
                    };
                    if (op.type == OP_R0) {
                        if (kList) {
#pragma clang fp contract(off)
                            for (int j = 0; j < temp; ++j) {
                                const double l = lval(j);
                                pm += (double)(float)(l < 0) * fabs(l);
                            }
                        }
                        for (int w = 0; w < nwo; ++w) store_node_word(P, wsc, d, to_r, w, 0u, lane);
                    } else if (op.type == OP_REP) {
                        uint32_t fill = 0;
                        if (!kList) {
                            double S = 0;
                            for (int j = 0; j < temp; ++j) S += lval(j);
                            fill = S <= 0 ? 0xffffffffu : 0u;
                        } else {
#pragma clang fp contract(off)
                            double kk = pm, kf = pm;
                            for (int j = 0; j < temp; ++j) {
                                const double l = lval(j);
                                kk += (double)(l < 0) * fabs(l);
                                kf += (double)(l >= 0) * fabs(l);
                            }
                            check_keys<DOM>(P, kk, kf);
                            const Sel sl = gselect<ML>(kk, kf, gl, gbase, L, sh);
                            const int p = gbase + sl.parent;
                            pm = pick(sl.upper, shfld(kf, p), shfld(kk, p));
                            ps = gp_shfl<ML>(ps, p);
                            pu = gp_shfl<ML>(pu, p);
                            fill = sl.upper ? 0xffffffffu : 0u;
                        }
                        const uint32_t m = temp < 32 ? ((1u << temp) - 1u) : 0xffffffffu;
                        for (int w = 0; w < nwo; ++w) store_node_word(P, wsc, d, to_r, w, fill & m, lane);
                    } else if (op.type == OP_SPC) {  // FastSC only
                        uint32_t parity = 0;
                        double best = 0;
                        int bi = 0;
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = 0;
                            for (int i = 0; i < 32 && 32 * w + i < temp; ++i) {
                                const int j = 32 * w + i;
                                const double l = lval(j);
                                const uint32_t h = l <= 0;
                                word |= h << i;
                                parity ^= h;
                                const double a = fabs(l);
                                if (j == 0 || a < best) {  // first minimum (H6)
                                    best = a;
                                    bi = j;
                                }
                            }
                            store_node_word(P, wsc, d, to_r, w, word, lane);
                        }
                        if (parity) {
                            uint32_t *pw = to_r ? &row_ptr(wsc, P.Ro + (bi >> 5))[lane]
                                                : &row_ptr(wsc, P.Uo[d] + (bi >> 5))[lane];
                            *pw ^= 1u << (bi & 31);
                        }
                    } else if (!kList) {  // OP_R1, FastSC: `<= 0`
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = 0;
                            for (int i = 0; i < 32 && 32 * w + i < temp; ++i) {
                                const int j = 32 * w + i;
                                word |= (uint32_t)(lval(j) <= 0) << i;
                            }
                            store_node_word(P, wsc, d, to_r, w, word, lane);
                        }
                    } else if constexpr (KIND == K_FASTSCL_LUT) {  // OP_R1, FastSCL: FastSCLLUTDecoder.cpp:99-166
                        const int m = (L - 1) < temp ? (L - 1) : temp;
                        // hard decisions (`< 0`) to own H rows, magnitudes to own key rows
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = 0;
                            for (int i = 0; i < 32 && 32 * w + i < temp; ++i) {
                                const int j = 32 * w + i;
                                const double l = lval(j);
                                word |= (uint32_t)(l < 0) << i;
                                ((double *)row_ptr(wsc, P.Ko + 2 * j))[lane] = fabs(l);
                            }
                            row_ptr(wsc, P.Ho + w)[lane] = word;
                        }
                        // first m entries of argsort(|l|) (argsort :7-17, H1)
                        int ord[MM];
                        double ms[MM];
                        int flip[MM];
#pragma unroll
                        for (int q = 0; q < MM; ++q) {
                            ord[q] = 0;
                            ms[q] = 0;
                            flip[q] = -1;
                        }
                        LaneSortSeq seq{wsc, P.Io, P.Ko, lane};
                        if (temp <= stl::kThreshold) {
                            // insertion sort is stable: order by (|l|, index)
                            uint32_t taken = 0;
#pragma unroll
                            for (int q = 0; q < MM; ++q) {
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
                            for (int q = 0; q < MM; ++q) {
                                if (q < m) {
                                    ord[q] = seq.get(q);
                                    ms[q] = seq.key(ord[q]);
                                }
                            }
                        }
                        wave_sync();  // H rows visible to the other lanes of the group
                        int origin = gl;
#pragma unroll
                        for (int layer = 0; layer < MM; ++layer) {
                            if (layer < m) {
                                const double kf = pm + ms[layer];
                                check_keys<DOM>(P, pm, kf);
                                const Sel sl = gselect<ML>(pm, kf, gl, gbase, L, sh);
                                const int p = gbase + sl.parent;
                                const int pos_old = ord[layer];  // H2: own pre-permutation order
                                pm = pick(sl.upper, shfld(kf, p), shfld(pm, p));
                                ps = gp_shfl<ML>(ps, p);
                                pu = gp_shfl<ML>(pu, p);
                                origin = __shfl(origin, p);
#pragma unroll
                                for (int q = 0; q < MM; ++q) {
                                    ord[q] = __shfl(ord[q], p);
                                    ms[q] = shfld(ms[q], p);
                                    if (q < layer) flip[q] = __shfl(flip[q], p);
                                }
                                flip[layer] = sl.upper ? pos_old : -1;
                            }
                        }
                        for (int w = 0; w < nwo; ++w) {
                            uint32_t word = row_ptr(wsc, P.Ho + w)[gbase + origin];
#pragma unroll
                            for (int q = 0; q < MM; ++q)
                                if (q < m && flip[q] >= 0 && (flip[q] >> 5) == w) word ^= 1u << (flip[q] & 31);
                            if (temp < 32) word &= (1u << temp) - 1u;
                            store_node_word(P, wsc, d, to_r, w, word, lane);
                        }
                    }
                    if (!to_r) pu = gp_set<ML>(pu, d, gl);
                    break;
                }
            }
            wave_sync();  // scratch writes of this op visible to the whole wave
        }

        // Root partial sums (N bits) are in the own R rows.  u = x F^{(x)n}
        // (re-encoding, FastSCLUT.cpp:186-198; for SC/SCL this reproduces the
        // leaf decisions the reference reads directly, SCLUTDecoder.cpp:116-123).
        const int nwr = (N + 31) >> 5;
        for (int w = 0; w < nwr; ++w) {
            uint32_t x = row_ptr(wsc, P.Ro + w)[lane];
            if (N < 32) x &= (1u << N) - 1u;
            x ^= (x >> 1) & 0x55555555u;
            x ^= (x >> 2) & 0x33333333u;
            x ^= (x >> 4) & 0x0f0f0f0fu;
            x ^= (x >> 8) & 0x00ff00ffu;
            x ^= (x >> 16) & 0x0000ffffu;
            row_ptr(wsc, P.Ro + w)[lane] = x;
        }
        for (int mw = 1; mw < nwr; mw *= 2)
            for (int i = 0; i < nwr; i += 2 * mw)
                for (int j = 0; j < mw; ++j) {
                    uint32_t *a = &row_ptr(wsc, P.Ro + i + j)[lane];
                    *a ^= row_ptr(wsc, P.Ro + i + mw + j)[lane];
                }
        wave_sync();
        // best path: first minimum of the path metrics (H6, SCLLUTDecoder.cpp:244)
        int best = 0;
        if (kList && P.crc_n > 0) {
            check_keys<DOM>(P, pm, pm);  // the CA epilogue sorts the metrics
            best = ca_winner_ranked(grank<ML>(pm, gl, gbase, L, sh), gl, gbase, L, P.N, P.info_mask, P.ca_A, P.ca_chk,
                                    P.crc_n, P.crc_q, [&](int w) { return row_ptr(wsc, P.Ro + w)[lane]; });
        } else if (kList) {
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
            const uint32_t *rb = row_ptr(wsc, P.Ro);
            for (int t = gl; t < P.out_k; t += gs) {
                const int pos = P.info_pos[t];
                out[frame * P.out_k + t] = (uint8_t)((rb[(size_t)(pos >> 5) * 64 + gbase + best] >> (pos & 31)) & 1u);
            }
        }
        wave_sync();
    }
}

}  // namespace qpd
