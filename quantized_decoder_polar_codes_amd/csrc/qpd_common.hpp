// qpd_common.hpp -- device-side pieces shared by the decode kernels:
// schedule op encoding, list-pointer helpers, cross-lane helpers and the
// survivor selection that reproduces the reference's mink tie order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qpd_types.hpp"

namespace qpd {

// Task queue of the persistent decode kernels.
#ifndef QPD_DYN
#define QPD_DYN 1  // tasks from a device queue (0: static grid-stride with evened rounds)
#endif

// One atomic per wave (lane 0, a vector atomic), the old value broadcast,
// relative to the launch's base.  The counter is never reset: a launch of T
// tasks on a grid of G <= T waves takes exactly T values (T - G successful
// takes, then one failed take per wave), so the host advances the base by T
// per launch (qpd_capi.hip: qpd_decoder::task_base) and the next launch on the decoder
// starts where this one ended.  uint32 arithmetic: wrap-around is harmless.
// Launches on one decoder are ordered by the host (stream events), so no
// launch ever sees another's takes.
__device__ __forceinline__ int64_t wave_take(uint32_t *ctr, uint32_t base) {
    uint32_t v = 0;
    if (threadIdx.x == 0) v = atomicAdd(ctr, 1u);
    return (int64_t)(uint32_t)(__builtin_amdgcn_readfirstlane(v) - base);
}

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t *row_ptr(uint32_t *wsc, int r) { return wsc + (size_t)r * 64; }

__device__ __forceinline__ int ptr_get(uint64_t p, int d) { return (int)((p >> (4 * d)) & 15u); }

__device__ __forceinline__ uint64_t ptr_set(uint64_t p, int d, int lane_in_group) {
    const uint64_t m = 15ull << (4 * d);
    return (p & ~m) | ((uint64_t)lane_in_group << (4 * d));
}

// Lane `src` (0..63, taken mod 64) of x: one ds_bpermute at byte address
// src * 4.  HIP's __shfl computes the same read but first rebuilds the lane id
// (two mbcnt) and re-bases the source on it; the wave is 64 wide, so there is
// nothing to re-base (SCL-LUT +0.7 %, profiles/r03t_ab_lane_read.txt).  The
// FastSCL-LUT unit (qpd_fast_fscl.hip) keeps __shfl (QPD_LANE_READ_SHFL): there
// the change moves its register allocation and costs 12 %.  Internal linkage,
// so the two units' definitions stay separate.
#ifdef QPD_LANE_READ_SHFL
static __device__ __forceinline__ uint32_t lane_read(uint32_t x, int src) { return __shfl(x, src); }
static __device__ __forceinline__ int lane_read(int x, int src) { return __shfl(x, src); }
#else
static __device__ __forceinline__ uint32_t lane_read(uint32_t x, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)x);
}
static __device__ __forceinline__ int lane_read(int x, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, x); }
#endif

static __device__ __forceinline__ uint64_t shfl64(uint64_t x, int src) {
    const uint32_t lo = lane_read((uint32_t)x, src);
    const uint32_t hi = lane_read((uint32_t)(x >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

#ifdef QPD_LANE_READ_SHFL
static __device__ __forceinline__ double shfld(double x, int src) { return __shfl(x, src); }
#else
static __device__ __forceinline__ double shfld(double x, int src) {
    return __builtin_bit_cast(double, shfl64(__builtin_bit_cast(uint64_t, x), src));
}
#endif

// Cross-lane reads (ds_bpermute) see 0 from lanes that are inactive for the
// instruction, so every shuffle runs with the whole wave active: evaluate both
// sides first, then select (never `c ? lane_read(a) : lane_read(b)`).
__device__ __forceinline__ double pick(bool c, double a, double b) { return c ? a : b; }

__device__ __forceinline__ void wave_sync() { __syncthreads(); }  // 64-thread block: one wave

// Compiler-only ordering point for LDS accesses of a single wave.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }




// ---------------------------------------------------------------------------
// Survivor selection: keep the L best of 2L candidates {keep_j = c_j,
// flip_j = c_{j+L}} exactly as std::sort(index, key<) + take L (mink,
// src/SCLLUTDecoder.cpp:8-21).  For 2L <= 16 libstdc++ runs a stable
// insertion sort, i.e. order by (key, candidate index); rank each candidate by
// counting the candidates before it, then invert the ranks through LDS.
// ---------------------------------------------------------------------------
struct Sel {
    int parent;  // lane-in-group of the surviving candidate's path
    bool upper;  // candidate came from the second half (flip / penalty branch)
};

// Group-of-8 exchange by DPP (VALU, no LDS round trip): partner m (1..7) of
// lane i is lane i^m.  quad_perm gives XOR 1/2/3, row_half_mirror XOR 7, and
// their composition XOR 4/5/6.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppXor3 = 0x1B, kDppHalfMirror = 0x141;
constexpr int kDppRowShl1 = 0x101;  // lane i <- lane i+1 within a row of 16
constexpr int kDppQuadBcast3 = 0xFF;  // quad_perm(3,3,3,3): lane i <- lane 4*(i/4)+3

template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, true);
    return ((uint64_t)hi << 32) | lo;
}

template <int M>
__device__ __forceinline__ uint64_t xor_lane8(uint64_t x, uint64_t hm) {  // hm = x of lane i^7
    if constexpr (M == 1) return dpp64<kDppXor1>(x);
    if constexpr (M == 2) return dpp64<kDppXor2>(x);
    if constexpr (M == 3) return dpp64<kDppXor3>(x);
    if constexpr (M == 4) return dpp64<kDppXor3>(hm);
    if constexpr (M == 5) return dpp64<kDppXor2>(hm);
    if constexpr (M == 6) return dpp64<kDppXor1>(hm);
    return hm;
}

// Rank contribution of partner gl^M.  Keys are non-negative doubles (or +inf),
// so their order is the order of their bit patterns as unsigned integers.
// The candidate-index tie break (partner j < gl) holds iff gl has the highest
// bit of M set.
template <int M>
__device__ __forceinline__ void rank8_partner(uint64_t K, uint64_t F, uint64_t F1, uint64_t hk, uint64_t hf, int gl,
                                              int &rk, int &rf) {
    constexpr int hb = M >= 4 ? 2 : (M >= 2 ? 1 : 0);
    const uint64_t t = (uint64_t)((gl >> hb) & 1);
    const uint64_t ok = xor_lane8<M>(K, hk), of = xor_lane8<M>(F, hf);
    // (o < X) || (o == X && partner index below) == o < X + t  (no overflow: X <= +inf bits)
    rk += ok < K + t;
    rk += of < K;
    rf += ok < F1;
    rf += of < F + t;
}

// Generic form: any L <= 8 (lane groups of G = pow2 >= L), `sel` = 64 ints.
__device__ __forceinline__ Sel select_survivors(double kk, double kf, int gl, int gbase, int L, int *sel) {
    int rk = 0, rf = 0;
    for (int j = 0; j < L; ++j) {
        const double ok = shfld(kk, gbase + j);
        const double of = shfld(kf, gbase + j);
        rk += (ok < kk) || (ok == kk && j < gl);
        rk += (of < kk);
        rf += (ok <= kf);
        rf += (of < kf) || (of == kf && j < gl);
    }
    if (gl < L) {
        if (rk < L) sel[gbase + rk] = gl;
        if (rf < L) sel[gbase + rf] = gl + L;
    }
    // One wave per workgroup and LDS instructions of a wave complete in order:
    // the scatter above is visible to the gather below without s_barrier or a
    // vmcnt drain (which would also stall on in-flight global prefetches).
    lds_order();
    int c = (gl < L) ? sel[gbase + gl] : gl;
    lds_order();
    Sel s;
    s.upper = c >= L;
    s.parent = s.upper ? c - L : c;
    return s;
}

// L = 8 (lane groups of 8): ranks from the 7 DPP partners, branch-free
// scatter (ranks >= 8 go to a per-lane junk slot at sel[junk + lane]), so
// several independent selections can interleave in one basic block.
// QPD_SEL_OPAQUE: the lane values pass through an empty volatile asm first, so the
// selection's lane terms (partner tie bits, scatter addresses) are derived here,
// behind the caller's identity test (keep_all8) -- otherwise the compiler computes
// them before the test, on every information leaf, identity or not.  SCL-LUT
// +0.5 %, FastSCL-LUT +1.4 %, SCL-LUT scratch 104 -> 84 B per lane
// (profiles/r06zc_ab_fork_opaque.txt, r06zd_ab_sel_opaque.txt).
#ifndef QPD_SEL_OPAQUE
#define QPD_SEL_OPAQUE 1
#endif
__device__ __forceinline__ Sel select_survivors8(double kk, double kf, int gl, int gbase, int lane, int *sel,
                                                 int junk = 64) {
#if QPD_SEL_OPAQUE
    asm volatile("" : "+v"(gl), "+v"(gbase), "+v"(lane));
#endif
    const uint64_t K = __builtin_bit_cast(uint64_t, kk), F = __builtin_bit_cast(uint64_t, kf);
    const uint64_t hk = dpp64<kDppHalfMirror>(K), hf = dpp64<kDppHalfMirror>(F);
    const uint64_t F1 = F + 1;
    int rk = F < K, rf = K < F1;
    rank8_partner<1>(K, F, F1, hk, hf, gl, rk, rf);
    rank8_partner<2>(K, F, F1, hk, hf, gl, rk, rf);
    rank8_partner<3>(K, F, F1, hk, hf, gl, rk, rf);
    rank8_partner<4>(K, F, F1, hk, hf, gl, rk, rf);
    rank8_partner<5>(K, F, F1, hk, hf, gl, rk, rf);
    rank8_partner<6>(K, F, F1, hk, hf, gl, rk, rf);
    rank8_partner<7>(K, F, F1, hk, hf, gl, rk, rf);
    sel[rk < 8 ? gbase + rk : junk + lane] = gl;
    sel[rf < 8 ? gbase + rf : junk + lane] = gl + 8;
    lds_order();
    const int c = sel[gbase + gl];
    lds_order();
    Sel s;
    s.upper = c >= 8;
    s.parent = c & 7;
    return s;
}

// CRC-aided choice of the output path (CASCLLUTDecoder.cpp:263-290,
// CAFastSCLLUTDecoder.cpp:333-371, CASCLDecoder.cpp:202-235): the paths in
// stable path-metric order (argsort of L <= 8 doubles is libstdc++'s
// insertion sort, H1); the first whose info bits [0, A) reproduce the `chk`
// bits [A, A + chk) under CRC::encoding (utils.cpp:77-92), else the first in
// that order.  chk = K - A for the LUT kinds (CASCLLUTDecoder.cpp:279), crc_n
// for the float CA-SCL (CASCLDecoder.cpp:223).  The reference's bit-array
// long division is run as the equivalent MSB-first register: the divisor's
// leading coefficient only clears the current bit, `crc_q` holds
// coefficients 1..crc_n.  `word(w)` = this lane's decoded bits 32w..32w+31;
// `info_mask` = wave-uniform information-position mask words.
// Stable rank of this lane's path metric among the group's L (argsort by
// insertion sort: L <= 16).
__device__ __forceinline__ int stable_rank(double pm, int gl, int gbase, int L) {
    int rank = 0;
    for (int j = 0; j < L; ++j) {
        const double o = shfld(pm, gbase + j);
        rank += (o < pm) || (o == pm && j < gl);
    }
    return rank;
}

// `rank` = this path's position in the argsort(PML) order.
template <class WordFn>
__device__ __forceinline__ int ca_winner_ranked(int rank, int gl, int gbase, int L, int N, const uint32_t *info_mask,
                                                int A, int chk, int crc_n, uint32_t crc_q, WordFn word) {
    const int K = A + chk;
    const uint32_t top = 1u << (crc_n - 1);
    const uint32_t mask = (top << 1) - 1u;  // crc_n = 32: 0 - 1 = all ones
    uint32_t r = 0;
    bool pass = true;
    int t = 0;
    const int nw = (N + 31) >> 5;
    for (int w = 0; w < nw && t < K; ++w) {
        uint32_t m = info_mask[w];
        if (!m) continue;
        const uint32_t x = word(w);
        while (m) {
            const int b = __builtin_ctz(m);
            m &= m - 1u;
            const uint32_t bit = (x >> b) & 1u;
            if (t < A) {
                const uint32_t fb = bit ^ ((r & top) ? 1u : 0u);
                r = ((r << 1) & mask) ^ (crc_q & (0u - fb));
            } else {
                pass = pass && bit == ((r >> (crc_n - 1 - (t - A))) & 1u);
            }
            ++t;
        }
    }
    const int key = gl < L ? (pass ? rank : kMaxLWide + rank) : 2 * kMaxLWide;
    int best = 0, bk = 1 << 30;
    for (int j = 0; j < L; ++j) {
        const int kj = lane_read(key, gbase + j);
        if (kj < bk) {
            bk = kj;
            best = j;
        }
    }
    return best;
}

template <class WordFn>
__device__ __forceinline__ int ca_winner(double pm, int gl, int gbase, int L, int N, const uint32_t *info_mask, int A,
                                         int chk, int crc_n, uint32_t crc_q, WordFn word) {
    return ca_winner_ranked(stable_rank(pm, gl, gbase, L), gl, gbase, L, N, info_mask, A, chk, crc_n, crc_q, word);
}

}  // namespace qpd
