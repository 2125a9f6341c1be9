// qpd_mc.hip -- GPU-resident Monte-Carlo front end.
//
// Replaces the reference driver's per-frame Python loop
// (mainQuantizedDecoder_LLRDomain.py:151-176): message bits, optional CRC
// (CRCEnc, :153-156), polar encoding (the un-vendored PolarEnc, restated:
// u[info] = msg, x = u F^{(x)n} in natural order), BPSK, AWGN in float64
// (`y = bpsk + normal(0, sigma)`, `llr = y * 2 / sigma**2`, :161-165, no fused
// multiply-add; the division by sigma**2 is a multiplication by its reciprocal,
// within an ulp of the driver's quotient) and the driver's channel quantizer
// (saturate at the outer edges, else channel_lut[bisect_left(edges[:-1], llr) - 1],
// :167-176).
//
// Every random number is a pure function of (seed, GLOBAL frame id, word):
// Philox4x32-10 with counter = (frame_lo, frame_hi, word, stream tag), so a
// frame's content does not depend on batch size, grid, or how frames are
// sharded across GPUs -- the 1/2/4/8-GPU runs of one frame range see the same
// frames.  Gaussians: Box-Muller in float64 on 52-bit
// uniforms (two Philox words each), u1 in (0, 1], u2 in [0, 1).
//
// bisect_left is exact for any ascending edges: a guess from the mean bin
// width, checked against its two neighbouring edges (one LDS read); only a
// wrong guess walks, and the walk ends at the first edge >= llr whatever the
// guess (uniform edges, the driver's linspace, are almost never wrong).
//
// PRE mode (qpd_mc_decode): the frame's symbols are staged in LDS and the
// kernel writes the decoder's root pre-pass row instead (root_pre_kernel,
// qpd_fast.hip), so generation feeds the decode kernel directly: no int32
// symbols (4 KB per frame at N = 1024) written to HBM and read back.
//
// Work mapping: one wave per frame (grid-stride).  The frame's bits are
// handled bit-packed (32 positions per dword): lane d draws message dword d,
// the CRC is a table XOR (the register is linear in the message bits), the
// info bits are deposited into u words by the per-word info masks, and the
// encoder runs 5 in-word butterfly stages as shift/mask XORs plus log2(N/32)
// word stages in LDS.  Noise, LLR and quantizer: one position pair per lane
// and round, stored as int2 (512 B per wave-instruction, coalesced).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qpd {

constexpr int kMcMaxEdges = 257;  // channel quantizer with up to 256 bins
constexpr uint32_t kTagMsg = 0x4d534731u, kTagNoise = 0x4e4f4931u;

struct Philox4 {
    uint32_t v[4];
};

__device__ inline Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                  uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
        // the round keys stay two SGPRs advanced per round (SALU) instead of
        // 20 hoisted loop invariants, which would spill the kernel's SGPRs
        asm volatile("" : "+s"(k0), "+s"(k1));
    }
    Philox4 o;
    o.v[0] = c0;
    o.v[1] = c1;
    o.v[2] = c2;
    o.v[3] = c3;
    return o;
}

struct McChannel {
    int32_t N, K, q, n_edges;
    int32_t A, crc_n;     // crc_n > 0: A message bits + first K-A bits of their CRC
    double sigma, inv_s2; // AWGN std and 1 / (sigma*sigma): llr = (2y) * inv_s2
    uint32_t seed_lo, seed_hi;
    const uint32_t *info_mask;  // [N/32] bit i of word w: position 32w+i is an information bit
    const int32_t *info_pref;   // [N/32] information bits before word w
    const uint32_t *crc_tab;    // [A] CRC register contribution of message bit j (CA kinds)
    double edges[kMcMaxEdges];  // [n_edges], ascending (kernel arguments; staged in LDS)
    int32_t lut[kMcMaxEdges - 1];
    // PRE mode (qpd_mc_decode on a fast-engine decoder in pre-mode): instead
    // of int32 symbols, each frame's root pre-pass row (root_pre_kernel's
    // layout: f(y), g(y, 0), g(y, 1) as nibble words, N/4 dwords per frame),
    // computed from the frame's symbols staged in LDS with the root's tables.
    const uint32_t *f_tab, *g_tab;  // node 0's nibble tables (FastPlan f_tab / g_tab)
};

// The double 1.m in [1, 2) whose 52 mantissa bits are (a >> 12) : b -- two
// Philox words; 2 - x is then uniform on (0, 1], x - 1 on [0, 1) (52-bit grid).
__device__ __host__ inline double mc_one_m(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(double, ((uint64_t)(0x3FF00000u | (a >> 12)) << 32) | b);
}

// One Horner step a * b + c with the constant c as an SGPR operand of a VOP3
// v_fma_f64: the compiler otherwise keeps the polynomial constants in VGPRs and
// evaluates every step as a copy + v_fmac_f64 (two VALU instructions instead
// of one plus two scalar moves).
__device__ __forceinline__ double hfma(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

// sin and cos of x in [0, 2 pi] for the Box-Muller angle: reduction by
// q = rint(x * 2/pi) against pi/2 in three parts (Cody-Waite), then the
// fdlibm kernel polynomials (__kernel_sin / __kernel_cos, |r| <= pi/4, < 1 ulp).
// The angle never needs the large-argument (Payne-Hanek) path a general
// libm sin/cos carries (scratch memory, registers).
__device__ inline void mc_sincos(double x, double *sn, double *cs) {
    const double q = rint(x * 0.63661977236758134308);  // 2/pi
    double r = fma(-q, 1.57079632673412561417e+00, x);
    r = fma(-q, 6.07710050630396597660e-11, r);
    r = fma(-q, 2.02226624879595063154e-21, r);
    const double z = r * r;
    const double ps = hfma(z, hfma(z, hfma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                           2.75573137070700676789e-06), -1.98412698298579493134e-04),
                           8.33333333332248946124e-03);
    const double sr = fma(r * z, hfma(z, ps, -1.66666666666666324348e-01), r);
    const double pc = z * hfma(z, hfma(z, hfma(z, hfma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                      -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                                         -1.38888888888741095749e-03), 4.16666666666666019037e-02);
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * pc);
    // quadrant q & 3: (sr, cr), (cr, -sr), (-sr, -cr), (-cr, sr) -- as selects
    const int qi = (int)q;
    const double s0 = (qi & 1) ? cr : sr, c0 = (qi & 1) ? sr : cr;
    *sn = (qi & 2) ? -s0 : s0;
    *cs = ((qi + 1) & 2) ? -c0 : c0;
}

// log(u) for u in (0, 1]: fdlibm's __ieee754_log (u = m 2^k with m in
// [sqrt(2)/2, sqrt(2)), f = m - 1, s = f / (2 + f), the Remez polynomial in
// s^2; < 1 ulp) with its one division as a Newton-refined reciprocal plus a
// residual correction -- s enters only through s (hfsq + R), an O(f^3) term.
// A third of the instructions of the double-double device log.
__device__ inline double mc_log(double u) {
    int k;
    double m = frexp(u, &k);  // [0.5, 1)
    if (m < 0.70710678118654752440) {
        m += m;
        --k;
    }
    const double f = m - 1.0, dd = 2.0 + f;
    double r = __builtin_amdgcn_rcp(dd);
    r = fma(fma(-dd, r, 1.0), r, r);
    r = fma(fma(-dd, r, 1.0), r, r);
    double s = f * r;
    s = fma(fma(-dd, s, f), r, s);
    const double z = s * s, w = z * z;
    // fdlibm's Horner steps as fused multiply-adds
    const double t1 = w * hfma(w, fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01), 3.999999999940941908e-01);
    const double t2 = z * hfma(w, hfma(w, fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01), 2.857142874366239149e-01),
                               6.666666666666735130e-01);
    const double R = t2 + t1, hfsq = 0.5 * f * f, dk = (double)k;
    return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
}

#ifndef QPD_MC_PAIRS
#define QPD_MC_PAIRS 1  // noise pairs per lane and round: 1 measured best (2: +1 %, 4: +5 % generator time; profiles/r03n_ab_generator_pairs.txt)
#endif
#ifndef QPD_MC_WPE
#define QPD_MC_WPE 6  // 6 waves per SIMD: -2.5 % generator time vs 5 (profiles/r03j_ab_generator.txt)
#endif
template <bool PRE>
__global__ __launch_bounds__(64, QPD_MC_WPE) void mc_frames_kernel(McChannel C, int64_t frame0, int64_t B,
                                                       uint8_t *__restrict__ msg_out, int32_t *__restrict__ sym_out) {
#pragma clang fp contract(off)
    extern __shared__ uint32_t lds_mc[];
    // PRE: sym_out holds pre-pass rows (N/4 dwords per frame), see McChannel
    uint32_t Tf = 0, Tg = 0;
    if (PRE) {
        Tf = C.f_tab[threadIdx.x & 31];
        Tg = C.g_tab[threadIdx.x];
    }
    const int t = threadIdx.x;
    const int N = C.N, K = C.K, A = C.A, M = C.n_edges - 1;
    const int nw = (N + 31) >> 5;        // u / x words
    const int kw = (K + 31) >> 5;        // information-bit words (message + CRC)
    // E[0] = -inf, E[1 + i] = edges[i]: E[lo] = edges[lo - 1] and E[lo + 1] = edges[lo] need no guards
    double *E = reinterpret_cast<double *>(lds_mc);
    int32_t *lut = reinterpret_cast<int32_t *>(E + kMcMaxEdges + 1);
    uint32_t *xw = reinterpret_cast<uint32_t *>(lut + kMcMaxEdges);
    uint32_t *bw = xw + nw;               // message + CRC bits (kw + 2 words)
    uint8_t *sy = reinterpret_cast<uint8_t *>(bw + kw + 2);  // PRE: the frame's N channel symbols
    for (int i = t; i < C.n_edges; i += 64) E[1 + i] = C.edges[i];
    if (t == 0) E[0] = -__builtin_inf();
    for (int i = t; i < M; i += 64) lut[i] = C.lut[i];
    const double lo_edge = C.edges[0], hi_edge = C.edges[M];
    const double inv_w = hi_edge > lo_edge ? M / (hi_edge - lo_edge) : 0.0;
    for (int64_t f = blockIdx.x; f < B; f += gridDim.x) {
        const uint64_t gid = (uint64_t)(frame0 + f);
        const uint32_t glo = (uint32_t)gid, ghi = (uint32_t)(gid >> 32);
        // message dword d = Philox(w = d / 4).v[d % 4]; bits >= A cleared
        uint32_t crc_part = 0;
        for (int d = t; d < kw + 2; d += 64) {  // + 2 zero words: funnel reads past the last
            uint32_t m = 0;
            if (32 * d < A) {
                const Philox4 r = philox4x32_10(glo, ghi, (uint32_t)(d >> 2), kTagMsg, C.seed_lo, C.seed_hi);
                // r.v[d & 3] as selects (a dynamic index would go through scratch)
                const uint32_t lo2 = (d & 1) ? r.v[1] : r.v[0], hi2 = (d & 1) ? r.v[3] : r.v[2];
                m = (d & 2) ? hi2 : lo2;
                if (A - 32 * d < 32) m &= (1u << (A - 32 * d)) - 1u;
                // msg bytes 32d .. 32d+31 (A % 8 == 0: 8 B stores)
                uint8_t *mo = msg_out + f * A + 32 * d;
                const int nb = min(32, A - 32 * d);
                if ((A & 7) == 0 && nb == 32) {
                    uint32_t w4[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const uint32_t nib = (m >> (4 * k)) & 0xFu;
                        w4[k] = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
                    }
                    uint2 *o2 = reinterpret_cast<uint2 *>(mo);
#pragma unroll
                    for (int k = 0; k < 4; ++k) o2[k] = make_uint2(w4[2 * k], w4[2 * k + 1]);
                } else {
                    for (int b = 0; b < nb; ++b) mo[b] = (uint8_t)((m >> b) & 1u);
                }
                if (C.crc_n > 0)
                    for (uint32_t mm = m; mm; mm &= mm - 1u) crc_part ^= C.crc_tab[32 * d + __builtin_ctz(mm)];
            }
            bw[d] = m;
        }
        if (C.crc_n > 0) {  // CRC::encoding (utils.cpp:77-92): XOR of the set bits' contributions
            for (int s = 32; s >= 1; s >>= 1) crc_part ^= (uint32_t)__shfl_xor((int)crc_part, s, 64);
            __syncthreads();
            if (t == 0)
                for (int j = 0; j < K - A; ++j) {
                    const uint32_t bit = (crc_part >> (C.crc_n - 1 - j)) & 1u;
                    bw[(A + j) >> 5] |= bit << ((A + j) & 31);
                }
        }
        __syncthreads();
        // u word w = the info bits [pref_w, pref_w + popc(mask_w)) deposited at the mask's set bits,
        // one 16-bit half per lane (the deposit loop runs popc(half) <= 16 times);
        // then the 5 in-word stages of x = u F^{(x)n} (bit i ^= bit i + m for i with bit m clear)
        for (int h0 = 0; h0 < 2 * nw; h0 += 64) {  // whole-wave rounds: the halves meet by a shuffle
            const int h = h0 + t, w = h >> 1;
            uint32_t u = 0;
            if (h < 2 * nw) {
                const uint32_t wm = C.info_mask[w];
                uint32_t mask = (h & 1) ? wm >> 16 : wm & 0xFFFFu;
                const int s = C.info_pref[w] + ((h & 1) ? __builtin_popcount(wm & 0xFFFFu) : 0);
                const uint32_t lo = bw[s >> 5], hi = bw[(s >> 5) + 1];
                uint32_t src = (s & 31) ? ((lo >> (s & 31)) | (hi << (32 - (s & 31)))) : lo;
                for (; mask; mask &= mask - 1u) {
                    u |= (src & 1u) << __builtin_ctz(mask);
                    src >>= 1;
                }
            }
            u |= (uint32_t)__shfl_xor((int)u, 1, 64) << 16;  // even lane: low | high << 16
            if (h < 2 * nw && !(h & 1)) {
                u ^= (u >> 1) & 0x55555555u;
                u ^= (u >> 2) & 0x33333333u;
                u ^= (u >> 4) & 0x0F0F0F0Fu;
                u ^= (u >> 8) & 0x00FF00FFu;
                u ^= (u >> 16) & 0x0000FFFFu;
                xw[w] = u;
            }
        }
        __syncthreads();
        for (int sw = 1; sw < nw; sw <<= 1) {  // word stages (m = 32 sw)
            for (int w = t; w < nw; w += 64)
                if (!(w & sw)) xw[w] ^= xw[w + sw];
            __syncthreads();
        }
        // AWGN + LLR + channel quantizer, positions 2p and 2p+1, QPD_MC_PAIRS
        // pairs per lane and round (p, p + 64, ...): their Philox / log / sincos
        // chains are independent straight-line code the scheduler interleaves
        auto noise = [&](int p, double (&nz)[2]) {
            const Philox4 r = philox4x32_10(glo, ghi, (uint32_t)p, kTagNoise, C.seed_lo, C.seed_hi);
            const double u1 = 2.0 - mc_one_m(r.v[0], r.v[1]);  // (0, 1]
            const double u2 = mc_one_m(r.v[2], r.v[3]) - 1.0;  // [0, 1)
            const double rad = sqrt(-2.0 * mc_log(u1));
            double sn, cs;
            mc_sincos(6.283185307179586 * u2, &sn, &cs);
            nz[0] = rad * cs;
            nz[1] = rad * sn;
        };
        auto quantize = [&](int p, const double (&nz)[2]) {
            const uint32_t xbits = xw[(2 * p) >> 5] >> ((2 * p) & 31);
            int s_out[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const double bpsk = (xbits >> h) & 1u ? -1.0 : 1.0;
                const double y = bpsk + C.sigma * nz[h];
                const double llr = y * 2.0 * C.inv_s2;
                // bisect_left over edges[0..M-1] for lo_edge < llr < hi_edge: lo in [1, M]
                // with edges[lo - 1] < llr <= edges[lo]; guessed, checked, walked if wrong
                const bool inner = llr > lo_edge && llr < hi_edge;
                const double gi = fmin(fmax((llr - lo_edge) * inv_w + 1.0, 1.0), (double)M);
                int lo = (int)gi;
                if (inner && !(E[lo] < llr && llr <= E[lo + 1])) {
                    while (E[lo] >= llr) --lo;     // stops at lo >= 1: E[1] = lo_edge < llr
                    while (E[lo + 1] < llr) ++lo;  // stops at lo <= M: E[M + 1] = hi_edge > llr
                }
                const int sl = lut[lo - 1];
                s_out[h] = inner ? sl : (llr <= lo_edge ? 0 : C.q - 1);
            }
            if (PRE)
                *reinterpret_cast<uint16_t *>(sy + 2 * p) = (uint16_t)(s_out[0] | (s_out[1] << 8));
            else
                *reinterpret_cast<int2 *>(sym_out + f * N + 2 * p) = make_int2(s_out[0], s_out[1]);
        };
        for (int p0 = 0; 2 * p0 < N; p0 += 64 * QPD_MC_PAIRS) {
            double nz[QPD_MC_PAIRS][2];
#pragma unroll
            for (int i = 0; i < QPD_MC_PAIRS; ++i) noise(p0 + 64 * i + t, nz[i]);
#pragma unroll
            for (int i = 0; i < QPD_MC_PAIRS; ++i)
                if (2 * (p0 + 64 * i + t) < N) quantize(p0 + 64 * i + t, nz[i]);
        }
        __syncthreads();
        if (PRE) {
            // root_pre_kernel's row from the staged symbols: word w of f(y),
            // g(y, 0), g(y, 1) from symbols [8w, 8w+8) and [N/2 + 8w, ...);
            // whole waves stay active through the lookups (inactive lanes
            // would read 0 from the table registers)
            const int nwh = N >> 4;  // words per segment (N >= 16)
            uint32_t *row = reinterpret_cast<uint32_t *>(sym_out) + f * (N >> 2);
            for (int w0 = 0; w0 < nwh; w0 += 64) {
                const int w = min(w0 + t, nwh - 1);
                uint32_t a = 0, b = 0;
                for (int i = 0; i < 8; ++i) {
                    a |= (uint32_t)sy[8 * w + i] << (4 * i);
                    b |= (uint32_t)sy[(N >> 1) + 8 * w + i] << (4 * i);
                }
                const uint32_t fw = lut_vec<8>(Tf, a, b, 0u);
                const uint32_t g0 = lut_vec<8>(Tg, a, b, 0u);
                const uint32_t g1 = lut_vec<8>(Tg, a, b, 0xFFu);
                if (w0 + t < nwh) {
                    row[w] = fw;
                    row[nwh + w] = g0;
                    row[2 * nwh + w] = g1;
                }
            }
            __syncthreads();
        }
    }
}

// Bit and block errors of decoded frames against their messages, added to
// counts[0] / counts[1] (the driver's counters, mainQuantizedDecoder_LLRDomain.py:181-183):
// one wave per frame (grid-stride, four frames' loads in flight per wave), 8
// bytes per lane per step -- the bytes are 0 / 1, so popcount(a ^ b) counts the
// differing ones; a frame's block error is one ballot, the bit errors are
// reduced once per wave; two atomics per wave.
__global__ __launch_bounds__(256) void mc_count_kernel(const uint8_t *__restrict__ bits,
                                                       const uint8_t *__restrict__ msg, int64_t B, int K,
                                                       unsigned long long *__restrict__ counts) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    unsigned be = 0, fe = 0;  // be: this lane's share of the bit errors
    const bool vec = (K & 7) == 0 && ((uintptr_t)bits & 7) == 0 && ((uintptr_t)msg & 7) == 0;
    if (vec && K <= 512) {  // one 8-byte step per lane covers a frame
        const bool on = 8 * lane < K;
        for (int64_t f0 = wave; f0 < B; f0 += 4 * waves) {
            unsigned long long x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t f = f0 + u * waves;
                x[u] = 0;
                if (f < B && on)
                    x[u] = *(const unsigned long long *)(bits + f * K + 8 * lane) ^
                           *(const unsigned long long *)(msg + f * K + 8 * lane);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                be += __popcll(x[u]);
                fe += __ballot(x[u] != 0) != 0;
            }
        }
    } else {
        for (int64_t f = wave; f < B; f += waves) {
            const uint8_t *a = bits + f * K, *b = msg + f * K;
            unsigned e = 0;
            if (vec) {
                for (int i = 8 * lane; i < K; i += 512)
                    e += __popcll(*(const unsigned long long *)(a + i) ^ *(const unsigned long long *)(b + i));
            } else {
                for (int i = lane; i < K; i += 64) e += (a[i] ^ b[i]) & 1u;
            }
            be += e;
            fe += __ballot(e != 0) != 0;
        }
    }
    for (int m = 32; m >= 1; m >>= 1) be += (unsigned)__shfl_xor((int)be, m, 64);
    if (lane == 0 && be) {
        atomicAdd(counts, (unsigned long long)be);
        atomicAdd(counts + 1, (unsigned long long)fe);
    }
}

// Dynamic LDS of mc_frames_kernel.
inline size_t mc_lds_bytes(int N, int K, bool pre) {
    return (kMcMaxEdges + 1) * sizeof(double) + kMcMaxEdges * sizeof(int32_t) + 4 * (((N + 31) >> 5) + ((K + 31) >> 5) + 2) +
           (pre ? (size_t)N : 0);
}

}  // namespace qpd
