// qpd_mc.hip -- GPU-resident Monte-Carlo front end.
//
// Replaces the reference driver's per-frame Python loop
// (mainQuantizedDecoder_LLRDomain.py:151-176): message bits, polar encoding
// (the un-vendored PolarEnc, restated: u[info] = msg, x = u F^{(x)n} in natural
// order), BPSK, AWGN, LLR = 2y/sigma^2 and the driver's channel quantizer
// (saturate at the outer edges, else channel_lut[bisect_left(edges[:-1], llr) - 1]).
//
// Every random number is a pure function of (seed, GLOBAL frame id, word):
// Philox4x32-10 with counter = (frame_lo, frame_hi, word, stream tag), so a
// frame's content does not depend on batch size, grid, or how frames are
// sharded across GPUs -- the 1/2/4/8-GPU runs of one frame range see the same
// frames.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qpd {

constexpr int kMcMaxEdges = 257;  // channel quantizer with up to 256 bins
constexpr uint32_t kTagMsg = 0x4d534731u, kTagNoise = 0x4e4f4931u;

struct Philox4 {
    uint32_t v[4];
};

__host__ __device__ inline Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                  uint32_t k1) {
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
    int32_t A, crc_n;  // crc_n > 0: A message bits + first K-A bits of their CRC
    uint32_t crc_q;    // CRC register taps (coefficients 1..crc_n, as ca_winner)
    uint32_t seed_lo, seed_hi;
    float sigma, llr_scale;  // AWGN std and 2/sigma^2
    const int32_t *info_pos; // [K] information positions, ascending
    double edges[kMcMaxEdges];
    int32_t lut[kMcMaxEdges - 1];
};

// One 64-lane workgroup per frame (grid-stride).  LDS: N bytes of u / x.
__global__ __launch_bounds__(64) void mc_frames_kernel(McChannel C, int64_t frame0, int64_t B,
                                                       uint8_t *__restrict__ msg_out, int32_t *__restrict__ sym_out) {
    extern __shared__ uint8_t ux[];
    const int t = threadIdx.x;
    const int N = C.N, K = C.K;
    for (int64_t f = blockIdx.x; f < B; f += gridDim.x) {
        const uint64_t gid = (uint64_t)(frame0 + f);
        const uint32_t glo = (uint32_t)gid, ghi = (uint32_t)(gid >> 32);
        for (int e = t; e < N; e += 64) ux[e] = 0;
        __syncthreads();
        const int A = C.A;  // message bits (= K without CRC)
        for (int w = t; w * 128 < A; w += 64) {
            const Philox4 r = philox4x32_10(glo, ghi, (uint32_t)w, kTagMsg, C.seed_lo, C.seed_hi);
            for (int b = 0; b < 128 && 128 * w + b < A; ++b) {
                const uint8_t bit = (r.v[b >> 5] >> (b & 31)) & 1u;
                const int j = 128 * w + b;
                msg_out[f * A + j] = bit;
                ux[C.info_pos[j]] = bit;
            }
        }
        __syncthreads();
        if (C.crc_n > 0 && t == 0) {  // CRC::encoding (utils.cpp:77-92) as a register, one lane
            const uint32_t top = 1u << (C.crc_n - 1), mask = (top << 1) - 1u;
            uint32_t r = 0;
            for (int j = 0; j < A; ++j) {
                const uint32_t fb = (uint32_t)ux[C.info_pos[j]] ^ ((r & top) ? 1u : 0u);
                r = ((r << 1) & mask) ^ (C.crc_q & (0u - fb));
            }
            for (int j = 0; j < K - A; ++j) ux[C.info_pos[A + j]] = (uint8_t)((r >> (C.crc_n - 1 - j)) & 1u);
        }
        __syncthreads();
        for (int m = 1; m < N; m *= 2) {  // x = u F^{(x)n}
            for (int e = t; e < N / 2; e += 64) {
                const int i = (e / m) * 2 * m + (e % m);
                ux[i] ^= ux[i + m];
            }
            __syncthreads();
        }
        for (int p = t; 2 * p < N; p += 64) {
            const Philox4 r = philox4x32_10(glo, ghi, (uint32_t)p, kTagNoise, C.seed_lo, C.seed_hi);
            const float u1 = ((float)(r.v[0] >> 8) + 0.5f) * (1.0f / 16777216.0f);
            const float u2 = (float)(r.v[1] >> 8) * (1.0f / 16777216.0f);
            const float rad = sqrtf(-2.0f * logf(u1));
            float s, c;
            sincosf(6.283185307179586f * u2, &s, &c);
            const float nz[2] = {rad * c, rad * s};
            for (int h = 0; h < 2; ++h) {
                const int e = 2 * p + h;
                const float y = (1.0f - 2.0f * (float)ux[e]) + C.sigma * nz[h];
                const double llr = (double)(y * C.llr_scale);
                int s_out;
                const int M = C.n_edges - 1;
                if (llr <= C.edges[0]) {
                    s_out = 0;
                } else if (llr >= C.edges[M]) {
                    s_out = C.q - 1;
                } else {  // bisect_left over edges[0..M-1]
                    int lo = 0, hi = M;
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (C.edges[mid] < llr)
                            lo = mid + 1;
                        else
                            hi = mid;
                    }
                    s_out = C.lut[lo - 1];
                }
                sym_out[f * N + e] = s_out;
            }
        }
        __syncthreads();
    }
}

}  // namespace qpd
