// qpd_lutgen.cpp -- host-side MinDistortion LUT generator.
//
// Restates, without OpenCV and in one native pass, the reference's offline
// table design that produces the decoders' inputs:
//
//   LLRQuantizer::find_OptLS_quantizer
//       Quantizers/quantizers/_cpp/LLRQuantizer/LLRQuantizer.cpp:67-165
//       (its pure-Python twin QuantizeDensityEvolution/MinDistortionQuantizer.py:28-99):
//       minimum-squared-error merge of M sorted LLR quanta into K, by dynamic
//       programming over contiguous groups.
//   LLRQuantizerSC.run
//       QuantizeDensityEvolution/QLLRDensityEvolution_MinDistortion.py:73-126:
//       density evolution down the code tree with f = min-sum and
//       g = (1-2u)a + b on the quantized alphabet, merge of equal values
//       (np.unique), then the DP quantizer back to v symbols; one f and one g
//       table per node plus the per-level quanta (the decoders' vcl).
//
// Summation order.  The reference generator is numpy glue around the C++ DP,
// so sums inside the DP are sequential (C++ loops) and the glue's sums are
// numpy's pairwise reduction.  `order` selects the DP's summation:
// QPD_SUM_SEQUENTIAL reproduces the C++ quantizer the reference generator
// calls; QPD_SUM_NUMPY reproduces its Python twin (used to pin this code
// against the reference here, where the OpenCV build is unavailable).
// The glue always sums like numpy.
//
// Quirk kept: the DP's output density/quanta re-index the already-permuted
// arrays through the permutation again (LLRQuantizer.cpp:151-163,
// MinDistortionQuantizer.py:88-99).  Every caller passes ascending quanta
// (np.unique output, binned channel quanta), so the permutation is the
// identity and the quirk is a no-op; it is restated for other inputs.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace qpd_lutgen {

enum SumOrder { SUM_SEQUENTIAL = 0, SUM_NUMPY = 1 };

// numpy's float64 add-reduction (pairwise_sum, numpy/_core/src/umath/
// loops_utils.h.src): blocks of <= 128 with 8 interleaved partial sums.
double pairwise_sum(const double *a, long n) {
    if (n < 8) {
        double r = 0.;
        for (long i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        long i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

double sum(const double *a, long n, int order) {
    if (order == SUM_NUMPY) return pairwise_sum(a, n);
    double r = 0.;
    for (long i = 0; i < n; ++i) r += a[i];
    return r;
}

struct Quantized {
    std::vector<double> density, quanta;
    std::vector<int> lut;
    double distortion = 0;
};

// Squared-error cost of merging sorted symbols [a', a) into one
// (compute_partial_quantization_noise, LLRQuantizer.cpp:28-48 /
// MinDistortionQuantizer.py:3-7).
double merge_cost(const double *d, const double *q, int len, int order, std::vector<double> &tmp) {
    tmp.resize(len);
    for (int i = 0; i < len; ++i) tmp[i] = d[i] * q[i];
    const double mean = sum(tmp.data(), len, order) / sum(d, len, order);
    for (int i = 0; i < len; ++i) {
        const double e = q[i] - mean;
        tmp[i] = e * e * d[i];
    }
    return sum(tmp.data(), len, order);
}

// LLRQuantizer::find_OptLS_quantizer (LLRQuantizer.cpp:67-165).
Quantized optls(const double *density_in, const double *quanta_in, int M, int K, int order) {
    std::vector<int> perm(M);
    for (int i = 0; i < M; ++i) perm[i] = i;
    std::sort(perm.begin(), perm.end(), [&](int a, int b) { return quanta_in[a] < quanta_in[b]; });
    std::vector<double> d(M), q(M);
    for (int i = 0; i < M; ++i) {
        d[i] = density_in[perm[i]];
        q[i] = quanta_in[perm[i]];
    }
    // cost table [a'][a], a in (a', a' + M - K + 1]  (:50-65)
    const int W = M + 1;
    std::vector<double> table((size_t)M * W, 0.0), tmp;
    for (int ap = 0; ap < M; ++ap) {
        const int max_a = std::min(ap + M - K + 1, M);
        for (int a = ap + 1; a <= max_a; ++a) table[(size_t)ap * W + a] = merge_cost(&d[ap], &q[ap], a - ap, order, tmp);
    }
    // dynamic programme (:85-130): state[a - z][z] = best cost of z groups over [0, a)
    const int R = M - K + 1;
    std::vector<double> state((size_t)R * (K + 1), 0.0);
    std::vector<int> arg((size_t)R * (K + 1), 0);
    auto S = [&](int r, int z) -> double & { return state[(size_t)r * (K + 1) + z]; };
    auto A = [&](int r, int z) -> int & { return arg[(size_t)r * (K + 1) + z]; };
    for (int i = 0; i < R; ++i) S(i, 1) = table[(size_t)0 * W + 1 + i];
    for (int z = 2; z <= K; ++z) {
        const int a_lo = z < K ? z : M, a_hi = z < K ? z + M - K : M;
        for (int a = a_lo; a <= a_hi; ++a) {
            const int row = z < K ? a - z : M - K;
            double best = 0;
            int best_ap = -1;
            for (int ap = z - 1; ap <= a - 1; ++ap) {
                const double t = S(ap - (z - 1), z - 1) + table[(size_t)ap * W + a];
                if (best_ap < 0 || t < best) {  // first minimum (std::min_element / np.argmin)
                    best = t;
                    best_ap = ap;
                }
            }
            A(row, z) = best_ap;
            S(row, z) = best;
        }
    }
    // backward trace (:131-137)
    std::vector<int> Az(K + 1, 0);
    Az[K] = M;
    if (K >= 2) {
        Az[K - 1] = A(M - K, K);
        int opt = Az[K - 1];
        for (int z = K - 1; z > 1; --z) {
            opt = A(opt - z, z);
            Az[z - 1] = opt;
        }
    }
    Quantized out;
    out.density.assign(K, 0.0);
    out.quanta.assign(K, 0.0);
    out.lut.assign(M, 0);
    out.distortion = K >= 2 ? S(M - K, K) : S(M - K, 1);
    // output (:139-163), re-indexing the permuted arrays through perm (quirk)
    std::vector<double> dd, qd;
    for (int i = 0; i < K; ++i) {
        dd.clear();
        qd.clear();
        for (int j = Az[i]; j < Az[i + 1]; ++j) {
            out.lut[perm[j]] = i;
            dd.push_back(d[perm[j]]);
            qd.push_back(d[perm[j]] * q[perm[j]]);
        }
        out.density[i] = sum(dd.data(), (long)dd.size(), order);
        out.quanta[i] = sum(qd.data(), (long)qd.size(), order) / out.density[i];
    }
    return out;
}

// np.unique + per-value density sums + index map (get_unique_quanta,
// QLLRDensityEvolution_MinDistortion.py:40-47).  -0.0 and +0.0 are one value.
void unique_merge(const std::vector<double> &dens, const std::vector<double> &quanta, std::vector<double> &ud,
                  std::vector<double> &uq, std::vector<int> &map) {
    std::vector<double> s(quanta);
    for (double &x : s)
        if (x == 0) x = 0.0;
    std::sort(s.begin(), s.end());
    uq.clear();
    for (size_t i = 0; i < s.size(); ++i)
        if (i == 0 || s[i] != s[i - 1]) uq.push_back(s[i]);
    map.assign(quanta.size(), 0);
    ud.assign(uq.size(), 0.0);
    std::vector<std::vector<double>> parts(uq.size());
    for (size_t i = 0; i < quanta.size(); ++i) {
        const int k = (int)(std::lower_bound(uq.begin(), uq.end(), quanta[i] == 0 ? 0.0 : quanta[i]) - uq.begin());
        map[i] = k;
        parts[k].push_back(dens[i]);  // index order, as the boolean mask selects them
    }
    for (size_t k = 0; k < uq.size(); ++k) ud[k] = pairwise_sum(parts[k].data(), (long)parts[k].size());
}

inline double npsign(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0); }

struct Tree {
    int N, n, v, order;
    uint8_t *lut_f, *lut_g;
    double *dens, *quant;  // [n+1][N][v]
    int err = 0;

    double *D(int level, int pos) { return dens + ((size_t)level * N + pos) * v; }
    double *Q(int level, int pos) { return quant + ((size_t)level * N + pos) * v; }

    // One node of LLRQuantizerSC.run (:86-126).
    void node(int level, int nd) {
        const int bits = N >> level, stride = bits / 2, offset = nd * bits;
        const int posi = (1 << level) + nd - 1;
        const double *d1 = D(level, offset), *d2 = D(level, offset + stride);
        const double *q1 = Q(level, offset), *q2 = Q(level, offset + stride);
        const int vv = v * v;
        std::vector<double> df(vv), qf(vv), dg(2 * vv), qg(2 * vv);
        for (int i = 0; i < v; ++i)
            for (int j = 0; j < v; ++j) {  // get_llr_density_quanta_after_f / _g (:22-38)
                df[i * v + j] = d1[i] * d2[j];
                qf[i * v + j] = npsign(q1[i]) * npsign(q2[j]) * std::min(std::fabs(q1[i]), std::fabs(q2[j]));
                for (int u = 0; u < 2; ++u) {
                    qg[u * vv + i * v + j] = (1 - 2 * u) * q1[i] + q2[j];
                    dg[u * vv + i * v + j] = 0.5 * d1[i] * d2[j];
                }
            }
        for (int side = 0; side < 2; ++side) {
            const std::vector<double> &dd = side ? dg : df, &qq = side ? qg : qf;
            std::vector<double> ud, uq;
            std::vector<int> emap;
            unique_merge(dd, qq, ud, uq, emap);
            if ((int)uq.size() < v) {  // CV_Assert(M >= K) in the reference
                err = 1;
                return;
            }
            Quantized c = optls(ud.data(), uq.data(), (int)uq.size(), v, order);
            // get_LUT (:49-71)
            if (!side) {
                for (int k = 0; k < vv; ++k) lut_f[(size_t)posi * vv + k] = (uint8_t)c.lut[emap[k]];
            } else {
                for (int k = 0; k < 2 * vv; ++k) lut_g[(size_t)posi * 2 * vv + k] = (uint8_t)c.lut[emap[k]];
            }
            const int base = offset + (side ? stride : 0);
            for (int p = 0; p < bits / 2; ++p) {
                std::memcpy(D(level + 1, base + p), c.density.data(), sizeof(double) * v);
                std::memcpy(Q(level + 1, base + p), c.quanta.data(), sizeof(double) * v);
            }
        }
    }
};

}  // namespace qpd_lutgen

extern "C" {

// Declared in include/qpd.h.
int qpd_optls_quantizer(const double *density, const double *quanta, int32_t M, int32_t K, int32_t sum_order,
                        double *out_density, double *out_quanta, int32_t *out_lut, double *out_distortion) {
    if (!density || !quanta || M < 1 || K < 1 || K > M) return -1;
    qpd_lutgen::Quantized c = qpd_lutgen::optls(density, quanta, M, K, sum_order);
    if (out_density) std::memcpy(out_density, c.density.data(), sizeof(double) * K);
    if (out_quanta) std::memcpy(out_quanta, c.quanta.data(), sizeof(double) * K);
    if (out_lut)
        for (int i = 0; i < M; ++i) out_lut[i] = c.lut[i];
    if (out_distortion) *out_distortion = c.distortion;
    return 0;
}

int qpd_lutgen_mindistortion(int32_t N, int32_t v, const double *ch_density, const double *ch_quanta,
                             int32_t sum_order, int32_t threads, uint8_t *lut_f, uint8_t *lut_g, double *llr_density,
                             double *llr_quanta) {
    int n = 0;
    while ((1 << n) < N) ++n;
    if (N < 2 || (1 << n) != N || v < 2 || v > 256 || !ch_density || !ch_quanta || !lut_f || !lut_g || !llr_density ||
        !llr_quanta)
        return -1;
    qpd_lutgen::Tree t{N, n, v, sum_order, lut_f, lut_g, llr_density, llr_quanta};
    for (int p = 0; p < N; ++p) {  // level 0 = the channel (:79-82)
        std::memcpy(t.D(0, p), ch_density, sizeof(double) * v);
        std::memcpy(t.Q(0, p), ch_quanta, sizeof(double) * v);
    }
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    for (int level = 0; level < n; ++level) {  // nodes of one level are independent
        const int nodes = 1 << level;
        const int T = std::min(threads, nodes);
        std::vector<qpd_lutgen::Tree> part(T, t);
        std::vector<std::thread> pool;
        for (int w = 0; w < T; ++w)
            pool.emplace_back([&, w] {
                for (int nd = w; nd < nodes; nd += T) part[w].node(level, nd);
            });
        for (auto &th : pool) th.join();
        for (auto &p : part)
            if (p.err) return -2;
    }
    return 0;
}

}  // extern "C"
