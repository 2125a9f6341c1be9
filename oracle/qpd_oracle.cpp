// =============================================================================
// qpd_oracle.cpp -- CPU restatement of the reference LUT polar decoders.
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
// product path and the `cpu_baseline` leg of bench.py.  Nothing in
// quantized_decoder_polar_codes_amd/ links, loads or calls it.  It restates,
// from scratch and in its own structure (explicit recursion instead of the
// reference's node_state machine), the algorithms of
//
//   SC   (float)    /root/reference/PolarDecoder/PolarDecoder/_cpp/src/SCDecoder.cpp:14-89
//   SC-LUT          .../src/SCLUTDecoder.cpp:21-124
//   SCL-LUT         .../src/SCLLUTDecoder.cpp:47-253   (mink :8-21, argmin :25-29)
//   FastSC-LUT      .../src/FastSCLUT.cpp:27-206
//   FastSCL-LUT     .../src/FastSCLLUTDecoder.cpp:57-408 (argsort :7-17)
//   CA-SCL-LUT      .../src/CASCLLUTDecoder.cpp:47-303   (CRC epilogue :263-302)
//   CA-FastSCL-LUT  .../src/CAFastSCLLUTDecoder.cpp:57-454 (CRC epilogue :332-453)
//   CRC::encoding   .../src/utils.cpp:77-92
//   partial sums    .../src/utils.cpp:62-67 (u), min-sum f/g utils.cpp:26-36
//
// It keeps the reference's per-fork deep copies of the whole list state, so
// that its speed is representative of the reference CPU decoder (SURVEY.md
// §8(d)), and it calls libstdc++ std::sort with the same comparator as the
// reference so that tie order is identical (hazard H1).  Parity is pinned by
// tests/test_oracle_vs_reference.py against the reference compiled from its
// own sources (oracle/build_ref.sh -> oracle/_ref/).
//
// Table layout shared with the product C-ABI (include/qpd.h):
//   f table t : lut_f[t*v*v + a*v + b]                     (a = first half)
//   g table t : lut_g[(t*2 + u)*v*v + a*v + b]
//   node p (node_posi = 2^depth + node - 1), element j uses table
//        f_base[p] + j*f_step   (f_step 0 = one table per node, 1 = per element)
//   vcl       : vcl[((row*N) + pos)*v + sym], rows = vcl_rows
// =============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace {

struct Code {
    int N, K, L, v, n;
    const int32_t *frozen;
    const int32_t *node_type;  // may be null (no special nodes)
    const uint8_t *lut_f;
    const int32_t *f_base;
    int f_step;
    const uint8_t *lut_g;
    const int32_t *g_base;
    int g_step;
    const double *vcl;
    int vcl_rows;

    int F(int posi, int j, int a, int b) const {
        size_t t = (size_t)f_base[posi] + (size_t)j * f_step;
        return lut_f[t * v * v + (size_t)a * v + b];
    }
    int G(int posi, int j, int u, int a, int b) const {
        size_t t = (size_t)g_base[posi] + (size_t)j * g_step;
        return lut_g[(t * 2 + u) * v * v + (size_t)a * v + b];
    }
    double Q(int row, int pos, int sym) const {
        return vcl[((size_t)row * N + pos) * v + sym];
    }
    int type(int posi) const { return node_type ? node_type[posi] : -1; }
};

const double kInf = std::numeric_limits<double>::infinity();

int ilog2(int N) {
    int n = 0;
    while ((1 << n) < N) ++n;
    return n;
}

// Partial-sum combine, utils.cpp:62-67: out = [l ^ r, r].
void combine(uint8_t *out, const uint8_t *l, const uint8_t *r, int half) {
    for (int j = 0; j < half; ++j) out[j] = l[j] ^ r[j];
    std::memcpy(out + half, r, half);
}

// Polar re-encoding of the root partial sums, FastSCLUT.cpp:186-198.
void reencode(std::vector<uint8_t> &x, int N) {
    for (int m = 1; m < N; m *= 2)
        for (int i = 0; i < N; i += 2 * m)
            for (int j = 0; j < m; ++j) x[i + j] ^= x[i + m + j];
}

void emit_info(const Code &c, const uint8_t *bits, uint8_t *out) {
    int t = 0;
    for (int i = 0; i < c.N; ++i)
        if (c.frozen[i] == 0) out[t++] = bits[i];
}

// std::sort of an index vector by key -- the reference's mink/argsort
// (SCLLUTDecoder.cpp:8-21, FastSCLLUTDecoder.cpp:7-34).  Same libstdc++ call,
// same comparator, hence the same order among ties.
std::vector<int> sort_index(const std::vector<double> &key) {
    std::vector<int> idx(key.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
    std::sort(idx.begin(), idx.end(), [&key](int p, int q) { return key[p] < key[q]; });
    return idx;
}

// CRC::encoding, utils.cpp:77-92: long division of info || 0^crc_n by the
// coefficient vector p (p[loc] = 1, utils.cpp:69-75); returns the crc_n bits
// that follow the info bits after the division.
std::vector<uint8_t> crc_encoding(const std::vector<uint8_t> &info, int crc_n, const std::vector<int> &p) {
    const int A = (int)info.size();
    std::vector<uint8_t> u(A + crc_n, 0);
    std::memcpy(u.data(), info.data(), A);
    for (int i = 0; i < A; ++i)
        if (u[i] == 1)
            for (int j = 0; j <= crc_n; ++j) u[j + i] = (uint8_t)((u[j + i] + p[j]) % 2);
    return std::vector<uint8_t>(u.begin() + A, u.end());
}

// CRC-aided list output (CASCLLUTDecoder.cpp:263-302): walk the paths in
// argsort(PML) order (L <= 8: libstdc++ insertion sort, stable, H1); the
// first whose decoded info bits [0, A) reproduce bits [A, K) under the CRC
// wins, else the first in that order.
struct CaSpec {
    int A = 0, crc_n = 0;
    std::vector<int> p;  // crc_n + 1 coefficients
};

int first_argmin(const std::vector<double> &x) {
    return (int)std::distance(x.begin(), std::min_element(x.begin(), x.end()));
}

// ---------------------------------------------------------------------------
// SC (float, min-sum) -- SCDecoder.cpp:14-89, f/g utils.cpp:26-36
// ---------------------------------------------------------------------------
struct FloatSC {
    const Code &c;
    std::vector<double> alpha;
    std::vector<uint8_t> beta;
    explicit FloatSC(const Code &c_) : c(c_), alpha((c_.n + 1) * c_.N), beta((c_.n + 1) * c_.N) {}

    static int sgn(double x) { return x < 0 ? -1 : (x > 0); }

    void leaf(int k) {
        const int N = c.N, n = c.n;
        beta[n * N + k] = c.frozen[k] == 1 ? 0 : (uint8_t)(alpha[n * N + k] <= 0);
    }
    void visit(int d, int node) {
        const int N = c.N, n = c.n;
        if (d == n) { leaf(node); return; }
        const int temp = N >> d, half = temp / 2;
        const double *a = &alpha[d * N + temp * node];
        const double *b = a + half;
        double *lo = &alpha[(d + 1) * N + half * (2 * node)];
        for (int j = 0; j < half; ++j)
            lo[j] = (sgn(a[j]) * sgn(b[j])) * std::min(std::fabs(a[j]), std::fabs(b[j]));
        visit(d + 1, 2 * node);
        const uint8_t *ul = &beta[(d + 1) * N + half * (2 * node)];
        double *hi = &alpha[(d + 1) * N + half * (2 * node + 1)];
        for (int j = 0; j < half; ++j) hi[j] = (1 - 2 * ul[j]) * a[j] + b[j];
        visit(d + 1, 2 * node + 1);
        combine(&beta[d * N + temp * node], ul, &beta[(d + 1) * N + half * (2 * node + 1)], half);
    }
    void run(const double *llr, uint8_t *out) {
        std::memcpy(alpha.data(), llr, sizeof(double) * c.N);
        visit(0, 0);
        emit_info(c, &beta[c.n * c.N], out);
    }
};

// ---------------------------------------------------------------------------
// SC-LUT -- SCLUTDecoder.cpp:21-124 (and the non-special part of
// FastSCLUT.cpp:27-206 when `fast` is set).
// ---------------------------------------------------------------------------
struct LutSC {
    const Code &c;
    bool fast;
    std::vector<int> sym;
    std::vector<uint8_t> ucap;
    LutSC(const Code &c_, bool fast_) : c(c_), fast(fast_), sym((c_.n + 1) * c_.N), ucap((c_.n + 1) * c_.N) {}

    // Leaf decision from a node at depth n-1 (SCLUTDecoder.cpp:59-66, 90-97).
    // Hazard H4: SC family decides `llr <= 0`.  Frozen leaves skip the LUT.
    void leaf(int posi, int k, bool right, const int *pa, const int *pb, int ul) {
        const int N = c.N, n = c.n;
        if (c.frozen[k] == 1) { ucap[n * N + k] = 0; return; }
        int s = right ? c.G(posi, 0, ul, pa[0], pb[0]) : c.F(posi, 0, pa[0], pb[0]);
        ucap[n * N + k] = (uint8_t)(c.Q(n - 1, k, s) <= 0);
    }

    // Special nodes of FastSC-LUT, FastSCLUT.cpp:46-107.  vcl row depth-1 (H3).
    bool special(int d, int node) {
        const int N = c.N;
        const int posi = (1 << d) + node - 1;
        const int t = c.type(posi);
        if (!fast || t < 0 || t > 3) return false;
        const int temp = N >> d;
        const int *ps = &sym[d * N + temp * node];
        uint8_t *pu = &ucap[d * N + temp * node];
        if (t == 0) {  // R0, :46-54
            std::memset(pu, 0, temp);
        } else if (t == 1) {  // R1, :55-66
            for (int i = 0; i < temp; ++i) pu[i] = c.Q(d - 1, temp * node + i, ps[i]) <= 0;
        } else if (t == 2) {  // REP, :67-80 (sequential fp64 sum, H5)
            double S = 0;
            for (int i = 0; i < temp; ++i) S += c.Q(d - 1, temp * node + i, ps[i]);
            std::memset(pu, (uint8_t)(S <= 0), temp);
        } else {  // SPC, :81-107 (first-min flip, H6)
            std::vector<double> mag(temp);
            int parity = 0;
            for (int i = 0; i < temp; ++i) {
                double l = c.Q(d - 1, temp * node + i, ps[i]);
                pu[i] = (uint8_t)(l <= 0);
                parity += pu[i];
                mag[i] = std::fabs(l);
            }
            if (parity % 2) {
                int m = first_argmin(mag);
                pu[m] = 1 - pu[m];
            }
        }
        return true;
    }

    void visit(int d, int node) {
        const int N = c.N, n = c.n;
        if (special(d, node)) return;
        const int posi = (1 << d) + node - 1;
        const int temp = N >> d, half = temp / 2;
        const int *pa = &sym[d * N + temp * node];
        const int *pb = pa + half;
        const int l = 2 * node, r = 2 * node + 1;
        if (d + 1 < n) {
            int *lo = &sym[(d + 1) * N + half * l];
            for (int j = 0; j < half; ++j) lo[j] = c.F(posi, j, pa[j], pb[j]);
            visit(d + 1, l);
        } else {
            leaf(posi, l, false, pa, pb, 0);
        }
        const uint8_t *ul = &ucap[(d + 1) * N + half * l];
        if (d + 1 < n) {
            int *hi = &sym[(d + 1) * N + half * r];
            for (int j = 0; j < half; ++j) hi[j] = c.G(posi, j, ul[j], pa[j], pb[j]);
            visit(d + 1, r);
        } else {
            leaf(posi, r, true, pa, pb, ul[0]);
        }
        combine(&ucap[d * N + temp * node], ul, &ucap[(d + 1) * N + half * r], half);
    }

    int run(const int32_t *y, uint8_t *out) {
        const int N = c.N, n = c.n;
        if (fast && c.type(0) >= 0 && c.type(0) <= 3) return -2;  // reference UB (root special)
        for (int i = 0; i < N; ++i) sym[i] = y[i];
        visit(0, 0);
        if (!fast) {
            emit_info(c, &ucap[n * N], out);  // SCLUTDecoder.cpp:116-123
        } else {
            std::vector<uint8_t> x(ucap.begin(), ucap.begin() + N);  // FastSCLUT.cpp:186-205
            reencode(x, N);
            emit_info(c, x.data(), out);
        }
        return 0;
    }
};

// ---------------------------------------------------------------------------
// SCL-LUT -- SCLLUTDecoder.cpp:47-253, and FastSCL-LUT (FastSCLLUTDecoder.cpp:
// 57-408) when `fast` is set.  State is L full copies of the symbol tree and
// partial sums, deep-copied at every fork exactly as the reference does.
// ---------------------------------------------------------------------------
struct LutSCL {
    const Code &c;
    bool fast;
    int L;
    std::vector<std::vector<int>> sym;
    std::vector<std::vector<uint8_t>> ucap;
    std::vector<double> pm;

    CaSpec ca;  // ca.A > 0: CRC-aided output of A bits

    LutSCL(const Code &c_, bool fast_) : c(c_), fast(fast_), L(c_.L) {}

    // Keep L survivors of the 2L candidates `pm2` (mink, :8-21).  Returns the
    // parent path and whether the candidate came from the upper half.
    void select(const std::vector<double> &pm2, std::vector<int> &parent, std::vector<bool> &upper) {
        std::vector<int> order = sort_index(pm2);
        parent.assign(L, 0);
        upper.assign(L, false);
        for (int i = 0; i < L; ++i) {
            pm[i] = pm2[order[i]];
            upper[i] = order[i] >= L;
            parent[i] = upper[i] ? order[i] - L : order[i];
        }
    }
    void permute(const std::vector<int> &parent) {
        std::vector<std::vector<int>> s2(L);
        std::vector<std::vector<uint8_t>> u2(L);
        for (int i = 0; i < L; ++i) {
            s2[i] = sym[parent[i]];
            u2[i] = ucap[parent[i]];
        }
        sym.swap(s2);
        ucap.swap(u2);
    }

    // Leaf k from a node at depth n-1 (left :91-145, right :166-221).
    // H3: vcl row n-1.  H4: decisions `DM < 0`.
    void leaf(int posi, int d, int node, int k, bool right) {
        const int N = c.N, n = c.n;
        const int temp = N >> d, half = temp / 2;
        std::vector<double> dm(L);
        for (int i = 0; i < L; ++i) {
            const int *p = &sym[i][d * N + temp * node];
            int s = right ? c.G(posi, 0, ucap[i][(d + 1) * N + half * (2 * node)], p[0], p[half])
                          : c.F(posi, 0, p[0], p[half]);
            dm[i] = c.Q(n - 1, k, s);
        }
        if (c.frozen[k] == 1) {
            for (int i = 0; i < L; ++i) {
                ucap[i][n * N + k] = 0;
                pm[i] += std::fabs(dm[i]) * (double)(dm[i] < 0);
            }
            return;
        }
        std::vector<double> pm2(2 * L);
        std::vector<uint8_t> dec(L);
        for (int i = 0; i < L; ++i) {
            pm2[i] = pm[i];
            pm2[i + L] = pm[i] + std::fabs(dm[i]);
            dec[i] = (uint8_t)(dm[i] < 0);
        }
        std::vector<int> parent;
        std::vector<bool> upper;
        select(pm2, parent, upper);
        permute(parent);
        for (int i = 0; i < L; ++i) {
            uint8_t b = dec[parent[i]];
            ucap[i][n * N + k] = upper[i] ? (uint8_t)(1 - b) : b;
        }
    }

    // FastSCL-LUT special nodes, FastSCLLUTDecoder.cpp:82-213.  SPC (type 3)
    // has no handler in the reference (:215 TODO) and falls through (H7).
    bool special(int d, int node) {
        const int N = c.N;
        const int posi = (1 << d) + node - 1;
        const int t = c.type(posi);
        if (!fast || t < 0 || t > 2) return false;
        const int temp = N >> d;
        const int off = d * N + temp * node;
        if (t == 0) {  // R0, :83-96
            for (int i = 0; i < L; ++i) {
                std::memset(&ucap[i][off], 0, temp);
                for (int j = 0; j < temp; ++j) {
                    double l = c.Q(d - 1, temp * node + j, sym[i][off + j]);
                    pm[i] += (float)(l < 0) * std::fabs(l);
                }
            }
        } else if (t == 1) {  // R1, :99-166
            const int depth = std::min(L - 1, temp);
            std::vector<std::vector<uint8_t>> dec(L, std::vector<uint8_t>(temp));
            std::vector<std::vector<double>> mag(L, std::vector<double>(temp));
            std::vector<std::vector<int>> order(L);
            for (int i = 0; i < L; ++i) {
                for (int j = 0; j < temp; ++j) {
                    double l = c.Q(d - 1, temp * node + j, sym[i][off + j]);
                    dec[i][j] = (uint8_t)(l < 0);
                    mag[i][j] = std::fabs(l);
                }
                order[i] = sort_index(mag[i]);
            }
            for (int layer = 0; layer < depth; ++layer) {
                std::vector<double> pm2(2 * L);
                for (int i = 0; i < L; ++i) {
                    pm2[i] = pm[i];
                    pm2[i + L] = pm[i] + mag[i][order[i][layer]];
                }
                std::vector<int> parent;
                std::vector<bool> upper;
                select(pm2, parent, upper);
                std::vector<std::vector<uint8_t>> dec2(L);
                std::vector<std::vector<double>> mag2(L);
                std::vector<std::vector<int>> order2(L);
                for (int i = 0; i < L; ++i) {
                    dec2[i] = dec[parent[i]];
                    // H2: the flipped position comes from slot i's own (pre-
                    // permutation) order, not from the parent's (:145).
                    if (upper[i]) {
                        int q = order[i][layer];
                        dec2[i][q] = 1 - dec2[i][q];
                    }
                    mag2[i] = mag[parent[i]];
                    order2[i] = order[parent[i]];
                }
                permute(parent);
                dec.swap(dec2);
                mag.swap(mag2);
                order.swap(order2);
            }
            for (int i = 0; i < L; ++i) std::memcpy(&ucap[i][off], dec[i].data(), temp);
        } else {  // REP, :169-213
            std::vector<double> pm2(2 * L);
            for (int i = 0; i < L; ++i) {
                pm2[i] = pm[i];
                pm2[i + L] = pm[i];
            }
            for (int i = 0; i < L; ++i) {
                for (int j = 0; j < temp; ++j) {
                    double l = c.Q(d - 1, temp * node + j, sym[i][off + j]);
                    pm2[i] += (double)(l < 0) * std::fabs(l);
                    pm2[i + L] += (double)(l >= 0) * std::fabs(l);
                }
            }
            std::vector<int> parent;
            std::vector<bool> upper;
            select(pm2, parent, upper);
            permute(parent);
            for (int i = 0; i < L; ++i) std::memset(&ucap[i][off], upper[i] ? 1 : 0, temp);
        }
        return true;
    }

    void visit(int d, int node) {
        const int N = c.N, n = c.n;
        if (special(d, node)) return;
        const int posi = (1 << d) + node - 1;
        const int temp = N >> d, half = temp / 2;
        const int l = 2 * node, r = 2 * node + 1;
        const int off = d * N + temp * node;
        // f (:83-90 / :223-230)
        if (d + 1 < n) {
            for (int i = 0; i < L; ++i) {
                int *s = sym[i].data();
                for (int j = 0; j < half; ++j)
                    s[(d + 1) * N + half * l + j] = c.F(posi, j, s[off + j], s[off + half + j]);
            }
            visit(d + 1, l);
        } else {
            leaf(posi, d, node, l, false);
        }
        // g (:157-165 / :297-305)
        if (d + 1 < n) {
            for (int i = 0; i < L; ++i) {
                int *s = sym[i].data();
                const uint8_t *ul = &ucap[i][(d + 1) * N + half * l];
                for (int j = 0; j < half; ++j)
                    s[(d + 1) * N + half * r + j] = c.G(posi, j, ul[j], s[off + j], s[off + half + j]);
            }
            visit(d + 1, r);
        } else {
            leaf(posi, d, node, r, true);
        }
        // combine (:226-241 / :366-384)
        for (int i = 0; i < L; ++i)
            combine(&ucap[i][off], &ucap[i][(d + 1) * N + half * l], &ucap[i][(d + 1) * N + half * r], half);
    }

    int run(const int32_t *y, uint8_t *out) {
        const int N = c.N, n = c.n;
        if (fast && c.type(0) >= 0 && c.type(0) <= 2) return -2;  // reference UB (root special)
        sym.assign(L, std::vector<int>((n + 1) * N));
        ucap.assign(L, std::vector<uint8_t>((n + 1) * N));
        pm.assign(L, kInf);
        pm[0] = 0;
        for (int i = 0; i < L; ++i)
            for (int k = 0; k < N; ++k) sym[i][k] = y[k];
        visit(0, 0);
        if (ca.A > 0) {
            // decoded info bits of a path: ucap[n] (SCL, :268-275) or the re-encoded
            // root partial sums (FastSCL, :338-355)
            auto info_of = [&](int path) {
                std::vector<uint8_t> x(ucap[path].begin() + (fast ? 0 : n * N), ucap[path].begin() + (fast ? N : (n + 1) * N));
                if (fast) reencode(x, N);
                std::vector<uint8_t> info;
                for (int k = 0; k < N; ++k)
                    if (c.frozen[k] == 0) info.push_back(x[k]);
                return info;
            };
            std::vector<int> order = sort_index(pm);
            int winner = order[0];
            for (int i = 0; i < L; ++i) {
                std::vector<uint8_t> info = info_of(order[i]);
                std::vector<uint8_t> head(info.begin(), info.begin() + ca.A);
                std::vector<uint8_t> chk = crc_encoding(head, ca.crc_n, ca.p);
                bool pass = true;
                for (int j = 0; j < c.K - ca.A; ++j)
                    if (chk[j] != info[ca.A + j]) {
                        pass = false;
                        break;
                    }
                if (pass) {
                    winner = order[i];
                    break;
                }
            }
            std::vector<uint8_t> info = info_of(winner);
            std::memcpy(out, info.data(), ca.A);
            return 0;
        }
        int best = first_argmin(pm);  // H6
        if (!fast) {
            emit_info(c, &ucap[best][n * N], out);  // :244-252
        } else {
            std::vector<uint8_t> x(ucap[best].begin(), ucap[best].begin() + N);  // :387-406
            reencode(x, N);
            emit_info(c, x.data(), out);
        }
        return 0;
    }
};

Code make_code(int32_t N, int32_t K, int32_t L, int32_t v, const int32_t *frozen, const int32_t *node_type,
               const uint8_t *lut_f, const int32_t *f_base, int32_t f_step, const uint8_t *lut_g,
               const int32_t *g_base, int32_t g_step, const double *vcl, int32_t vcl_rows) {
    Code c;
    c.N = N;
    c.K = K;
    c.L = L;
    c.v = v;
    c.n = ilog2(N);
    c.frozen = frozen;
    c.node_type = node_type;
    c.lut_f = lut_f;
    c.f_base = f_base;
    c.f_step = f_step;
    c.lut_g = lut_g;
    c.g_base = g_base;
    c.g_step = g_step;
    c.vcl = vcl;
    c.vcl_rows = vcl_rows;
    return c;
}

}  // namespace

extern "C" {

// kind: 1 = SC-LUT, 2 = SCL-LUT, 3 = FastSC-LUT, 4 = FastSCL-LUT.
// Decodes frames [0, B) of `sym` (int32 [B][N]) into `out` (uint8 [B][K]).
int orc_decode_lut(int32_t kind, int32_t N, int32_t K, int32_t L, int32_t v, const int32_t *frozen,
                   const int32_t *node_type, const uint8_t *lut_f, const int32_t *f_base, int32_t f_step,
                   const uint8_t *lut_g, const int32_t *g_base, int32_t g_step, const double *vcl,
                   int32_t vcl_rows, const int32_t *sym, int64_t B, uint8_t *out) {
    Code c = make_code(N, K, kind == 2 || kind == 4 ? L : 1, v, frozen, node_type, lut_f, f_base, f_step, lut_g,
                       g_base, g_step, vcl, vcl_rows);
    if (N < 2 || (1 << c.n) != N) return -1;
    if (kind == 1 || kind == 3) {
        LutSC dec(c, kind == 3);
        for (int64_t b = 0; b < B; ++b) {
            int rc = dec.run(sym + b * N, out + b * K);
            if (rc) return rc;
        }
        return 0;
    }
    if (kind == 2 || kind == 4) {
        LutSCL dec(c, kind == 4);
        for (int64_t b = 0; b < B; ++b) {
            int rc = dec.run(sym + b * N, out + b * K);
            if (rc) return rc;
        }
        return 0;
    }
    return -3;
}

// CRC-aided list decoders: kind 2 = CA-SCL-LUT, 4 = CA-FastSCL-LUT (the
// list kinds above plus the CRC epilogue).  crc_loc lists the nonzero
// coefficient indices (CRC::CRC, utils.cpp:69-75).  Output uint8 [B][A].
int orc_decode_lut_ca(int32_t kind, int32_t N, int32_t K, int32_t A, int32_t L, int32_t v, const int32_t *frozen,
                      const int32_t *node_type, const uint8_t *lut_f, const int32_t *f_base, int32_t f_step,
                      const uint8_t *lut_g, const int32_t *g_base, int32_t g_step, const double *vcl,
                      int32_t vcl_rows, int32_t crc_n, const int32_t *crc_loc, int32_t n_loc, const int32_t *sym,
                      int64_t B, uint8_t *out) {
    if (kind != 2 && kind != 4) return -3;
    if (A < 1 || A > K || K - A > crc_n) return -1;
    Code c = make_code(N, K, L, v, frozen, node_type, lut_f, f_base, f_step, lut_g, g_base, g_step, vcl, vcl_rows);
    if (N < 2 || (1 << c.n) != N) return -1;
    LutSCL dec(c, kind == 4);
    dec.ca.A = A;
    dec.ca.crc_n = crc_n;
    dec.ca.p.assign(crc_n + 1, 0);
    for (int i = 0; i < n_loc; ++i) dec.ca.p[crc_loc[i]] = 1;
    for (int64_t b = 0; b < B; ++b) {
        int rc = dec.run(sym + b * N, out + b * A);
        if (rc) return rc;
    }
    return 0;
}

// Float SC (min-sum), SCDecoder.cpp:14-89.  llr is float64 [B][N].
int orc_decode_sc_float(int32_t N, int32_t K, const int32_t *frozen, const double *llr, int64_t B, uint8_t *out) {
    Code c = make_code(N, K, 1, 1, frozen, nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr, 0);
    if (N < 2 || (1 << c.n) != N) return -1;
    FloatSC dec(c);
    for (int64_t b = 0; b < B; ++b) dec.run(llr + b * N, out + b * K);
    return 0;
}

}  // extern "C"
