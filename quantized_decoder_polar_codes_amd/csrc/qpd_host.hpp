// qpd_host.hpp -- the host engine of libqpd.so: decodes a few frames on the
// CPU, one after another, for the reference drivers' per-frame call
// (`decode(symbols)` once per frame, mainQuantizedDecoder_LLRDomain.py:178;
// mainFPDecoder.py:113).  A GPU launch costs ~0.1 ms before any decoding
// (launch, copies, synchronization), ten times the reference's whole SC-LUT
// call at N = 128 (SCLUTDecoder.cpp:21-124, ~10 us), so the host-buffer entry
// points send batches this small here (qpd_capi.hip: host_engine_takes).
// Batches go to the GPU kernels; this engine is product code with its own
// parity tests (tests/test_gpu_host_engine.py), not the test oracle.
//
// Same algorithm as the GPU kernels (the static schedule of qpd_capi.hip:
// visit, pointer memory instead of the reference's per-fork deep copies,
// the reference's mink / argsort ties through stl_sort.hpp), laid out for one
// core: per path byte / double arrays per tree depth, an F or G whose inputs
// several paths share computed once and pointed to.
//
// Domains: LUT symbols (SC-, SCL-, FastSC-, FastSCL-LUT, the CRC-aided
// kinds) and plain float64 LLRs (SC, SCL, CA-SCL, FastSC, FastSCL); the
// re-quantized float kinds (uniform / Lloyd) stay on the GPU.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include <memory>

#include "qpd.h"
#include "qpd_schedule.hpp"
#include "qpd_types.hpp"
#include "stl_sort.hpp"

namespace qpd_host {

using qpd::Op;

struct Plan {
    int fam = 0;  // qpd::Kind family
    int dom = 0;  // qpd::DOM_LUT or qpd::DOM_FLOAT
    int N = 0, n = 0, K = 0, L = 1, v = 0;
    std::vector<Op> ops;
    std::vector<uint8_t> lut_f, lut_g;  // [count][v][v], [count][2][v][v]
    std::vector<int32_t> f_base, g_base;
    int f_step = 0, g_step = 0;
    std::vector<double> vcl;  // [rows][N][v]
    std::vector<int32_t> info_pos;
    int out_k = 0, ca_A = 0, ca_chk = 0, crc_n = 0;
    uint32_t crc_q = 0;
    double pm_init = 0;
};

// The host engine's plan from a validated configuration (qpd_create has
// checked it): the schedule, the tables and the CRC / list parameters, as
// qpd_create derives them for the GPU plans.  Null for the kinds the engine
// does not decode (uniform / Lloyd re-quantized float domains).
inline std::unique_ptr<Plan> make_plan(const qpd_config *c) {
    int fam = 0, dom = 0;
    if (!qpd_sched::family_of(c->kind, &fam, &dom)) return nullptr;
    if (dom != qpd::DOM_LUT && dom != qpd::DOM_FLOAT) return nullptr;
    auto h = std::make_unique<Plan>();
    int n = 0;
    while ((1 << n) < c->N) ++n;
    const bool list = fam == QPD_SCL_LUT || fam == QPD_FASTSCL_LUT;
    const bool fast = fam == QPD_FASTSC_LUT || fam == QPD_FASTSCL_LUT;
    h->fam = fam;
    h->dom = dom;
    h->N = c->N;
    h->n = n;
    h->K = c->K;
    h->L = list ? c->L : 1;
    h->v = dom == qpd::DOM_LUT ? c->v : 0;
    qpd_sched::Schedule s;
    qpd_sched::visit(s, fam, c->N, n, c->frozen_bits, fast ? c->node_type : nullptr, 0, 0);
    h->ops = s.ops;
    if (dom == qpd::DOM_LUT) {
        const size_t vv = (size_t)c->v * c->v;
        h->lut_f.assign(c->lut_f, c->lut_f + (size_t)c->lut_f_count * vv);
        h->lut_g.assign(c->lut_g, c->lut_g + (size_t)c->lut_g_count * 2 * vv);
        h->f_base.assign(c->f_base, c->f_base + (c->N - 1));
        h->g_base.assign(c->g_base, c->g_base + (c->N - 1));
        h->f_step = c->f_step;
        h->g_step = c->g_step;
        h->vcl.assign(c->vcl, c->vcl + (size_t)c->vcl_rows * c->N * c->v);
    }
    for (int i = 0; i < c->N; ++i)
        if (c->frozen_bits[i] == 0) h->info_pos.push_back(i);
    const bool ca = qpd_sched::is_ca(c->kind);
    h->out_k = ca ? c->A : c->K;
    if (ca) {
        h->ca_A = c->A;
        h->crc_n = c->crc_n;
        for (int i = 0; i < c->crc_loc_count; ++i) {
            const int j = c->crc_loc[i];  // coefficient j -> register bit crc_n - j (j = 0: leading, drops out)
            if (j >= 1) h->crc_q |= 1u << (c->crc_n - j);
        }
        // bits compared after the A info bits: K - A (LUT kinds), crc_n (CASCLDecoder.cpp:223)
        h->ca_chk = c->kind == QPD_CASCL_FLOAT ? c->crc_n : c->K - c->A;
    }
    // DOUBLE_INF of each class (SCLLUTDecoder.h:16, FastSCLDecoder.h:7: 1/0;
    // SCLDecoder.h:8, CASCLDecoder.h:9: 1e300)
    h->pm_init = (dom == qpd::DOM_LUT || fam == QPD_FASTSCL_LUT) ? __builtin_huge_val() : 1e300;
    return h;
}

// Index array sorted by keys, stl_sort.hpp's Seq interface (the reference's
// std::sort(index, key<) of mink / argsort, tie order included).
struct KeySeq {
    int *idx;
    const double *key;
    int get(int p) const { return idx[p]; }
    void set(int p, int e) { idx[p] = e; }
    bool less(int a, int b) const { return key[a] < key[b]; }
};

inline void std_sort_index(int *idx, const double *key, int n) {
    for (int i = 0; i < n; ++i) idx[i] = i;
    KeySeq s{idx, key};
    qpd::stl::sort(s, 0, n);
}

inline int sgn(double x) { return x < 0 ? -1 : (x > 0); }  // utils.h:13

template <class T>
class Engine {
  public:
    explicit Engine(const Plan &p) : P(p) {
        const int N = P.N, n = P.n, L = P.L;
        So.assign(n + 1, 0);
        Uo.assign(n + 1, 0);
        for (int d = 1; d <= n - 1; ++d) {
            So[d] = ssz;
            ssz += N >> d;
        }
        for (int d = 1; d <= n; ++d) {
            Uo[d] = usz;
            usz += N >> d;
        }
        S.assign((size_t)L * ssz + 1, T(0));
        U.assign((size_t)L * usz + 1, 0);
        R.assign((size_t)L * N, 0);
        ps.assign((size_t)L * (n + 1), 0);
        pu.assign((size_t)L * (n + 1), 0);
        tps.assign(ps.size(), 0);
        tpu.assign(pu.size(), 0);
        pm.assign(L, 0.0);
        key.assign(4 * L + 2, 0.0);
        idx.assign(4 * L + 2, 0);
        chan.assign(N, T(0));
        uw.assign((N + 63) / 64, 0);
        int max_r1 = 0;
        // ops with their tables / quanta rows resolved (the host twin of the
        // GPU's micro-op records)
        const size_t vv = (size_t)P.v * P.v;
        for (const Op &o : P.ops) {
            HOp h;
            h.type = o.type;
            h.d = o.d;
            h.node = o.node;
            h.aux = o.aux;
            h.posi = (1 << o.d) + o.node - 1;
            h.ct = N >> (o.d + 1);
            h.temp = N >> o.d;
            h.to_r = o.d == 0 || (o.node & 1);
            if (o.type == qpd::OP_R1) max_r1 = std::max(max_r1, h.temp);
            if (sizeof(T) == 1 && (o.type <= qpd::OP_LEAF_R)) {
                h.tf = P.lut_f.data() + (size_t)P.f_base[h.posi] * vv;
                h.tg = P.lut_g.data() + (size_t)P.g_base[h.posi] * 2 * vv;
                h.fstep = (size_t)P.f_step * vv;
                h.gstep = (size_t)P.g_step * 2 * vv;
            }
            if (sizeof(T) == 1 && (o.type == qpd::OP_LEAF_L || o.type == qpd::OP_LEAF_R))
                h.vrow = P.vcl.data() + ((size_t)(n - 1) * N + 2 * o.node + (o.type == qpd::OP_LEAF_R)) * P.v;  // H3
            if (sizeof(T) == 1 && o.type >= qpd::OP_R0)
                h.vrow = P.vcl.data() + ((size_t)(o.d - 1) * N + (size_t)h.temp * o.node) * P.v;  // H3
            hops.push_back(h);
        }
        // single-path kinds: a depth n-1 node's LEAF_L, LEAF_R and COMB as one
        // op (both decisions and their combine, no dispatch in between)
        if (P.L == 1) {
            std::vector<HOp> f;
            for (size_t k = 0; k < hops.size(); ++k) {
                if (k + 2 < hops.size() && hops[k].type == qpd::OP_LEAF_L && hops[k + 1].type == qpd::OP_LEAF_R &&
                    hops[k + 2].type == qpd::OP_COMB && hops[k + 2].d == hops[k].d) {
                    HOp h = hops[k];
                    h.type = kLeafPair;
                    h.aux = (hops[k].aux ? 1 : 0) | (hops[k + 1].aux ? 2 : 0);
                    h.vrow2 = hops[k + 1].vrow;
                    h.to_r = hops[k + 2].to_r;
                    f.push_back(h);
                    k += 2;
                } else {
                    f.push_back(hops[k]);
                }
            }
            hops.swap(f);
        }
        r1_h.assign((size_t)L * (max_r1 + 1), 0);
        r1_a.assign((size_t)L * (max_r1 + 1), 0.0);
        r1_ord.assign((size_t)L * (max_r1 + 1), 0);
    }

    // One frame: y[N] (int32 symbols or float64 LLRs) -> out[out_k].
    // Returns 0, or qpd::ERR_SYMBOL for a channel symbol outside [0, v).
    template <class In>
    int decode(const In *y, uint8_t *out) {
        const int N = P.N;
        if constexpr (sizeof(T) == 1) {
            uint32_t bad = 0;
            for (int i = 0; i < N; ++i) {
                const int32_t s = (int32_t)y[i];
                bad |= (uint32_t)((uint32_t)s >= (uint32_t)P.v);
                chan[i] = (T)s;
            }
            if (bad) return qpd::ERR_SYMBOL;
        } else {
            for (int i = 0; i < N; ++i) chan[i] = (T)y[i];
        }
        flags = 0;
        if (P.L == 1)
            run<false>();
        else
            run<true>();
        if (flags) return flags;  // NaN metric: the reference's sort is undefined there, stop
        finish(out);
        return flags;
    }

  private:
    struct HOp {
        int type = 0, d = 0, node = 0, aux = 0, posi = 0, ct = 0, temp = 0;
        bool to_r = false;
        const uint8_t *tf = nullptr, *tg = nullptr;
        size_t fstep = 0, gstep = 0;
        const double *vrow = nullptr, *vrow2 = nullptr;
    };
    static constexpr int kLeafPair = 100;
    const Plan &P;
    int flags = 0;  // qpd::ErrFlag of the frame being decoded
    int ssz = 0, usz = 0;

    // A NaN path metric reaching a list sort (float domains; undefined in the
    // reference's std::sort): flagged as the GPU engine flags it (ERR_NAN_PM).
    bool nan_key(const double *k, int n) {
        if (sizeof(T) == 1) return false;  // LUT quanta are finite
        for (int i = 0; i < n; ++i)
            if (k[i] != k[i]) {
                flags |= qpd::ERR_NAN_PM;
                return true;
            }
        return false;
    }
    std::vector<HOp> hops;
    std::vector<int> So, Uo;
    std::vector<T> S, chan;
    std::vector<uint8_t> U, R, ps, pu, tps, tpu, r1_h;
    std::vector<uint64_t> uw;
    std::vector<double> pm, key, r1_a;
    std::vector<int> idx, r1_ord;

    const T *srow(int path, int d) const { return d == 0 ? chan.data() : S.data() + (size_t)path * ssz + So[d]; }
    T *srow_w(int path, int d) { return S.data() + (size_t)path * ssz + So[d]; }
    const uint8_t *urow(int path, int d) const { return U.data() + (size_t)path * usz + Uo[d]; }
    uint8_t *urow_w(int path, int d) { return U.data() + (size_t)path * usz + Uo[d]; }
    uint8_t &PS(int i, int d) { return ps[i * (P.n + 1) + d]; }
    uint8_t &PU(int i, int d) { return pu[i * (P.n + 1) + d]; }

    template <bool LIST>
    void run() {
        const int n = P.n, L = P.L;
        for (int i = 0; i < L; ++i) {
            pm[i] = i == 0 ? 0.0 : P.pm_init;
            for (int d = 0; d <= n; ++d) ps[i * (n + 1) + d] = pu[i * (n + 1) + d] = (uint8_t)i;
        }
        for (const HOp &op : hops) {
            if (flags) return;
            switch (op.type) {
                case qpd::OP_F: fg<LIST, false>(op); break;
                case qpd::OP_G: fg<LIST, true>(op); break;
                case qpd::OP_LEAF_L: leaf<LIST, false>(op); break;
                case qpd::OP_LEAF_R: leaf<LIST, true>(op); break;
                case qpd::OP_COMB: comb<LIST>(op); break;
                case kLeafPair: leaf_pair(op); break;
                default: special(op); break;
            }
        }
    }

    // f / g of one node's ct elements (SCLLUTDecoder.cpp:83-89 / :157-164;
    // utils.cpp:26-36 with contraction off, as the reference rounds)
    template <bool ISG>
    void fg_node(const HOp &op, const T *a, const uint8_t *uu, T *o) const {
#pragma clang fp contract(off)
        const int ct = op.ct;
        const T *b = a + ct;
        if constexpr (sizeof(T) == 1) {
            const int v = P.v;
            const size_t vv = (size_t)v * v;
            if (!ISG) {
                const uint8_t *t = op.tf;
                if (op.fstep == 0)
                    for (int e = 0; e < ct; ++e) o[e] = t[a[e] * v + b[e]];
                else
                    for (int e = 0; e < ct; ++e, t += op.fstep) o[e] = t[a[e] * v + b[e]];
            } else {
                const uint8_t *t = op.tg;
                if (op.gstep == 0)
                    for (int e = 0; e < ct; ++e) o[e] = t[uu[e] * vv + a[e] * v + b[e]];
                else
                    for (int e = 0; e < ct; ++e, t += op.gstep) o[e] = t[uu[e] * vv + a[e] * v + b[e]];
            }
        } else {
            for (int e = 0; e < ct; ++e) {
                if (ISG) {
                    o[e] = (double)(1 - 2 * (int)uu[e]) * a[e] + b[e];
                } else {
                    const double fa = std::fabs(a[e]), fb = std::fabs(b[e]);
                    o[e] = (double)(sgn(a[e]) * sgn(b[e])) * ((fb < fa) ? fb : fa);
                }
            }
        }
    }

    template <bool LIST, bool ISG>
    void fg(const HOp &op) {
        const int d = op.d;
        if (!LIST) {
            fg_node<ISG>(op, srow(0, d), ISG ? urow(0, d + 1) : nullptr, srow_w(0, d + 1));
            return;
        }
        const int L = P.L;
        for (int i = 0; i < L; ++i) {
            // the channel (d = 0) is every path's source
            const int src = d == 0 ? 0 : PS(i, d), us = ISG ? PU(i, d + 1) : 0;
            int dup = -1;  // an earlier path with the same inputs computed this node already
            for (int j = 0; j < i && dup < 0; ++j)
                if ((d == 0 ? 0 : PS(j, d)) == src && (!ISG || PU(j, d + 1) == us) && PS(j, d + 1) == j) dup = j;
#ifdef QPD_HOST_FG_HOOK
            QPD_HOST_FG_HOOK(d, ISG, dup >= 0);  // diagnostic builds: how many path rows an f / g op shares
#endif
            if (dup >= 0) {
                PS(i, d + 1) = (uint8_t)dup;
                continue;
            }
            fg_node<ISG>(op, srow(src, d), ISG ? urow(us, d + 1) : nullptr, srow_w(i, d + 1));
#ifdef QPD_HOST_FG_ELEMS
            QPD_HOST_FG_ELEMS(op, ISG, i, srow(src, d), ISG ? urow(us, d + 1) : nullptr);  // diagnostic builds
#endif
            PS(i, d + 1) = (uint8_t)i;
        }
    }

    // the LLR a decision reads: vcl[row][pos][sym] through the op's quanta
    // row (H3) or the value itself
    double llr(const HOp &op, int j, T s) const {
        if constexpr (sizeof(T) == 1)
            return op.vrow[(size_t)j * P.v + s];
        else
            return s;
    }

    double leaf_llr(const HOp &op, const T *s, int uu, bool right) const {
#pragma clang fp contract(off)
        if constexpr (sizeof(T) == 1) {
            const int v = P.v;
            const int sym = right ? op.tg[(size_t)uu * v * v + s[0] * v + s[1]] : op.tf[s[0] * v + s[1]];
            return op.vrow[sym];
        } else {
            if (right) return (double)(1 - 2 * uu) * s[0] + s[1];
            const double fa = std::fabs(s[0]), fb = std::fabs(s[1]);
            return (double)(sgn(s[0]) * sgn(s[1])) * ((fb < fa) ? fb : fa);
        }
    }

    // Survivors of 2L candidates key[0, 2L) (mink, SCLLUTDecoder.cpp:8-21):
    // slot i takes candidate idx[i]; pointers move with the parents.
    void select() {
        const int L = P.L, n1 = P.n + 1;
        if (nan_key(key.data(), 2 * L)) {  // as the GPU engine's check_keys: a NaN never reaches the sort
            for (int i = 0; i < 2 * L; ++i) idx[i] = i;
            return;
        }
        std_sort_index(idx.data(), key.data(), 2 * L);
        std::memcpy(tps.data(), ps.data(), ps.size());
        std::memcpy(tpu.data(), pu.data(), pu.size());
        for (int i = 0; i < L; ++i) {
            const int c = idx[i], par = c % L;
            pm[i] = key[c];
            std::memcpy(&ps[i * n1], &tps[par * n1], n1);
            std::memcpy(&pu[i * n1], &tpu[par * n1], n1);
        }
    }

    template <bool LIST, bool RIGHT>
    void leaf(const HOp &op) {
        const bool frozen = op.aux != 0;
        const int n = P.n;
        if (!LIST) {  // SCLUTDecoder.cpp:60-65: frozen leaves are 0, else `<= 0` (H4)
            uint8_t dec = 0;
            if (!frozen) dec = leaf_llr(op, srow(0, op.d), RIGHT ? urow(0, n)[0] : 0, RIGHT) <= 0;
            if (RIGHT)
                R[0] = dec;
            else
                urow_w(0, n)[0] = dec;
            return;
        }
        const int L = P.L;
        uint8_t hd[qpd::kMaxLWide];
        double dm[qpd::kMaxLWide];
        for (int i = 0; i < L; ++i) dm[i] = leaf_llr(op, srow(PS(i, op.d), op.d), RIGHT ? urow(PU(i, n), n)[0] : 0, RIGHT);
        if (frozen) {
#pragma clang fp contract(off)
            for (int i = 0; i < L; ++i) {
                pm[i] += std::fabs(dm[i]) * (double)(dm[i] < 0);  // :100-104
                hd[i] = 0;
            }
        } else {
            uint8_t h0[qpd::kMaxLWide];
            for (int i = 0; i < L; ++i) {
                h0[i] = dm[i] < 0;  // H4: SCL family `< 0`
                key[i] = pm[i];
                key[L + i] = pm[i] + std::fabs(dm[i]);
            }
#ifdef QPD_HOST_FORK_HOOK
            QPD_HOST_FORK_HOOK(key.data(), L);  // diagnostic builds: statistics of the info-leaf forks
#endif
            select();
            for (int i = 0; i < L; ++i) hd[i] = h0[idx[i] % L] ^ (idx[i] >= L ? 1 : 0);
        }
        for (int i = 0; i < L; ++i) {
            if (RIGHT) {
                R[(size_t)i * P.N] = hd[i];
            } else {
                urow_w(i, n)[0] = hd[i];
                PU(i, n) = (uint8_t)i;
            }
        }
    }

    // SC family: both leaves of a depth n-1 node and its combine
    // (SCLUTDecoder.cpp:60-65, frozen leaves 0, else `<= 0` (H4); utils.cpp:62-67)
    void leaf_pair(const HOp &op) {
        const T *s = srow(0, op.d);
        uint8_t l = 0, r = 0;
        if (!(op.aux & 1)) l = leaf_llr(op, s, 0, false) <= 0;
        if (!(op.aux & 2)) {
            HOp o2 = op;
            o2.vrow = op.vrow2;
            r = leaf_llr(o2, s, l, true) <= 0;
        }
        uint8_t *o = op.to_r ? &R[0] : urow_w(0, op.d);
        o[0] = l ^ r;
        o[1] = r;
    }

    template <bool LIST>
    void comb(const HOp &op) {
        const int d = op.d, ct = op.ct, L = LIST ? P.L : 1;
        for (int i = 0; i < L; ++i) {
            const uint8_t *l = urow(LIST ? PU(i, d + 1) : 0, d + 1);
            uint8_t *r = &R[(size_t)i * P.N];
            if (op.to_r) {
                std::memcpy(r + ct, r, ct);
                for (int e = 0; e < ct; ++e) r[e] ^= l[e];
            } else {
                uint8_t *o = urow_w(i, d);
                for (int e = 0; e < ct; ++e) o[e] = l[e] ^ r[e];
                std::memcpy(o + ct, r, ct);
                if (LIST) PU(i, d) = (uint8_t)i;
            }
        }
    }

    uint8_t *node_out(int i, int d, bool to_r) { return to_r ? &R[(size_t)i * P.N] : urow_w(i, d); }

    // Special nodes (FastSCLUT.cpp:46-107, FastSCLLUTDecoder.cpp:82-213 and
    // the float twins FastSCDecoder.cpp:45-106 / FastSCLDecoder.cpp:122-251).
    void special(const HOp &op) {
#pragma clang fp contract(off)
        const int d = op.d, L = P.L, temp = op.temp;
        const bool to_r = op.to_r;
        const bool list = P.fam == qpd::K_FASTSCL_LUT;
        auto lv = [&](int i, int j) { return llr(op, j, srow(PS(i, d), d)[j]); };
        if (op.type == qpd::OP_R0) {
            if (list)
                for (int i = 0; i < L; ++i)
                    for (int j = 0; j < temp; ++j) {
                        const double l = lv(i, j);
                        pm[i] += (double)(float)(l < 0) * std::fabs(l);  // H5, :90
                    }
            for (int i = 0; i < L; ++i) std::memset(node_out(i, d, to_r), 0, temp);
        } else if (op.type == qpd::OP_REP) {
            if (!list) {
                double s = 0;
                for (int j = 0; j < temp; ++j) s += lv(0, j);
                std::memset(node_out(0, d, to_r), s <= 0 ? 1 : 0, temp);  // H4: `S <= 0`
            } else {
                for (int i = 0; i < L; ++i) {
                    double kk = pm[i], kf = pm[i];
                    for (int j = 0; j < temp; ++j) {
                        const double l = lv(i, j);
                        kk += (double)(l < 0) * std::fabs(l);
                        kf += (double)(l >= 0) * std::fabs(l);
                    }
                    key[i] = kk;
                    key[L + i] = kf;
                }
                select();
                for (int i = 0; i < L; ++i) std::memset(node_out(i, d, to_r), idx[i] >= L ? 1 : 0, temp);
            }
        } else if (op.type == qpd::OP_SPC) {  // FastSC only
            uint8_t *o = node_out(0, d, to_r);
            uint8_t parity = 0;
            double best = 0;
            int bi = 0;
            for (int j = 0; j < temp; ++j) {
                const double l = lv(0, j);
                o[j] = l <= 0;
                parity ^= o[j];
                const double a = std::fabs(l);
                if (j == 0 || a < best) {  // first minimum (H6)
                    best = a;
                    bi = j;
                }
            }
            if (parity) o[bi] ^= 1;
        } else if (!list) {  // R1, FastSC: `<= 0`
            uint8_t *o = node_out(0, d, to_r);
            for (int j = 0; j < temp; ++j) o[j] = lv(0, j) <= 0;
        } else {
            r1_list(op, temp, to_r, lv);
        }
        if (!to_r)
            for (int i = 0; i < L; ++i) PU(i, d) = (uint8_t)i;
    }

    // FastSCL R1 (FastSCLLUTDecoder.cpp:99-166): per path hard decisions and
    // argsort(|l|) (H1); then min(L-1, temp) layers, each a mink over
    // [PML, PML + |l|[sorted[layer]]], the survivor taking its parent's arrays
    // and, for a flip, flipping the element its OWN slot's old array names
    // (H2, :145).  The arrays never move: a slot holds the index of the path
    // whose arrays it inherited (origin) and its flip positions.
    template <class LV>
    void r1_list(const HOp &op, int temp, bool to_r, LV &&lv) {
        const int L = P.L, m = (L - 1) < temp ? (L - 1) : temp, st = temp + 1;
        for (int i = 0; i < L; ++i) {
            for (int j = 0; j < temp; ++j) {
                const double l = lv(i, j);
                r1_h[i * st + j] = l < 0;
                r1_a[i * st + j] = std::fabs(l);
            }
            std_sort_index(&r1_ord[i * st], &r1_a[i * st], temp);
        }
        int origin[qpd::kMaxLWide], to[qpd::kMaxLWide], nf[qpd::kMaxLWide], tnf[qpd::kMaxLWide];
        int flips[qpd::kMaxLWide][qpd::kMaxLWide], tfl[qpd::kMaxLWide][qpd::kMaxLWide];
        for (int i = 0; i < L; ++i) {
            origin[i] = i;
            nf[i] = 0;
        }
        for (int layer = 0; layer < m; ++layer) {
            int pos_old[qpd::kMaxLWide];
            for (int i = 0; i < L; ++i) {
                const int o = origin[i];
                pos_old[i] = r1_ord[o * st + layer];
                key[i] = pm[i];
                key[L + i] = pm[i] + r1_a[o * st + pos_old[i]];
            }
#ifdef QPD_HOST_R1_HOOK
            QPD_HOST_R1_HOOK(key.data(), L, layer, m, temp);  // diagnostic builds: R1 layer statistics
#endif
            select();
            for (int i = 0; i < L; ++i) {
                const int c = idx[i], par = c % L;
                to[i] = origin[par];
                tnf[i] = nf[par];
                std::memcpy(tfl[i], flips[par], sizeof(int) * nf[par]);
                if (c >= L) tfl[i][tnf[i]++] = pos_old[i];  // H2: the slot's own old order
            }
            for (int i = 0; i < L; ++i) {
                origin[i] = to[i];
                nf[i] = tnf[i];
                std::memcpy(flips[i], tfl[i], sizeof(int) * tnf[i]);
            }
        }
        for (int i = 0; i < L; ++i) {
            uint8_t *o = node_out(i, op.d, to_r);
            std::memcpy(o, &r1_h[origin[i] * st], temp);
            for (int q = 0; q < nf[i]; ++q) o[flips[i][q]] ^= 1;
        }
    }

    // u = x F^{(x)n} of path i's root partial sums (FastSCLUT.cpp:186-198;
    // for SC / SCL the leaf decisions themselves), bit-packed: the stages
    // inside a 64-bit word by masks, the others word against word.
    const uint64_t *reencode(int i) {
        const int N = P.N, nw = (N + 63) / 64;
        const uint8_t *x = &R[(size_t)i * N];
        uint64_t *w = uw.data();
        for (int k = 0; k < nw; ++k) {
            uint64_t a = 0;
            const int e = std::min(64, N - 64 * k);
            for (int j = 0; j < e; ++j) a |= (uint64_t)(x[64 * k + j] & 1u) << j;
            a ^= (a >> 1) & 0x5555555555555555ull;
            a ^= (a >> 2) & 0x3333333333333333ull;
            a ^= (a >> 4) & 0x0f0f0f0f0f0f0f0full;
            a ^= (a >> 8) & 0x00ff00ff00ff00ffull;
            a ^= (a >> 16) & 0x0000ffff0000ffffull;
            a ^= (a >> 32);
            w[k] = a;
        }
        for (int h = 1; h < nw; h <<= 1)
            for (int b = 0; b < nw; b += 2 * h)
                for (int j = b; j < b + h; ++j) w[j] ^= w[j + h];
        return w;
    }
    static uint8_t bit(const uint64_t *w, int pos) { return (uint8_t)((w[pos >> 6] >> (pos & 63)) & 1u); }

    void finish(uint8_t *out) {
        const int L = P.L;
        int best = 0;
        if (L > 1 && P.crc_n > 0) {
            // CA epilogue (CASCLLUTDecoder.cpp:263-290): paths in argsort(PML)
            // order, the first whose A info bits reproduce the check bits under
            // CRC::encoding (utils.cpp:77-92), else the first
            if (nan_key(pm.data(), L)) return;
            std_sort_index(idx.data(), pm.data(), L);
            best = idx[0];
            const uint32_t top = 1u << (P.crc_n - 1), mask = (top << 1) - 1u;
            for (int r = 0; r < L; ++r) {
                const uint64_t *x = reencode(idx[r]);
                uint32_t reg = 0;
                bool pass = true;
                for (int t = 0; t < P.ca_A + P.ca_chk; ++t) {
                    const uint32_t bit = Engine::bit(x, P.info_pos[t]);
                    if (t < P.ca_A) {
                        const uint32_t fb = bit ^ ((reg & top) ? 1u : 0u);
                        reg = ((reg << 1) & mask) ^ (P.crc_q & (0u - fb));
                    } else {
                        pass = pass && bit == ((reg >> (P.crc_n - 1 - (t - P.ca_A))) & 1u);
                    }
                }
                if (pass) {
                    best = idx[r];
                    break;
                }
            }
        } else if (L > 1) {
            for (int j = 1; j < L; ++j)
                if (pm[j] < pm[best]) best = j;  // first minimum (H6, SCLLUTDecoder.cpp:244)
        }
        const uint64_t *x = reencode(best);
        for (int t = 0; t < P.out_k; ++t) out[t] = bit(x, P.info_pos[t]);
    }
};

}  // namespace qpd_host
