// Scalar emulation of the W16 survivor selection (qpd_fast.hip select_survivors16:
// dense key ranks, the group-parallel replay of stl::partition_prefix by scan-stop
// masks and all of a partition's swaps at once (stop ranks and slots), and the
// final (rank, position) selection), step for step as one lane group runs it,
// checked against std::sort on the 2L candidate indices (mink,
// SCLLUTDecoder.cpp:8-21) -- the first L outputs must be identical.
// Inputs: path-metric-like keys (keeps roughly ascending, flips = keep + penalty)
// drawn from few distinct values (ties at almost every selection), all-equal and
// +inf keys, and arrays that push the introsort toward its depth limit.
// usage: w16_replay_check [trials]; prints "mismatches=N fallbacks=M".
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

static int lg(int n) {
    int r = 0;
    while (n >>= 1) ++r;
    return r;
}

// Returns false when the replay needs its serial fallback (the depth limit).
static bool emulate(const std::vector<double> &key, int L, std::vector<int> &out) {
    const int n2 = 2 * L;
    std::vector<uint32_t> lt(n2), ent(n2);
    for (int i = 0; i < n2; ++i) {
        int c = 0;
        for (int j = 0; j < n2; ++j) c += key[j] < key[i];
        lt[i] = (uint32_t)c;
        ent[i] = (lt[i] << 5) | (uint32_t)i;  // position i holds candidate i
    }
    int f = 0, l = n2, dl = 2 * lg(n2), end = n2;
    bool live = true;
    while (live) {
        if (dl == 0) return false;
        --dl;
        const int mid = f + (l - f) / 2;
        const uint32_t ea = ent[f + 1], eb = ent[mid], ec = ent[l - 1], ef = ent[f];
        const uint32_t ra = ea >> 5, rb = eb >> 5, rc = ec >> 5;
        int pick;
        if (ra < rb) pick = rb < rc ? mid : ra < rc ? l - 1 : f + 1;
        else pick = ra < rc ? f + 1 : rb < rc ? l - 1 : mid;
        const uint32_t em = pick == mid ? eb : pick == f + 1 ? ea : ec;
        ent[f] = em;
        ent[pick] = ef;
        const uint32_t pv = em >> 5;
        const uint32_t in = ((l < 32 ? (1u << l) : 0u) - 1u) & ~((2u << f) - 1u);
        uint32_t GE = 0, LE = 0;
        for (int p = 0; p < n2; ++p) {
            GE |= (uint32_t)((ent[p] >> 5) >= pv) << p;
            LE |= (uint32_t)((ent[p] >> 5) <= pv) << p;
        }
        GE &= in;
        LE &= in;
        // all swaps at once, as the kernel: ranks, byte slots, partners
        int slotA[32], slotB[32];
        for (int p = 0; p < n2; ++p) {
            if ((GE >> p) & 1u) slotA[__builtin_popcount(GE & ((1u << p) - 1u))] = p;
            if ((LE >> p) & 1u) slotB[__builtin_popcount(LE & ~((p < 31 ? (2u << p) : 0u) - 1u))] = p;
        }
        const int nA = __builtin_popcount(GE), nB = __builtin_popcount(LE);
        std::vector<uint32_t> nxt(ent);
        int S = 0;
        for (int p = 0; p < n2; ++p) {
            const int kA = __builtin_popcount(GE & ((1u << p) - 1u));
            const int kB = __builtin_popcount(LE & ~((p < 31 ? (2u << p) : 0u) - 1u));
            const int bk = ((GE >> p) & 1u) && kA < nB ? slotB[kA] : -1;
            const int ak = ((LE >> p) & 1u) && kB < nA ? slotA[kB] : 64;
            if (p < bk) {
                nxt[p] = ent[bk];
                ++S;
            } else if (ak < p) {
                nxt[p] = ent[ak];
            }
        }
        ent = nxt;
        const int cut_a = S < nA ? slotA[S] : n2, cut_b = S >= 1 ? slotB[S - 1] : n2;
        const int cut = cut_a < cut_b ? cut_a : cut_b;
        if (cut >= L && cut < end) end = cut;
        if (l - cut > 16) {
            if (cut >= end) live = false;
            else f = cut;
        } else {
            l = cut;
        }
        live = live && l - f > 16;
    }
    std::vector<uint32_t> comp(n2);
    for (int p = 0; p < n2; ++p) comp[p] = p < end ? ((ent[p] & 0xFFE0u) | (uint32_t)p) : 0xFFFFu;
    out.assign(L, -1);
    for (int p = 0; p < n2; ++p) {
        int r = 0;
        for (int q = 0; q < n2; ++q) r += comp[q] < comp[p];
        if (r < L) out[r] = (int)(ent[p] & 31u);
    }
    return true;
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(12345);
    long mism = 0, fall = 0, total = 0;
    const double inf = INFINITY;
    for (int t = 0; t < trials; ++t) {
        const int L = 9 + (int)(rng() % 8);
        const int n2 = 2 * L;
        std::vector<double> key(n2);
        const int mode = (int)(rng() % 6);
        const int nv = 1 + (int)(rng() % 5);
        for (int j = 0; j < L; ++j) {
            double k;
            switch (mode) {
                case 0: k = (double)(rng() % nv); break;                              // few values, any order
                case 1: k = (double)(j / (1 + (int)(rng() % 3))); break;              // ascending keeps with runs
                case 2: k = j < (int)(rng() % L) ? (double)(rng() % 3) : inf; break;  // dead paths
                case 3: k = 7.0; break;                                               // all equal
                case 4: k = (double)((j * 7919) % 11 < 4 ? j % 3 : 10 + j); break;    // mixed
                default: k = std::ldexp((double)(rng() % 8), -(int)(rng() % 3)); break;
            }
            key[j] = k;
        }
        for (int j = 0; j < L; ++j) {
            const double pen = (mode == 3 || rng() % 4 == 0) ? 0.0 : (double)(1 + rng() % nv);
            key[L + j] = key[j] + pen;
        }
        std::vector<int> idx(n2);
        for (int i = 0; i < n2; ++i) idx[i] = i;
        std::sort(idx.begin(), idx.end(), [&](int p, int q) { return key[p] < key[q]; });  // mink
        std::vector<int> got;
        if (!emulate(key, L, got)) {
            ++fall;
            continue;
        }
        ++total;
        for (int r = 0; r < L; ++r)
            if (got[r] != idx[r]) {
                if (mism < 5) {
                    printf("mismatch L=%d mode=%d slot %d: %d vs std::sort %d\n", L, mode, r, got[r], idx[r]);
                }
                ++mism;
                break;
            }
    }
    printf("trials=%ld mismatches=%ld fallbacks=%ld\n", total, mism, fall);
    return mism != 0;
}
