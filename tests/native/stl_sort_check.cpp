// Host check: qpd::stl::sort (csrc/stl_sort.hpp) == libstdc++ std::sort on
// index arrays ordered by tie-heavy double keys.  Built and run by
// tests/test_stl_sort.py.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "stl_sort.hpp"

struct VecSeq {
    std::vector<int> &idx;
    const std::vector<double> &key;
    int get(int p) { return idx[p]; }
    void set(int p, int e) { idx[p] = e; }
    bool less(int a, int b) { return key[a] < key[b]; }
};

int main(int argc, char **argv) {
    long trials = argc > 1 ? atol(argv[1]) : 200000;
    std::mt19937_64 rng(12345);
    long bad = 0;
    for (long t = 0; t < trials; ++t) {
        int n = 1 + rng() % 300;
        if (t % 3 == 0) n = 17 + rng() % 48;  // the R1-node sizes of interest
        if (t % 3 == 1) n = 1 + rng() % 33;   // sort_small's range
        int distinct = 1 + rng() % 8;
        std::vector<double> key(n);
        for (auto &k : key) k = (double)(rng() % distinct) * 0.5;
        if (t % 11 == 0)  // organ pipe / sawtooth: drives introsort into heap sort
            for (int i = 0; i < n; ++i) key[i] = (t % 2) ? (i < n / 2 ? i : n - i) : (double)((i * 7919) % n);
        if (t % 5 == 0) std::sort(key.begin(), key.end());           // presorted
        if (t % 7 == 0) std::sort(key.rbegin(), key.rend());         // reversed
        std::vector<int> a(n), b(n);
        for (int i = 0; i < n; ++i) a[i] = b[i] = i;
        std::sort(a.begin(), a.end(), [&](int p, int q) { return key[p] < key[q]; });
        VecSeq s{b, key};
        qpd::stl::sort(s, 0, n);
        if (a != b) {
            if (++bad < 5) printf("mismatch n=%d distinct=%d\n", n, distinct);
        }
        if (n <= 2 * qpd::stl::kThreshold + 1) {  // the stack-free form used on the device for R1 <= 32
            std::vector<int> c(n);
            for (int i = 0; i < n; ++i) c[i] = i;
            VecSeq s2{c, key};
            qpd::stl::sort_small(s2, 0, n);
            if (a != c && ++bad < 5) printf("sort_small mismatch n=%d distinct=%d\n", n, distinct);
            for (int m = 1; m <= 8; ++m) {  // the R1 layers read the first min(L-1, n) entries
                std::vector<int> e(n);
                for (int i = 0; i < n; ++i) e[i] = i;
                VecSeq s3{e, key};
                qpd::stl::sort_small_prefix(s3, 0, n, m);
                const int k = std::min(m, n);
                if (!std::equal(a.begin(), a.begin() + k, e.begin()) && ++bad < 5)
                    printf("sort_small_prefix mismatch n=%d m=%d distinct=%d\n", n, m, distinct);
                // partition_prefix + the m smallest by (key, block position): the device's selection
                std::vector<int> g(n);
                for (int i = 0; i < n; ++i) g[i] = i;
                VecSeq s4{g, key};
                const int end = n ? qpd::stl::partition_prefix(s4, 0, n, m) : 0;
                std::vector<int> pos(end);
                for (int i = 0; i < end; ++i) pos[i] = i;
                std::stable_sort(pos.begin(), pos.end(), [&](int p, int q) { return key[g[p]] < key[g[q]]; });
                bool ok = end >= k;
                for (int q = 0; q < k && ok; ++q) ok = g[pos[q]] == a[q];
                if (!ok && ++bad < 5) printf("partition_prefix selection mismatch n=%d m=%d distinct=%d\n", n, m, distinct);
            }
        }
    }
    printf("trials=%ld mismatches=%ld\n", trials, bad);
    return bad ? 1 : 0;
}
