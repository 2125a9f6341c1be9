// Diagnostic (dev tool): how the SCL info-leaf forks of a set of frames split
// into the survivor-selection cases the GPU kernel could special-case, per
// frame.  Built by tools/fork_cases.py with g++ around the host engine.
#include <cstdio>
#include <vector>
struct ForkStats;
static std::vector<int> *g_cases = nullptr;  // per fork: 0 identity, 1 one swap, 2 other
static void fork_hook(const double *key, int L) {
    // keeps key[0..L), flips key[L..2L): stable order by (key, index)
    bool sorted = true;
    for (int j = 0; j + 1 < L; ++j) sorted = sorted && key[j] <= key[j + 1];
    const double kmax = key[L - 1];
    int below = 0, a = -1;
    for (int j = 0; j < L; ++j)
        if (key[L + j] < kmax) {
            ++below;
            if (a < 0 || key[L + j] < key[L + a]) a = j;
        }
    int c = 2;
    if (sorted && below == 0) c = 0;
    else if (sorted && below == 1 && key[L + a] >= key[L - 2]) c = 1;
    // 2L > 16 (the W16 kernel, qpd_fast.hip select_survivors16): strict identity, and a tie
    // among the first L stable ranks (the introsort replay)
    bool strict = true;
    for (int j = 0; j + 1 < L; ++j) strict = strict && key[j] < key[j + 1];
    for (int j = 0; j < L; ++j) strict = strict && key[L + j] > key[L - 1];
    bool tie = false;
    for (int i = 0; i < 2 * L && !tie; ++i) {
        int r = 0;
        bool eq = false;
        for (int k = 0; k < 2 * L; ++k) {
            if (k == i) continue;
            r += key[k] < key[i] || (key[k] == key[i] && k < i);
            eq = eq || key[k] == key[i];
        }
        tie = r < L && eq;
    }
    // detail: 10 * min(below, 8) + (sorted ? 0 : 100) + c + (strict ? 1000 : 0) + (tie ? 2000 : 0)
    g_cases->push_back(c + 10 * (below < 9 ? below : 9) + (sorted ? 0 : 100) + (strict ? 1000 : 0) + (tie ? 2000 : 0));
}
#define QPD_HOST_FORK_HOOK(k, L) fork_hook(k, L)
#include "qpd_host.hpp"

extern "C" int fc_run(const qpd_config *c, const int32_t *in, int64_t B, int32_t *cases, int64_t cap, int64_t *per_frame) {
    std::unique_ptr<qpd_host::Plan> p = qpd_host::make_plan(c);
    qpd_host::Engine<uint8_t> e(*p);
    std::vector<int> v;
    g_cases = &v;
    std::vector<uint8_t> out(p->out_k);
    for (int64_t b = 0; b < B; ++b) {
        const size_t before = v.size();
        e.decode(in + b * p->N, out.data());
        per_frame[b] = (int64_t)(v.size() - before);
    }
    for (size_t i = 0; i < v.size() && (int64_t)i < cap; ++i) cases[i] = v[i];
    return (int)v.size();
}
