// Diagnostic (dev tool): for every R1 node of FastSCL-LUT decodes, the first
// survivor-selection layer whose selection is the identity in a frame (the GPU
// kernel's r1_layers stops there for a wave when all its 8 frames have reached
// such a layer).  Built by tools/r1_layers.py with g++ around the host engine.
#include <cstdio>
#include <vector>
static std::vector<int> *g_rec = nullptr;  // per node: temp * 100 + first identity layer (m if none)
static int g_first = -1, g_m = 0, g_temp = 0;
static void r1_hook(const double *key, int L, int layer, int m, int temp) {
    if (layer == 0) {
        if (g_first >= -1 && g_m > 0) g_rec->push_back(g_temp * 100 + (g_first < 0 ? g_m : g_first));
        g_first = -1;
        g_m = m;
        g_temp = temp;
    }
    if (g_first >= 0) return;
    bool sorted = true;
    for (int j = 0; j + 1 < L; ++j) sorted = sorted && key[j] <= key[j + 1];
    double kmax = key[0];
    for (int j = 1; j < L; ++j) kmax = key[j] > kmax ? key[j] : kmax;
    bool keep = sorted;
    for (int j = 0; j < L && keep; ++j) keep = key[L + j] >= kmax;
    if (keep) g_first = layer;
}
#define QPD_HOST_R1_HOOK(k, L, layer, m, temp) r1_hook(k, L, layer, m, temp)
#include "qpd_host.hpp"

extern "C" int r1_run(const qpd_config *c, const int32_t *in, int64_t B, int32_t *rec, int64_t cap) {
    std::unique_ptr<qpd_host::Plan> p = qpd_host::make_plan(c);
    qpd_host::Engine<uint8_t> e(*p);
    std::vector<int> v;
    g_rec = &v;
    std::vector<uint8_t> out(p->out_k);
    for (int64_t b = 0; b < B; ++b) {
        e.decode(in + b * p->N, out.data());
        if (g_m > 0) v.push_back(g_temp * 100 + (g_first < 0 ? g_m : g_first));  // the frame's last node
        g_m = 0;
        g_first = -1;
    }
    for (size_t i = 0; i < v.size() && (int64_t)i < cap; ++i) rec[i] = v[i];
    return (int)v.size();
}
