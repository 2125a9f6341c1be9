// qpd_capi.hip -- C-ABI of libqpd.so (include/qpd.h): validation, the static
// traversal-schedule compiler, device residency of the tables and kernel
// launches.  Host code only; kernels in qpd_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "qpd.h"
#include "qpd_generic.hip"
#include "qpd_fast.hip"

// Kernel instantiations, each in its own translation unit (build.py UNITS:
// the units compile in parallel).
namespace qpd {
const void *fast_kernel_single(int kind, int sets);              // qpd_k_fast.hip
const void *prefix_kernel(int kind, int sets, bool pw1);         // qpd_k_fast.hip
const void *fast_kernel_scl(int sets, bool l8, bool w16);        // qpd_k_scl.hip
const void *fast_kernel_scl_pw1(int sets, bool l8, bool w16);    // qpd_k_scl1.hip
const void *fast_kernel_fscl(int sets, bool l8, bool r1l);       // qpd_fast_fscl.hip
const void *fast_kernel_fscl_pw1(int sets, bool l8, bool r1l);   // qpd_fast_fscl1.hip
const void *generic_kernel(int fam, int dom, bool wide);         // qpd_k_generic.hip
}  // namespace qpd
#include "qpd_mc.hip"
#include "qpd_probe.hip"
#include "qpd_host.hpp"
#include "qpd_schedule.hpp"

#include <memory>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define QPD_HIP(call)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) return fail(QPD_E_DEVICE, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)

using qpd::DevPlan;
using qpd::Op;
using qpd_sched::Schedule;
using qpd_sched::special_of;
using qpd_sched::visit;
using qpd_sched::family_of;
using qpd_sched::is_ca;

int ilog2_exact(int N) {
    int n = 0;
    while ((1 << n) < N) ++n;
    return ((1 << n) == N) ? n : -1;
}

struct DeviceBuf {
    void *p = nullptr;
    ~DeviceBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct qpd_decoder {
    int kind, N, n, K, L, v, device;  // kind: the kernel family (SC/SCL/FastSC/FastSCL LUT ids)
    int dom = 0;                      // qpd::Dom symbol domain
    int max_waves;
    int64_t scratch_bytes_per_wave;
    int engine = QPD_ENGINE_GENERIC;
    int lds_bytes = 0;
    int lds_tab_bytes = 0;  // of lds_bytes: the f / g ops' byte tables (SCL-LUT)
    int pub_kind = 0;  // the kind the caller asked for (CRC-aided kinds map to their list kind)
    int out_bits = 0;  // bits per decoded frame: K, or A for the CRC-aided kinds
    int ca_A = 0, crc_n = 0;
    uint32_t crc_q = 0;
    DeviceBuf info_mask;
    DeviceBuf mc_pref, mc_crc;  // qpd_mc_frames: info bits before each word; CRC contribution per message bit
    int sets = 1;  // fast engine: frame sets per wave (lut_fast_kernel NS)
    bool l8 = false;  // fast engine: list decoder with L = 8 (select_survivors8)
    bool w16 = false; // fast engine: SCL-LUT with 9 <= L <= 16 (lane groups of 16, select_survivors16)
    bool r1l = false;  // fast engine: an R1 node needs r1_large (the R1L instantiation)
    bool pw1 = false;  // fast engine: one pointer word per path (compact_pointer_fields)
    bool pre = false;         // fast engine pre-mode: root_pre_kernel, then the decode on its rows
    int64_t pre_chunk = 0;    // frames per pre-pass chunk
    int64_t pre_cap = 0;      // frames pre_buf holds
    bool pre_fell_back = false;  // an allocation of pre-pass rows failed: pre_cap is the chunk from then on
    DeviceBuf pre_buf;
    DeviceBuf mc_sym;        // qpd_mc_decode without a fused pre-pass: int32 symbols of one chunk
    int64_t mc_sym_cap = 0;  // frames mc_sym holds
    bool mc_sym_fell_back = false;
    DevPlan plan{};
    qpd::FastPlan fplan{};
    DeviceBuf f_tab, g_tab, fscratch, mops, r1_rank, task_ctr;
    int num_mops = 0;
    DeviceBuf pfx_mops;  // frozen-prefix stages' ops (lut_prefix_kernel): stage 1, then stage 2
    int pfx_nops = 0;    // stage 1 (one path per frame); 0: no split
    int pfx1b_nops = 0;  // stage 1b (<= 2 live paths); 0: stage 2 resumes from stage 1
    int pfx2_nops = 0;   // stage 2 (<= 4 live paths); 0: the decode kernel resumes from stage 1
    int pfx_sets = 1;    // frame sets per wave of the prefix stages (QPD_PFX_SETS)
    int pfx1_rec = 0, pfx1_pm = 0;  // stage 1: words per record, metric word in it
    int pfx1b_rec = 0, pfx1b_pm = 0;  // stage 1b: words per path record, metric word in it
    int pfx2_rec = 0, pfx2_pm = 0;    // stage 2: words per path record, metric word in it
    DeviceBuf pfx1_buf, pfx1b_buf, pfx2_buf;  // the stages' records (interleaved, see FastPlan::pfx)
    size_t pfx1_cap = 0, pfx1b_cap = 0, pfx2_cap = 0;
    std::vector<qpd::MOp> pfx_ops_host, main_ops_host;  // host copies of the split schedule (patch_imports)
    const void *xin_at[3] = {nullptr, nullptr, nullptr};         // the buffer addresses the device copies hold
    std::vector<Op> ops_host;
    DeviceBuf lut_f, f_base, lut_g, g_base, vcl, ops, info_pos, scratch, err;
    DeviceBuf r_f, r_g, q_bnd, q_rec, bnd_off, bnd_len, rec_off, rec_len;  // float-domain re-quantizers
    // staging for the host-buffer entry points
    DeviceBuf h_in, h_out;
    size_t h_in_bytes = 0, h_out_bytes = 0;
    // The decoder's own stream (created with the handle): every upload of
    // qpd_create, the host-buffer entry points (pinned staging, one stream
    // synchronization per call: copy in, decode, copy out + error word) and
    // the error-word checks run on it.
    hipStream_t hs = nullptr;
    void *pin = nullptr;
    size_t pin_bytes = 0;
    // Ordering across streams (thread-safe per handle per
    // stream).  The work buffers (slab, pre-pass rows, task queue, error word,
    // staging) are per decoder, so every call first makes its stream wait for
    // the decoder's previous work when that ran on another stream
    // (hipStreamWaitEvent on `last_ev`), and records `last_ev` on its own
    // stream after its launches.  `mu` serializes host threads on one handle.
    std::mutex mu;
    hipEvent_t last_ev = nullptr;
    hipStream_t last_st = nullptr;
    bool last_valid = false;
    uint32_t task_base = 0;  // task queue counter at the start of the next launch (wave_take)
    // Host engine (qpd_host.hpp) for the host-buffer entry points' small
    // batches: the per-frame drop-in call.  Null for the kinds it does not
    // decode (re-quantized float domains).
    std::unique_ptr<qpd_host::Plan> hplan;
    std::unique_ptr<qpd_host::Engine<uint8_t>> heng_lut;
    std::unique_ptr<qpd_host::Engine<double>> heng_f64;
    int host_mode = QPD_HOST_AUTO;
    int64_t host_max_frames = 0;  // QPD_HOST_AUTO: batches up to this size run on the host engine
    int last_engine = QPD_RAN_NONE;  // what served the last decode call (qpd_info.last_engine)
    // qpd_profile: HIP events around every launch, per kernel class
    bool prof = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev[QPD_KC_COUNT];
    ~qpd_decoder() {
        if (last_valid) (void)hipEventSynchronize(last_ev);  // no buffer is freed under a running launch
        if (hs) (void)hipStreamSynchronize(hs);
        if (last_ev) (void)hipEventDestroy(last_ev);
        if (hs) (void)hipStreamDestroy(hs);
        if (pin) (void)hipHostFree(pin);
        for (auto &v : prof_ev)
            for (auto &e : v) {
                (void)hipEventDestroy(e.first);
                (void)hipEventDestroy(e.second);
            }
    }
};

namespace {

// Device copy of a host array on the decoder's own stream, complete on return
// (qpd_create: every table is resident before the handle is handed out, so no
// decode on any stream can overtake an upload).
template <class T>
int upload(DeviceBuf &b, const T *src, size_t count, hipStream_t st) {
    const size_t bytes = std::max<size_t>(1, count * sizeof(T));
    QPD_HIP(hipMalloc(&b.p, bytes));
    if (count) {
        QPD_HIP(hipMemcpyAsync(b.p, src, count * sizeof(T), hipMemcpyHostToDevice, st));
        QPD_HIP(hipStreamSynchronize(st));
    }
    return QPD_OK;
}

int set_device(const qpd_decoder *d) {
    if (d->device >= 0) QPD_HIP(hipSetDevice(d->device));
    return QPD_OK;
}

// Cross-stream ordering of one decoder's work (see qpd_decoder::last_ev):
// `order_on` before a call's first operation on stream st, `mark_on` after
// its last.
int order_on(qpd_decoder *d, hipStream_t st) {
    if (d->last_valid && d->last_st != st) QPD_HIP(hipStreamWaitEvent(st, d->last_ev, 0));
    return QPD_OK;
}

int mark_on(qpd_decoder *d, hipStream_t st) {
    if (!d->last_ev) QPD_HIP(hipEventCreateWithFlags(&d->last_ev, hipEventDisableTiming));
    QPD_HIP(hipEventRecord(d->last_ev, st));
    d->last_st = st;
    d->last_valid = true;
    return QPD_OK;
}

// One kernel launch of class kc on stream st; bracketed by HIP events on that
// stream while profiling is enabled (qpd_profile / qpd_kernel_times).
template <class F>
int timed_launch(qpd_decoder *d, int kc, hipStream_t st, F &&launch) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto drop = [&]() {  // no event outlives a failed record or launch
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    };
    if (d->prof) {
        hipError_t e = hipEventCreate(&e0);
        if (e == hipSuccess) e = hipEventCreate(&e1);
        if (e == hipSuccess) e = hipEventRecord(e0, st);
        if (e != hipSuccess) {
            drop();
            return fail(QPD_E_DEVICE, std::string("profiling event: ") + hipGetErrorString(e));
        }
    }
    const int rc = launch();
    if (d->prof) {
        const hipError_t e = rc ? hipSuccess : hipEventRecord(e1, st);
        if (rc || e != hipSuccess) {
            drop();
            return rc ? rc : fail(QPD_E_DEVICE, std::string("profiling event: ") + hipGetErrorString(e));
        }
        d->prof_ev[kc].emplace_back(e0, e1);
    }
    return rc;
}

// Kernel family (SC / SCL / FastSC / FastSCL, as the LUT kind ids) and symbol
// domain of every public kind; the CRC-aided kinds are their list family
// plus an output epilogue.
int validate(const qpd_config *c, int *n_out, int *fam_out, int *dom_out) {
    if (!c) return fail(QPD_E_INVALID, "null config");
    int fam = 0, dom = 0;
    if (!family_of(c->kind, &fam, &dom)) return fail(QPD_E_INVALID, "unknown decoder kind");
    if (is_ca(c->kind)) {
        if (c->crc_n < 1 || c->crc_n > 32) return fail(QPD_E_INVALID, "crc_n must be in [1, 32]");
        if (c->kind == QPD_CASCL_FLOAT) {
            // CASCLDecoder.cpp:218-226 compares crc_n bits after the A info bits:
            // A + crc_n > K would read past the decoded info bits (UB there).
            if (c->A < 1 || c->A + c->crc_n > c->K) return fail(QPD_E_INVALID, "CASCLDecoder needs 1 <= A and A + crc_n <= K");
        } else if (c->A < 1 || c->A > c->K || c->K - c->A > c->crc_n) {
            // CRC-aided LUT output (CASCLLUTDecoder.cpp:263-302): K - A > crc_n would
            // read past the reference's check code (UB there), so it is rejected here.
            return fail(QPD_E_INVALID, "CRC-aided kinds need 1 <= A <= K and K - A <= crc_n");
        }
        if (c->crc_loc_count < 0 || (c->crc_loc_count > 0 && !c->crc_loc)) return fail(QPD_E_INVALID, "bad crc_loc");
        for (int i = 0; i < c->crc_loc_count; ++i)
            if (c->crc_loc[i] < 0 || c->crc_loc[i] > c->crc_n) return fail(QPD_E_INVALID, "crc_loc entry outside [0, crc_n]");
    }
    const int n = ilog2_exact(c->N);
    if (c->N < 2 || n < 0 || n > qpd::kMaxDepth) return fail(QPD_E_INVALID, "N must be a power of two in [2, 65536]");
    if (!c->frozen_bits) return fail(QPD_E_INVALID, "frozen_bits is NULL");
    int zeros = 0;
    for (int i = 0; i < c->N; ++i) {
        if (c->frozen_bits[i] != 0 && c->frozen_bits[i] != 1)
            return fail(QPD_E_INVALID, "frozen_bits entries must be 0 or 1");
        zeros += c->frozen_bits[i] == 0;
    }
    if (zeros != c->K) return fail(QPD_E_INVALID, "K must equal the number of information (0) entries of frozen_bits");
    *n_out = n;
    *fam_out = fam;
    *dom_out = dom;
    const bool list = fam == QPD_SCL_LUT || fam == QPD_FASTSCL_LUT;
    if (list && (c->L < 1 || c->L > qpd::kMaxLWide))
        return fail(QPD_E_UNSUPPORTED, "list size L must be in [1, 32]");
    if (fam == QPD_FASTSC_LUT || fam == QPD_FASTSCL_LUT) {
        if (!c->node_type) return fail(QPD_E_INVALID, "node_type is required for the Fast decoders");
        if (special_of(fam, c->node_type, 0) >= 0)
            return fail(QPD_E_UNSUPPORTED, "root node labelled special (undefined behaviour in the reference)");
    }
    if (dom == qpd::DOM_UNIFORM && (!c->r_f || !c->r_g)) return fail(QPD_E_INVALID, "uniform kinds need r_f and r_g");
    if (dom == qpd::DOM_LLOYD) {
        if (!c->q_bnd || !c->q_rec || !c->bnd_off || !c->bnd_len || !c->rec_off || !c->rec_len)
            return fail(QPD_E_INVALID, "Lloyd kinds need boundary and reconstruction tables");
        for (int k = 0; k < 2 * (c->N - 1); ++k) {
            if (c->bnd_len[k] < 1 || c->bnd_off[k] < 0 || (long)c->bnd_off[k] + c->bnd_len[k] > c->q_bnd_count)
                return fail(QPD_E_INVALID, "Lloyd boundary list outside q_bnd (or empty)");
            if (c->rec_len[k] < 1 || c->rec_off[k] < 0 || (long)c->rec_off[k] + c->rec_len[k] > c->q_rec_count)
                return fail(QPD_E_INVALID, "Lloyd reconstruction list outside q_rec (or empty)");
        }
    }
    if (dom != qpd::DOM_LUT) return QPD_OK;
    if (c->v < 2 || c->v > 256) return fail(QPD_E_INVALID, "alphabet size v must be in [2, 256]");
    if (!c->lut_f || !c->lut_g || !c->f_base || !c->g_base || !c->vcl) return fail(QPD_E_INVALID, "null table pointer");
    if ((c->f_step != 0 && c->f_step != 1) || (c->g_step != 0 && c->g_step != 1))
        return fail(QPD_E_INVALID, "f_step/g_step must be 0 or 1");
    if (c->vcl_rows < n) return fail(QPD_E_INVALID, "vcl_rows must be >= log2(N)");
    const int vv = c->v * c->v;
    for (int p = 0; p < c->N - 1; ++p) {
        const int depth = 31 - __builtin_clz((unsigned)(p + 1));
        const int last = (c->N >> (depth + 1)) - 1;
        const long fl = (long)c->f_base[p] + (long)last * c->f_step;
        const long gl = (long)c->g_base[p] + (long)last * c->g_step;
        if (c->f_base[p] < 0 || fl >= c->lut_f_count) return fail(QPD_E_INVALID, "f_base/f_step index outside lut_f");
        if (c->g_base[p] < 0 || gl >= c->lut_g_count) return fail(QPD_E_INVALID, "g_base/g_step index outside lut_g");
    }
    for (long i = 0; i < (long)c->lut_f_count * vv; ++i)
        if (c->lut_f[i] >= c->v) return fail(QPD_E_INVALID, "lut_f entry outside [0, v)");
    for (long i = 0; i < (long)c->lut_g_count * 2 * vv; ++i)
        if (c->lut_g[i] >= c->v) return fail(QPD_E_INVALID, "lut_g entry outside [0, v)");
    for (long i = 0; i < (long)n * c->N * c->v; ++i)
        if (!std::isfinite(c->vcl[i])) return fail(QPD_E_INVALID, "vcl rows 0..n-1 must be finite");
    return QPD_OK;
}


// Fast-engine plan (qpd_fast.hip): per-depth placement of the path buffers
// (deep levels in LDS, shallow levels in a global slab, sized to the LDS
// budget per wave), nibble-packed per-node tables, and the micro-op list with
// every offset precomputed and plain height-3 subtrees fused into BOT3 ops.
struct FastLayout {
    int D = 0;
    int S[qpd::kMaxDepth + 1] = {}, U[qpd::kMaxDepth + 1] = {}, R[qpd::kMaxDepth + 1] = {};
    // LDS rows are grouped by depth (R, S, U of depth D, then of D+1, ...) and
    // followed by the set's selection scratch, so that the rows of all depths
    // > d form one contiguous tail: free scratch while a special node at
    // depth d (which replaces its whole subtree) runs.
    int lds_base[qpd::kMaxDepth + 2] = {};  // first LDS row of depth dd (dd >= D)
    int lds_end = 0;                        // rows incl. the selection scratch
    bool pre = false;    // root pre-pass (root_pre_kernel): MF_PRE / MF_GSEL ops at the root
    bool bfuse = false;  // BOT3 children of depth n-4 nodes fold in the parent's F / G / COMB
    int ns = 1;          // frame sets per wave (their rows interleave)
    bool botx = false;   // FastSCL-LUT, L = 8: height-3 subtrees with special nodes as BOT3 ops (MF_BOTX)
    bool lds(int dd) const { return dd >= D; }
};

// A plain height-3 subtree under (d = n-3, node): one BOT3 op.
bool bot3_plain(int kind, const int32_t *node_type, int n, int d, int node) {
    if (n < 3 || d != n - 3) return false;
    for (int dd = d; dd < n; ++dd)
        for (int k = 0; k < (1 << (dd - d)); ++k)
            if (special_of(kind, node_type, (1 << dd) + (node << (dd - d)) + k - 1) >= 0) return false;
    return true;
}

// The elements of the special node (d, node) share one quanta row vcl[d-1][pos]
// (MF_VUNI's condition; every MinDistortion table qualifies).
bool quanta_uniform(const double *vcl, int N, int v, int d, int node) {
    const int temp = N >> d;
    const uint64_t *q = (const uint64_t *)(vcl + ((size_t)(d - 1) * N + (size_t)temp * node) * v);
    for (int j = 1; j < temp; ++j)
        if (std::memcmp(q, q + (size_t)j * v, sizeof(double) * v) != 0) return false;
    return true;
}

// A height-3 subtree under (d = n-3, node) that botx_op (qpd_fast.hip) can run in
// registers: its nodes of size 4 and 2 plain or FastSCL special nodes (R0 / R1 /
// REP) with one quanta row each.  *ty = the types, two bits per node (q1, q2,
// then q3..q6; BX_* in qpd_fast.hip).
bool bot3_mixed(int kind, const int32_t *node_type, const double *vcl, int N, int n, int v, int node, int *ty) {
    if (kind != QPD_FASTSCL_LUT || n < 4 || v > 16) return false;
    const int d = n - 3;
    if (special_of(kind, node_type, (1 << d) + node - 1) >= 0) return false;
    int t = 0;
    bool any = false;
    for (int h = 0; h < 2; ++h) {
        const int q = 2 * node + h;  // size-4 node at depth n-2
        const int s4 = special_of(kind, node_type, (1 << (d + 1)) + q - 1);
        if (s4 >= 0) {
            if (!quanta_uniform(vcl, N, v, d + 1, q)) return false;
            t |= (1 + s4) << (2 * h);  // R0 / R1 / REP = 0 / 1 / 2 -> BX_R0 / BX_R1 / BX_REP
            any = true;
            continue;
        }
        for (int c = 0; c < 2; ++c) {
            const int k = 2 * h + c, q2 = 2 * q + c;  // size-2 node at depth n-1
            const int s2 = special_of(kind, node_type, (1 << (d + 2)) + q2 - 1);
            if (s2 < 0) continue;
            if (!quanta_uniform(vcl, N, v, d + 2, q2)) return false;
            t |= (1 + s2) << (4 + 2 * k);
            any = true;
        }
    }
#ifdef QPD_DIAG  // diagnostic builds only: QPD_BOTX_SEL = allowed types (bit 1 R0, 2 R1, 3 REP) | size-4 (bit 4) / size-2 (bit 5)
    if (const char *e = getenv("QPD_BOTX_SEL")) {
        const int sel = atoi(e);
        for (int i = 0; i < 6; ++i) {
            const int x = (t >> (2 * i)) & 3;
            if (x && (!(sel & (1 << x)) || !(sel & (i < 2 ? 16 : 32)))) return false;
        }
    }
#endif
    *ty = t;
    return any;
}

// R1 argsort keys of the fast engine (FastSCL, node size <= 32): for element j
// and symbol s of the node, (rank of |vcl[d-1][pos_j][s]| among all the node's
// magnitudes) << 1 | (vcl < 0).  Equal magnitudes get equal ranks, so
// comparing ranks is comparing the doubles (H1 tie behaviour intact).
void r1_rank_table(std::vector<uint16_t> &tab, const double *vcl, int N, int v, int d, int node) {
    const int temp = N >> d;
    const double *q = vcl + ((size_t)(d - 1) * N + (size_t)temp * node) * v;
    std::vector<double> mags;
    for (int i = 0; i < temp * v; ++i) mags.push_back(std::fabs(q[i]));
    std::sort(mags.begin(), mags.end());
    mags.erase(std::unique(mags.begin(), mags.end()), mags.end());
    for (int i = 0; i < temp * v; ++i) {
        const int r = (int)(std::lower_bound(mags.begin(), mags.end(), std::fabs(q[i])) - mags.begin());
        tab.push_back((uint16_t)((r << 1) | (q[i] < 0 ? 1 : 0)));
    }
}

void fast_ops(std::vector<qpd::MOp> &out, const FastLayout &Ly, int kind, int N, int n, int v, const int32_t *frozen,
              const int32_t *node_type, const double *vcl, std::vector<uint16_t> &r1tab, int d, int node) {
    using namespace qpd;
    const int posi = (1 << d) + node - 1;
    auto base = [&](int type) {
        MOp m;
        std::memset(&m, 0, sizeof(m));
        m.type = type;
        m.d = d;
        m.node = node;
        m.sh_src = 4 * d;
        if (d == 0)
            m.flags |= MF_CHAN;
        else if (Ly.pre && d == 1 && node == 0)
            m.flags |= MF_PRE;  // f(y) words at the start of the frame's pre-pass row (src_row 0)
        else {
            m.src_row = Ly.S[d];
            if (Ly.lds(d)) m.flags |= MF_SRC_LDS;
        }
        return m;
    };
    auto finish_node = [&](MOp &m) {  // destination of a finished node (d, node)
        const bool to_r = d == 0 || (node & 1);
        m.dst_row = to_r ? Ly.R[d] : Ly.U[d];
        if (to_r) m.flags |= MF_TO_R;
        if (Ly.lds(d)) m.flags |= MF_DST_LDS;
        m.sh_dst = 4 * d;
    };
    const int t = special_of(kind, node_type, posi);
    if (t >= 0) {
        MOp m = base(OP_R0 + t);
        m.cnt = N >> d;
        m.vrow = (d - 1) * N + (N >> d) * node;
        if (v <= 16 && !getenv("QPD_NO_VUNI")) {  // one quanta row for all the node's elements (MinDistortion tables)
            const uint64_t *q = (const uint64_t *)(vcl + (size_t)m.vrow * v);
            bool uni = true;
            for (int j = 1; j < m.cnt && uni; ++j) uni = std::memcmp(q, q + (size_t)j * v, sizeof(double) * v) == 0;
            if (uni) m.flags |= MF_VUNI;
        }
        if (kind == QPD_FASTSCL_LUT && OP_R0 + t == OP_R1 && m.cnt <= 32) {
            m.tab = (int)r1tab.size();  // rank-key table of this node
            r1_rank_table(r1tab, vcl, N, v, d, node);
            if ((m.flags & MF_VUNI) && !getenv("QPD_NO_R1RK")) {  // one row: the symbols' ranks (< 16) and signs in the record
                uint64_t rk = 0;
                uint32_t sg = 0;
                for (int sy = 0; sy < v; ++sy) {
                    const uint16_t e = r1tab[m.tab + sy];  // element 0's entry = every element's
                    rk |= (uint64_t)(e >> 1) << (4 * sy);
                    sg |= (uint32_t)(e & 1) << sy;
                }
                m.flags |= MF_R1_RK;
                m.r_row = (int32_t)(uint32_t)rk;
                m.tab2 = (int32_t)(uint32_t)(rk >> 32);
                m.pad1 = (int32_t)sg;
            }
            // > 16 elements: std::sort's introsort runs on 16-bit entries in the
            // free LDS tail of the wave (the sets' rows of depths > d + their
            // selection scratch; build_fast pads the LDS rows to make room)
            if (m.cnt > qpd::stl::kThreshold && Ly.lds(d + 1) && Ly.ns * (Ly.lds_end - Ly.lds_base[d + 1]) >= m.cnt / 2) {
                m.flags |= MF_R1_LDS;
                m.u_row = Ly.lds_base[d + 1];
            }
        }
        finish_node(m);
        out.push_back(m);
        return;
    }
    int bx_ty = 0;
    if (n >= 3 && d == n - 3) {
        const bool mixed = Ly.botx && bot3_mixed(kind, node_type, vcl, N, n, v, node, &bx_ty);
        if (mixed || bot3_plain(kind, node_type, n, d, node)) {
            MOp m = base(OP_BOT3);
            for (int j = 0; j < 8; ++j) m.cnt |= (frozen[8 * node + j] == 1) << j;
            if (mixed) {
                m.flags |= MF_BOTX;
                m.cnt |= bx_ty << 8;
            }
            m.tab = posi;
            m.vrow = ((n - 1) * N + 8 * node) * v;
            finish_node(m);
            out.push_back(m);
            return;
        }
    }
    if (d + 1 < n) {
        // Both children plain BOT3 subtrees of a depth n-4 node (d >= 2: S[d] is
        // a slab/LDS row): the left BOT3 takes this node's f, the right one its g
        // and then this node's combine -- no F / G / COMB ops, no S[n-3] rows.
        int t0 = 0;
        auto bot3_able = [&](int c) {  // the child (d + 1, c) becomes a BOT3 op
            return bot3_plain(kind, node_type, n, d + 1, c) ||
                   (Ly.botx && bot3_mixed(kind, node_type, vcl, N, n, v, c, &t0));
        };
        // FastSCL-LUT (L = 8): a size-8 special child takes this node's f / g and combine too
        // (MF_SFG / MF_SGG / MF_SCOMB: r0rep_multi, r1_multi in qpd_fast.hip); R1 only with its
        // ranks in the op record (MF_R1_RK: the record's tab field then holds this node's table)
        auto spec8_able = [&](int c) {
            const int cp = (1 << (d + 1)) + c - 1, ts = special_of(kind, node_type, cp);
            if (!Ly.botx || ts < 0 || getenv("QPD_NO_SFOLD")) return false;
            return OP_R0 + ts != OP_R1 ||
                   (v <= 16 && quanta_uniform(vcl, N, v, d + 1, c) && !getenv("QPD_NO_VUNI") && !getenv("QPD_NO_R1RK"));
        };
        const bool fuse = Ly.bfuse && d == n - 4 && d >= 2 && (bot3_able(2 * node) || spec8_able(2 * node)) &&
                          (bot3_able(2 * node + 1) || spec8_able(2 * node + 1));
        auto spec_child = [&](int c) { return !bot3_able(c); };  // (under `fuse`: a size-8 special child)
        for (int side = 0; side < 2; ++side) {
            MOp m = base(side ? OP_G : OP_F);
            m.cnt = N >> (d + 1);
            m.dst_row = Ly.S[d + 1];
            if (Ly.lds(d + 1)) m.flags |= MF_DST_LDS;
            m.sh_dst = 4 * (d + 1);
            if (side) {
                m.u_row = Ly.U[d + 1];
                if (Ly.lds(d + 1)) m.flags |= MF_U_LDS;
                m.sh_u = 4 * (d + 1);
                m.tab = posi * 64;
            } else {
                m.tab = posi * 32;
            }
            if (Ly.pre && d == 0) {  // root in pre-mode: f(y) comes from the pre-pass row, g(y, u) by selects
                m.flags = (m.flags & ~MF_CHAN) | MF_PRE | MF_GSEL;
                m.src_row = N >> 4;  // g(y, 0) words; g(y, 1) follow
            }
            if (fuse && spec_child(2 * node + side)) {
                const size_t at = out.size();
                fast_ops(out, Ly, kind, N, n, v, frozen, node_type, vcl, r1tab, d + 1, 2 * node + side);
                MOp &b = out[at];  // the child's special op: this node's f / g (and combine) folded in
                b.flags = (b.flags & ~MF_SRC_LDS) | (m.flags & MF_SRC_LDS) | MF_SFG;
                b.src_row = m.src_row;
                b.sh_src = m.sh_src;
                b.tab = m.tab;
                if (side) {
                    b.flags = (b.flags & ~(MF_DST_LDS | MF_TO_R)) | MF_SGG | MF_SCOMB | (m.flags & MF_U_LDS);
                    b.u_row = m.u_row;  // U[n-3] of the left child: g's u bits, then the combine's left half
                    b.sh_u = m.sh_u;
                    finish_node(b);  // this node's destination
                }
                continue;
            }
            if (fuse) {
                const size_t at = out.size();
                fast_ops(out, Ly, kind, N, n, v, frozen, node_type, vcl, r1tab, d + 1, 2 * node + side);
                MOp &b = out[at];  // the child's BOT3
                b.flags = (b.flags & ~MF_SRC_LDS) | (m.flags & MF_SRC_LDS) | MF_BFG;
                b.src_row = m.src_row;
                b.sh_src = m.sh_src;
                b.tab2 = m.tab;
                if (side) {
                    b.flags = (b.flags & ~(MF_DST_LDS | MF_TO_R)) | MF_BG | MF_BCOMB | (m.flags & MF_U_LDS);
                    b.u_row = m.u_row;  // U[n-3]: g's u bits, then the left half of the combine
                    b.sh_u = m.sh_u;
                    finish_node(b);  // this node's destination
                }
                continue;
            }
            if (!(Ly.pre && d == 0 && side == 0)) out.push_back(m);
            fast_ops(out, Ly, kind, N, n, v, frozen, node_type, vcl, r1tab, d + 1, 2 * node + side);
        }
        if (fuse) return;
    } else {
        for (int side = 0; side < 2; ++side) {
            const int k = 2 * node + side;
            MOp m = base(side ? OP_LEAF_R : OP_LEAF_L);
            m.cnt = frozen[k] == 1;
            m.dst_row = side ? Ly.R[n] : Ly.U[n];
            if (Ly.lds(n)) m.flags |= MF_DST_LDS;
            m.sh_dst = 4 * n;
            if (side) {
                m.u_row = Ly.U[n];
                if (Ly.lds(n)) m.flags |= MF_U_LDS;
                m.sh_u = 4 * n;
                m.tab = posi * 64;
            } else {
                m.tab = posi * 32;
            }
            m.vrow = ((n - 1) * N + k) * v;
            out.push_back(m);
        }
    }
    MOp m = base(OP_COMB);
    m.cnt = N >> (d + 1);
    m.u_row = Ly.U[d + 1];
    m.r_row = Ly.R[d + 1];
    if (Ly.lds(d + 1)) m.flags |= MF_U_LDS | MF_R_LDS;
    m.sh_u = 4 * (d + 1);
    finish_node(m);
    out.push_back(m);
}

// Fold an F at depth d+1 into the F / G right before it that produced its
// input (MF_FF, ff_op in qpd_fast.hip): the child's f reads the words the
// parent just computed from registers instead of re-reading S[d+1] from the
// slab.  Pairs are taken greedily down each descent (G1+F2, F3+F4, ...);
// S[d] and S[d+1] as the slab rows ff_op reads, S[d+1] of at least 4 words.
// The rows written are the same as before, so the prefix split's analysis
// (op_rows on the unfused list) and the stores' order are unchanged.
void fuse_descent(std::vector<qpd::MOp> &ops) {
    using namespace qpd;
    std::vector<MOp> out;
    out.reserve(ops.size());
    for (size_t i = 0; i < ops.size(); ++i) {
        MOp a = ops[i];
        if (i + 1 < ops.size() && (a.type == OP_F || a.type == OP_G) &&
            !(a.flags & (MF_CHAN | MF_PRE | MF_GSEL | MF_SRC_LDS | MF_FF)) && a.cnt >= 32) {
            const MOp &b = ops[i + 1];
            const bool dl = a.flags & MF_DST_LDS, cdl = b.flags & MF_DST_LDS;
            if (b.type == OP_F && b.d == a.d + 1 && b.src_row == a.dst_row && b.sh_src == a.sh_dst &&
                ((b.flags & MF_SRC_LDS) != 0) == dl && !(dl && !cdl) && !(b.flags & (MF_CHAN | MF_PRE | MF_GSEL)) &&
                b.cnt * 2 == a.cnt) {
                a.flags |= MF_FF | (cdl ? MF_FF_DL : 0);
                a.r_row = b.dst_row;
                a.tab2 = b.tab;
                a.pad1 = b.sh_dst;
                out.push_back(a);
                ++i;
                continue;
            }
        }
        out.push_back(a);
    }
    ops.swap(out);
}

// Fold the combine at depth n-5 into the right BOT3 before it (MF_BC2, the
// end of bot3_op in qpd_fast.hip): a right BOT3 that already runs its
// parent's combine (MF_BCOMB) and writes R[n-4] is followed by the COMB that
// reads that row and its left sibling's U[n-4]; the BOT3 computes that
// combine from its result in registers and writes the COMB's destination, so
// R[n-4] is neither stored nor loaded and the COMB op goes.  SCL-LUT only.
void fold_combine(std::vector<qpd::MOp> &ops) {
    using namespace qpd;
    std::vector<MOp> out;
    out.reserve(ops.size());
    for (size_t i = 0; i < ops.size(); ++i) {
        MOp a = ops[i];
        if (i + 1 < ops.size() && a.type == OP_BOT3 && (a.flags & MF_BCOMB) && (a.flags & MF_TO_R) && !(a.flags & MF_BC2)) {
            const MOp &b = ops[i + 1];
            if (b.type == OP_COMB && b.d == a.d - 2 && b.cnt == 16 && b.r_row == a.dst_row &&
                ((b.flags & MF_R_LDS) != 0) == ((a.flags & MF_DST_LDS) != 0) && b.sh_u < 256 && b.sh_dst < 256 &&
                b.dst_row >= 0 && b.dst_row < 32768) {
                a.flags |= MF_BC2 | ((b.flags & MF_U_LDS) ? MF_BC2_ULDS : 0) | ((b.flags & MF_DST_LDS) ? MF_BC2_DLDS : 0) |
                           ((b.flags & MF_TO_R) ? MF_BC2_TOR : 0);
                a.r_row = b.u_row;
                a.pad1 = b.sh_u | (b.sh_dst << 8) | (b.dst_row << 16);
                out.push_back(a);
                ++i;
                continue;
            }
        }
        out.push_back(a);
    }
    ops.swap(out);
}

// Place the global-slab drains (MF_SYNC: vmcnt(0) + barrier BEFORE the op).
// A path reads another path's slab rows only through pointer fields copied
// at a fork, and every op that writes a depth's rows writes all lanes' own
// columns and re-points them at themselves.  So a drain is needed only before
// an op that reads global rows through a pointer when some global write
// precedes a fork since the last drain; by then the stores have long
// completed and the drain costs almost nothing.  Single-path kinds (SC, Fast
// SC) never read another lane's rows.  A BOT3 with the parent's combine
// folded in (MF_BCOMB) reads U[n-3] through a pointer AFTER its own forks, so
// any global write before it is drained at its start.
void place_syncs(std::vector<qpd::MOp> &ops, bool list) {
    using namespace qpd;
    bool dirty = false, exposed = false;
    for (MOp &m : ops) {
        m.flags &= ~MF_SYNC;
        if (!list) continue;
        bool forks = false;
        switch (m.type) {
            case OP_BOT3: forks = m.cnt != 0xff; break;
            case OP_LEAF_L:
            case OP_LEAF_R: forks = m.cnt == 0; break;
            case OP_REP:
            case OP_R1: forks = true; break;
            default: break;
        }
        const bool src_glb = !(m.flags & (MF_SRC_LDS | MF_CHAN | MF_PRE));
        const bool spec_u = m.type >= OP_R0 && m.type <= OP_SPC && (m.flags & (MF_SGG | MF_SCOMB));
        const bool u_glb = ((m.type == OP_G || m.type == OP_COMB || m.type == OP_LEAF_R || spec_u ||
                             (m.type == OP_BOT3 && (m.flags & (MF_BG | MF_BCOMB)))) &&
                            !(m.flags & MF_U_LDS)) ||
                           (m.type == OP_BOT3 && (m.flags & MF_BC2) && !(m.flags & MF_BC2_ULDS));
        const bool late_u = (m.type == OP_BOT3 && forks &&
                             (((m.flags & MF_BCOMB) && !(m.flags & MF_U_LDS)) || ((m.flags & MF_BC2) && !(m.flags & MF_BC2_ULDS)))) ||
                            (forks && (m.flags & MF_SCOMB) && spec_u && !(m.flags & MF_U_LDS));
        if ((exposed && (src_glb || u_glb)) || (late_u && dirty)) {
            m.flags |= MF_SYNC;
            exposed = dirty = false;
        }
        if (!(m.flags & ((m.type == OP_BOT3 && (m.flags & MF_BC2)) ? MF_BC2_DLDS : MF_DST_LDS))) dirty = true;
        if (forks && dirty) exposed = true;
    }
}

// Row ownership of a fast layout: (space, row) -> slot (0 R, 1 S, 2 U) and tree
// depth, for the frozen-prefix split.
struct FastOwner {
    std::vector<int8_t> slot[2], depth[2];  // per space (0 slab, 1 LDS); slot -1: unowned
    void add(bool lds, int base, int cnt, int sl, int dd) {
        const int sp = lds ? 1 : 0;
        if ((int)slot[sp].size() < base + cnt) {
            slot[sp].resize(base + cnt, -1);
            depth[sp].resize(base + cnt, -1);
        }
        for (int r = 0; r < cnt; ++r) {
            slot[sp][base + r] = (int8_t)sl;
            depth[sp][base + r] = (int8_t)dd;
        }
    }
    int of(int sp, int row) const { return row >= 0 && row < (int)slot[sp].size() ? slot[sp][row] : -1; }
    int rows(int sp) const { return (int)slot[sp].size(); }
};

// Rows of the fast engine's slab / LDS an op reads and writes (space, first
// row, count), from the access pattern of its code in qpd_fast.hip.  Reads of
// the channel or a pre-pass row (MF_CHAN / MF_PRE) are not row reads.
template <class Fn>
void op_rows(const qpd::MOp &m, Fn &&acc) {
    using namespace qpd;
    const int fl = m.flags;
    const bool src_row = !(fl & (MF_CHAN | MF_PRE));
    const int sp_s = (fl & MF_SRC_LDS) ? 1 : 0, sp_u = (fl & MF_U_LDS) ? 1 : 0, sp_d = (fl & MF_DST_LDS) ? 1 : 0;
    const int c = m.cnt;
    switch (m.type) {
        case OP_F:
        case OP_G:
            if (src_row) acc(false, sp_s, m.src_row, c >= 8 ? 2 * (c >> 3) : 1);
            if (m.type == OP_G) acc(false, sp_u, m.u_row, std::max(1, c >> 5));
            acc(true, sp_d, m.dst_row, c >= 8 ? c >> 3 : 1);
            if (fl & MF_FF) acc(true, (fl & MF_FF_DL) ? 1 : 0, m.r_row, c >> 4);
            break;
        case OP_COMB: {
            const int cw = c < 32 ? 1 : c >> 5;
            acc(false, sp_u, m.u_row, cw);
            acc(false, (fl & MF_R_LDS) ? 1 : 0, m.r_row, cw);
            acc(true, sp_d, m.dst_row, c < 32 ? 1 : 2 * cw);
            break;
        }
        case OP_LEAF_L:
        case OP_LEAF_R:
            if (src_row) acc(false, sp_s, m.src_row, 1);
            if (m.type == OP_LEAF_R) acc(false, sp_u, m.u_row, 1);
            acc(true, sp_d, m.dst_row, 1);
            break;
        case OP_BOT3:
            if (src_row) acc(false, sp_s, m.src_row, (fl & MF_BFG) ? 2 : 1);
            if (fl & (MF_BG | MF_BCOMB)) acc(false, sp_u, m.u_row, 1);
            if (fl & MF_BC2) {
                acc(false, (fl & MF_BC2_ULDS) ? 1 : 0, m.r_row, 1);
                acc(true, (fl & MF_BC2_DLDS) ? 1 : 0, m.pad1 >> 16, 1);
            } else {
                acc(true, sp_d, m.dst_row, 1);
            }
            break;
        case OP_IMPORT: acc(true, sp_d, m.dst_row, c); break;
        case OP_EXPORT: acc(false, sp_s, m.src_row, c); break;
        default:  // special nodes: temp symbols in, temp bits out
            acc(false, sp_s, m.src_row, (c + 7) >> 3);
            acc(true, sp_d, m.dst_row, (c + 31) >> 5);
            break;
    }
}

// Frozen-prefix stages of an SCL schedule (see lut_prefix_kernel).
//   stage 1:  ops [0, s1) -- up to the first forking op: one path, gs = 1;
//   stage 1b: ops [s1, sb) -- up to the op with the second information leaf: at
//             most 2 live paths, run with L = 2, gs = 2 (opt-in: QPD_PFX1B=1);
//   stage 2:  ops [sb, s2) -- up to the op with the third information leaf: at
//             most 4 live paths, run with L = 4;
//   decode:   ops [s2, end) with the full list.
// For 2L <= 16 mink's sort is stable (SCLLUTDecoder.cpp:8-21, H1): the live
// candidates (keeps before flips, each in slot order) take slots 0..2k-1 in the
// same order at L = 2, 4 or 8, and the other slots' metrics are infinite.
// Each stage ends with OP_EXPORT of the words the later ops read before
// writing them (live-in) and begins with OP_IMPORT of its predecessor's.
struct PrefixPlan {
    std::vector<qpd::MOp> st1, st1b, st2, rest;
    int rec1 = 0, pm1 = 0;    // stage 1: words per record, metric word in it
    int rec1b = 0, pm1b = 0;  // stage 1b: words per path record, metric word in it
    int rec2 = 0, pm2 = 0;    // stage 2: words per path record, metric word in it
};

bool is_fork(const qpd::MOp &m) {
    using namespace qpd;
    return (m.type == OP_BOT3 && m.cnt != 0xff) || ((m.type == OP_LEAF_L || m.type == OP_LEAF_R) && m.cnt == 0) ||
           m.type == OP_R1 || m.type == OP_REP || m.type == OP_SPC;
}

int info_leaves(const qpd::MOp &m) {
    using namespace qpd;
    if (m.type == OP_BOT3) return __builtin_popcount(~m.cnt & 0xff);
    if (m.type == OP_LEAF_L || m.type == OP_LEAF_R) return m.cnt == 0;
    return 0;
}

// Live-in words of ops[from, end): live[sp][row].  False if an unowned row is read.
bool live_in(const std::vector<qpd::MOp> &ops, size_t from, const FastOwner &own, std::vector<char> (&live)[2]) {
    std::vector<char> def[2];
    for (int sp = 0; sp < 2; ++sp) {
        def[sp].assign(own.rows(sp), 0);
        live[sp].assign(own.rows(sp), 0);
    }
    bool ok = true;
    for (size_t i = from; i < ops.size() && ok; ++i)
        op_rows(ops[i], [&](bool wr, int sp, int row, int cnt) {
            for (int r = row; r < row + cnt; ++r) {
                if (own.of(sp, r) < 0) {
                    if (!wr) ok = false;
                    continue;
                }
                if (wr) def[sp][r] = 1;
                else if (!def[sp][r]) live[sp][r] = 1;
            }
        });
    return ok;
}

// Runs of live words with one slot and depth: fn(sp, first row, count, slot, depth).
template <class Fn>
void live_runs(const std::vector<char> (&live)[2], const FastOwner &own, Fn &&fn) {
    for (int sp = 0; sp < 2; ++sp)
        for (int r = 0; r < own.rows(sp);) {
            if (!live[sp][r]) {
                ++r;
                continue;
            }
            int e = r;
            while (e < own.rows(sp) && live[sp][e] && own.slot[sp][e] == own.slot[sp][r] && own.depth[sp][e] == own.depth[sp][r])
                ++e;
            fn(sp, r, e - r, (int)own.slot[sp][r], (int)own.depth[sp][r]);
            r = e;
        }
}

qpd::MOp blank_op(int type) {
    qpd::MOp m;
    std::memset(&m, 0, sizeof(m));
    m.type = type;
    return m;
}

bool plan_prefix(const std::vector<qpd::MOp> &ops, const FastOwner &own, int L, PrefixPlan &pp) {
    using namespace qpd;
    size_t s1 = 0;
    while (s1 < ops.size() && !is_fork(ops[s1])) ++s1;
    if (s1 == 0 || s1 == ops.size()) return false;
    // stage 1 -> one-path records (geometry G = 6, PS = 0): S words (computed) and the
    // metric; U / R words are zeros (every decision of the prefix is a frozen 0)
    std::vector<char> live1[2];
    if (!live_in(ops, s1, own, live1)) return false;
    std::vector<MOp> imp1, exp1;
    int w1 = 0;
    live_runs(live1, own, [&](int sp, int r, int cnt, int slot, int) {
        MOp m = blank_op(OP_IMPORT);
        m.dst_row = r;
        m.cnt = cnt;
        m.flags = sp ? MF_DST_LDS : 0;
        if (slot == 1) {
            m.flags |= MF_XBUF;
            m.src_row = w1;
            MOp x = blank_op(OP_EXPORT);
            x.flags = sp ? MF_SRC_LDS : 0;
            x.src_row = r;
            x.dst_row = w1;
            x.cnt = cnt;
            exp1.push_back(x);
            w1 += cnt;
        } else {
            m.flags |= MF_ZERO;
        }
        imp1.push_back(m);
    });
    pp.pm1 = w1;
    pp.rec1 = w1 + 2;
    MOp pm = blank_op(OP_IMPORT);
    pm.flags = MF_XBUF | MF_PM;
    pm.src_row = pp.pm1;
    imp1.insert(imp1.begin(), pm);
    for (MOp &m : imp1) {  // record words, geometry and live paths; the address is patched per buffer
        m.tab = pp.rec1;
        m.vrow = 6;
        m.tab2 = 1;
        m.node = 1;  // buffer: stage 1's
    }
    pp.st1.assign(ops.begin(), ops.begin() + s1);
    pp.st1.insert(pp.st1.end(), exp1.begin(), exp1.end());
    // stage 2 (4 < L <= 8): up to the op with the third information leaf.  Not above L = 8:
    // mink's 2L > 16 candidates go through libstdc++'s introsort there, whose order of tied
    // live metrics the stable L = 4 selection would not reproduce (H1).
    size_t s2 = s1;
    for (int inf = 0; s2 < ops.size() && inf + info_leaves(ops[s2]) <= 2; ++s2) inf += info_leaves(ops[s2]);
    std::vector<char> live2[2];
    if (L <= 4 || L > qpd::kMaxL || getenv("QPD_NO_PFX2") || s2 <= s1 || s2 >= ops.size() || !live_in(ops, s2, own, live2)) {
        pp.rest = imp1;
        pp.rest.insert(pp.rest.end(), ops.begin() + s1, ops.end());
        return true;
    }
    // stage 2 -> four-path records (G = 4, PS = 2), stage 1b -> two-path records (G = 5,
    // PS = 1): every live word, read through the lineage's pointer of its depth, and the metric
    auto path_records = [&](const std::vector<char> (&live)[2], int G, int PS, int node, std::vector<MOp> &imp,
                            std::vector<MOp> &exp, int &rec, int &pmw) {
        int w = 0;
        live_runs(live, own, [&](int sp, int r, int cnt, int slot, int dd) {
            MOp x = blank_op(OP_EXPORT);
            x.flags = (sp ? MF_SRC_LDS : 0) | (slot == 1 ? MF_VIA_PS : slot == 2 ? MF_VIA_PU : 0);
            x.sh_src = 4 * dd;
            x.src_row = r;
            x.dst_row = w;
            x.cnt = cnt;
            exp.push_back(x);
            MOp m = blank_op(OP_IMPORT);
            m.flags = MF_XBUF | (sp ? MF_DST_LDS : 0);
            m.src_row = w;
            m.dst_row = r;
            m.cnt = cnt;
            imp.push_back(m);
            w += cnt;
        });
        pmw = w;
        rec = w + 2;
        MOp pm = blank_op(OP_IMPORT);
        pm.flags = MF_XBUF | MF_PM;
        pm.src_row = pmw;
        imp.insert(imp.begin(), pm);
        for (MOp &m : imp) {
            m.tab = rec;
            m.vrow = G | (PS << 8);
            m.tab2 = 1 << PS;  // live paths of the record
            m.node = node;     // buffer: 2 stage 2's, 3 stage 1b's
        }
    };
    std::vector<MOp> imp2, exp2;
    path_records(live2, 4, 2, 2, imp2, exp2, pp.rec2, pp.pm2);
    // stage 1b (opt-in, QPD_PFX1B=1): the ops up to the one with the second information
    // leaf, run by 2 lanes per frame instead of stage 2's 4 (a third of the stages' lane
    // lookups on the bench code).  Measured -0.7 % on the bench workload: stage 2 2.19 ->
    // 1.30 ms, but stage 1b's own launch, drain and records take 1.07 ms (profiles/r06m_*).
    size_t sb = s1;
    for (int inf = 0; sb < ops.size() && inf + info_leaves(ops[sb]) <= 1; ++sb) inf += info_leaves(ops[sb]);
    std::vector<char> liveb[2];
    if (sb > s1 && sb < s2 && getenv("QPD_PFX1B") && live_in(ops, sb, own, liveb)) {
        std::vector<MOp> impb, expb;
        path_records(liveb, 5, 1, 3, impb, expb, pp.rec1b, pp.pm1b);
        pp.st1b = imp1;
        pp.st1b.insert(pp.st1b.end(), ops.begin() + s1, ops.begin() + sb);
        pp.st1b.insert(pp.st1b.end(), expb.begin(), expb.end());
        imp1 = impb;  // stage 2 starts from stage 1b's records
        s1 = sb;
    }
    pp.st2 = imp1;
    pp.st2.insert(pp.st2.end(), ops.begin() + s1, ops.begin() + s2);
    pp.st2.insert(pp.st2.end(), exp2.begin(), exp2.end());
    pp.rest = imp2;
    pp.rest.insert(pp.rest.end(), ops.begin() + s2, ops.end());
    return true;
}

// Point the import ops of a prefix-split schedule at the stage buffers (op.node: 1 / 2 /
// 3 = stage 1b), on the launch stream, when a buffer moved.
int patch_imports(qpd_decoder *d, hipStream_t st) {
    const void *b1 = d->pfx1_buf.p, *b2 = d->pfx2_buf.p, *b3 = d->pfx1b_buf.p;
    if (d->xin_at[0] == b1 && d->xin_at[1] == b2 && d->xin_at[2] == b3) return QPD_OK;
    auto patch = [&](std::vector<qpd::MOp> &v) {
        for (qpd::MOp &m : v)
            if (m.type == qpd::OP_IMPORT && (m.flags & qpd::MF_XBUF)) {
                const uint64_t a = (uint64_t)(uintptr_t)(m.node == 3 ? b3 : m.node == 2 ? b2 : b1);
                m.u_row = (int32_t)(uint32_t)a;
                m.r_row = (int32_t)(uint32_t)(a >> 32);
            }
    };
    patch(d->pfx_ops_host);
    patch(d->main_ops_host);
    QPD_HIP(hipMemcpyAsync(d->pfx_mops.p, d->pfx_ops_host.data(), d->pfx_ops_host.size() * sizeof(qpd::MOp),
                           hipMemcpyHostToDevice, st));
    QPD_HIP(hipMemcpyAsync(d->mops.p, d->main_ops_host.data(), d->main_ops_host.size() * sizeof(qpd::MOp),
                           hipMemcpyHostToDevice, st));
    d->xin_at[0] = b1;
    d->xin_at[1] = b2;
    d->xin_at[2] = b3;
    return QPD_OK;
}

// A stage's record buffer for Bc frames (rounded up to whole 64-frame groups), grown on demand.
int ensure_records(DeviceBuf &b, size_t &cap, int64_t Bc, int rec, int paths) {
    const size_t need = (size_t)((Bc + 63) / 64 * 64) * (size_t)rec * paths * sizeof(uint32_t);
    if (cap >= need) return QPD_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    cap = 0;
    const hipError_t e = hipMalloc(&b.p, need);
    if (e != hipSuccess) return fail(QPD_E_DEVICE, std::string("prefix records hipMalloc: ") + hipGetErrorString(e));
    cap = need;
    return QPD_OK;
}

#ifndef QPD_DEFAULT_SETS
#define QPD_DEFAULT_SETS 2
#endif
constexpr int kDefaultSets = QPD_DEFAULT_SETS;

// The decode kernel instantiation of a plan (nullptr: none, the launch fails).
// pw1: the op list's pointer fields fit one word (compact_pointer_fields).
const void *fast_kernel(int kind, int sets, bool l8, bool r1l, bool pw1, bool w16) {
    switch (kind) {
        case QPD_SC_LUT:
        case QPD_FASTSC_LUT: return pw1 || r1l ? nullptr : qpd::fast_kernel_single(kind, sets);
        case QPD_SCL_LUT: return r1l ? nullptr : pw1 ? qpd::fast_kernel_scl_pw1(sets, l8, w16) : qpd::fast_kernel_scl(sets, l8, w16);
        case QPD_FASTSCL_LUT: return w16 ? nullptr : pw1 ? qpd::fast_kernel_fscl_pw1(sets, l8, r1l) : qpd::fast_kernel_fscl(sets, l8, r1l);
        default: return nullptr;
    }
}
using qpd::generic_kernel;
using qpd::prefix_kernel;

// One pointer word per path (PathT<true>, qpd_fast.hip): the S-row and U-row
// pointer fields the op lists read or set, by op type (the access pattern of
// each op's code), packed into consecutive 4-bit positions of one word.
// False (lists unchanged) when they need more than 16 fields.
bool compact_pointer_fields(const std::vector<std::vector<qpd::MOp> *> &lists) {
    using namespace qpd;
    int pos[2][kMaxDepth + 1];
    for (auto &a : pos)
        for (int &x : a) x = -1;
    int bc_u = 0, bc_dst = 0;  // an MF_BC2 op's two fields (pad1), unpacked before each()
    auto each = [&](qpd::MOp &m, auto &&fn) {  // fn(slot 0 = S / 1 = U, int &sh)
        const int fl = m.flags;
        const bool src_row = !(fl & (MF_CHAN | MF_PRE));
        switch (m.type) {
            case OP_F:
            case OP_G:
                if (src_row) fn(0, m.sh_src);
                if (m.type == OP_G) fn(1, m.sh_u);  // (MF_GSEL reads U[1] through it too)
                fn(0, m.sh_dst);
                if (fl & MF_FF) fn(0, m.pad1);
                break;
            case OP_LEAF_L:
            case OP_LEAF_R:
                if (src_row) fn(0, m.sh_src);
                if (m.type == OP_LEAF_R) fn(1, m.sh_u);
                else fn(1, m.sh_dst);
                break;
            case OP_COMB:
                fn(1, m.sh_u);
                if (!(fl & MF_TO_R)) fn(1, m.sh_dst);
                break;
            case OP_BOT3:
                if (src_row) fn(0, m.sh_src);
                if (fl & (MF_BG | MF_BCOMB)) fn(1, m.sh_u);
                if (!(fl & MF_TO_R)) fn(1, m.sh_dst);
                if (fl & MF_BC2) {  // (the fields packed in pad1, unpacked into bc_u / bc_dst)
                    fn(1, bc_u);
                    if (!(fl & MF_BC2_TOR)) fn(1, bc_dst);
                }
                break;
            case OP_IMPORT: break;
            case OP_EXPORT:
                if (fl & MF_VIA_PS) fn(0, m.sh_src);
                if (fl & MF_VIA_PU) fn(1, m.sh_src);
                break;
            default:  // special nodes
                fn(0, m.sh_src);
                if (fl & (MF_SGG | MF_SCOMB)) fn(1, m.sh_u);
                if (!(fl & MF_TO_R)) fn(1, m.sh_dst);
                break;
        }
    };
    auto unpack = [&](const qpd::MOp &m) {
        bc_u = m.pad1 & 255;
        bc_dst = (m.pad1 >> 8) & 255;
    };
    int used = 0;
    for (auto *l : lists)
        for (qpd::MOp &m : *l)
            unpack(m), each(m, [&](int sl, int &sh) {
                int &p = pos[sl][sh / 4];
                if (p < 0) p = used++;
            });
    if (used > 16) return false;
    for (auto *l : lists)
        for (qpd::MOp &m : *l) {
            // every field of an op is rewritten once (fields shared by two
            // roles, e.g. sh_src of a special node, are read before any write)
            int sh_src = m.sh_src, sh_u = m.sh_u, sh_dst = m.sh_dst, pad1 = m.pad1;
            unpack(m);
            int nbc_u = bc_u, nbc_dst = bc_dst;
            each(m, [&](int sl, int &sh) {
                const int np = 4 * pos[sl][sh / 4];
                if (&sh == &m.sh_src) sh_src = np;
                else if (&sh == &m.sh_u) sh_u = np;
                else if (&sh == &m.pad1) pad1 = np;
                else if (&sh == &bc_u) nbc_u = np;
                else if (&sh == &bc_dst) nbc_dst = np;
                else sh_dst = np;
            });
            if (m.type == OP_BOT3 && (m.flags & MF_BC2)) pad1 = (m.pad1 & ~0xFFFF) | nbc_u | (nbc_dst << 8);
            m.sh_src = sh_src;
            m.sh_u = sh_u;
            m.sh_dst = sh_dst;
            m.pad1 = pad1;
        }
    return true;
}

// Task queue of the persistent kernels: one counter, never reset (wave_take).
// QPD_TASK_BASE0 (tests only) starts it elsewhere, e.g. just below 2^32 so
// that the first launches wrap around.
int init_task_queue(qpd_decoder *d) {
    uint32_t v0 = 0;
    if (const char *e = getenv("QPD_TASK_BASE0")) v0 = (uint32_t)strtoull(e, nullptr, 0);
    const uint32_t init[2] = {v0, 0u};
    const int rc = upload(d->task_ctr, init, 2, d->hs);
    if (rc) return rc;
    d->task_base = v0;
    return QPD_OK;
}

#ifdef QPD_STAMPS
// Diagnostic builds: the per-op-class cycle accumulators every decoder's
// kernels add to (qpd_debug_stamps), one device buffer per device (qpd_debug_stamps reads the
// current device's).
unsigned long long *stamp_buffer() {  // one per device (the current one)
    static std::mutex mu;
    static std::map<int, unsigned long long *> bufs;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    unsigned long long *&buf = bufs[dev];
    if (!buf && hipMalloc(&buf, 64 * sizeof(unsigned long long)) == hipSuccess)
        (void)hipMemset(buf, 0, 64 * sizeof(unsigned long long));
    return buf;
}
#endif

int build_fast(qpd_decoder *d, const qpd_config *c, const Schedule &s) {
    qpd::FastPlan &F = d->fplan;
#ifdef QPD_STAMPS
    F.stamps = stamp_buffer();
#endif
    const int N = c->N, n = d->n, v = c->v;
    F.N = N;
    F.n = n;
    F.K = c->K;
    F.L = d->L;
    F.v = v;
    F.gs = d->plan.gs;
    F.fpw = d->plan.fpw;
    F.max_r1 = s.max_r1;
    auto srows = [&](int dd) { return std::max(1, (N >> dd) / 8); };
    auto brows = [&](int dd) { return std::max(1, (N >> dd) / 32); };
    // Row slots per depth: 0 = R, 1 = S, 2 = U.  `use` keeps all of them, or
    // (trimmed layout) only those some op touches: BOT3 subtrees keep depths
    // n-2..n in registers and the fused BOT3s also skip S/R[n-3], which frees
    // LDS for a shallower lds_from.
    bool use[3][qpd::kMaxDepth + 1];
    for (auto &u : use)
        for (bool &b : u) b = true;
    auto rows_of = [&](int slot, int dd) {
        if (slot == 1) return (dd >= 1 && dd <= n - 1) ? srows(dd) : 0;
        if (slot == 2) return dd >= 1 ? brows(dd) : 0;
        return brows(dd);
    };
    auto assign = [&](FastLayout &L, int &rl, int &rg) {
        rl = rg = 0;
        for (int dd = 0; dd <= n; ++dd) {  // grouped by depth (see FastLayout)
            int &r = L.lds(dd) ? rl : rg;
            if (L.lds(dd)) L.lds_base[dd] = r;
            L.R[dd] = r;
            if (use[0][dd]) r += rows_of(0, dd);
            L.S[dd] = r;
            if (use[1][dd]) r += rows_of(1, dd);
            L.U[dd] = r;
            if (use[2][dd]) r += rows_of(2, dd);
        }
        L.lds_base[n + 1] = rl;
        L.lds_end = rl + qpd::kSelInts / 64;
    };
    // one frame set for FastSC-LUT (N=1024: 171 -> 241 M frames/s with one set,
    // profiles/r03z_sets.txt); two for the list kinds, FastSCL-LUT included (round 5:
    // the SCL-LUT kernel's two-set machinery with the special-node ops)
    d->sets = c->kind == QPD_FASTSC_LUT ? 1 : kDefaultSets;
    if (const char *e = getenv("QPD_SETS")) d->sets = std::min(2, std::max(1, atoi(e)));
#ifdef QPD_SETS3
    if (const char *e = getenv("QPD_SETS")) if (atoi(e) == 3 && c->kind == QPD_SCL_LUT && d->L == 8) d->sets = 3;
#endif
    d->l8 = (c->kind == QPD_SCL_LUT || c->kind == QPD_FASTSCL_LUT) && d->L == 8;
    d->w16 = c->kind == QPD_SCL_LUT && d->L > qpd::kMaxL;
    const int NS = d->sets;
    FastLayout Ly;
    Ly.ns = NS;
    const int32_t *nt_fast = (c->kind == QPD_FASTSC_LUT || c->kind == QPD_FASTSCL_LUT) ? c->node_type : nullptr;
    // pre-mode: S[1] is whole words (N >= 16) and the root's left child a plain node
    Ly.pre = n >= 4 && special_of(c->kind, nt_fast, 1) < 0 && !getenv("QPD_NO_PRE");
    Ly.bfuse = !getenv("QPD_NO_BFUSE");
    Ly.botx = c->kind == QPD_FASTSCL_LUT && d->l8 && !getenv("QPD_NO_BOTX");
    // Trimmed layout: probe the op list on an all-global layout and keep the
    // slots it touches.  (FastSCL's R1 argsorts of > 16 elements borrow the LDS
    // tail of the deeper levels; it is padded below where it is too short.)
    if (!getenv("QPD_NO_TRIM")) {
        FastLayout Lp = Ly;
        Lp.D = n + 1;
        int pl = 0, pg = 0;
        assign(Lp, pl, pg);
        std::vector<qpd::MOp> probe;
        std::vector<uint16_t> r1p;
        fast_ops(probe, Lp, c->kind, N, n, v, c->frozen_bits, nt_fast, c->vcl, r1p, 0, 0);
        std::vector<int> owner(std::max(pg, 1), -1);  // row -> slot * 32 + depth
        for (int dd = 0; dd <= n; ++dd)
            for (int sl = 0; sl < 3; ++sl) {
                const int b = sl == 0 ? Lp.R[dd] : sl == 1 ? Lp.S[dd] : Lp.U[dd];
                for (int r = 0; r < rows_of(sl, dd); ++r) owner[b + r] = sl * 32 + dd;
            }
        bool used[3][qpd::kMaxDepth + 1] = {};
        auto mark = [&](int row) {
            if (row >= 0 && row < pg && owner[row] >= 0) used[owner[row] / 32][owner[row] % 32] = true;
        };
        for (const qpd::MOp &m : probe) {
            using namespace qpd;
            if (!(m.flags & (MF_CHAN | MF_PRE))) mark(m.src_row);
            mark(m.dst_row);
            if (m.type == OP_G || m.type == OP_LEAF_R || m.type == OP_COMB ||
                (m.type == OP_BOT3 && (m.flags & (MF_BG | MF_BCOMB))) ||
                (m.type >= OP_R0 && m.type <= OP_SPC && (m.flags & (MF_SGG | MF_SCOMB))))
                mark(m.u_row);
            if (m.type == OP_COMB) mark(m.r_row);
        }
        used[0][0] = true;  // R[0]: the tail re-encodes it
        std::memcpy(use, used, sizeof(use));
    }
    // the list kinds' byte tables of the f / g ops at two frame sets (stage_tab in
    // qpd_fast.hip: 512 B for the op's table, 256 B for a folded child's f), after the
    // sets' selection scratch
    const bool list_kind = c->kind == QPD_SCL_LUT || c->kind == QPD_FASTSCL_LUT;
    d->lds_tab_bytes = list_kind && NS >= 2 ? 768 : 0;
    // LDS per wave = NS * (selection scratch + rows of depths >= D) + the byte
    // tables; the budget is measured: occupancy beats LDS residency of the
    // shallow depths.
    int budget = NS == 1 ? 6 * 1024 : NS == 2 ? 10 * 1024 : 15 * 1024;
    if (const char *e = getenv("QPD_LDS_BUDGET")) budget = atoi(e);
    // FastSCL R1 nodes of 17..32 elements sort in the wave's LDS tail of the
    // deeper levels (MF_R1_LDS): rows of padding so that the tail holds cnt / 2
    // rows -- part of the LDS the budget bounds
    auto r1_pad = [&](const FastLayout &Lt) {
        int pad = 0;
        for (const qpd::Op &o : s.ops)
            if (c->kind == QPD_FASTSCL_LUT && o.type == qpd::OP_R1 && (N >> o.d) > qpd::stl::kThreshold &&
                (N >> o.d) <= 32 && Lt.lds(o.d + 1)) {
                const int have = NS * (Lt.lds_end - Lt.lds_base[o.d + 1]), need = (N >> o.d) / 2;
                if (have < need) pad = std::max(pad, (need - have + NS - 1) / NS);
            }
        return pad;
    };
    int rl = 0, rg = 0;
    for (;; ++Ly.D) {
        assign(Ly, rl, rg);
        const int pad = r1_pad(Ly);
        if (Ly.D > n || NS * (qpd::kSelInts * 4 + (rl + pad) * 256) + d->lds_tab_bytes <= budget) {
            rl += pad;
            Ly.lds_end += pad;
            break;
        }
    }
    F.lds_from = Ly.D;
    F.R0_row = Ly.R[0];
    F.R0_lds = Ly.lds(0);
    F.H_row = F.K_row = F.I_row = rg;
    if (c->kind == QPD_FASTSCL_LUT && s.max_r1 > 0) {
        F.H_row = rg;
        rg += (s.max_r1 + 31) / 32;
        F.K_row = rg;
        rg += 2 * s.max_r1;
        F.I_row = rg;
        if (s.max_r1 > qpd::stl::kThreshold) rg += s.max_r1;
    }
    F.lds_rows = rl;
    F.glb_rows = std::max(rg, 1);
    d->lds_bytes = NS * (qpd::kSelInts * 4 + rl * 256) + d->lds_tab_bytes;
    std::vector<qpd::MOp> mops;
    std::vector<uint16_t> r1tab;
    d->pre = Ly.pre;
    // pre-pass rows: N bytes per frame, <= 2 GB (2^21 frames at N = 1024: each
    // decode launch ends in a drain where its SIMDs idle one by one, so fewer,
    // larger launches are faster -- SCL-LUT 35.9 / 37.5 / 38.3 M frames/s at
    // 2^18 / 2^20 / 2^21 frames per launch)
    // <= 8 GB of rows per chunk (2^23 frames at N = 1024): one decode launch, one
    // drain and one set of prefix-stage launches per 2^23 frames (SCL-LUT bench
    // workload: 2 GB chunks 53.5 M frames/s at 2^22 frames per call, 4 GB 54.3 M;
    // at 2^23 4 GB 54.8 M, 8 GB 55.2 M -- profiles/r06q_ab_chunk.txt)
    d->pre_chunk = std::max<int64_t>(1, ((int64_t)8 << 30) / N);
    if (const char *e = getenv("QPD_PRE_CHUNK")) d->pre_chunk = std::max<int64_t>(1, atoll(e));
    fast_ops(mops, Ly, c->kind, N, n, v, c->frozen_bits, nt_fast, c->vcl, r1tab, 0, 0);
    if (r1tab.empty()) r1tab.push_back(0);
    {
        int rc = upload(d->r1_rank, r1tab.data(), r1tab.size(), d->hs);
        if (rc) return rc;
    }
    F.r1_rank = (const uint16_t *)d->r1_rank.p;
    // Frozen-prefix stages (lut_prefix_kernel, plan_prefix): SCL-LUT in pre-mode.
    // FastSCL's R0 / REP nodes already take most of the prefix (4 ops of the bench
    // code; the one-stage split measured -3 % there, profiles/r03ab_*).
    PrefixPlan pp;
    // The split needs every live path metric finite: stage 2 and the decode
    // kernel seed the dead slots with path 0's rows and +inf, where the
    // reference holds copies of other dead paths (SCLLUTDecoder.cpp:117-144);
    // the two agree while no live metric reaches +inf and ties with a dead one.
    // A metric is a sum of at most N leaf quanta (row n-1), so quanta below
    // DBL_MAX / 2N keep it finite; tables beyond that decode unsplit, exactly
    // as the reference does with its infinities.
    double qmax = 0.0;
    for (size_t i = (size_t)(n - 1) * N * v; i < (size_t)n * N * v; ++i) qmax = std::max(qmax, std::fabs(c->vcl[i]));
    const bool pm_finite = qmax <= __DBL_MAX__ / (2.0 * N);
    if (Ly.pre && d->L > 1 && c->kind == QPD_SCL_LUT && pm_finite && !getenv("QPD_NO_PFX")) {
        FastOwner own;
        for (int dd = 0; dd <= n; ++dd)
            for (int sl = 0; sl < 3; ++sl) {
                const int b = sl == 0 ? Ly.R[dd] : sl == 1 ? Ly.S[dd] : Ly.U[dd];
                own.add(Ly.lds(dd), b, use[sl][dd] ? rows_of(sl, dd) : 0, sl == 0 ? 0 : sl == 1 ? 1 : 2, dd);
            }
        if (plan_prefix(mops, own, d->L, pp)) mops.swap(pp.rest);
    }
    d->pfx_sets = std::min(d->sets, 2);
    // prefix_kernel() instantiates NS = 1 and 2 only: fast_launch's task count
    // (fgroups) must use the NS the launched kernel has
    if (const char *e = getenv("QPD_PFX_SETS")) d->pfx_sets = std::min(std::min(d->sets, 2), std::max(1, atoi(e)));
    // folded descents: the list kernels with two frame sets (ff_op)
    if (list_kind && !getenv("QPD_NO_FF")) {
        if (d->sets == 2) fuse_descent(mops);
        if (d->pfx_sets == 2) {
            fuse_descent(pp.st1);
            fuse_descent(pp.st1b);
            fuse_descent(pp.st2);
        }
    }
    if (list_kind && !getenv("QPD_NO_BC2")) {  // folded depth n-5 combines (any NS)
        fold_combine(mops);
        fold_combine(pp.st1);
        fold_combine(pp.st1b);
        fold_combine(pp.st2);
    }
    place_syncs(pp.st1, true);
    place_syncs(pp.st1b, true);
    place_syncs(pp.st2, true);
    place_syncs(mops, c->kind == QPD_SCL_LUT || c->kind == QPD_FASTSCL_LUT);
    // one pointer word: the list kinds at one or two frame sets (the instantiations
    // fast_kernel() has); FastSCL-LUT only at two sets with L = 8 and no r1_large
    // Special nodes the lean code of the R1L = false kernels cannot take: R1 nodes of > 16
    // elements without their LDS tail (r1_large), or (L = 8) R1 nodes without ranks in the
    // op record and R0 / REP nodes without one quanta row
    for (const qpd::MOp &m : mops)
        if (c->kind == QPD_FASTSCL_LUT &&
            ((m.type == qpd::OP_R1 &&
              ((m.cnt > qpd::stl::kThreshold && !(m.flags & qpd::MF_R1_LDS)) || (d->l8 && !(m.flags & qpd::MF_R1_RK)))) ||
             (d->l8 && (m.type == qpd::OP_R0 || m.type == qpd::OP_REP) && !(m.flags & qpd::MF_VUNI))))
            d->r1l = true;
    // (SCL-LUT only with the root pre-pass: those kernels have no channel reads, lut_fast_kernel kChan)
    const bool pw1_ok = c->kind == QPD_SCL_LUT ? NS <= 2 && Ly.pre : (c->kind == QPD_FASTSCL_LUT && NS == 2 && d->l8 && !d->r1l);
    if (pw1_ok && !getenv("QPD_NO_PW1")) d->pw1 = compact_pointer_fields({&mops, &pp.st1, &pp.st1b, &pp.st2});
    d->pfx_nops = (int)pp.st1.size();
    d->pfx1b_nops = (int)pp.st1b.size();
    d->pfx2_nops = (int)pp.st2.size();
    d->pfx1_rec = pp.rec1;
    d->pfx1_pm = pp.pm1;
    d->pfx1b_rec = pp.rec1b;
    d->pfx1b_pm = pp.pm1b;
    d->pfx2_rec = pp.rec2;
    d->pfx2_pm = pp.pm2;
    d->pfx_ops_host = pp.st1;  // one device array: stage 1, stage 1b, then stage 2
    d->pfx_ops_host.insert(d->pfx_ops_host.end(), pp.st1b.begin(), pp.st1b.end());
    d->pfx_ops_host.insert(d->pfx_ops_host.end(), pp.st2.begin(), pp.st2.end());
    if (!d->pfx_ops_host.empty()) {
        int rc = upload(d->pfx_mops, d->pfx_ops_host.data(), d->pfx_ops_host.size(), d->hs);
        if (rc) return rc;
        d->main_ops_host = mops;  // the import ops get the record buffers' addresses (patch_imports)
    }
    for (const qpd::MOp &m : mops)  // the kernel's f / g ops have no (S[d] in LDS, S[d+1] in the slab) variant
        if ((m.type == qpd::OP_F || m.type == qpd::OP_G) && (m.flags & qpd::MF_SRC_LDS) && !(m.flags & qpd::MF_DST_LDS))
            return fail(QPD_E_INVALID, "fast plan: an f/g op reads LDS rows and writes slab rows");
    F.nops = (int)mops.size();
    d->num_mops = F.nops + d->pfx_nops + d->pfx1b_nops + d->pfx2_nops;
    {
        int rc = upload(d->mops, mops.data(), mops.size(), d->hs);
        if (rc) return rc;
    }
    // nibble-packed tables: entry (u, a, b) of node p at bit 4*(idx&7) of dword idx>>3, idx =
    // u * 256 + a * 16 + b; the leaf pairs' nodes (depth n-1: only the leaf lookups read them)
    // transposed, idx = u * 256 + b * 16 + a (qpd_fast.hip leaf_idx, QPD_LEAF_T)
    std::vector<uint32_t> ft((size_t)(N - 1) * 32, 0), gt((size_t)(N - 1) * 64, 0);
    const size_t vv = (size_t)v * v;
    for (int p = 0; p < N - 1; ++p) {
        const uint8_t *tf = c->lut_f + (size_t)c->f_base[p] * vv;
        const uint8_t *tg = c->lut_g + (size_t)c->g_base[p] * 2 * vv;
        const bool leafpair = QPD_LEAF_T && p >= (N >> 1) - 1;
        for (int a = 0; a < v; ++a)
            for (int b = 0; b < v; ++b) {
                const int idx = leafpair ? b * 16 + a : a * 16 + b;
                ft[(size_t)p * 32 + (idx >> 3)] |= (uint32_t)tf[a * v + b] << (4 * (idx & 7));
                for (int u = 0; u < 2; ++u) {
                    const int gi = u * 256 + idx;
                    gt[(size_t)p * 64 + (gi >> 3)] |= (uint32_t)tg[u * vv + a * v + b] << (4 * (gi & 7));
                }
            }
    }
    int rc = upload(d->f_tab, ft.data(), ft.size(), d->hs);
    if (rc) return rc;
    rc = upload(d->g_tab, gt.data(), gt.size(), d->hs);
    if (rc) return rc;
    const int64_t per_wave = (int64_t)NS * F.glb_rows * 64 * 4;
    {
        // the byte tables' lookups address LDS offset 0 as the start of the dynamic
        // allocation (qpd_fast.hip lut_lds): the kernel must declare no static LDS
        hipFuncAttributes fa;
        const void *kfn = fast_kernel(d->kind, d->sets, d->l8, d->r1l, d->pw1, d->w16);
        if (!kfn) return fail(QPD_E_UNSUPPORTED, "fast plan: no decode kernel instantiation for this plan");
        QPD_HIP(hipFuncGetAttributes(&fa, kfn));
        if (fa.sharedSizeBytes != 0) return fail(QPD_E_DEVICE, "fast decode kernel declares static LDS");
    }
    // Persistent grid: as many waves as can be resident at once.
    int mw = c->max_waves;
    if (mw <= 0) {
        int dev = 0, ncu = 256, per_cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        const hipError_t oe =
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fast_kernel(d->kind, d->sets, d->l8, d->r1l, d->pw1, d->w16), 64,
                                                         d->lds_bytes);
        if (oe != hipSuccess || per_cu <= 0) per_cu = 16;
        mw = std::max(1, ncu) * per_cu;
    }
    mw = (int)std::max<int64_t>(1, std::min<int64_t>(mw, ((int64_t)2 << 30) / per_wave));
    d->max_waves = mw;
    d->scratch_bytes_per_wave = per_wave;
    QPD_HIP(hipMalloc(&d->fscratch.p, (size_t)per_wave * mw));
    F.f_tab = (const uint32_t *)d->f_tab.p;
    F.g_tab = (const uint32_t *)d->g_tab.p;
    F.vcl = (const double *)d->vcl.p;
    F.ops = (const qpd::MOp *)d->mops.p;
    F.info_pos = (const int32_t *)d->info_pos.p;
    F.scratch = (uint32_t *)d->fscratch.p;
    F.err = (int32_t *)d->err.p;
    rc = init_task_queue(d);
    if (rc) return rc;
    F.task_ctr = (uint32_t *)d->task_ctr.p;
    return QPD_OK;
}


template <class In>
int launch_generic(qpd_decoder *d, const In *in, int64_t B, uint8_t *out, int grid, hipStream_t st) {
    const void *kfn = generic_kernel(d->kind, d->dom, d->L > qpd::kMaxL);
    if (!kfn) return fail(QPD_E_INVALID, "bad kind");
    qpd::DevPlan P = d->plan;
    P.task_base = d->task_base;
    const In *in_arg = in;
    void *args[] = {&P, &in_arg, &B, &out};
    const int rc = timed_launch(d, QPD_KC_DECODE, st, [&]() -> int {
        QPD_HIP(hipLaunchKernel(kfn, dim3(grid), dim3(64), args, 0, st));
        QPD_HIP(hipGetLastError());
        return QPD_OK;
    });
    if (!rc) d->task_base += (uint32_t)((B + d->plan.fpw - 1) / d->plan.fpw);  // takes of this launch (wave_take)
    return rc;
}

// The host engine's copy of the plan (qpd_host.hpp) and the batch size up to
// which QPD_HOST_AUTO prefers it.  The crossover is a cost model fitted to the
// per-call latencies measured on MI355X (tools/latency.py,
// profiles/r02_latency.jsonl, re-checked on profiles/r03af_latency.jsonl): a GPU call costs a fixed launch / copy /
// synchronization overhead plus one wave running the whole serial schedule,
// whatever the batch up to thousands of frames; the host engine costs its
// per-frame work times the batch.
int build_host(qpd_decoder *d, const qpd_config *cfg, size_t nops) {
    std::unique_ptr<qpd_host::Plan> h = qpd_host::make_plan(cfg);
    if (!h) return QPD_OK;  // re-quantized float kinds: GPU only
    if (h->dom == qpd::DOM_LUT)
        d->heng_lut = std::make_unique<qpd_host::Engine<uint8_t>>(*h);
    else
        d->heng_f64 = std::make_unique<qpd_host::Engine<double>>(*h);
    // Per frame on the host engine ~ its lookups (N log2 N per path) plus,
    // for lists, the forks (re-fitted to the round-3 engine, profiles/
    // r03af_latency.jsonl: SC-LUT N=128 2.8 us, N=1024 15.5 us, SCL-LUT
    // N=1024 L=8 0.154 ms); a GPU call ~ 55 us of launches, copies and
    // synchronization plus one wave running the serial schedule (SC-LUT N=128
    // 0.11 ms, N=1024 0.91 ms, SCL-LUT N=1024 L=8 1.07 ms, same file) -- flat
    // in the batch up to thousands of frames.
    const double nn = (double)h->N * h->n;
    const double host_us = 0.00136 * nn * h->L + (h->L > 1 ? 0.005 * h->L * h->N : 0.0) + 1.6;
    const double gpu_us = 55.0 + 0.083 * nn + (h->L > 1 ? 0.02 * nn : 0.0);
    (void)nops;
    d->host_max_frames = std::max<int64_t>(1, (int64_t)(gpu_us / host_us));
    d->hplan = std::move(h);
    if (const char *e = getenv("QPD_HOST_ENGINE")) {
        if (!strcmp(e, "gpu")) d->host_mode = QPD_HOST_GPU;
        if (!strcmp(e, "cpu")) d->host_mode = QPD_HOST_CPU;
    }
    return QPD_OK;
}

}  // namespace

extern "C" {

int qpd_abi_version(void) { return QPD_ABI_VERSION; }

// Source hash of the tree this library was built from (build.py:
// source_hash); the tagged string is also found in the file's bytes.
#ifndef QPD_BUILD_ID
#define QPD_BUILD_ID "unstamped-build"
#endif
__attribute__((used)) static const char kBuildIdTag[] = "qpd-build-id:" QPD_BUILD_ID;

const char *qpd_build_id(void) { return kBuildIdTag + sizeof("qpd-build-id:") - 1; }

const char *qpd_last_error(void) { return g_err.c_str(); }

int qpd_create(const qpd_config *cfg, qpd_decoder **out) {
    if (!out) return fail(QPD_E_INVALID, "null output handle");
    *out = nullptr;
    int n = 0, fam = 0, dom = 0;
    int rc = validate(cfg, &n, &fam, &dom);
    if (rc) return rc;
    // Every public kind is a kernel family in a symbol domain (family_of); the
    // CRC-aided kinds add an output epilogue.
    qpd_config cc = *cfg;
    const bool ca = is_ca(cfg->kind);
    cc.kind = fam;
    const qpd_config *c = &cc;
    if (c->device >= 0) QPD_HIP(hipSetDevice(c->device));

    qpd_decoder *d = new qpd_decoder();
    {
        const hipError_t e = hipStreamCreateWithFlags(&d->hs, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete d;
            return fail(QPD_E_DEVICE, std::string("decoder stream: ") + hipGetErrorString(e));
        }
    }
    d->pub_kind = cfg->kind;
    d->dom = dom;
    d->out_bits = ca ? cfg->A : cfg->K;
    if (ca) {
        d->ca_A = cfg->A;
        d->crc_n = cfg->crc_n;
        for (int i = 0; i < cfg->crc_loc_count; ++i) {
            const int j = cfg->crc_loc[i];  // coefficient j -> register bit crc_n - j (j = 0: leading, drops out)
            if (j >= 1) d->crc_q |= 1u << (cfg->crc_n - j);
        }
    }
    d->kind = c->kind;
    d->N = c->N;
    d->n = n;
    d->K = c->K;
    const bool list = c->kind == QPD_SCL_LUT || c->kind == QPD_FASTSCL_LUT;
    d->L = list ? c->L : 1;
    d->v = (dom == qpd::DOM_LUT || dom == qpd::DOM_UNIFORM) ? c->v : 0;
    d->device = c->device;

    Schedule s;
    visit(s, c->kind, c->N, n, c->frozen_bits, (c->kind == QPD_FASTSC_LUT || c->kind == QPD_FASTSCL_LUT) ? c->node_type : nullptr, 0, 0);
    d->ops_host = s.ops;
    {
        // L > 8 (2L > 16: libstdc++ introsort, replayed where ties make it matter): SCL-LUT up to
        // L = 16 on the fast engine (lane groups of 16, select_survivors16), the others on the generic one
        const bool fast_ok = dom == qpd::DOM_LUT && c->f_step == 0 && c->g_step == 0 && c->v <= 16 &&
                             (d->L <= qpd::kMaxL || (c->kind == QPD_SCL_LUT && d->L <= 2 * qpd::kMaxL));
        int want = c->engine;
        if (const char *e = getenv("QPD_ENGINE")) want = atoi(e);
        if (want == QPD_ENGINE_FAST && !fast_ok) {
            delete d;
            return fail(QPD_E_UNSUPPORTED,
                        "fast engine needs LUT symbols with one table per node (f_step = g_step = 0), v <= 16 and L <= 8 "
                        "(SCL-LUT: L <= 16)");
        }
        d->engine = (want == QPD_ENGINE_GENERIC || !fast_ok) ? QPD_ENGINE_GENERIC : QPD_ENGINE_FAST;
    }

    DevPlan &P = d->plan;
    P.N = c->N;
    P.n = n;
    P.K = c->K;
    P.L = d->L;
    P.v = d->v;
    int gs = 1;
    while (gs < d->L) gs *= 2;
    P.gs = gs;
    P.fpw = 64 / gs;
    P.nops = (int)s.ops.size();
    P.max_r1 = s.max_r1;
    // scratch layout, in 64-lane dword rows
    int r = 0;
    const int N = c->N;
    for (int dd = 0; dd <= qpd::kMaxDepth; ++dd) P.So[dd] = P.Uo[dd] = 0;
    for (int dd = 1; dd <= n - 1; ++dd) {
        P.So[dd] = r;
        r += dom != qpd::DOM_LUT ? 2 * (N >> dd) : std::max(1, ((N >> dd) + 3) / 4);
    }
    for (int dd = 1; dd <= n; ++dd) {
        P.Uo[dd] = r;
        r += std::max(1, ((N >> dd) + 31) / 32);
    }
    P.Ro = r;
    r += std::max(1, (N + 31) / 32);
    P.Ho = P.Ko = P.Io = r;
    if (c->kind == QPD_FASTSCL_LUT && s.max_r1 > 0) {
        P.Ho = r;
        r += (s.max_r1 + 31) / 32;
        P.Ko = r;
        r += 2 * s.max_r1;
        P.Io = r;
        if (s.max_r1 > qpd::stl::kThreshold) r += s.max_r1;
    }
    P.rows_per_wave = r;
    P.f_step = c->f_step;
    P.g_step = c->g_step;
    d->scratch_bytes_per_wave = (int64_t)r * 64 * 4;
    int mw = c->max_waves > 0 ? c->max_waves : 256 * 8;
    const int64_t cap = (int64_t)2 << 30;  // <= 2 GiB of scratch
    mw = (int)std::max<int64_t>(1, std::min<int64_t>(mw, cap / d->scratch_bytes_per_wave));
    d->max_waves = mw;

    std::vector<int32_t> info;
    for (int i = 0; i < N; ++i)
        if (c->frozen_bits[i] == 0) info.push_back(i);

#define QPD_TRY(x)            \
    do {                      \
        int rc_ = (x);        \
        if (rc_) {            \
            delete d;         \
            return rc_;       \
        }                     \
    } while (0)
    QPD_TRY(upload(d->ops, s.ops.data(), s.ops.size(), d->hs));
    QPD_TRY(upload(d->info_pos, info.data(), info.size(), d->hs));
    {
        std::vector<uint32_t> mask((N + 31) / 32, 0u);
        for (int i : info) mask[i >> 5] |= 1u << (i & 31);
        QPD_TRY(upload(d->info_mask, mask.data(), mask.size(), d->hs));
    }
    if (dom == qpd::DOM_UNIFORM) {
        QPD_TRY(upload(d->r_f, c->r_f, (size_t)N - 1, d->hs));
        QPD_TRY(upload(d->r_g, c->r_g, (size_t)N - 1, d->hs));
    } else if (dom == qpd::DOM_LLOYD) {
        QPD_TRY(upload(d->q_bnd, c->q_bnd, (size_t)c->q_bnd_count, d->hs));
        QPD_TRY(upload(d->q_rec, c->q_rec, (size_t)c->q_rec_count, d->hs));
        QPD_TRY(upload(d->bnd_off, c->bnd_off, 2 * ((size_t)N - 1), d->hs));
        QPD_TRY(upload(d->bnd_len, c->bnd_len, 2 * ((size_t)N - 1), d->hs));
        QPD_TRY(upload(d->rec_off, c->rec_off, 2 * ((size_t)N - 1), d->hs));
        QPD_TRY(upload(d->rec_len, c->rec_len, 2 * ((size_t)N - 1), d->hs));
    }
    if (dom == qpd::DOM_LUT) {
        const size_t vv = (size_t)c->v * c->v;
        QPD_TRY(upload(d->lut_f, c->lut_f, (size_t)c->lut_f_count * vv, d->hs));
        QPD_TRY(upload(d->lut_g, c->lut_g, (size_t)c->lut_g_count * 2 * vv, d->hs));
        QPD_TRY(upload(d->f_base, c->f_base, (size_t)N - 1, d->hs));
        QPD_TRY(upload(d->g_base, c->g_base, (size_t)N - 1, d->hs));
        QPD_TRY(upload(d->vcl, c->vcl, (size_t)c->vcl_rows * N * c->v, d->hs));
    }
    {
        hipError_t e = hipSuccess;
        if (d->engine == QPD_ENGINE_GENERIC) e = hipMalloc(&d->scratch.p, (size_t)d->scratch_bytes_per_wave * mw);
        if (e != hipSuccess) {
            delete d;
            return fail(QPD_E_DEVICE, std::string("scratch hipMalloc: ") + hipGetErrorString(e));
        }
        e = hipMalloc(&d->err.p, sizeof(int32_t));
        if (e == hipSuccess) e = hipMemsetAsync(d->err.p, 0, sizeof(int32_t), d->hs);
        if (e == hipSuccess) e = hipStreamSynchronize(d->hs);
        if (e != hipSuccess) {
            delete d;
            return fail(QPD_E_DEVICE, std::string("err hipMalloc: ") + hipGetErrorString(e));
        }
    }
    if (d->engine == QPD_ENGINE_FAST) QPD_TRY(build_fast(d, c, s));
#undef QPD_TRY
    P.lut_f = (const uint8_t *)d->lut_f.p;
    P.f_base = (const int32_t *)d->f_base.p;
    P.lut_g = (const uint8_t *)d->lut_g.p;
    P.g_base = (const int32_t *)d->g_base.p;
    P.vcl = (const double *)d->vcl.p;
    P.ops = (const Op *)d->ops.p;
    P.info_pos = (const int32_t *)d->info_pos.p;
    P.scratch = (uint32_t *)d->scratch.p;
    P.err = (int32_t *)d->err.p;
    if (!d->task_ctr.p) {
        const int rc = init_task_queue(d);
        if (rc) {
            delete d;
            return rc;
        }
    }
    P.task_ctr = (uint32_t *)d->task_ctr.p;
    P.r_f = (const double *)d->r_f.p;
    P.r_g = (const double *)d->r_g.p;
    P.q_bnd = (const double *)d->q_bnd.p;
    P.q_rec = (const double *)d->q_rec.p;
    P.bnd_off = (const int32_t *)d->bnd_off.p;
    P.bnd_len = (const int32_t *)d->bnd_len.p;
    P.rec_off = (const int32_t *)d->rec_off.p;
    P.rec_len = (const int32_t *)d->rec_len.p;
    // DOUBLE_INF of each class: 1.0/0.0 for the LUT decoders and FastSCL
    // (SCLLUTDecoder.h:16, FastSCLDecoder.h:7), 1e300 for the float SCL family
    // (SCLDecoder.h:8, CASCLDecoder.h:9, SCL{Uniform,Lloyd}QuantizedDecoder.h)
    P.pm_init = (dom == qpd::DOM_LUT || c->kind == QPD_FASTSCL_LUT) ? __builtin_huge_val() : 1e300;
    P.out_k = d->out_bits;
    P.ca_A = d->ca_A;
    P.crc_n = d->crc_n;
    // bits compared after the A info bits: K - A (LUT kinds), crc_n (CASCLDecoder)
    P.ca_chk = cfg->kind == QPD_CASCL_FLOAT ? d->crc_n : d->K - d->ca_A;
    P.crc_q = d->crc_q;
    P.info_mask = (const uint32_t *)d->info_mask.p;
    d->fplan.out_k = d->out_bits;
    d->fplan.ca_A = d->ca_A;
    d->fplan.crc_n = d->crc_n;
    d->fplan.crc_q = d->crc_q;
    d->fplan.info_mask = (const uint32_t *)d->info_mask.p;
    {
        const int rc = build_host(d, cfg, s.ops.size());
        if (rc) {
            delete d;
            return rc;
        }
    }
    *out = d;
    return QPD_OK;
}

void qpd_destroy(qpd_decoder *d) {
    if (!d) return;
    if (d->device >= 0) (void)hipSetDevice(d->device);
    delete d;  // ~qpd_decoder waits for the decoder's last work before any buffer is freed
}

int qpd_get_info(const qpd_decoder *d, qpd_info *info) {
    if (!d || !info) return fail(QPD_E_INVALID, "null argument");
    info->kind = d->pub_kind;
    info->out_bits = d->out_bits;
    info->host_max_frames = !d->hplan ? 0 : d->host_mode == QPD_HOST_GPU ? 0
                            : d->host_mode == QPD_HOST_CPU ? INT64_MAX : d->host_max_frames;
    info->N = d->N;
    info->K = d->K;
    info->L = d->L;
    info->v = d->v;
    info->num_ops = d->engine == QPD_ENGINE_FAST ? d->num_mops : (int32_t)d->ops_host.size();
    info->frames_per_wave = d->engine == QPD_ENGINE_FAST ? d->plan.fpw * d->sets : d->plan.fpw;
    info->lanes_per_frame = d->plan.gs;
    info->max_waves = d->max_waves;
    info->scratch_bytes_per_wave = d->scratch_bytes_per_wave;
    info->engine = d->engine;
    info->lds_bytes_per_wave = d->lds_bytes;
    info->lds_from_depth = d->engine == QPD_ENGINE_FAST ? d->fplan.lds_from : -1;
    info->prefix_ops = d->engine == QPD_ENGINE_FAST ? d->pfx_nops + d->pfx1b_nops + d->pfx2_nops : 0;
    info->last_engine = d->last_engine;
    // f / g ops of a node at depth d look up N >> (d + 1) symbols each; a leaf
    // pair's two decisions one each (SCLLUTDecoder.cpp:83-89, :157-164)
    int64_t lk = 0;
    for (const Op &o : d->ops_host)
        if (o.type == qpd::OP_F || o.type == qpd::OP_G) lk += d->N >> (o.d + 1);
        else if (o.type == qpd::OP_LEAF_L || o.type == qpd::OP_LEAF_R) lk += 1;
    info->lookups_per_path = lk;
    info->fast_variant = d->engine == QPD_ENGINE_FAST ? (d->pw1 ? 1 : 0) | (d->r1l ? 2 : 0) : 0;
    info->reserved0 = 0;
    return QPD_OK;
}

}  // extern "C"

namespace {

// Launches of one device-buffer decode on stream st (caller: lock held,
// stream ordered).
// One fast-engine decode launch over Bc frames whose rows start at `in`
// (channel symbols, in_shift = n; or pre-pass rows, in_shift = n - 2).
int fast_launch(qpd_decoder *d, qpd::FastPlan fp, const int32_t *in, int64_t Bc, uint8_t *out, hipStream_t st,
                bool prefix = false) {
    const int sets = prefix ? d->pfx_sets : d->sets;
    const int64_t tw = (int64_t)fp.fpw * sets;  // frames per wave task
    const void *kfn = prefix ? prefix_kernel(d->kind, sets, d->pw1) : fast_kernel(d->kind, d->sets, d->l8, d->r1l, d->pw1, d->w16);
    if (!kfn) return fail(QPD_E_INVALID, "bad kind");
    const int64_t fgroups = (Bc + tw - 1) / tw;
    int fgrid = (int)std::min<int64_t>(fgroups, d->max_waves);
    if (!QPD_DYN) {
        // even out the rounds of the grid-stride loop (no partial last round)
        const int64_t rounds = (fgroups + fgrid - 1) / fgrid;
        fgrid = (int)((fgroups + rounds - 1) / rounds);
    }
    const qpd::MOp *ops_arg = fp.ops;
    fp.task_base = d->task_base;
    void *args[] = {&fp, &in, &Bc, &out, &ops_arg};
    // the prefix stages run pfx_sets frame sets per wave in the same per-set layout
    const size_t lds = (size_t)((d->lds_bytes - d->lds_tab_bytes) / d->sets * sets + d->lds_tab_bytes);
    const int rc = timed_launch(d, prefix ? QPD_KC_PFX : QPD_KC_DECODE, st, [&]() -> int {
        QPD_HIP(hipLaunchKernel(kfn, dim3(fgrid), dim3(64), args, lds, st));
        QPD_HIP(hipGetLastError());
        return QPD_OK;
    });
    if (!rc) d->task_base += (uint32_t)fgroups;  // takes of this launch (wave_take)
    return rc;
}

// The decode of Bc frames from their root pre-pass rows (pre-mode decoders).
int decode_pre_rows(qpd_decoder *d, const uint32_t *rows, int64_t Bc, uint8_t *out, hipStream_t st) {
    qpd::FastPlan fp = d->fplan;
    fp.in_vec = 1;
    fp.in_shift = fp.n - 2;
    if (d->pfx_nops > 0) {  // the frozen-prefix stages, then the decode
        int rc = ensure_records(d->pfx1_buf, d->pfx1_cap, Bc, d->pfx1_rec, 1);
        if (!rc && d->pfx1b_nops > 0) rc = ensure_records(d->pfx1b_buf, d->pfx1b_cap, Bc, d->pfx1b_rec, 2);
        if (!rc && d->pfx2_nops > 0) rc = ensure_records(d->pfx2_buf, d->pfx2_cap, Bc, d->pfx2_rec, 4);
        if (!rc) rc = patch_imports(d, st);
        if (rc) return rc;
        qpd::FastPlan pp = fp;  // stage 1: one path per frame
        pp.ops = (const qpd::MOp *)d->pfx_mops.p;
        pp.nops = d->pfx_nops;
        pp.gs = 1;
        pp.fpw = 64;
        pp.L = 1;
        pp.pfx = (uint32_t *)d->pfx1_buf.p;
        pp.pfx_rec = d->pfx1_rec;
        pp.pfx_geo = 6;
        pp.pm_off = d->pfx1_pm;
        rc = fast_launch(d, pp, (const int32_t *)rows, Bc, nullptr, st, true);
        if (rc) return rc;
        if (d->pfx1b_nops > 0) {  // stage 1b: <= 2 live paths, L = 2
            pp.ops = (const qpd::MOp *)d->pfx_mops.p + d->pfx_nops;
            pp.nops = d->pfx1b_nops;
            pp.gs = 2;
            pp.fpw = 32;
            pp.L = 2;
            pp.pfx = (uint32_t *)d->pfx1b_buf.p;
            pp.pfx_rec = d->pfx1b_rec;
            pp.pfx_geo = 5 | (1 << 8);
            pp.pm_off = d->pfx1b_pm;
            rc = fast_launch(d, pp, (const int32_t *)rows, Bc, nullptr, st, true);
            if (rc) return rc;
        }
        if (d->pfx2_nops > 0) {  // stage 2: <= 4 live paths, L = 4
            pp.ops = (const qpd::MOp *)d->pfx_mops.p + d->pfx_nops + d->pfx1b_nops;
            pp.nops = d->pfx2_nops;
            pp.gs = 4;
            pp.fpw = 16;
            pp.L = 4;
            pp.pfx = (uint32_t *)d->pfx2_buf.p;
            pp.pfx_rec = d->pfx2_rec;
            pp.pfx_geo = 4 | (2 << 8);
            pp.pm_off = d->pfx2_pm;
            rc = fast_launch(d, pp, (const int32_t *)rows, Bc, nullptr, st, true);
            if (rc) return rc;
        }
    }
    return fast_launch(d, fp, (const int32_t *)rows, Bc, out, st);
}

// pre-pass rows for `chunk` frames (N bytes each), grown on demand; on an
// allocation failure the chunk halves (fewer frames per decode launch, same
// results).  Returns the frames the buffer holds.
int64_t ensure_pre_rows(qpd_decoder *d, int64_t chunk, int *rc) {
    *rc = QPD_OK;
    // after a fallback the smaller buffer is the chunk: no device-wide hipFree
    // and failing hipMallocs on every later call
    if (d->pre_fell_back) chunk = std::min<int64_t>(chunk, d->pre_cap);
    if (d->pre_cap >= chunk) return std::min<int64_t>(chunk, d->pre_cap);
    if (d->pre_buf.p) (void)hipFree(d->pre_buf.p);
    d->pre_buf.p = nullptr;
    d->pre_cap = 0;
    const int64_t want = chunk;
    hipError_t e = hipErrorOutOfMemory;
    while (chunk >= 1 && (e = hipMalloc(&d->pre_buf.p, (size_t)chunk * (size_t)d->N)) != hipSuccess) {
        (void)hipGetLastError();
        d->pre_buf.p = nullptr;
        chunk /= 2;
    }
    if (e != hipSuccess) {
        *rc = fail(QPD_E_DEVICE, std::string("pre-pass rows hipMalloc: ") + hipGetErrorString(e));
        return 0;
    }
    d->pre_fell_back = d->pre_fell_back || e != hipSuccess || chunk < want;
    d->pre_cap = chunk;
    return chunk;
}

// Launches of one device-buffer decode on stream st (caller: lock held,
// stream ordered).
int decode_impl(qpd_decoder *d, const int32_t *d_symbols, int64_t B, uint8_t *d_out, hipStream_t st) {
    int rc = QPD_OK;
    d->last_engine = QPD_RAN_GPU;
    if (d->engine != QPD_ENGINE_FAST) {
        const int64_t groups = (B + d->plan.fpw - 1) / d->plan.fpw;
        return launch_generic(d, d_symbols, B, d_out, (int)std::min<int64_t>(groups, d->max_waves), st);
    }
    qpd::FastPlan fp = d->fplan;
    fp.in_vec = ((uintptr_t)d_symbols & 15u) == 0 && (fp.N & 3) == 0;
    if (!d->pre) {
        fp.in_shift = fp.n;
        return fast_launch(d, fp, d_symbols, B, d_out, st);
    }
    // pre-mode: root pre-pass, then the decode on its rows, chunk by chunk
    const int64_t chunk = ensure_pre_rows(d, std::min<int64_t>(B, d->pre_chunk), &rc);
    if (rc) return rc;
    uint32_t *pre = (uint32_t *)d->pre_buf.p;
    for (int64_t f0 = 0; f0 < B; f0 += chunk) {
        int64_t Bc = std::min<int64_t>(chunk, B - f0);
        const int32_t *sym = d_symbols + f0 * fp.N;
        fp.in_shift = fp.n;
        const int pgrid = (int)std::min<int64_t>(((Bc << (fp.n - 4)) + 255) / 256, 8192);
        void *pargs[] = {&fp, &sym, &Bc, &pre};
        rc = timed_launch(d, QPD_KC_PRE, st, [&]() -> int {
            QPD_HIP(hipLaunchKernel(reinterpret_cast<const void *>(&qpd::root_pre_kernel), dim3(pgrid), dim3(256),
                                    pargs, 0, st));
            QPD_HIP(hipGetLastError());
            return QPD_OK;
        });
        if (rc) return rc;
        rc = decode_pre_rows(d, pre, Bc, d_out + f0 * fp.out_k, st);
        if (rc) return rc;
    }
    return QPD_OK;
}

int decode_f64_impl(qpd_decoder *d, const double *d_llr, int64_t B, uint8_t *d_out, hipStream_t st) {
    d->last_engine = QPD_RAN_GPU;
    const int64_t groups = (B + d->plan.fpw - 1) / d->plan.fpw;
    const int grid = (int)std::min<int64_t>(groups, d->max_waves);
    return launch_generic(d, d_llr, B, d_out, grid, st);
}

int check_channel(const qpd_mc_channel *ch) {
    if (ch->n_edges < 2 || ch->n_edges > qpd::kMcMaxEdges) return fail(QPD_E_INVALID, "n_edges must be in [2, 257]");
    if (!ch->edges || !ch->lut) return fail(QPD_E_INVALID, "null channel quantizer");
    if (!(ch->sigma > 0) || ch->q < 2) return fail(QPD_E_INVALID, "sigma must be > 0 and q >= 2");
    for (int i = 0; i + 1 < ch->n_edges; ++i) {
        if (!(ch->edges[i] <= ch->edges[i + 1])) return fail(QPD_E_INVALID, "edges must be ascending");
        if (ch->lut[i] < 0 || ch->lut[i] >= ch->q) return fail(QPD_E_INVALID, "lut entry outside [0, q)");
    }
    return QPD_OK;
}

// The Monte-Carlo generator on stream st: int32 symbols to `rows`, or (pre)
// the decoder's root pre-pass rows.  Caller: lock held, stream ordered.
int mc_launch(qpd_decoder *d, const qpd_mc_channel *ch, uint64_t seed, int64_t frame0, int64_t B, uint8_t *d_msg,
              int32_t *rows, bool pre, hipStream_t st) {
    if (!d->mc_pref.p) {  // per-decoder constants of the generator, built at the first call
        const int nw = (d->N + 31) / 32;
        std::vector<int32_t> pref(nw, 0);
        std::vector<uint32_t> mask(nw, 0u);
        QPD_HIP(hipMemcpyAsync(mask.data(), d->info_mask.p, nw * sizeof(uint32_t), hipMemcpyDeviceToHost, d->hs));
        QPD_HIP(hipStreamSynchronize(d->hs));
        for (int w = 1; w < nw; ++w) pref[w] = pref[w - 1] + __builtin_popcount(mask[w - 1]);
        // CRC register after message bit j and A-1-j zero bits (the register is
        // linear in the message bits, utils.cpp:77-92): tab[A-1] = taps,
        // tab[j] = one zero step of tab[j+1]
        const int A = d->crc_n > 0 ? d->ca_A : 0;
        std::vector<uint32_t> tab(std::max(A, 1), 0u);
        if (A > 0) {
            const uint32_t top = 1u << (d->crc_n - 1), msk = (top << 1) - 1u;
            tab[A - 1] = d->crc_q & msk;
            for (int j = A - 2; j >= 0; --j) {
                const uint32_t r = tab[j + 1];
                tab[j] = ((r << 1) & msk) ^ ((r & top) ? d->crc_q : 0u);
            }
        }
        int rc2 = upload(d->mc_pref, pref.data(), pref.size(), d->hs);
        if (rc2) return rc2;
        rc2 = upload(d->mc_crc, tab.data(), tab.size(), d->hs);
        if (rc2) return rc2;
    }
    qpd::McChannel C;
    std::memset(&C, 0, sizeof(C));
    C.N = d->N;
    C.K = d->K;
    C.A = d->crc_n > 0 ? d->ca_A : d->K;
    C.crc_n = d->crc_n;
    C.q = ch->q;
    C.n_edges = ch->n_edges;
    C.seed_lo = (uint32_t)seed;
    C.seed_hi = (uint32_t)(seed >> 32);
    C.sigma = ch->sigma;
    C.inv_s2 = 1.0 / (ch->sigma * ch->sigma);  // the driver's sigma ** 2, inverted once
    C.info_mask = (const uint32_t *)d->info_mask.p;
    C.info_pref = (const int32_t *)d->mc_pref.p;
    C.crc_tab = (const uint32_t *)d->mc_crc.p;
    C.f_tab = d->fplan.f_tab;
    C.g_tab = d->fplan.g_tab;
    for (int i = 0; i < ch->n_edges; ++i) C.edges[i] = ch->edges[i];
    for (int i = 0; i + 1 < ch->n_edges; ++i) C.lut[i] = ch->lut[i];
    int dev = 0, ncu = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t lds = qpd::mc_lds_bytes(d->N, d->K, pre);
    // one resident round of workgroups (grid-stride over frames): a grid
    // larger than what fits at once runs its last workgroups as a tail
    const void *kfn = pre ? reinterpret_cast<const void *>(&qpd::mc_frames_kernel<true>)
                          : reinterpret_cast<const void *>(&qpd::mc_frames_kernel<false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 64, lds) != hipSuccess || per_cu <= 0) per_cu = 8;
    const int grid = (int)std::min<int64_t>(B, (int64_t)ncu * per_cu);
    return timed_launch(d, QPD_KC_MC, st, [&]() -> int {
        if (pre)
            hipLaunchKernelGGL(qpd::mc_frames_kernel<true>, dim3(grid), dim3(64), lds, st, C, frame0, B, d_msg, rows);
        else
            hipLaunchKernelGGL(qpd::mc_frames_kernel<false>, dim3(grid), dim3(64), lds, st, C, frame0, B, d_msg, rows);
        QPD_HIP(hipGetLastError());
        return QPD_OK;
    });
}

// One call's work on stream st, ordered after the decoder's previous work on
// any other stream, under the handle's lock.
template <class F>
int ordered(qpd_decoder *d, hipStream_t st, F &&work) {
    std::lock_guard<std::mutex> lk(d->mu);
    int rc = set_device(d);
    if (rc) return rc;
    if ((rc = order_on(d, st))) return rc;
    rc = work();
    const int mrc = mark_on(d, st);  // also after a failed launch: earlier launches of the call may be queued
    return rc ? rc : mrc;
}

}  // namespace

extern "C" {

int qpd_decode(qpd_decoder *d, const int32_t *d_symbols, int64_t B, uint8_t *d_out, void *stream) {
    if (!d) return fail(QPD_E_INVALID, "null decoder");
    if (d->dom != qpd::DOM_LUT) return fail(QPD_E_INVALID, "this decoder takes float64 LLRs: use qpd_decode_f64");
    if (B < 0) return fail(QPD_E_INVALID, "negative batch");
    if (B == 0) return QPD_OK;
    if (!d_symbols || !d_out) return fail(QPD_E_INVALID, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    return ordered(d, st, [&]() { return decode_impl(d, d_symbols, B, d_out, st); });
}

int qpd_decode_f64(qpd_decoder *d, const double *d_llr, int64_t B, uint8_t *d_out, void *stream) {
    if (!d) return fail(QPD_E_INVALID, "null decoder");
    if (d->dom == qpd::DOM_LUT) return fail(QPD_E_INVALID, "LUT decoders take int32 channel symbols: use qpd_decode");
    if (B < 0) return fail(QPD_E_INVALID, "negative batch");
    if (B == 0) return QPD_OK;
    if (!d_llr || !d_out) return fail(QPD_E_INVALID, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    return ordered(d, st, [&]() { return decode_f64_impl(d, d_llr, B, d_out, st); });
}

}  // extern "C"

static int input_error(int32_t flag) {
    std::string msg;
    if (flag & qpd::ERR_SYMBOL) msg += "channel symbol outside [0, v) in decoder input; ";
    if (flag & qpd::ERR_LLOYD) msg += "Lloyd bisect index outside the reconstruction list (reference UB); ";
    if (flag & qpd::ERR_NAN_PM) msg += "NaN path metric reached the list sort (reference UB); ";
    msg.resize(msg.size() - 2);
    return fail(QPD_E_INPUT, msg);
}

static int ensure(DeviceBuf &b, size_t &have, size_t need) {
    if (have >= need) return QPD_OK;
    if (b.p) {
        QPD_HIP(hipFree(b.p));
        b.p = nullptr;
    }
    QPD_HIP(hipMalloc(&b.p, need));
    have = need;
    return QPD_OK;
}

// One synchronous host-buffer decode: input staged through pinned memory,
// H2D copy, decode and D2H copies of the bits and the error word queued on
// the handle's own stream, one stream synchronization.  (What a per-frame
// decode(symbols) call of the reference drivers costs here: tools/latency.py.)
// Whether a host-buffer call of B frames runs on the host engine.
static bool host_engine_takes(const qpd_decoder *d, int64_t B) {
    if (!d->hplan || d->host_mode == QPD_HOST_GPU) return false;
    return d->host_mode == QPD_HOST_CPU || B <= d->host_max_frames;
}

// B frames on the host engine, one after another, under the handle's lock.
// The GPU work of the decoder is not touched (the engine has its own state),
// so no stream ordering is needed.
template <class Eng, class In>
static int host_engine_run(qpd_decoder *d, Eng *eng, const In *h_in, int64_t B, uint8_t *h_out) {
    std::lock_guard<std::mutex> lk(d->mu);
    d->last_engine = QPD_RAN_HOST;
    int32_t flag = 0;
    for (int64_t b = 0; b < B; ++b) flag |= eng->decode(h_in + b * d->N, h_out + b * d->out_bits);
    return flag ? input_error(flag) : QPD_OK;
}

template <class In, class Dec>
static int host_roundtrip(qpd_decoder *d, const In *h_in, int64_t B, uint8_t *h_out, Dec dec) {
    const size_t in_b = (size_t)B * d->N * sizeof(In), out_b = (size_t)B * d->out_bits;
    const size_t out_at = (in_b + 15) & ~(size_t)15, err_at = out_at + ((out_b + 15) & ~(size_t)15);
    hipStream_t hs = d->hs;
    return ordered(d, hs, [&]() -> int {
        // the staging buffers may still be read by the previous call's work
        // only if that ran on hs, which the synchronization below has drained
        int rc = ensure(d->h_in, d->h_in_bytes, in_b);
        if (rc) return rc;
        if ((rc = ensure(d->h_out, d->h_out_bytes, std::max<size_t>(1, out_b)))) return rc;
        if (d->pin_bytes < err_at + 16) {
            if (d->pin) QPD_HIP(hipHostFree(d->pin));
            d->pin = nullptr;
            d->pin_bytes = 0;
            QPD_HIP(hipHostMalloc(&d->pin, err_at + 16, hipHostMallocDefault));
            d->pin_bytes = err_at + 16;
        }
        char *pin = (char *)d->pin;
        std::memcpy(pin, h_in, in_b);
        QPD_HIP(hipMemcpyAsync(d->h_in.p, pin, in_b, hipMemcpyHostToDevice, hs));
        if ((rc = dec((const In *)d->h_in.p, (uint8_t *)d->h_out.p, hs))) return rc;
        if (out_b) QPD_HIP(hipMemcpyAsync(pin + out_at, d->h_out.p, out_b, hipMemcpyDeviceToHost, hs));
        QPD_HIP(hipMemcpyAsync(pin + err_at, d->err.p, sizeof(int32_t), hipMemcpyDeviceToHost, hs));
        QPD_HIP(hipStreamSynchronize(hs));
        std::memcpy(h_out, pin + out_at, out_b);
        int32_t flag = 0;
        std::memcpy(&flag, pin + err_at, sizeof(flag));
        if (flag) {
            QPD_HIP(hipMemsetAsync(d->err.p, 0, sizeof(int32_t), hs));
            QPD_HIP(hipStreamSynchronize(hs));
            return input_error(flag);
        }
        return QPD_OK;
    });
}

extern "C" {

int qpd_check_input_error(qpd_decoder *d) {
    if (!d) return fail(QPD_E_INVALID, "null decoder");
    hipStream_t hs = d->hs;
    return ordered(d, hs, [&]() -> int {
        // hs waits for the decoder's last launch (any stream); the flag is
        // read and cleared on hs, which later calls on other streams wait for
        int32_t flag = 0;
        QPD_HIP(hipMemcpyAsync(&flag, d->err.p, sizeof(flag), hipMemcpyDeviceToHost, hs));
        QPD_HIP(hipStreamSynchronize(hs));
        if (flag) {
            QPD_HIP(hipMemsetAsync(d->err.p, 0, sizeof(int32_t), hs));
            QPD_HIP(hipStreamSynchronize(hs));
            return input_error(flag);
        }
        return QPD_OK;
    });
}

int qpd_decode_host(qpd_decoder *d, const int32_t *h_symbols, int64_t B, uint8_t *h_out) {
    if (!d) return fail(QPD_E_INVALID, "null decoder");
    if (d->dom != qpd::DOM_LUT) return fail(QPD_E_INVALID, "this decoder takes float64 LLRs: use qpd_decode_f64_host");
    if (B <= 0) return B == 0 ? QPD_OK : fail(QPD_E_INVALID, "negative batch");
    if (!h_symbols || !h_out) return fail(QPD_E_INVALID, "null buffer");
    if (host_engine_takes(d, B)) return host_engine_run(d, d->heng_lut.get(), h_symbols, B, h_out);
    return host_roundtrip(d, h_symbols, B, h_out,
                          [&](const int32_t *in, uint8_t *out, hipStream_t st) { return decode_impl(d, in, B, out, st); });
}

int qpd_decode_f64_host(qpd_decoder *d, const double *h_llr, int64_t B, uint8_t *h_out) {
    if (!d) return fail(QPD_E_INVALID, "null decoder");
    if (d->dom == qpd::DOM_LUT) return fail(QPD_E_INVALID, "LUT decoders take int32 channel symbols: use qpd_decode_host");
    if (B <= 0) return B == 0 ? QPD_OK : fail(QPD_E_INVALID, "negative batch");
    if (!h_llr || !h_out) return fail(QPD_E_INVALID, "null buffer");
    if (host_engine_takes(d, B)) return host_engine_run(d, d->heng_f64.get(), h_llr, B, h_out);
    return host_roundtrip(d, h_llr, B, h_out,
                          [&](const double *in, uint8_t *out, hipStream_t st) { return decode_f64_impl(d, in, B, out, st); });
}

int qpd_set_host_engine(qpd_decoder *d, int32_t mode) {
    if (!d) return fail(QPD_E_INVALID, "null decoder");
    if (mode < QPD_HOST_AUTO || mode > QPD_HOST_CPU) return fail(QPD_E_INVALID, "mode must be QPD_HOST_AUTO, _GPU or _CPU");
    if (mode == QPD_HOST_CPU && !d->hplan)
        return fail(QPD_E_UNSUPPORTED, "the host engine does not decode the re-quantized float kinds");
    std::lock_guard<std::mutex> lk(d->mu);
    d->host_mode = mode;
    return QPD_OK;
}

int qpd_mc_frames(qpd_decoder *d, const qpd_mc_channel *ch, uint64_t seed, int64_t frame0, int64_t B, uint8_t *d_msg,
                  int32_t *d_symbols, void *stream) {
    if (!d || !ch) return fail(QPD_E_INVALID, "null argument");
    if (B < 0 || frame0 < 0) return fail(QPD_E_INVALID, "negative frame range");
    if (B == 0) return QPD_OK;
    if (!d_msg || !d_symbols) return fail(QPD_E_INVALID, "null buffer");
    int rc = check_channel(ch);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    return ordered(d, st, [&]() { return mc_launch(d, ch, seed, frame0, B, d_msg, d_symbols, false, st); });
}

int qpd_mc_decode(qpd_decoder *d, const qpd_mc_channel *ch, uint64_t seed, int64_t frame0, int64_t B, uint8_t *d_msg,
                  uint8_t *d_out, int64_t *d_counts, void *stream) {
    if (!d || !ch) return fail(QPD_E_INVALID, "null argument");
    if (d->dom != qpd::DOM_LUT) return fail(QPD_E_INVALID, "qpd_mc_decode needs a LUT decoder (int32 channel symbols)");
    if (B < 0 || frame0 < 0) return fail(QPD_E_INVALID, "negative frame range");
    if (B == 0) return QPD_OK;
    if (!d_msg || !d_out) return fail(QPD_E_INVALID, "null buffer");
    int rc = check_channel(ch);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    return ordered(d, st, [&]() -> int {
        // fused: the generator writes the root pre-pass rows the decode
        // kernel reads (fast engine in pre-mode; symbols < q <= v need no
        // range check); else int32 symbols in a buffer of its own
        const bool fused = d->engine == QPD_ENGINE_FAST && d->pre && ch->q <= d->v;
        d->last_engine = QPD_RAN_GPU;
        int64_t chunk;
        if (fused) {
            int r0 = QPD_OK;
            chunk = ensure_pre_rows(d, std::min<int64_t>(B, d->pre_chunk), &r0);
            if (r0) return r0;
        } else {
            // int32 symbols of <= 1 GB per chunk (2^18 frames at N = 1024); halved
            // on an allocation failure, and the smaller buffer kept from then on
            chunk = std::min<int64_t>(B, std::max<int64_t>(1, ((int64_t)1 << 30) / ((int64_t)d->N * 4)));
            if (d->mc_sym_fell_back) chunk = std::min(chunk, d->mc_sym_cap);
            if (d->mc_sym_cap < chunk) {
                if (d->mc_sym.p) QPD_HIP(hipFree(d->mc_sym.p));
                d->mc_sym.p = nullptr;
                d->mc_sym_cap = 0;
                hipError_t e = hipErrorOutOfMemory;
                const int64_t want = chunk;
                while (chunk >= 1 && (e = hipMalloc(&d->mc_sym.p, (size_t)chunk * d->N * sizeof(int32_t))) != hipSuccess) {
                    (void)hipGetLastError();
                    d->mc_sym.p = nullptr;
                    chunk /= 2;
                }
                if (e != hipSuccess) return fail(QPD_E_DEVICE, std::string("Monte-Carlo symbols hipMalloc: ") + hipGetErrorString(e));
                d->mc_sym_fell_back = chunk < want;
                d->mc_sym_cap = chunk;
            }
            chunk = std::min(chunk, d->mc_sym_cap);
        }
        DeviceBuf &buf = fused ? d->pre_buf : d->mc_sym;
        for (int64_t f0 = 0; f0 < B; f0 += chunk) {
            const int64_t Bc = std::min<int64_t>(chunk, B - f0);
            int r = mc_launch(d, ch, seed, frame0 + f0, Bc, d_msg + f0 * d->out_bits, (int32_t *)buf.p, fused, st);
            if (r) return r;
            uint8_t *out = d_out + f0 * d->out_bits;
            r = fused ? decode_pre_rows(d, (const uint32_t *)buf.p, Bc, out, st)
                      : decode_impl(d, (const int32_t *)buf.p, Bc, out, st);
            if (r) return r;
        }
        if (d_counts) {  // the driver's error counters over the whole range
            int dev = 0, ncu = 256;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
            const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((B + 3) / 4, (int64_t)ncu * 8));
            hipLaunchKernelGGL(qpd::mc_count_kernel, dim3(grid), dim3(256), 0, st, d_out, d_msg, B, d->out_bits,
                               (unsigned long long *)d_counts);
            QPD_HIP(hipGetLastError());
        }
        return QPD_OK;
    });
}

int qpd_probe_lds(int32_t device, int32_t op, double *gbps) {
    if (!gbps || op < 0 || op > 2) return fail(QPD_E_INVALID, "bad probe op / null output");
    if (device >= 0) QPD_HIP(hipSetDevice(device));
    QPD_HIP(qpd::probe_lds_run(op, gbps));
    return QPD_OK;
}

int qpd_profile(qpd_decoder *d, int32_t enable) {
    if (!d) return fail(QPD_E_INVALID, "null decoder");
    std::lock_guard<std::mutex> lk(d->mu);
    d->prof = enable != 0;
    return QPD_OK;
}

int qpd_kernel_times(qpd_decoder *d, double *ms, int64_t *launches) {
    if (!d || !ms || !launches) return fail(QPD_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(d->mu);
    int rc = set_device(d);
    if (rc) return rc;
    for (int k = 0; k < QPD_KC_COUNT; ++k) {
        ms[k] = 0.0;
        launches[k] = (int64_t)d->prof_ev[k].size();
        for (auto &e : d->prof_ev[k]) {
            float t = 0.f;
            QPD_HIP(hipEventSynchronize(e.second));
            QPD_HIP(hipEventElapsedTime(&t, e.first, e.second));
            ms[k] += t;
            QPD_HIP(hipEventDestroy(e.first));
            QPD_HIP(hipEventDestroy(e.second));
        }
        d->prof_ev[k].clear();
    }
    return QPD_OK;
}

#ifdef QPD_STAMPS
// Diagnostic builds only (not declared in qpd.h): read and clear the per-class
// cycle / count accumulators of lut_fast_kernel.
int qpd_debug_stamps(unsigned long long *out64) {
    QPD_HIP(hipDeviceSynchronize());
    unsigned long long *acc = stamp_buffer();
    if (!acc) return fail(QPD_E_DEVICE, "stamp buffer");
    QPD_HIP(hipMemcpy(out64, acc, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    QPD_HIP(hipMemset(acc, 0, 64 * sizeof(unsigned long long)));
    return QPD_OK;
}
#endif
}  // extern "C"

