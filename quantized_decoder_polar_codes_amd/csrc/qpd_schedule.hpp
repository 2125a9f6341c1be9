// qpd_schedule.hpp -- the static traversal schedule (host code), shared by
// the C-ABI (qpd_capi.hip: GPU plans) and the host engine (qpd_host.hpp).
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

#include "qpd.h"
#include "qpd_types.hpp"

namespace qpd_sched {

using qpd::Op;

// Static traversal schedule.  The reference walks the
// tree with a node_state machine (src/SCLLUTDecoder.cpp:62-243); the walk does
// not depend on data, so it is compiled once per code into a flat op list that
// every frame replays.  Special nodes follow node_type AS PASSED (H7):
// FastSC-LUT handles R0/R1/REP/SPC (FastSCLUT.cpp:46-107), FastSCL-LUT handles
// R0/R1/REP only (FastSCLLUTDecoder.cpp:82-215); other labels decode as plain
// f/g nodes.
struct Schedule {
    std::vector<Op> ops;
    int max_r1 = 0;
};

inline int special_of(int kind, const int32_t *node_type, int posi) {
    if (!node_type) return -1;
    const int t = node_type[posi];
    if (kind == QPD_FASTSC_LUT && t >= 0 && t <= 3) return t;
    if (kind == QPD_FASTSCL_LUT && t >= 0 && t <= 2) return t;
    return -1;
}

inline void emit(Schedule &s, int type, int d, int node, int aux) {
    Op op;
    op.type = type;
    op.d = d;
    op.node = node;
    op.aux = aux;
    s.ops.push_back(op);
}

inline void visit(Schedule &s, int kind, int N, int n, const int32_t *frozen, const int32_t *node_type, int d, int node) {
    const int posi = (1 << d) + node - 1;
    const int t = special_of(kind, node_type, posi);
    if (t >= 0) {
        emit(s, qpd::OP_R0 + t, d, node, 0);
        if (t == 1) s.max_r1 = std::max(s.max_r1, N >> d);
        return;
    }
    if (d + 1 < n) {
        emit(s, qpd::OP_F, d, node, 0);
        visit(s, kind, N, n, frozen, node_type, d + 1, 2 * node);
        emit(s, qpd::OP_G, d, node, 0);
        visit(s, kind, N, n, frozen, node_type, d + 1, 2 * node + 1);
    } else {
        emit(s, qpd::OP_LEAF_L, d, node, frozen[2 * node] == 1);
        emit(s, qpd::OP_LEAF_R, d, node, frozen[2 * node + 1] == 1);
    }
    emit(s, qpd::OP_COMB, d, node, 0);
}

// Kernel family (SC / SCL / FastSC / FastSCL, as the LUT kind ids) and symbol
// domain of every public kind; the CRC-aided kinds are their list family
// plus an output epilogue.
inline bool family_of(int kind, int *fam, int *dom) {
    using namespace qpd;
    switch (kind) {
        case QPD_SC_FLOAT: *fam = QPD_SC_LUT; *dom = DOM_FLOAT; return true;
        case QPD_SC_LUT:
        case QPD_SCL_LUT:
        case QPD_FASTSC_LUT:
        case QPD_FASTSCL_LUT: *fam = kind; *dom = DOM_LUT; return true;
        case QPD_CASCL_LUT: *fam = QPD_SCL_LUT; *dom = DOM_LUT; return true;
        case QPD_CAFASTSCL_LUT: *fam = QPD_FASTSCL_LUT; *dom = DOM_LUT; return true;
        case QPD_SCL_FLOAT:
        case QPD_CASCL_FLOAT: *fam = QPD_SCL_LUT; *dom = DOM_FLOAT; return true;
        case QPD_FASTSC_FLOAT: *fam = QPD_FASTSC_LUT; *dom = DOM_FLOAT; return true;
        case QPD_FASTSCL_FLOAT: *fam = QPD_FASTSCL_LUT; *dom = DOM_FLOAT; return true;
        case QPD_SC_UNIFORM: *fam = QPD_SC_LUT; *dom = DOM_UNIFORM; return true;
        case QPD_SCL_UNIFORM: *fam = QPD_SCL_LUT; *dom = DOM_UNIFORM; return true;
        case QPD_SC_LLOYD: *fam = QPD_SC_LUT; *dom = DOM_LLOYD; return true;
        case QPD_SCL_LLOYD: *fam = QPD_SCL_LUT; *dom = DOM_LLOYD; return true;
        default: return false;
    }
}

inline bool is_ca(int kind) { return kind == QPD_CASCL_LUT || kind == QPD_CAFASTSCL_LUT || kind == QPD_CASCL_FLOAT; }

}  // namespace qpd_sched
