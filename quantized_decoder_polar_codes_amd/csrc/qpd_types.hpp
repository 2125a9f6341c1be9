// qpd_types.hpp -- plain types and constants shared by the device kernels,
// the C-ABI and the host engine (no HIP: the host engine's CPU test builds it
// with g++).
#pragma once
#include <stdint.h>

namespace qpd {

enum OpType : int32_t {
    OP_F = 0,       // left child symbols  (f LUT), depth d -> d+1
    OP_G = 1,       // right child symbols (g LUT), depth d -> d+1
    OP_LEAF_L = 2,  // left leaf 2*node of a depth n-1 node (f LUT at j=0)
    OP_LEAF_R = 3,  // right leaf 2*node+1                  (g LUT at j=0)
    OP_COMB = 4,    // partial-sum combine u(), utils.cpp:62-67
    OP_R0 = 5,
    OP_R1 = 6,
    OP_REP = 7,
    OP_SPC = 8
};

struct Op {
    int32_t type, d, node, aux;  // aux: frozen flag for leaves
};

constexpr int kMaxDepth = 16;  // N <= 65536
constexpr int kMaxL = 8;       // fast engine: 2L <= 16, libstdc++ sorts by insertion (stable)
constexpr int kMaxM = kMaxL - 1;
constexpr int kMaxLWide = 32;  // generic engine: 2L <= 64, libstdc++ introsort replayed (stl_sort.hpp)

// Decoder families of the kernels (the float-domain decoders use the same
// family ids with a DOM_* symbol domain; K_SC_FLOAT is the C-ABI's kind 0).
enum Kind : int32_t { K_SC_FLOAT = 0, K_SC_LUT = 1, K_SCL_LUT = 2, K_FASTSC_LUT = 3, K_FASTSCL_LUT = 4 };

// Symbol domains of the generic engine: LUT symbols (int, f/g by tables) or
// fp64 LLRs (min-sum f/g), optionally re-quantized after every f/g.
enum Dom : int32_t { DOM_LUT = 0, DOM_FLOAT = 1, DOM_UNIFORM = 2, DOM_LLOYD = 3 };

// Device error flags (DevPlan/FastPlan err word).
enum ErrFlag : int32_t { ERR_SYMBOL = 1, ERR_LLOYD = 2, ERR_NAN_PM = 4 };

}  // namespace qpd
