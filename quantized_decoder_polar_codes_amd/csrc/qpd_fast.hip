// qpd_fast.hip -- the fast gfx950 LUT decode kernel (one table per node, v <= 16).
//
// Same algorithm, traversal and list management as the generic kernel
// (qpd_generic.hip: one lane per list path, G = pow2 >= L lanes per frame,
// per-depth 4-bit slot pointers instead of deep copies), laid out for the
// CDNA4 memory hierarchy and for instruction count:
//
//  * Host-compiled micro-op records (MOp, 64 B, one s_load_dwordx16 each)
//    carry every row offset, shift and flag an op needs, so the wave-uniform
//    interpreter does almost no scalar arithmetic per op.
//  * Symbols are 4-bit nibbles, 8 per dword.  Per tree depth d a path owns
//    S[d] (symbols of the active depth-d node), U[d] (partial sums of the
//    finished left child) and R[d] (partial sums of a finished right child).
//    Deep levels (d >= lds_from) sit in LDS, shallow levels in a per-wave
//    global slab; both are laid out [row][64 lanes].  LDS instructions of one
//    wave complete in order, so LDS-only ops need no barrier.
//  * The last three tree levels of every plain subtree are one BOT3 op held
//    entirely in registers: 8 symbols in, 8 leaves decided (with list forks
//    moving the whole in-register state from the parent lane), 8 partial-sum
//    bits out -- 21 interpreted ops become one straight-line block.
//  * The current node's f/g table sits in ONE VGPR per lane (f: 256 nibbles =
//    32 dwords, g: 512 nibbles = 64 dwords), read with ds_bpermute; the next
//    op's table / leaf quanta row are prefetched while the current op runs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qpd_common.hpp"
#include "stl_sort.hpp"

namespace qpd {

constexpr int OP_BOT3 = 9;    // fused bottom subtree of height 3 (fast engine only)
constexpr int OP_IMPORT = 10; // frozen-prefix stages (see lut_prefix_kernel): rows / metric from a stage's records, or zeros
constexpr int OP_EXPORT = 11; // lut_prefix_kernel only: live rows into the stage's records (FastPlan::pfx)

enum MopFlag : int32_t {
    MF_SRC_LDS = 1,   // S[d] in LDS
    MF_DST_LDS = 2,   // destination rows in LDS
    MF_U_LDS = 4,     // U rows read by the op in LDS
    MF_TO_R = 8,      // finished node is a right child (or the root): write R, not U
    MF_SYNC = 16,     // drain the global slab before this op (see place_syncs)
    MF_R_LDS = 32,    // R rows read by the op (COMB) in LDS
    MF_CHAN = 64,     // S[d] is the channel input (d == 0)
    MF_R1_LDS = 128,  // R1 (> 16 elements): argsort in the free LDS tail starting at row u_row
    MF_PRE = 256,     // S[1] of the root's left child / the root g inputs: words of the frame's
                      // pre-pass row (root_pre_kernel), read without a slot pointer
    MF_GSEL = 512,    // root g in pre-mode: nibble select between g(y, 0) and g(y, 1) by u
    MF_BFG = 1024,    // BOT3 whose 8 input symbols are f (or g, MF_BG) of its depth n-4 parent's 16:
    MF_BG = 2048,     //   the parent's F / G op folded in (src = S[n-4], table at tab2, U[n-3] at u_row)
    MF_BCOMB = 4096,  // right BOT3 that also runs its parent's combine (dst = U/R[n-4])
    MF_VUNI = 8192,   // special node whose elements share one quanta row (v <= 16): quanta and
                      //   R1 ranks are looked up in a register row instead of gathered per element
    MF_ZERO = 16384,  // OP_IMPORT: zero rows (partial sums of the frozen prefix) instead of record words
    MF_PM = 32768,    // OP_IMPORT: the path metric (a double in words src_row, src_row + 1 of the record)
    MF_VIA_PS = 65536,   // OP_EXPORT: the row is read through the path's S pointer of depth sh_src / 4
    MF_VIA_PU = 131072,  //   ... or its U pointer (else the lane's own row: R rows)
    MF_XBUF = 262144,    // OP_IMPORT: from a prefix stage's records (address and layout in the op record)
    MF_FF = 524288,      // F / G (SCL-LUT) that also runs the f of its left child at depth d+1 from
                         //   the words it just computed (fuse_descent): S[d+2] at r_row, the
                         //   child's table at tab2, its S pointer field at pad1
    MF_FF_DL = 1048576,  //   ... S[d+2] in LDS
    MF_BC2 = 2097152,    // right BOT3 with MF_BCOMB and MF_TO_R that also runs the combine of its
                         //   grandparent at depth n-5 (fold_combine): U[n-4] of the left sibling at
                         //   r_row (pointer field pad1 & 255), result to row pad1 >> 16 (its U
                         //   pointer field (pad1 >> 8) & 255) instead of R[n-4] at dst_row
    MF_BC2_ULDS = 4194304,  //   ... that U row in LDS
    MF_BC2_DLDS = 8388608,  //   ... the result row in LDS
    MF_BC2_TOR = 16777216,  //   ... the grandparent is a right child (R row: no pointer update)
    MF_BOTX = 33554432,     // BOT3 of a subtree with FastSCL special nodes of size 4 / 2 (botx_op)
    MF_R1_RK = 67108864,    // R1 with one quanta row: symbol s's rank in bits 4s..4s+3 of r_row | tab2 << 32 and
                            //   its sign in bit s of pad1 (r1_prep: no per-element rank lookups)
    MF_SFG = 134217728,     // size-8 special node (FastSCL-LUT, L = 8) that computes its 8 symbols as f of its
                            //   depth n-4 parent's 16 (src = S[n-4], the parent's table at tab): no F op
    MF_SGG = 268435456,     //   ... as g of them, u = the left sibling's U[n-3] at u_row (sh_u): no G op
    MF_SCOMB = 536870912,   //   ... and runs the parent's combine with that U[n-3] (dst = the parent's): no COMB
};

struct MOp {
    int32_t type, flags, d, node;
    int32_t cnt;      // F/G/COMB: ctemp = N>>(d+1); special: temp = N>>d; LEAF: frozen; BOT3: frozen mask
    int32_t src_row;  // S[d]
    int32_t dst_row;  // F/G: S[d+1]; COMB/special/BOT3: U[d] or R[d]; LEAF_L: U[n]; LEAF_R: R[n]
    int32_t u_row;    // G/COMB: U[d+1]; LEAF_R: U[n]
    int32_t r_row;    // COMB: R[d+1]; F/G with MF_FF: S[d+2]
    int32_t sh_src;   // 4*d: ps field of S[d]
    int32_t sh_u;     // G/COMB: 4*(d+1); LEAF_R: 4*n
    int32_t sh_dst;   // F/G: 4*(d+1) (ps); COMB/special/BOT3 left child: 4*d (pu); LEAF_L: 4*n (pu)
    int32_t tab;      // F/LEAF_L: posi*32; G/LEAF_R: posi*64; BOT3: posi of the subtree root; R1: r1_rank offset
    int32_t vrow;     // LEAF: ((n-1)*N + k)*v; special: (d-1)*N + temp*node; BOT3: ((n-1)*N + 8*node)*v
    int32_t tab2;     // MF_BFG: the parent's table (f: posi*32, g: posi*64); MF_FF: the child's f table
    int32_t pad1;     // MF_FF: the child's S pointer field (4*(d+2))
};

struct FastPlan {
    int32_t N, n, K, L, v, gs, fpw, nops, max_r1;
    int32_t in_vec;               // per launch: input rows are 16-byte aligned
    int32_t in_shift;             // per launch: log2 int32 words per frame row of `in` (n: channel
                                  // symbols; n - 2: pre-pass rows, root_pre_kernel)
    int32_t out_k;                // output bits per frame: K, or A (CRC-aided kinds)
    int32_t ca_A, crc_n;          // crc_n > 0: CRC-aided output (ca_winner)
    uint32_t crc_q;
    const uint32_t *info_mask;    // [N/32] information-position mask
    int32_t lds_rows, glb_rows, lds_from;
    int32_t R0_row, R0_lds;      // root partial sums (R[0])
    int32_t H_row, K_row, I_row;  // R1 scratch (global)
    const uint32_t *f_tab;        // [N-1][32] nibble-packed f tables
    const uint32_t *g_tab;        // [N-1][64] nibble-packed g tables (u=0: dwords 0..31)
    const double *vcl;            // [rows][N][v]
    const MOp *ops;
    const int32_t *info_pos;
    const uint16_t *r1_rank;      // FastSCL R1 (<= 32 elements): [temp][v] rank << 1 | sign, per node at op.tab
    uint32_t *scratch;            // [waves][glb_rows][64]
    int32_t *err;
    uint32_t *task_ctr;           // QPD_DYN task queue: tasks taken (never reset; see wave_take)
    uint32_t task_base;           // per launch: the counter's value when this launch's takes begin
    // Frozen-prefix stages (lut_prefix_kernel).  A stage writes, per frame f and path p,
    // its live rows (OP_EXPORT) and metric (two words from pm_off) as a record of pfx_rec
    // words in a buffer of its own, interleaved so that the 64 lanes of a wave store 64
    // consecutive words: word w of (f, p) at ((f >> G) * pfx_rec + w) * 64 + (f mod 2^G) *
    // 2^PS + p, pfx_geo = G | PS << 8 (2^G frames of 2^PS paths per 64 words; stage 1:
    // G = 6, PS = 0; stage 2: G = 4, PS = 2).  OP_IMPORT (MF_XBUF) reads records back with
    // the buffer address, record words, geometry and live paths in the op record (u_row |
    // r_row << 32, tab, vrow, tab2), not in the plan: plan fields the decode loop reads
    // cost it SGPRs (spill 149 -> 158).
    uint32_t *pfx;
    int32_t pfx_rec, pfx_geo, pm_off;
#ifdef QPD_STAMPS
    unsigned long long *stamps;   // diagnostic builds: [64] per-class cycle / count accumulators
#endif
};

// Timing experiments only (wrong results): 0 = every op reads node 0's
// tables / the slab drops every access.
#ifndef QPD_EXP_TABMUL
#define QPD_EXP_TABMUL 1
#endif
#ifndef QPD_EXP_SLABMUL
#define QPD_EXP_SLABMUL 1
#endif

#ifndef QPD_EXP_LUTMASK
#define QPD_EXP_LUTMASK 0xFFFF  // timing experiments only (wrong results): 0x7F keeps every byte-table
                                // lookup inside one 128-B LDS bank row (no bank conflicts)
#endif

#ifndef QPD_EXP_NO_BOTX
#define QPD_EXP_NO_BOTX 0  // register-allocation experiments: botx_op compiled out (MF_BOTX ops then wrong)
#endif
#ifndef QPD_EXP_FSCL
#define QPD_EXP_FSCL 0  // code-quality experiments (wrong results for those ops): 2 no special ops,
                        // 4 no R1, 8 no R1 LDS introsort, 16 no REP, 128 old partition loop, 256 no special
                        // ops at all, 512 no multi-set R0/REP, 1024 no multi-set R1
#endif

#ifndef QPD_SLAB_AUX
#define QPD_SLAB_AUX 0  // cache-policy bits of the slab's buffer ops (2 = nt)
#endif

// Row access in either space.  `in_lds` is wave-uniform.  The global slab is
// reached through a buffer descriptor (32-bit lane offsets; distinct
// instructions, so the compiler never folds the two spaces into one flat
// access that would wait on both counters).
// A wave's `ns` frame sets interleave their rows, in LDS and in the slab: row r
// of set s is the wave's row r * ns + s.  The sets share one LDS base and one
// slab descriptor and a set's view differs only by s rows -- an immediate
// offset in its LDS / buffer instructions (`so` bytes, constant after the set
// loops unroll) instead of a base register and a descriptor per set.
struct Mem {
    uint32_t *lds;              // this set's LDS row 0 (the wave's base + s rows)
    uint32_t *gp;               // this set's slab row 0 (R1 argsort arrays)
    __amdgpu_buffer_rsrc_t rs;  // the wave's slab, all sets
    int so;                     // this set's byte offset in a slab row group (s * 256)
    int ns;                     // frame sets of the wave: the row stride in rows
    __device__ __forceinline__ int rw(int row) const { return row * ns * 64; }  // words to row `row`
    // the view of set s (runtime) from set 0's
    __device__ __forceinline__ Mem set(int s) const {
        Mem m = *this;
        m.lds = lds + s * 64;
        m.gp = gp + s * 64;
        m.so = so + s * 256;
        return m;
    }
    // `row` wave-uniform: it rides in the buffer op's SGPR offset
    __device__ __forceinline__ uint32_t ld(bool in_lds, int row, int lane) const {
        if (in_lds) return lds[rw(row) + lane];
        return __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, row * ns * 256 + so, QPD_SLAB_AUX);
    }
    __device__ __forceinline__ void st(bool in_lds, int row, int lane, uint32_t v) const {
        if (in_lds)
            lds[rw(row) + lane] = v;
        else
            __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane * 4, row * ns * 256 + so, QPD_SLAB_AUX);
    }
    // any row (per-lane)
    __device__ __forceinline__ uint32_t ldv(bool in_lds, int row, int lane) const {
        if (in_lds) return lds[rw(row) + lane];
        return __builtin_amdgcn_raw_buffer_load_b32(rs, (rw(row) + lane) * 4 + so, 0, QPD_SLAB_AUX);
    }
    __device__ __forceinline__ void stv(bool in_lds, int row, int lane, uint32_t v) const {
        if (in_lds)
            lds[rw(row) + lane] = v;
        else
            __builtin_amdgcn_raw_buffer_store_b32(v, rs, (rw(row) + lane) * 4 + so, 0, QPD_SLAB_AUX);
    }
};

// Table dword `at + ldw` (at wave-uniform, ldw = the lane's dword) through a
// buffer descriptor: the uniform part rides in the SGPR offset, so a table
// fetch costs no per-lane 64-bit address arithmetic.
__device__ __forceinline__ uint32_t tab_ld(const uint32_t *base, int at, int ldw) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, 0x7fffffff, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b32(r, ldw * 4, at * 4, 0);
}

__device__ __forceinline__ uint32_t bperm(uint32_t table, uint32_t dword) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(dword << 2), (int)table);
}

// 4-bit LUT lookup from the table register: entry idx lives in dword idx>>3.
__device__ __forceinline__ uint32_t lut4(uint32_t table, uint32_t idx) {
    return (bperm(table, idx >> 3) >> ((idx & 7u) << 2)) & 15u;
}

// x F^{(x)5} inside one 32-bit word (the in-word stages of the re-encode).
__device__ __forceinline__ uint32_t polar_word(uint32_t x) {
    x ^= (x >> 1) & 0x55555555u;
    x ^= (x >> 2) & 0x33333333u;
    x ^= (x >> 4) & 0x0f0f0f0fu;
    x ^= (x >> 8) & 0x00ff00ffu;
    x ^= (x >> 16) & 0x0000ffffu;
    return x;
}

// Cross-word butterfly stage of the re-encode on a register row (nwr <= 32 words).
template <int MW>
__device__ __forceinline__ void xor_stage(uint32_t (&x)[32], int nwr) {
#pragma unroll
    for (int i = 0; i < 32; i += 2 * MW)
#pragma unroll
        for (int j = 0; j < MW; ++j)
            if (i + MW + j < nwr) x[i + j] ^= x[i + MW + j];
}

__device__ __forceinline__ int pfield(uint64_t p, int sh) { return (int)((p >> sh) & 15u); }
__device__ __forceinline__ uint64_t pset(uint64_t p, int sh, int gl) {
    return (p & ~(15ull << sh)) | ((uint64_t)gl << sh);
}

// Channel symbols: int32 input, range-checked (UB in the reference).
__device__ __forceinline__ uint32_t chan_sym(const int32_t *y, int e, int v, int32_t *err) {
    int s = y[e];
    if ((unsigned)s >= (unsigned)v) {
        atomicOr(err, 1);
        s = 0;
    }
    return (uint32_t)s;
}

__device__ __forceinline__ uint32_t chan_word(const int32_t *y, int e0, int cnt, int v, int32_t *err) {
    uint32_t w = 0;
    for (int i = 0; i < cnt; ++i) w |= chan_sym(y, e0 + i, v, err) << (4 * i);
    return w;
}

// Eight channel symbols e0..e0+7 as one nibble word; `vec` = the input rows
// are 16-byte aligned (two 128-bit loads instead of eight 32-bit ones).
__device__ __forceinline__ uint32_t chan_word8(const int32_t *y, int e0, bool vec, int v, int32_t *err) {
    if (!vec) return chan_word(y, e0, 8, v, err);
    const int4 a = *(const int4 *)(y + e0), b = *(const int4 *)(y + e0 + 4);
    const int e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t w = 0, bad = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t s = (uint32_t)e[i];
        bad |= s >= (uint32_t)v;
        w |= (s >= (uint32_t)v ? 0u : s) << (4 * i);
    }
    if (bad) atomicOr(err, 1);
    return w;
}

// Word w (8 symbols) of S[d] of the path whose slot is `src`.
// The first `cnt` channel symbols as one nibble word, a rolled loop: the
// channel reads of the ops that see the channel only in codes of N <= 8 (the
// BOT3 / leaf ops at the root) -- small code for a case that is never hot.
__device__ __forceinline__ uint32_t chan_small(const int32_t *y, int cnt, int v, int32_t *err) {
    uint32_t w = 0, bad = 0;
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const uint32_t s = (uint32_t)y[i];
        bad |= s >= (uint32_t)v;
        w |= (s >= (uint32_t)v ? 0u : s) << (4 * i);
    }
    if (bad) atomicOr(err, 1);
    return w;
}

// Word w of S[d]: the pre-pass row (MF_PRE), a slab / LDS row, or with CH the
// channel (MF_CHAN): the ops that read the channel only in codes of N <= 8
// (the BOT3 / leaf ops at the root; word 0, chan_small).  The f / g ops at
// the root read it in fg_chan_op.
template <bool CH = false>
__device__ __forceinline__ uint32_t sym_word(const FastPlan &P, const Mem &M, const MOp &op, const int32_t *y, int src,
                                             int w, int cnt = 8) {
    if (op.flags & MF_PRE) return ((const uint32_t *)y)[op.src_row + w];  // N >= 16: whole words
    if constexpr (CH)
        if (op.flags & MF_CHAN) return chan_small(y, cnt, P.v, P.err);
    return M.ld(op.flags & MF_SRC_LDS, op.src_row + w, src);
}

// NE table lookups T[a_i, b_i] (i < NE <= 8) packed as output nibbles, with
// a_i / b_i = nibble i of A / B and table half h_i = bit i of `hi` (the g
// table's u = 1 half, or the second of two packed f tables).  SWAR index
// build: byte j of X / Y is the 8-bit index of element 2j / 2j+1, from which
// one pass each derives the ds_bpermute byte address (idx >> 1, whose bits
// 7:2 select the dword; + 128 for the upper half) and the nibble offset
// ((idx & 7) * 4, used by v_bfe through its low 5 bits only).
// QPD_VEC_CHAIN: lut_vec joins its results by one v_lshl_or per element (the
// compiler otherwise shifts each and merges them with v_or3: +0.5 VALU per
// lookup).  On in the FastSCL-LUT units (+0.5 %), off for SCL-LUT (-0.25 %:
// the serial chain costs it latency), profiles/r06v_ab_vec_chain.txt.
#ifndef QPD_VEC_CHAIN
#define QPD_VEC_CHAIN 0
#endif
template <int NE>
__device__ __forceinline__ uint32_t lut_vec(uint32_t T, uint32_t A, uint32_t B, uint32_t hi) {
    const uint32_t X = ((A << 4) & 0xF0F0F0F0u) | (B & 0x0F0F0F0Fu);
    const uint32_t Y = (A & 0xF0F0F0F0u) | ((B >> 4) & 0x0F0F0F0Fu);
    uint32_t hx = 0, hy = 0;  // bit 2j / 2j+1 of hi -> bit 8j+7
    if constexpr (NE == 8) {  // one multiply spreads 4 bits (no carries reach the kept bits)
        hx = ((hi & 0x55u) * 0x02082080u) & 0x80808080u;
        hy = (((hi >> 1) & 0x55u) * 0x02082080u) & 0x80808080u;
    } else {
#pragma unroll
        for (int j = 0; 2 * j < NE; ++j) {
            hx |= ((hi >> (2 * j)) & 1u) << (8 * j + 7);
            hy |= ((hi >> (2 * j + 1)) & 1u) << (8 * j + 7);
        }
    }
    const uint32_t XA = ((X >> 1) & 0x7F7F7F7Fu) | hx;
    const uint32_t YA = ((Y >> 1) & 0x7F7F7F7Fu) | hy;
    const uint32_t XS = (X << 2) & 0x1C1C1C1Cu, YS = (Y << 2) & 0x1C1C1C1Cu;
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int j = k >> 1;
        const uint32_t WA = (k & 1) ? YA : XA, WS = (k & 1) ? YS : XS;
        // ds_bpermute reads lane (addr >> 2) & 63: the bytes above j need no mask
        const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(WA >> (8 * j)), (int)T);
        out |= __builtin_amdgcn_ubfe(v, WS >> (8 * j), 4) << (4 * k);
#if QPD_VEC_CHAIN
        if (k + 1 < NE) asm("" : "+v"(out));  // one v_lshl_or per element, not shifts + v_or3
#endif
    }
    return out;
}

// The same NE lookups from the op's table staged as bytes in LDS (SCL-LUT's
// f / g ops: stage_tab, then lut_lds): entry i of the f table (256) or of the
// g table (512: u = 0, then u = 1) at byte i, read by ds_read_u8.  The address
// of element k is byte j = k/2 of X / Y (one v_bfe; for g, v_perm_b32 puts the
// u bit above it), and the result is the nibble itself: two VALU per lookup
// against about five for the bpermute form, whose address and nibble offset
// need a shift each and the result a field extract.  The f table's 64 dwords
// sit one per LDS bank (conflict-free); the g table's two halves share banks.
__device__ __forceinline__ uint32_t nib2byte4(uint32_t x) {  // nibbles 0-3 of x -> bytes 0-3
    x = (x | (x << 8)) & 0x00FF00FFu;
    return (x | (x << 4)) & 0x0F0F0F0Fu;
}

// Table dword `dw` (8 entries: f lanes & 31, g all 64 lanes) as 8 bytes at tb + 8 * dw.
__device__ __forceinline__ void stage_tab(uint8_t *tb, uint32_t T, int dw) {
    uint2 b;
    b.x = nib2byte4(T & 0xFFFFu);
    b.y = nib2byte4(T >> 16);
    *(uint2 *)(tb + 8 * dw) = b;
}

// Bank swizzle of the g table's u = 1 half (QPD_GSWZ, a multiple of 8): entry
// (1, i) sits at byte 256 + (i ^ QPD_GSWZ), so that the lookups of one path
// pair that differ only in u -- the common case: a frame's paths share their
// symbols and differ in their decisions -- fall on different LDS banks instead
// of two dwords of one bank (ds_read_u8 banking: (byte / 4) mod 32 per 32-lane
// half-wave).  Simulated on the bench workload (tools/bank_sim.py): the g
// lookups' conflict cycles 44 % -> 17 % with 72; measured (profiles/r06f_*):
// SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 15.8 % -> 10.0 % (SCL-LUT), 17.6 % ->
// 11.1 % (FastSCL-LUT) -- but 3.3 % / 1.5 % slower: the swizzle's VALU (the
// index bytes XOR u_byte * M: 6 per word of 8 lookups; 4 for M = 8, still -2.3 %)
// costs more than the conflicts, VALU issue being the kernel's nearest ceiling
// (a what-if without any conflicts and no extra VALU: +3.5 %).  Off; stage_tab
// puts the u = 1 chunks at lane ^ QPD_GSWZ / 8 (gtab_dw).
#ifndef QPD_GSWZ
#define QPD_GSWZ 0
#endif
__device__ __forceinline__ int gtab_dw(int lane) { return lane ^ ((lane >> 5) * (QPD_GSWZ >> 3)); }

// The staged tables sit at LDS offset TOFF of the wave's allocation (the kernel's
// `tb`, offset 0: lut_fast_kernel puts them first; qpd_capi.hip checks that the
// kernel declares no static LDS before them): the lookups address LDS through a
// constant, which the compiler folds into each ds_read_u8's offset field.
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
#ifndef QPD_LUT_PACK2
#define QPD_LUT_PACK2 1  // lut_lds: the 8 results combined as 16-bit pairs (see there)
#endif
#ifndef QPD_LUT_OPAQUE
#define QPD_LUT_OPAQUE 1  // lut_lds: the odd elements' word kept whole for the last shift-or (see there)
#endif
#ifndef QPD_LUT_OPAQUE_XY  // lut_lds: X, Y whole before the index extraction (-3 % static VALU; SCL-LUT +0.7 %,
#define QPD_LUT_OPAQUE_XY 1  // FastSCL-LUT +0.9 %, profiles/r06za_ab_lut_xy.txt)
#endif
template <int NE, bool ISG, int TOFF = 0>
__device__ __forceinline__ uint32_t lut_lds(uint32_t A, uint32_t B, uint32_t hi) {
    lds_u8 *const tb = (lds_u8 *)(size_t)TOFF;
    uint32_t X = ((A << 4) & 0xF0F0F0F0u) | (B & 0x0F0F0F0Fu);
    uint32_t Y = (A & 0xF0F0F0F0u) | ((B >> 4) & 0x0F0F0F0Fu);
    uint32_t hx = 0, hy = 0;  // byte j = bit 2j / 2j+1 of hi (g: the u half)
    if constexpr (ISG) {
        hx = (((hi & 0x55u) * 0x02082080u) >> 7) & 0x01010101u;
        hy = ((((hi >> 1) & 0x55u) * 0x02082080u) >> 7) & 0x01010101u;
        if constexpr (QPD_GSWZ != 0) {  // bytes of hx, hy are 0 / 1: X ^= hx * M by shifts (a
            uint32_t sx = 0, sy = 0;      // 32-bit multiply is a quarter-rate VALU op)
#pragma unroll
            for (int bit = 3; bit < 8; ++bit)
                if ((QPD_GSWZ >> bit) & 1) {
                    sx |= hx << bit;
                    sy |= hy << bit;
                }
            X ^= sx;
            Y ^= sy;
        }
    }
#if QPD_LUT_OPAQUE_XY
    // the words whole: otherwise the compiler rebuilds each index's byte from A and B
    // (v_and + v_bitop3 chains) beside X / Y themselves -- 15 VALU for 8 f indices, not 12
    asm("" : "+v"(X), "+v"(Y));
#endif
    uint32_t idx[NE];
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int j = k >> 1;
        const uint32_t W = (k & 1) ? Y : X;
        if constexpr (ISG)  // byte 0 = byte j of W, byte 1 = byte j of the u bits, bytes 2-3 = 0
            idx[k] = __builtin_amdgcn_perm((k & 1) ? hy : hx, W, (uint32_t)(j | ((4 + j) << 8) | (0x0C << 16) | (0x0C << 24)));
        else
            idx[k] = __builtin_amdgcn_ubfe(W, 8 * j, 8);
#if QPD_EXP_LUTMASK != 0xFFFF
        idx[k] &= QPD_EXP_LUTMASK;
#endif
    }
#if QPD_LUT_PACK2
    if constexpr (NE == 8) {
        // The even elements' bytes as [e0, e2, e4, e6] (16-bit pairs: the compiler
        // joins two loaded bytes with one v_perm), the odd ones' likewise, then one
        // shift-or: 7 VALU for the 8 results (4 v_perm, 3 v_lshl_or) instead of a
        // shift per element and an or3 per two.  O passes through an empty asm so
        // that the compiler does not distribute the final shift over O's two
        // halves (v_lshlrev x2 + v_or3 instead of one v_lshl_or: +1 VALU per word).
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const u16x2 r0 = {tb[idx[0]], tb[idx[4]]}, r1 = {tb[idx[2]], tb[idx[6]]};
        const u16x2 s0 = {tb[idx[1]], tb[idx[5]]}, s1 = {tb[idx[3]], tb[idx[7]]};
        const uint32_t E = __builtin_bit_cast(uint32_t, r0) | (__builtin_bit_cast(uint32_t, r1) << 8);
        uint32_t O = __builtin_bit_cast(uint32_t, s0) | (__builtin_bit_cast(uint32_t, s1) << 8);
#if QPD_LUT_OPAQUE
        asm("" : "+v"(O));
#endif
        return E | (O << 4);
    }
#endif
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < NE; ++k) out |= (uint32_t)tb[idx[k]] << (4 * k);
    return out;
}

// f / g op (SCLLUTDecoder.cpp:83-89 / :157-164): child symbols at depth d+1,
// for each of the wave's NS frame sets.  Words are processed in chunks whose
// loads are all issued before the first lookup: the shallow levels live in
// the global slab, and one memory round trip per chunk instead of per word is
// what bounds these ops.
// Source word of an f/g op; RAW: S[d] is a slab/LDS row (no channel / pre-pass
// reads), decided once per op instead of per word.
// SL >= 0: the row space of S[d] fixed at compile time (0 slab, 1 LDS).
template <bool RAW, int SL = -1>
__device__ __forceinline__ uint32_t fg_word(const FastPlan &P, const Mem &M, const MOp &op, const int32_t *y, int src, int w,
                                            int cnt = 8) {
    if constexpr (RAW) return M.ld(SL >= 0 ? SL != 0 : (op.flags & MF_SRC_LDS) != 0, op.src_row + w, src);
    return sym_word(P, M, op, y, src, w, cnt);
}

// f / g op at the root on the channel symbols (MF_CHAN: codes without the
// root pre-pass), a rolled loop over its words -- one copy of the channel
// reads (range check, error flag) instead of one per unrolled word.
template <bool ISG, int NS>
__device__ __forceinline__ void fg_chan_op(const FastPlan &P, const Mem (&M)[NS], const MOp &op, const int32_t *const (&y)[NS],
                                           const int (&usrc)[NS], uint32_t T, int lane) {
    const int ctemp = op.cnt;
    const bool dl = op.flags & MF_DST_LDS, ul = op.flags & MF_U_LDS;
    if (ctemp >= 8) {
        const int nwo = ctemp >> 3;
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll 1
            for (int w = 0; w < nwo; ++w) {
                const uint32_t a = chan_word8(y[s], 8 * w, P.in_vec, P.v, P.err);
                const uint32_t b = chan_word8(y[s], 8 * (nwo + w), P.in_vec, P.v, P.err);
                const uint32_t ub = ISG ? M[s].ld(ul, op.u_row + (w >> 2), usrc[s]) >> ((w & 3) << 3) : 0u;
                M[s].st(dl, op.dst_row + w, lane, lut_vec<8>(T, a, b, ub));
            }
    } else {  // ctemp in {2, 4}: the whole root (a then b) in one word
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const uint32_t W = chan_small(y[s], 2 * ctemp, P.v, P.err);
            const uint32_t ub = ISG ? M[s].ld(ul, op.u_row, usrc[s]) : 0u;
            const uint32_t out = ctemp == 4 ? lut_vec<4>(T, W, W >> 16, ub) : lut_vec<2>(T, W, W >> 8, ub);
            M[s].st(dl, op.dst_row, lane, out);
        }
    }
}

// LT: lookups from the byte table staged at tb (lut_lds) instead of T.
template <bool ISG, bool RAW, int NS, int SL = -1, int DL = -1, bool LT = false>
__device__ __forceinline__ void fg_op(const FastPlan &P, const Mem (&M)[NS], const MOp &op, const int32_t *const (&y)[NS],
                                      const int (&src)[NS], const int (&usrc)[NS], uint32_t T, int lane,
                                      const uint8_t *tb = nullptr) {
    const int ctemp = op.cnt;
    const bool dl = DL >= 0 ? DL != 0 : (op.flags & MF_DST_LDS) != 0, ul = op.flags & MF_U_LDS;
    if (ctemp >= 64) {
        const int nwo = ctemp >> 3;  // multiple of 8
        if constexpr (NS >= 2) {
            // chunks of 4 words of both sets: the sets' loads are in flight together
            for (int w0 = 0; w0 < nwo; w0 += 4) {
                uint32_t A[NS][4], B[NS][4], ub[NS];
#pragma unroll
                for (int s = 0; s < NS; ++s) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        A[s][k] = fg_word<RAW, SL>(P, M[s], op, y[s], src[s], w0 + k);
                        B[s][k] = fg_word<RAW, SL>(P, M[s], op, y[s], src[s], nwo + w0 + k);
                    }
                    ub[s] = ISG ? M[s].ld(ul, op.u_row + (w0 >> 2), usrc[s]) : 0u;
                }
#pragma unroll
                for (int s = 0; s < NS; ++s)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        M[s].st(dl, op.dst_row + w0 + k, lane,
                                LT ? lut_lds<8, ISG>(A[s][k], B[s][k], ub[s] >> (k << 3))
                                   : lut_vec<8>(T, A[s][k], B[s][k], ub[s] >> (k << 3)));
            }
        } else {
            for (int w0 = 0; w0 < nwo; w0 += 8) {
                uint32_t A[8], B[8], ub[2] = {0u, 0u};
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    A[k] = fg_word<RAW, SL>(P, M[0], op, y[0], src[0], w0 + k);
                    B[k] = fg_word<RAW, SL>(P, M[0], op, y[0], src[0], nwo + w0 + k);
                }
                if (ISG) {
                    ub[0] = M[0].ld(ul, op.u_row + (w0 >> 2), usrc[0]);
                    ub[1] = M[0].ld(ul, op.u_row + (w0 >> 2) + 1, usrc[0]);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    M[0].st(dl, op.dst_row + w0 + k, lane, lut_vec<8>(T, A[k], B[k], ub[k >> 2] >> ((k & 3) << 3)));
            }
        }
    } else if (ctemp >= 8) {
        const int nwo = ctemp >> 3;  // 1, 2 or 4
        uint32_t A[NS][4], B[NS][4], ub[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                A[s][k] = B[s][k] = 0u;
                if (k < nwo) {
                    A[s][k] = fg_word<RAW, SL>(P, M[s], op, y[s], src[s], k);
                    B[s][k] = fg_word<RAW, SL>(P, M[s], op, y[s], src[s], nwo + k);
                }
            }
            ub[s] = ISG ? M[s].ld(ul, op.u_row, usrc[s]) : 0u;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < nwo)
                    M[s].st(dl, op.dst_row + k, lane,
                            LT ? lut_lds<8, ISG>(A[s][k], B[s][k], ub[s] >> (k << 3))
                               : lut_vec<8>(T, A[s][k], B[s][k], ub[s] >> (k << 3)));
    } else {  // ctemp in {2, 4}: the whole depth-d node (a then b) is one word
        uint32_t W[NS], ub[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            W[s] = fg_word<RAW, SL>(P, M[s], op, y[s], src[s], 0, 2 * ctemp);
            ub[s] = ISG ? M[s].ld(ul, op.u_row, usrc[s]) : 0u;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const uint32_t out = ctemp == 4 ? lut_vec<4>(T, W[s], W[s] >> 16, ub[s]) : lut_vec<2>(T, W[s], W[s] >> 8, ub[s]);
            M[s].st(dl, op.dst_row, lane, out);
        }
    }
}

// f / g op with its left child's f folded in (MF_FF, fuse_descent in
// qpd_capi.hip): SCLLUTDecoder.cpp:83-89 / :157-164 at depth d, then :83-89
// at depth d+1.  Word u of S[d+2] is f(word u, word u + nwc) of S[d+1], both
// produced by this lane, so the child's inputs come from registers instead of
// a re-read of the row just stored (S[d+1] is still stored: the child's g
// reads it later).  Chunks of two S[d+2] words per set; S[d] in the slab.
// The op's table is staged at tb, the child's f table at tb + 512 (lut_lds).
template <bool ISG, int DL, int CDL, int NS>
__device__ __forceinline__ void ff_op(const Mem (&M)[NS], const MOp &op, const int (&src)[NS], const int (&usrc)[NS],
                                      const uint8_t *tb, int lane) {
    const int nwo = op.cnt >> 3, nwc = nwo >> 1;  // nwc even (op.cnt >= 32)
    const bool ul = op.flags & MF_U_LDS;
    for (int u0 = 0; u0 < nwc; u0 += 2) {
        uint32_t A[NS][4], B[NS][4], ub[NS][2], X[NS][4];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int w = (k < 2 ? 0 : nwc) + u0 + (k & 1);
                A[s][k] = M[s].ld(false, op.src_row + w, src[s]);
                B[s][k] = M[s].ld(false, op.src_row + nwo + w, src[s]);
            }
            ub[s][0] = ub[s][1] = 0u;
            if (ISG) {
                ub[s][0] = M[s].ld(ul, op.u_row + (u0 >> 2), usrc[s]);
                ub[s][1] = M[s].ld(ul, op.u_row + ((nwc + u0) >> 2), usrc[s]);
            }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int w = (k < 2 ? 0 : nwc) + u0 + (k & 1);
                X[s][k] = lut_lds<8, ISG>(A[s][k], B[s][k], ub[s][k >> 1] >> ((w & 3) << 3));
                M[s].st(DL != 0, op.dst_row + w, lane, X[s][k]);
            }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int k = 0; k < 2; ++k)
                M[s].st(CDL != 0, op.r_row + u0 + k, lane, lut_lds<8, false, 512>(X[s][k], X[s][k + 2], 0u));
    }
}

// Bit i of b (i < 8) -> nibble i all ones.
__device__ __forceinline__ uint32_t nib_mask(uint32_t b) {
    b &= 0xFFu;
    b = (b | (b << 12)) & 0x000F000Fu;
    b = (b | (b << 6)) & 0x03030303u;
    b = (b | (b << 3)) & 0x11111111u;
    return b * 15u;
}

// Root g in pre-mode (MF_GSEL; SCLLUTDecoder.cpp:157-164 at depth 0): the
// pre-pass row holds g(y, 0) and g(y, 1) of every root position, so the
// path's symbols are a nibble select by its left-half partial sums u.
template <int NS>
__device__ __forceinline__ void gsel_op(const Mem (&M)[NS], const MOp &op, const int32_t *const (&y)[NS],
                                        const int (&usrc)[NS], int lane) {
    const int nwo = op.cnt >> 3;  // 1, 2, 4 or a multiple of 8
    const bool dl = op.flags & MF_DST_LDS, ul = op.flags & MF_U_LDS;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const uint32_t *g = (const uint32_t *)y[s] + op.src_row;  // g(y, 0) words; g(y, 1) at + nwo
        for (int w0 = 0; w0 < nwo; w0 += 8) {
            uint32_t g0[8], g1[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                g0[k] = g1[k] = 0u;
                if (k == 0 || w0 + k < nwo) {
                    g0[k] = g[w0 + k];
                    g1[k] = g[nwo + w0 + k];
                }
            }
            const uint32_t u0 = M[s].ld(ul, op.u_row + (w0 >> 2), usrc[s]);
            const uint32_t u1 = nwo - w0 > 4 ? M[s].ld(ul, op.u_row + (w0 >> 2) + 1, usrc[s]) : 0u;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (k == 0 || w0 + k < nwo) {
                    const uint32_t m = nib_mask((k < 4 ? u0 : u1) >> ((k & 3) << 3));
                    M[s].st(dl, op.dst_row + w0 + k, lane, g0[k] ^ ((g0[k] ^ g1[k]) & m));
                }
        }
    }
}

// Per-lane argsort arrays (global scratch) for the R1 node; rows of this set
// (stride `rs` words, see Mem), a key's double as two rows (low, high word).
struct FastSortSeq {
    uint32_t *glb;
    int io, ko, lane, rs;
    __device__ int get(int p) { return (int)glb[(size_t)(io + p) * rs + lane]; }
    __device__ void set(int p, int e) { glb[(size_t)(io + p) * rs + lane] = (uint32_t)e; }
    __device__ double key(int e) {
        const uint64_t lo = glb[(size_t)(ko + 2 * e) * rs + lane], hi = glb[(size_t)(ko + 2 * e + 1) * rs + lane];
        return __builtin_bit_cast(double, lo | (hi << 32));
    }
    __device__ bool less(int a, int b) { return key(a) < key(b); }
};

// Prefetch of the per-op operands held in registers.
struct Pre {
    uint32_t T;   // f or g table dword of this lane
    uint32_t T2;  // MF_BFG: the folded parent op's table dword
    double V;     // leaf: vcl row entry of this lane (lanes < v)
};

__device__ __forceinline__ Pre fetch_pre(const FastPlan &P, const MOp &op, int lane, int vlane) {
    Pre p;
    p.T = p.T2 = 0;
    p.V = 0;
    if (op.type == OP_F || op.type == OP_LEAF_L) p.T = tab_ld(P.f_tab, op.tab * QPD_EXP_TABMUL, lane & 31);
    if ((op.type == OP_G && !(op.flags & MF_GSEL)) || op.type == OP_LEAF_R) p.T = tab_ld(P.g_tab, op.tab * QPD_EXP_TABMUL, lane);
    if ((op.type == OP_F || op.type == OP_G) && (op.flags & MF_FF)) p.T2 = tab_ld(P.f_tab, op.tab2 * QPD_EXP_TABMUL, lane & 31);
    if (op.type == OP_BOT3) {
        p.T = tab_ld(P.f_tab, op.tab * QPD_EXP_TABMUL * 32, lane & 31);
        if (op.flags & MF_BFG)
            p.T2 = (op.flags & MF_BG) ? tab_ld(P.g_tab, op.tab2 * QPD_EXP_TABMUL, lane)
                                      : tab_ld(P.f_tab, op.tab2 * QPD_EXP_TABMUL, lane & 31);
    }
    if (op.type == OP_LEAF_L || op.type == OP_LEAF_R) p.V = P.vcl[op.vrow + vlane];
    if (op.type >= OP_R0 && op.type <= OP_SPC && (op.flags & MF_SFG))  // the folded parent's table (tab)
        p.T2 = (op.flags & MF_SGG) ? tab_ld(P.g_tab, op.tab, lane) : tab_ld(P.f_tab, op.tab, lane & 31);
    return p;
}

// ---------------------------------------------------------------------------
// List state and the fork (mink, SCLLUTDecoder.cpp:105-144).
//
// The speculative right-leaf lookup (bot_pair): +1.3 % at 4 waves per SIMD,
// -1 % at the 5 the SCL-LUT kernel runs now (its registers; r04g / r04j): off.
#ifndef QPD_SPEC_RIGHT
#define QPD_SPEC_RIGHT 0
#endif
// A wave runs NS independent frame sets through the same op stream.  The op
// records, the per-node tables and all scalar control are shared; the sets'
// dependency chains (LDS lookups, survivor selection, fork shuffles) are
// independent and interleave, which hides the LDS latency that bounds a
// single set.
// ---------------------------------------------------------------------------
// A path's metric and slot pointers: ps holds the S-row pointer fields, pu
// the U-row ones.  PW1: the host packed every field the op list uses into one
// word (at most 16 of them: SCL-LUT up to N = 2048, qpd_capi.hip:
// compact_pointer_fields), so U() is the same word -- two registers and two
// shuffles per fork less per frame set.
template <bool PW1>
struct PathT;
template <>
struct PathT<false> {
    double pm;
    uint64_t ps, pu;
    __device__ __forceinline__ uint64_t &U() { return pu; }
    __device__ __forceinline__ void move(int p) {  // take lane p's pointers (a fork)
        ps = shfl64(ps, p);
        pu = shfl64(pu, p);
    }
};
template <>
struct PathT<true> {
    double pm;
    uint64_t ps;
    __device__ __forceinline__ uint64_t &U() { return ps; }
    __device__ __forceinline__ void move(int p) { ps = shfl64(ps, p); }
};

// Move every set's state one slot down (set s + 1 into slot s, slot 0 to the
// end): a loop over the sets that runs set s in slot 0 has its own state back
// in place after NS steps.
template <class T, int NS>
__device__ __forceinline__ void rotate_sets(T (&a)[NS]) {
    if constexpr (NS > 1) {
        T t = a[0];
#pragma unroll
        for (int i = 0; i + 1 < NS; ++i) a[i] = a[i + 1];
        a[NS - 1] = t;
    }
}
template <class T, int NS, int W>
__device__ __forceinline__ void rotate_sets(T (&a)[NS][W]) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
        T c[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) c[i] = a[i][w];
        rotate_sets(c);
#pragma unroll
        for (int i = 0; i < NS; ++i) a[i][w] = c[i];
    }
}

constexpr int kSelInts = 128;  // per set: 64 slots + 64 junk slots (select_survivors8): two rows after the set's

// max of two non-negative doubles given as bits (one v_max_f64).
__device__ __forceinline__ uint64_t dmax_bits(uint64_t a, uint64_t b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(__builtin_bit_cast(double, a)), "v"(__builtin_bit_cast(double, b)));
    return __builtin_bit_cast(uint64_t, r);
}

// max(-x, 0) in one v_max_f64 (the builtin would canonicalize its operand first).
__device__ __forceinline__ double neg_max0(double x) {
    double r;
    asm("v_max_f64 %0, -%1, 0" : "=v"(r) : "v"(x));
    return r;
}

// Identity test of the L = 8 survivor selection, for every lane group of the
// wave at once: the keeps K_j (this lane's keep key) are already in stable
// order (K_0 <= ... <= K_7) and no flip F_j beats the largest keep (a flip
// equal to a keep loses the tie: its candidate index is higher).  The stable
// sort of the 16 candidates then puts keep_j in slot j -- nothing moves and
// no flip survives.  Keys are >= +0 or +inf, never NaN (a NaN metric raises
// ERR_NAN_PM in the generic engine; LUT quanta are finite): max over doubles =
// max over their bits.  v_max_f64 by inline asm: the builtin would
// canonicalize the DPP operands first (two more VALU per step).
//
// First a conservative test on the high words alone (sign, exponent and the
// top 20 mantissa bits; keys are >= +0, so a larger high word is a larger
// double): strictly increasing keeps and every flip strictly above the
// largest keep's high word imply the identity.  32-bit words take the DPP
// lane moves inside the max / compare instructions (one VALU per step instead
// of two moves and a v_max_f64); only when it cannot decide (equal high words:
// near-ties) does the exact 64-bit test run.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
}

__device__ __forceinline__ bool keep_all8(uint64_t K, uint64_t F, int gl) {
#if defined(QPD_EXP_IDENT)  // timing experiments only (wrong results): every selection the identity / none
    return QPD_EXP_IDENT;
#endif
#ifdef QPD_HI_IDENT  // measured -0.5 % on SCL-LUT (r04e): off
    {
        const uint32_t kh = (uint32_t)(K >> 32), fh = (uint32_t)(F >> 32);
        uint32_t m = kh;
        m = max(m, dpp32<kDppXor1>(m));
        m = max(m, dpp32<kDppXor2>(m));
        m = max(m, dpp32<kDppHalfMirror>(m));
        const uint32_t khn = dpp32<kDppRowShl1>(kh);
        // lanes with gl == 7 (every 8th) have no next slot: their sortedness bit is set
        const uint64_t up = __builtin_amdgcn_ballot_w64(fh > m);
        const uint64_t srt = __builtin_amdgcn_ballot_w64(khn > kh) | 0x8080808080808080ull;
        if ((up & srt) == ~0ull) return true;
    }
#endif
#ifndef QPD_IDENT_MAX  // the group maximum by a 3-step DPP reduction (round 3): 1.1 % slower (r04q)
    // With the keeps in order the largest is slot 7's, so no reduction: lanes
    // 4-7 of each group take K_7 (quad broadcast) and the flips of slots 7-4
    // (own) and 3-0 (half-row mirror) and compare both -- three independent
    // lane moves instead of a dependent max chain.  (Unordered keeps fail the
    // order ballot whatever K_7 is.)
    const uint64_t k7 = dpp64<kDppQuadBcast3>(K);
    const uint64_t fm = dpp64<kDppHalfMirror>(F);
    const uint64_t Kn = dpp64<kDppRowShl1>(K);  // keep of slot gl+1
    (void)gl;
    const uint64_t up = (__builtin_amdgcn_ballot_w64(F >= k7) & __builtin_amdgcn_ballot_w64(fm >= k7)) | 0x0F0F0F0F0F0F0F0Full;
    return (up & (__builtin_amdgcn_ballot_w64(K <= Kn) | 0x8080808080808080ull)) == ~0ull;
#else
    uint64_t mk = K;
    mk = dmax_bits(mk, dpp64<kDppXor1>(mk));
    mk = dmax_bits(mk, dpp64<kDppXor2>(mk));
    mk = dmax_bits(mk, dpp64<kDppHalfMirror>(mk));  // lane i^7 lies in the other quad
    const uint64_t Kn = dpp64<kDppRowShl1>(K);       // keep of slot gl+1
    (void)gl;
    return (__builtin_amdgcn_ballot_w64(F >= mk) & (__builtin_amdgcn_ballot_w64(K <= Kn) | 0x8080808080808080ull)) == ~0ull;
#endif
}

// ---------------------------------------------------------------------------
// List sizes 9..16 (LM = 16: lane groups of 16 = one DPP row, 4 frames per
// set).  mink (SCLLUTDecoder.cpp:8-21) sorts 2L > 16 candidates, so libstdc++
// runs its introsort, which is NOT stable: with tied keys the survivors' order
// is whatever the partitions leave (H1).  Without ties every correct sort
// gives the same first L outputs, so the kernel ranks by counting and replays
// the introsort only for a group whose first L ranks hold a tie:
//  * strict identity (keep_all16): keeps strictly increasing, every flip
//    strictly above the largest keep -- the unique sorted order puts keep j in
//    slot j whatever the algorithm;
//  * select_survivors16: dense key ranks against the 15 row partners by DPP
//    row rotations, then every group replays libstdc++'s partitions
//    (stl::partition_prefix, stl_sort.hpp) on its 2L ranks in parallel (scan-stop
//    masks, all of a partition's swaps at once); only a group that reaches the
//    introsort's depth limit replays stl::sort_small_prefix serially on its first lane.
// Candidates are encoded keep j -> j, flip j -> 16 + j (flips after keeps, as
// the reference's indices j < L <= L + j); lanes gl >= L are padding (+inf
// keys, never scattered below L).
// ---------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ uint32_t dpp_ror(uint32_t x) {  // rotate within a row of 16 lanes
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x120 + R, 0xF, 0xF, false);
}
template <int R>
__device__ __forceinline__ uint64_t dpp_ror64(uint64_t x) {
    return ((uint64_t)dpp_ror<R>((uint32_t)(x >> 32)) << 32) | dpp_ror<R>((uint32_t)x);
}

__device__ __forceinline__ bool keep_all16(uint64_t K, uint64_t F, int gl, int gbase, int L) {
    const uint64_t Kn = dpp64<kDppRowShl1>(K);  // keep of slot gl + 1
    const uint64_t kl = shfl64(K, gbase + L - 1);
    const bool ok = (gl >= L - 1 || K < Kn) && (gl >= L || F > kl);
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// Dense key ranks: how many of the group's candidates have a strictly smaller
// key than this lane's keep / flip, counted against the 15 row partners (DPP
// row rotations).  lt preserves the order of the keys among the 2L
// candidates exactly (x < y <=> lt_x < lt_y), so the introsort replay below
// compares 5-bit ranks instead of doubles.  Padding lanes carry +inf: never
// smaller than anything.
template <int R>
__device__ __forceinline__ void lt16_all(uint64_t K, uint64_t F, int &lk, int &lf) {
    if constexpr (R < 16) {
        const uint64_t ok = dpp_ror64<R>(K), of = dpp_ror64<R>(F);
        lk += ok < K;
        lk += of < K;
        lf += ok < F;
        lf += of < F;
        lt16_all<R + 1>(K, F, lk, lf);
    }
}

// Index array of the serial replay in LDS (stl_sort.hpp Seq): keys by reference index.
struct SelReplay16 {
    int *idx;
    const double *key;
    __device__ int get(int p) { return idx[p]; }
    __device__ void set(int p, int e) { idx[p] = e; }
    __device__ bool less(int a, int b) { return key[a] < key[b]; }
};

// The group's array of 2L entries (lt << 5 | reference index), position p in
// lane p (p < L) or lane p - L (p >= L, upper half-word): every lane holds
// its keep's and its flip's starting positions.  w16_rd: the entry at a
// group-uniform position (a ds_bpermute: the whole wave executes it);
// w16_wr: this lane's word with that position's entry replaced.
__device__ __forceinline__ uint32_t w16_rd(uint32_t E, int gbase, int L, int p) {
    const bool hi = p >= L;
    const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((gbase + (hi ? p - L : p)) << 2, (int)E);
    return hi ? w >> 16 : w & 0xFFFFu;
}
__device__ __forceinline__ uint32_t w16_wr(uint32_t E, int gl, int L, int p, uint32_t e) {
    const bool hi = p >= L;
    if (gl != (hi ? p - L : p)) return E;
    return hi ? (E & 0xFFFFu) | (e << 16) : (E & 0xFFFF0000u) | e;
}

// The group's mask of positions (bit p) whose flag is set, from the lanes'
// flags for their two positions (ballots; every lane gets its group's mask).
__device__ __forceinline__ uint32_t w16_mask(bool c0, bool c1, int gbase, int L) {
    const uint64_t b0 = __builtin_amdgcn_ballot_w64(c0), b1 = __builtin_amdgcn_ballot_w64(c1);
    const uint32_t m = (1u << L) - 1u;
    return ((uint32_t)(b0 >> gbase) & m) | (((uint32_t)(b1 >> gbase) & m) << L);
}

// Ranks of this lane's two packed u16 composites against the row partners' (R..15 lanes away).
template <int R, class LessM, class V>
__device__ __forceinline__ void rank16_packed(uint32_t X, LessM &lessm, V &acc) {
    if constexpr (R < 16) {
        const uint32_t Y = dpp_ror<R>(X);
        acc += lessm(__builtin_bit_cast(V, Y));
        acc += lessm(__builtin_bit_cast(V, __builtin_amdgcn_alignbit(Y, Y, 16)));
        rank16_packed<R + 1>(X, lessm, acc);
    }
}

__device__ __forceinline__ Sel select_survivors16(double kk, double kf, int gl, int gbase, int L, int lane, int *sel,
                                                  int sj) {
    const uint64_t kInfBits = 0x7ff0000000000000ull;
    const bool pad = gl >= L;
    const uint64_t K = pad ? kInfBits : __builtin_bit_cast(uint64_t, kk);
    const uint64_t F = pad ? kInfBits : __builtin_bit_cast(uint64_t, kf);
    int lk = F < K, lf = K < F;
    lt16_all<1>(K, F, lk, lf);
    uint32_t E = pad ? 0xFFFFFFFFu : (((uint32_t)lk << 5) | (uint32_t)gl) | ((((uint32_t)lf << 5) | (uint32_t)(L + gl)) << 16);
    // stl::partition_prefix(seq, 0, 2L, L) replayed by each group on its array
    // (libstdc++ __introsort_loop's partitions, stl_sort.hpp): group-uniform f,
    // l, depth limit and end in every lane of the group.
    const int n2 = 2 * L;
    int f = 0, l = n2, dl = 2 * stl::lg(n2), end = n2;
    bool live = true, serial = false;
#pragma unroll 1
    while (__builtin_amdgcn_ballot_w64(live)) {
        if (live && dl == 0) {  // heap-sort fallback: the group replays serially below
            serial = true;
            live = false;
        }
        --dl;
        const int mid = f + (l - f) / 2;
        // move_median_to_first(f, f + 1, mid, l - 1) on the ranks
        const uint32_t ea = w16_rd(E, gbase, L, f + 1), eb = w16_rd(E, gbase, L, mid), ec = w16_rd(E, gbase, L, l - 1);
        const uint32_t ef = w16_rd(E, gbase, L, f);
        const uint32_t ra = ea >> 5, rb = eb >> 5, rc = ec >> 5;
        int pick;
        if (ra < rb) pick = rb < rc ? mid : ra < rc ? l - 1 : f + 1;
        else pick = ra < rc ? f + 1 : rb < rc ? l - 1 : mid;
        const uint32_t em = pick == mid ? eb : pick == f + 1 ? ea : ec;
        if (live) {
            E = w16_wr(E, gl, L, f, em);
            E = w16_wr(E, gl, L, pick, ef);
        }
        // unguarded_partition(f + 1, l, pivot f): the left scan stops at ranks >= the
        // pivot's, the right scan at ranks <= it.  A swap leaves the untouched
        // positions as they were, so the k-th stops are the k-th such positions of
        // the array before the partition (from the left / from the right) while they
        // have not crossed; the scan that then runs on stops at the last right stop
        // at the latest (its swapped-in entry): cut = min(next left stop, last right stop).
        // All swaps at once: every stop position learns its rank among the left /
        // right stops (popcounts of the masks), publishes itself in the group's byte
        // slots (left stops at [0, 32), right stops at [32, 64) of the set's selection
        // scratch) and reads the stop of the same rank on the other side: the k-th pair
        // swaps iff its left stop lies below its right stop (a prefix of the k), and a
        // position is in at most one swapping pair.
        const uint32_t pv = em >> 5;
        const uint32_t in = ((l < 32 ? (1u << l) : 0u) - 1u) & ~((2u << f) - 1u);  // positions [f + 1, l)
        const uint32_t r0 = (E & 0xFFFFu) >> 5, r1 = E >> 21;
        const uint32_t GE = w16_mask(!pad && r0 >= pv, !pad && r1 >= pv, gbase, L) & in;
        const uint32_t LE = w16_mask(!pad && r0 <= pv, !pad && r1 <= pv, gbase, L) & in;
        uint8_t *const slot = (uint8_t *)sel + 4 * gbase;  // the group's 64 bytes
        const int q[2] = {gl, L + gl};
        int kA[2], kB[2];
        bool ge[2], le[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            ge[h] = !pad && ((GE >> q[h]) & 1u);
            le[h] = !pad && ((LE >> q[h]) & 1u);
            kA[h] = __builtin_popcount(GE & ((1u << q[h]) - 1u));                      // rank from the left
            kB[h] = __builtin_popcount(LE & ~((q[h] < 31 ? (2u << q[h]) : 0u) - 1u));  // rank from the right
            if (live && ge[h]) slot[kA[h]] = (uint8_t)q[h];
            if (live && le[h]) slot[32 + kB[h]] = (uint8_t)q[h];
        }
        lds_order();
        const int nA = __builtin_popcount(GE), nB = __builtin_popcount(LE);
        int part[2];
        bool lsw[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            part[h] = q[h];
            lsw[h] = false;
            const int bk = ge[h] && kA[h] < nB ? slot[32 + kA[h]] : -1;  // this left stop's right partner
            const int ak = le[h] && kB[h] < nA ? slot[kB[h]] : 64;       // this right stop's left partner
            if (q[h] < bk) {
                part[h] = bk;
                lsw[h] = true;
            } else if (ak < q[h]) {
                part[h] = ak;
            }
        }
        const int S = __builtin_popcount(w16_mask(lsw[0], lsw[1], gbase, L));  // swaps of this partition
        const int cut_a = S < nA ? slot[S] : n2, cut_b = S >= 1 ? slot[32 + S - 1] : n2;
        lds_order();
        const uint32_t x0 = w16_rd(E, gbase, L, part[0]), x1 = w16_rd(E, gbase, L, part[1]);
        if (live && !pad) E = x0 | (x1 << 16);
        if (live) {
            const int cut = cut_a < cut_b ? cut_a : cut_b;
            if (cut >= L && cut < end) end = cut;  // a block boundary past the first L positions
            if (l - cut > stl::kThreshold) {
                if (cut >= end) live = false;  // the reference's recursion on [cut, l) lies past the prefix
                else f = cut;
            } else {
                l = cut;
            }
            live = live && l - f > stl::kThreshold;
        }
    }
    // The final insertion sort of [0, end) is stable on the positions the partitions
    // left: its first L outputs are the L smallest (rank, position) -- ranks of the
    // composites (lt << 5 | position) counted against the row partners, packed u16.
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const uint32_t p0 = (uint32_t)gl, p1 = (uint32_t)(L + gl);
    const uint32_t c0 = !pad && (int)p0 < end ? ((E & 0xFFE0u) | p0) : 0xFFFFu;
    const uint32_t c1 = !pad && (int)p1 < end ? (((E >> 16) & 0xFFE0u) | p1) : 0xFFFFu;
    const u16x2 X = __builtin_bit_cast(u16x2, c0 | (c1 << 16));
    const u16x2 one = {1, 1};
    auto lessm = [&](u16x2 y) { return __builtin_elementwise_min(__builtin_elementwise_sub_sat(X, y), one); };  // 1: y < x
    u16x2 R = lessm(__builtin_bit_cast(u16x2, __builtin_amdgcn_alignbit(c0 | (c1 << 16), c0 | (c1 << 16), 16)));
    rank16_packed<1>(c0 | (c1 << 16), lessm, R);
    const int rk0 = R.x, rk1 = R.y;
    const uint32_t cand0 = E & 31u, cand1 = (E >> 16) & 31u;
    sel[rk0 < L && !pad ? gbase + rk0 : sj + lane] = (int)(cand0 < (uint32_t)L ? cand0 : cand0 - L + 16);
    sel[rk1 < L && !pad ? gbase + rk1 : sj + lane] = (int)(cand1 < (uint32_t)L ? cand1 : cand1 - L + 16);
    lds_order();
    int c = pad ? gl : sel[gbase + gl];
    lds_order();
    const uint64_t slow = __builtin_amdgcn_ballot_w64(serial);
    if (slow) {
        // groups that reached the depth limit (heap-sort fallback), one after the other:
        // the whole replay on the group's first lane, keys by reference index at sel
        // (2L <= 32 doubles), the index array at the junk slots (2L ints)
        double *key = (double *)sel;
        int *idx = sel + sj;
#pragma unroll 1
        for (int g = 0; g < 64; g += 16) {
            if (!((slow >> g) & 0xFFFFull)) continue;
            if (gbase == g && !pad) {
                key[gl] = kk;
                key[L + gl] = kf;
            }
            lds_order();
            if (lane == g) {
                SelReplay16 seq{idx, key};
                for (int p = 0; p < 2 * L; ++p) idx[p] = p;
                stl::sort_small_prefix(seq, 0, 2 * L, L);  // libstdc++'s steps, first L outputs
            }
            lds_order();
            if (gbase == g && !pad) {
                const int e = idx[gl];
                c = e < L ? e : e - L + 16;
            }
            lds_order();
        }
    }
    Sel s;
    s.upper = c >= 16;
    s.parent = c & 15;
    return s;
}

// Info leaf with quanta dm: keep the L best of {keep, flip} candidates.
// Returns the new decision; `extra` words follow the surviving lineage.
// `moved` (wave-uniform): the selection was not the identity (paths moved).
// LM: the list mode -- 8 (L = 8, groups of 8: DPP ranks), 16 (L = 9..16,
// groups of 16), 0 (L <= 8, the generic stable ranks).
template <int LM, int NX, class Path>
__device__ __forceinline__ uint32_t leaf_fork(Path &st, double dm, int gl, int gbase, int L, int lane, int *sel, int sj,
                                              uint32_t (&extra)[NX], bool &moved) {
    const double kf = st.pm + fabs(dm);
    const uint32_t hd = dm < 0;  // H4: SCL family `< 0`
    // Fast path (about 2/3 of the info leaves on the bench channel): the
    // selection is the identity, the decision the hard one.
    moved = false;
    if constexpr (LM == 8)
        if (keep_all8(__builtin_bit_cast(uint64_t, st.pm), __builtin_bit_cast(uint64_t, kf), gl)) return hd;
    if constexpr (LM == 16)
        if (keep_all16(__builtin_bit_cast(uint64_t, st.pm), __builtin_bit_cast(uint64_t, kf), gl, gbase, L)) return hd;
    moved = true;
    const Sel sl = LM == 8    ? select_survivors8(st.pm, kf, gl, gbase, lane, sel, sj)
                   : LM == 16 ? select_survivors16(st.pm, kf, gl, gbase, L, lane, sel, sj)
                              : select_survivors(st.pm, kf, gl, gbase, L, sel);
    const int p = gbase + sl.parent;
    const uint32_t dec = (uint32_t)lane_read((int)hd, p) ^ (sl.upper ? 1u : 0u);
    st.pm = pick(sl.upper, shfld(kf, p), shfld(st.pm, p));
    st.move(p);
#pragma unroll
    for (int i = 0; i < NX; ++i) extra[i] = (uint32_t)lane_read((int)extra[i], p);
    return dec;
}

// One leaf decision for every set.  `frozen` is wave-uniform.
template <bool kList, int LM, int NS, int NX, class Path>
__device__ __forceinline__ void leaf_decide(Path (&st)[NS], const double (&dm)[NS], bool frozen, int gl, int gbase,
                                            int L, int lane, int *sel, int sstride, uint32_t (&extra)[NS][NX],
                                            uint32_t (&dec)[NS], bool (&moved)[NS]) {
#pragma unroll
    for (int s = 0; s < NS; ++s) moved[s] = false;
    if (!kList) {
#pragma unroll
        for (int s = 0; s < NS; ++s) dec[s] = frozen ? 0u : (uint32_t)(dm[s] <= 0);  // H4: SC family `<= 0`
        return;
    }
    if (frozen) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            // :100-104, |dm|·(dm<0) = max(-dm, 0): the same double (|dm|·1 = |dm| for
            // dm < 0; otherwise +0, or -0 for dm = +0, and pm + -0 = pm: pm is never -0)
            st[s].pm += neg_max0(dm[s]);
            dec[s] = 0u;
        }
        return;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
        dec[s] = leaf_fork<LM>(st[s], dm[s], gl, gbase, L, lane, sel + sstride * s, NS * sstride, extra[s], moved[s]);
}

// ---------------------------------------------------------------------------
// BOT3: the height-3 subtree under a depth n-3 node, fully in registers.
// Node numbering inside the subtree (posi): q0 = p0; q1,q2 = 2p0+1, 2p0+2;
// q3..q6 = 4p0+3 .. 4p0+6; leaves k0..k0+7 (k0 = 8*node).
// In-register lineage state per set: x[0] = W3 (8 symbols of q0) and x[1] =
// W2 (bits 0-15, 4 symbols of the current depth n-2 node) | W1 (bits 16-23,
// 2 symbols) | bL (bit 24, left leaf decision) | c2 (bits 25-26, left result
// at depth n-1) | c3 (bits 27-30, left result at depth n-2).
// ---------------------------------------------------------------------------
// Leaf lookups (the depth n-1 node's f / g table, lut4) of the leaf pair whose
// symbols a, b are nibbles 4, 5 of x1 (and, for g, the left decision u bit 24):
// QPD_LEAF_T = 1 -- the host stores the depth n-1 tables transposed (entry
// u * 256 + b * 16 + a, fast_tables in qpd_capi.hip), so the index is x1's
// bits 16..23 (..24) as they lie: one field extract instead of two extracts, a
// shift and an or per leaf.
#ifndef QPD_LEAF_T
#define QPD_LEAF_T 1
#endif
__device__ __forceinline__ uint32_t leaf_idx(uint32_t x1) {
    if constexpr (QPD_LEAF_T) return __builtin_amdgcn_ubfe(x1, 16, 8);
    return (((x1 >> 16) & 15u) << 4) | ((x1 >> 20) & 15u);
}
__device__ __forceinline__ uint32_t leaf_idx_g(uint32_t x1) {  // with u = bit 24
    if constexpr (QPD_LEAF_T) return __builtin_amdgcn_ubfe(x1, 16, 9);
    return (((x1 >> 24) & 1u) << 8) | leaf_idx(x1);
}

__device__ __forceinline__ uint32_t f_pair(uint32_t T, uint32_t hi, uint32_t w2) {  // 2 symbols of f(W2)
    return lut_vec<2>(T, w2, w2 >> 8, hi);
}
__device__ __forceinline__ uint32_t g_pair(uint32_t T, uint32_t c2, uint32_t w2) {  // 2 symbols of g(W2, c2)
    return lut_vec<2>(T, w2, w2 >> 8, c2);
}

template <bool kList, int LM, bool SPEC, int NS, class Path>
__device__ __forceinline__ void bot_pair(Path (&st)[NS], uint32_t (&x)[NS][2], uint32_t Tf, int fo, uint32_t Tg,
                                         double V, int vo, int fr, int gl, int gbase, int L, int lane, int *sel, int sstride,
                                         uint32_t (&c)[NS]) {
    double dm[NS];
    uint32_t bl[NS], br[NS];
    bool moved[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        dm[s] = 0;
        if (kList || !(fr & 1)) dm[s] = shfld(V, vo + (int)lut4(Tf, leaf_idx(x[s][1]) + fo));
    }
#if QPD_SPEC_RIGHT  // (SPEC: SCL-LUT; the FastSCL unit measured slower with it)
    // The right leaf's quanta for the decision the left leaf takes when its
    // selection is the identity (its hard decision, or 0 if frozen), looked up
    // before the left fork's test resolves: the lookup latency leaves the
    // chain of the ~2/3 of forks that move nothing; a fork that moves paths
    // looks it up again from the surviving lineage's word.
    double sdm[NS];
    if constexpr (kList && LM == 8 && SPEC) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const uint32_t hb = (fr & 1) ? 0u : (uint32_t)(dm[s] < 0);  // H4: SCL family `< 0`
            sdm[s] = shfld(V, vo + 16 + (int)lut4(Tg, (hb << 8) | leaf_idx(x[s][1])));
        }
    }
#endif
    leaf_decide<kList, LM>(st, dm, fr & 1, gl, gbase, L, lane, sel, sstride, x, bl, moved);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        x[s][1] = (x[s][1] & ~(1u << 24)) | (bl[s] << 24);
#if QPD_SPEC_RIGHT
        if constexpr (kList && LM == 8 && SPEC) {
            dm[s] = sdm[s];
            if (moved[s]) dm[s] = shfld(V, vo + 16 + (int)lut4(Tg, leaf_idx_g(x[s][1])));
            continue;
        }
#endif
        if (kList || !(fr & 2)) dm[s] = shfld(V, vo + 16 + (int)lut4(Tg, leaf_idx_g(x[s][1])));
    }
    leaf_decide<kList, LM>(st, dm, fr & 2, gl, gbase, L, lane, sel, sstride, x, br, moved);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const uint32_t bl2 = (x[s][1] >> 24) & 1u;
        c[s] = (bl2 ^ br[s]) | (br[s] << 1);
    }
}

// The subtree runs in four stages -- A: q0 left + leaves 0, 1; B: q1 g +
// leaves 2, 3; C: q0 right + leaves 4, 5; D: q2 g + leaves 6, 7 -- and each
// stage issues the table / quanta loads of the next one (LAZY: SCL-LUT, with
// QPD_BOT3_LAZY; +0.5 % there at 5 waves, r04h), so at most about
// 11 of them are live at once: the register budget of a fifth wave per SIMD.
// `prefetch_next` issues the next op's operand prefetch at the start of stage
// D instead of at the start of this op (4 registers less through stages A-C).
#ifndef QPD_BOT3_LAZY
#define QPD_BOT3_LAZY 1
#endif
// LT: the folded parent's lookups (MF_BFG) from its table staged as bytes at tb (lut_lds).
template <bool kList, int LM, bool LAZY, bool LT, bool CH, int NS, class PF, class Path>
__device__ __forceinline__ void bot3_op(const FastPlan &P, const Mem (&M)[NS], const MOp &op,
                                        const int32_t *const (&y)[NS], Path (&st)[NS], uint32_t Tf0, uint32_t T2, int gl,
                                        int gbase, int L, int *sel, int sstride, int lane, PF &&prefetch_next,
                                        uint8_t *tb) {
    const int p0 = op.tab * QPD_EXP_TABMUL;
    const int fr = op.cnt;
    const uint32_t *ft = P.f_tab, *gt = P.g_tab;
    // Tables of the 7 internal nodes (q0's f table arrives prefetched).  Two
    // 32-dword f tables share one register (lanes 0-31 | 32-63: p and p+1 are
    // adjacent), addressed by adding 256 to the nibble index of the second.
    const int p1 = 2 * p0 + 1, p3 = 4 * p0 + 3;
    // Leaf quanta vcl[n-1][8*node + j][s] of the 8 leaves, four leaves per
    // register: lane 16*jj + s holds leaf 4*h + jj (v <= 16).
    const int v = P.v;
    const int s16 = lane & 15, j16 = lane >> 4;
    const double *vb = P.vcl + op.vrow * QPD_EXP_TABMUL;
    // stage A's operands, and B's
    const uint32_t Tf12 = tab_ld(ft, p1 * 32, lane);
    const uint32_t Tf34 = tab_ld(ft, p3 * 32, lane), Tg3 = tab_ld(gt, p3 * 64, lane);
    const double Vlo = s16 < v ? vb[j16 * v + s16] : 0.0;
    const uint32_t Tg1 = tab_ld(gt, p1 * 64, lane), Tg4 = tab_ld(gt, (p3 + 1) * 64, lane);
    uint32_t Tg0 = 0, Tf56 = 0, Tg5 = 0, Tg2 = 0, Tg6 = 0;
    double Vhi = 0.0;
    if constexpr (!LAZY) {
        Tg0 = tab_ld(gt, p0 * 64, lane);
        Tf56 = tab_ld(ft, (p3 + 2) * 32, lane);
        Tg5 = tab_ld(gt, (p3 + 2) * 64, lane);
        Tg2 = tab_ld(gt, (p1 + 1) * 64, lane);
        Tg6 = tab_ld(gt, (p3 + 3) * 64, lane);
        Vhi = s16 < v ? vb[(4 + j16) * v + s16] : 0.0;
    }
    uint32_t x[NS][2], c[NS];
    if (op.flags & MF_BFG) {
        // The depth n-4 parent's f / g (SCLLUTDecoder.cpp:83-89 / :157-164,
        // ctemp = 8) folded in: W3 from the parent's 16 symbols, in registers.
        const bool sl = op.flags & MF_SRC_LDS, ul = op.flags & MF_U_LDS;
        if constexpr (LT) stage_tab(tb, T2, (op.flags & MF_BG) ? gtab_dw(lane) : (lane & 31));
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int src = gbase + pfield(st[s].ps, op.sh_src);
            const uint32_t a = M[s].ld(sl, op.src_row, src), b = M[s].ld(sl, op.src_row + 1, src);
            const uint32_t ub = (op.flags & MF_BG) ? M[s].ld(ul, op.u_row, gbase + pfield(st[s].U(), op.sh_u)) : 0u;
            x[s][0] = LT ? lut_lds<8, true>(a, b, ub) : lut_vec<8>(T2, a, b, ub);  // (ub = 0 for f: entries < 256)
        }
    } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) x[s][0] = sym_word<CH>(P, M[s], op, y[s], gbase + pfield(st[s].ps, op.sh_src), 0);  // W3
    }
    // ---- q0 left: W2 = f(W3); q1: W1 = f(W2)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const uint32_t w2 = lut_vec<4>(Tf0, x[s][0], x[s][0] >> 16, 0u);
        x[s][1] = w2 | (f_pair(Tf12, 0u, w2) << 16);
    }
    bot_pair<kList, LM, LAZY>(st, x, Tf34, 0, Tg3, Vlo, 0, fr, gl, gbase, L, lane, sel, sstride, c);  // leaves 0, 1
    if constexpr (LAZY) {  // stage C's operands
        Tg0 = tab_ld(gt, p0 * 64, lane);
        Tf56 = tab_ld(ft, (p3 + 2) * 32, lane);
        Tg5 = tab_ld(gt, (p3 + 2) * 64, lane);
        Vhi = s16 < v ? vb[(4 + j16) * v + s16] : 0.0;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {  // q1: W1 = g(W2, c2)
        x[s][1] = (x[s][1] & ~(3u << 25)) | (c[s] << 25);
        x[s][1] = (x[s][1] & ~(0xffu << 16)) | (g_pair(Tg1, c[s], x[s][1] & 0xffffu) << 16);
    }
    bot_pair<kList, LM, LAZY>(st, x, Tf34, 256, Tg4, Vlo, 32, fr >> 2, gl, gbase, L, lane, sel, sstride, c);  // leaves 2, 3
    if constexpr (LAZY) {  // stage D's operands
        Tg2 = tab_ld(gt, (p1 + 1) * 64, lane);
        Tg6 = tab_ld(gt, (p3 + 3) * 64, lane);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const uint32_t c2 = (x[s][1] >> 25) & 3u;
        const uint32_t c3 = (c2 ^ c[s]) | (c[s] << 2);  // combine at depth n-2
        // ---- q0 right: W2 = g(W3, c3); q2: W1 = f(W2)
        const uint32_t w2 = lut_vec<4>(Tg0, x[s][0], x[s][0] >> 16, c3);
        x[s][1] = w2 | (f_pair(Tf12, 3u, w2) << 16) | (c3 << 27);
    }
    bot_pair<kList, LM, LAZY>(st, x, Tf56, 0, Tg5, Vhi, 0, fr >> 4, gl, gbase, L, lane, sel, sstride, c);  // leaves 4, 5
    if constexpr (LAZY) prefetch_next();
#pragma unroll
    for (int s = 0; s < NS; ++s) {  // q2: W1 = g(W2, c2)
        x[s][1] = (x[s][1] & ~(3u << 25)) | (c[s] << 25);
        x[s][1] = (x[s][1] & ~(0xffu << 16)) | (g_pair(Tg2, c[s], x[s][1] & 0xffffu) << 16);
    }
    bot_pair<kList, LM, LAZY>(st, x, Tf56, 256, Tg6, Vhi, 32, fr >> 6, gl, gbase, L, lane, sel, sstride, c);  // leaves 6, 7
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const uint32_t c2 = (x[s][1] >> 25) & 3u;
        const uint32_t c3r = (c2 ^ c[s]) | (c[s] << 2);
        const uint32_t c3l = (x[s][1] >> 27) & 15u;
        uint32_t res = (c3l ^ c3r) | (c3r << 4);  // combine at depth n-3
        if (op.flags & MF_BCOMB)  // and the parent's (utils.cpp:62-67): U[n-3] of this lineage ^ res | res
            res = ((M[s].ld(op.flags & MF_U_LDS, op.u_row, gbase + pfield(st[s].U(), op.sh_u)) & 0xFFu) ^ res) | (res << 8);
        if (op.flags & MF_BC2) {  // and the grandparent's: U[n-4] ^ res | res, 32 bits
            const int e = op.pad1;
            res = ((M[s].ld(op.flags & MF_BC2_ULDS, op.r_row, gbase + pfield(st[s].U(), e & 255)) & 0xFFFFu) ^ res) |
                  (res << 16);
            M[s].st(op.flags & MF_BC2_DLDS, e >> 16, lane, res);
            if (!(op.flags & MF_BC2_TOR)) st[s].U() = pset(st[s].U(), (e >> 8) & 255, gl);
            continue;
        }
        M[s].st(op.flags & MF_DST_LDS, op.dst_row, lane, res);
        if (!(op.flags & MF_TO_R)) st[s].U() = pset(st[s].U(), op.sh_dst, gl);
    }
}

// ---------------------------------------------------------------------------
// BOTX (FastSCL-LUT, L = 8; MF_BOTX): a height-3 subtree whose nodes of size
// 4 or 2 include FastSCL special nodes (FastSCLLUTDecoder.cpp:83-213: R0, R1,
// REP), held in registers like BOT3.  The types ride in op.cnt bits 8-19, two
// bits per node: q1, q2 (size 4), then q3..q6 (size 2); 0 = plain (a size-4
// node of two size-2 children / a leaf pair), else BX_R0 / BX_R1 / BX_REP
// (nodes inside a special one: don't care).  Every special node's elements
// share one quanta row (MF_VUNI's condition, checked by the host), which sits
// in lanes 0-15 of the slot's quanta register.  The subtree runs as four leaf
// slots (the pairs under q3..q6), a loop that is not unrolled, each slot
// loading its own tables and quanta: a size-4 special node takes its half's
// first slot and skips the second.  Special-node forks move the in-register lineage
// state x as the leaf forks do.
// ---------------------------------------------------------------------------
constexpr int BX_PLAIN = 0, BX_R0 = 1, BX_R1 = 2, BX_REP = 3;

// One special node of t = 2 or 4 elements for one frame set: its symbols are
// nibbles `base`/4.. of x[1], its quanta row q[sym] = lane sym of Vq.
// Returns the node's partial-sum bits (the codeword the reference writes to
// ucap: R0 zeros, REP all equal, R1 the hard decisions with the layers' flips).
template <class Path>
__device__ __forceinline__ uint32_t bx_spec(Path &st, uint32_t (&x)[2], int type, int t, int base, double Vq, int gl,
                                            int gbase, int L, int lane, int *sel, int sj) {
    double l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) l[j] = shfld(Vq, (int)((x[1] >> (base + 4 * j)) & 15u));  // (j >= t: unused)
    if (type == BX_R0) {  // :83-98, (float)(l<0)·|l| as a select (H5: element order)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < t) st.pm += l[j] < 0 ? fabs(l[j]) : 0.0;
        return 0u;
    }
    if (type == BX_REP) {  // :169-213: the all-zeros / all-ones codewords as keep / flip
        double kk = st.pm, kf = st.pm;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < t) {
                kk += l[j] < 0 ? fabs(l[j]) : 0.0;
                kf += l[j] >= 0 ? fabs(l[j]) : 0.0;
            }
        if (keep_all8(__builtin_bit_cast(uint64_t, kk), __builtin_bit_cast(uint64_t, kf), gl)) {
            st.pm = kk;
            return 0u;
        }
        const Sel sx = select_survivors8(kk, kf, gl, gbase, lane, sel, sj);
        const int p = gbase + sx.parent;
        st.pm = pick(sx.upper, shfld(kf, p), shfld(kk, p));
        st.move(p);
        x[0] = (uint32_t)lane_read((int)x[0], p);
        x[1] = (uint32_t)lane_read((int)x[1], p);
        return sx.upper ? (1u << t) - 1u : 0u;
    }
    // R1 (:100-166): the stable argsort of |l| (std::sort of <= 16 elements is
    // an insertion sort, H1), packed with the lineage: r = ord (2 bits per rank)
    // | the ranked elements' symbols (4 bits each, from bit 8) | the decisions
    // (from bit 24, hard decisions l < 0, flipped per layer).  r follows the
    // survivors; a layer's flip position is the slot's own ord (H2).
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j < t) {
            const double aj = fabs(l[j]);
            int rk = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (i < t && i != j) rk += (fabs(l[i]) < aj) || (fabs(l[i]) == aj && i < j);
            r |= ((uint32_t)j << (2 * rk)) | ((((x[1] >> (base + 4 * j)) & 15u)) << (8 + 4 * rk)) |
                 ((uint32_t)(l[j] < 0) << (24 + j));
        }
    }
    const int m = (L - 1) < t ? (L - 1) : t;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q < m) {
            const double ms = fabs(shfld(Vq, (int)((r >> (8 + 4 * q)) & 15u)));
            const double kf = st.pm + ms;
            // identity in every group: the later layers' flips are no smaller (ascending |l|)
            if (keep_all8(__builtin_bit_cast(uint64_t, st.pm), __builtin_bit_cast(uint64_t, kf), gl)) break;
            const Sel sx = select_survivors8(st.pm, kf, gl, gbase, lane, sel, sj);
            const int p = gbase + sx.parent;
            st.pm = pick(sx.upper, shfld(kf, p), shfld(st.pm, p));
            st.move(p);
            x[0] = (uint32_t)lane_read((int)x[0], p);
            x[1] = (uint32_t)lane_read((int)x[1], p);
            // H2: the flip position is this slot's own ord[q] before the move
            // (sorted_absllr_idx[i][layer], :136-140), the decisions the parent's
            const uint32_t own = (r >> (2 * q)) & 3u;
            r = (uint32_t)lane_read((int)r, p);
            if (sx.upper) r ^= 1u << (24 + own);
        }
    }
    return (r >> 24) & ((1u << t) - 1u);
}

// bx_spec for all the wave's frame sets at once: the sums interleaved element
// by element, the R1 layers of the sets interleaved (each set stops at its
// first identity layer) -- the sets' dependency chains overlap.
template <int NS, class Path>
__device__ __forceinline__ void bx_spec_multi(Path (&st)[NS], uint32_t (&x)[NS][2], int type, int t, int base, double Vq, int gl,
                                              int gbase, int lane, int *sel_all, int sstride, uint32_t (&res)[NS]) {
    auto fork = [&](int s, double keep, double flip, Sel &sx) {  // survivor exchange of set s (keep / flip keys)
        sx = select_survivors8(keep, flip, gl, gbase, lane, sel_all + sstride * s, NS * sstride);
        const int p = gbase + sx.parent;
        st[s].pm = pick(sx.upper, shfld(flip, p), shfld(keep, p));
        st[s].move(p);
        x[s][0] = (uint32_t)lane_read((int)x[s][0], p);
        x[s][1] = (uint32_t)lane_read((int)x[s][1], p);
        return p;
    };
#ifdef QPD_BXE
    if (QPD_BXE & 1) return;
#endif
    if (type != BX_R1) {  // R0 (:83-98) / REP (:169-213)
        double kk[NS], kf[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) kk[s] = kf[s] = st[s].pm;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < t)
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const double l = shfld(Vq, (int)((x[s][1] >> (base + 4 * j)) & 15u));
                    kk[s] += l < 0 ? fabs(l) : 0.0;  // H5: element order
                    if (type == BX_REP) kf[s] += l >= 0 ? fabs(l) : 0.0;
                }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            res[s] = 0u;
            if (type == BX_R0 || keep_all8(__builtin_bit_cast(uint64_t, kk[s]), __builtin_bit_cast(uint64_t, kf[s]), gl)) {
                st[s].pm = kk[s];
            } else {
                Sel sx;
                fork(s, kk[s], kf[s], sx);
                res[s] = sx.upper ? (1u << t) - 1u : 0u;
            }
        }
        return;
    }
#ifdef QPD_BXE
    if (QPD_BXE & 2) return;
#endif
    // R1 (:100-166): per set r = ord | ranked symbols | decisions, as bx_spec
    uint32_t r[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        double a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = shfld(Vq, (int)((x[s][1] >> (base + 4 * j)) & 15u));
        r[s] = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j < t) {
                const double aj = fabs(a[j]);
                int rk = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i < t && i != j) rk += (fabs(a[i]) < aj) || (fabs(a[i]) == aj && i < j);
                r[s] |= ((uint32_t)j << (2 * rk)) | (((x[s][1] >> (base + 4 * j)) & 15u) << (8 + 4 * rk)) |
                        ((uint32_t)(a[j] < 0) << (24 + j));
            }
        }
    }
    bool done[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) done[s] = false;
#pragma unroll 1
    for (int q = 0; q < t; ++q) {  // m = min(L - 1, t) = t (L = 8, t <= 4)
        double kf[NS];
        bool all = true;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (done[s]) continue;
            kf[s] = st[s].pm + fabs(shfld(Vq, (int)((r[s] >> (8 + 4 * q)) & 15u)));
            done[s] = keep_all8(__builtin_bit_cast(uint64_t, st[s].pm), __builtin_bit_cast(uint64_t, kf[s]), gl);
            all = all && done[s];
        }
        if (all) break;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (done[s]) continue;
            Sel sx;
            const int p = fork(s, st[s].pm, kf[s], sx);
            const uint32_t own = (r[s] >> (2 * q)) & 3u;  // H2: this slot's own ord[q]
            r[s] = (uint32_t)lane_read((int)r[s], p);
            if (sx.upper) r[s] ^= 1u << (24 + own);
        }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) res[s] = (r[s] >> 24) & ((1u << t) - 1u);
}

// Operands of one leaf slot k (the pair under q3 + k): the table the half's W2
// comes from (k even: q0's f for k = 0, g for k = 2), the size-4 node's f (k
// even) or g table, the pair node's f and g tables, and the quanta register
// (lanes 0-15: the size-4 special node's row, the size-2 special node's row,
// or the left leaf's row; lanes 16-31: the right leaf's row).
struct BxSlot {
    uint32_t t2, t1, tf, tg;
    double V;
};

__device__ __forceinline__ BxSlot bx_load(const FastPlan &P, const MOp &op, int k, int ty, int lane) {
    const int p0 = op.tab, p1 = 2 * p0 + 1, p3 = 4 * p0 + 3;
    const int h = k >> 1, sub = k & 1;
    const int t4 = (ty >> (2 * h)) & 3, t2 = (ty >> (4 + 2 * k)) & 3;
    BxSlot s;
    s.t2 = 0u;
    if (!sub) s.t2 = h ? tab_ld(P.g_tab, p0 * 64, lane) : tab_ld(P.f_tab, p0 * 32, lane & 31);
    s.t1 = sub ? tab_ld(P.g_tab, (p1 + h) * 64, lane) : tab_ld(P.f_tab, (p1 + h) * 32, lane & 31);
    s.tf = tab_ld(P.f_tab, (p3 + k) * 32, lane & 31);
    s.tg = tab_ld(P.g_tab, (p3 + k) * 64, lane);
    // quanta rows vcl[row][pos][sym]: node8 = op.node (the subtree root at depth n-3)
    const int n = P.n, N = P.N, v = P.v, sym = lane & 15, j = (lane >> 4) & 1;
    const int pos8 = 8 * op.node;
    int row = n - 1, pos = pos8 + 2 * k + j;  // leaf rows
    if (t4 != BX_PLAIN) row = n - 3, pos = pos8 + 4 * h;  // size-4 special node (row d - 1, H3)
    else if (t2 != BX_PLAIN) row = n - 2, pos = pos8 + 2 * k;
    s.V = sym < v ? P.vcl[((size_t)row * N + pos) * v + sym] : 0.0;
    return s;
}

template <bool LT, bool CH, int NS, class Path>
__device__ __forceinline__ void botx_op(const FastPlan &P, const Mem (&M)[NS], const MOp &op, const int32_t *const (&y)[NS],
                                        Path (&st)[NS], uint32_t Tf0, uint32_t T2, int gl, int gbase, int L, int *sel,
                                        int sstride, int lane, uint8_t *tb) {
    const int fr = op.cnt & 0xff, ty = (op.cnt >> 8) & 0xfff;
    uint32_t x[NS][2], c[NS], c3r[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) x[s][1] = c3r[s] = 0u;
#if QPD_BX_PIPE
    BxSlot nx = bx_load(P, op, 0, ty, lane);
#endif
    if (op.flags & MF_BFG) {  // the depth n-4 parent's f / g folded in (as bot3_op)
        const bool sl = op.flags & MF_SRC_LDS, ul = op.flags & MF_U_LDS;
        if constexpr (LT) stage_tab(tb, T2, (op.flags & MF_BG) ? gtab_dw(lane) : (lane & 31));
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int src = gbase + pfield(st[s].ps, op.sh_src);
            const uint32_t a = M[s].ld(sl, op.src_row, src), b = M[s].ld(sl, op.src_row + 1, src);
            const uint32_t ub = (op.flags & MF_BG) ? M[s].ld(ul, op.u_row, gbase + pfield(st[s].U(), op.sh_u)) : 0u;
            x[s][0] = LT ? lut_lds<8, true>(a, b, ub) : lut_vec<8>(T2, a, b, ub);
        }
    } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) x[s][0] = sym_word<CH>(P, M[s], op, y[s], gbase + pfield(st[s].ps, op.sh_src), 0);
    }
    (void)Tf0;
#pragma unroll 1  // (unrolled: 18 % slower)
    for (int k = 0; k < 4; ++k) {
        const int h = k >> 1, sub = k & 1;
        const int t4 = (ty >> (2 * h)) & 3, t2 = (ty >> (4 + 2 * k)) & 3;
        if (t4 != BX_PLAIN && sub) continue;  // the half's size-4 special node ran at slot k - 1
#if QPD_BX_PIPE
        const BxSlot cur = nx;
        const int kn = t4 != BX_PLAIN ? k + 2 : k + 1;  // the next slot run
        if (kn < 4) nx = bx_load(P, op, kn, ty, lane);
#else
        const BxSlot cur = bx_load(P, op, k, ty, lane);
#endif
        if (!sub) {
#pragma unroll
            for (int s = 0; s < NS; ++s) {  // W2 = f(W3) / g(W3, c3) (q0, SCLLUTDecoder.cpp:83-89 / :157-164)
                const uint32_t w2 = lut_vec<4>(cur.t2, x[s][0], x[s][0] >> 16, h ? (x[s][1] >> 27) & 15u : 0u);
                x[s][1] = (x[s][1] & (15u << 27)) | w2;
            }
        }
        if (t4 != BX_PLAIN) {  // q1 / q2 special
            uint32_t res[NS];
            bx_spec_multi(st, x, t4, 4, 0, cur.V, gl, gbase, lane, sel, sstride, res);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                if (h) c3r[s] = res[s];
                else x[s][1] = (x[s][1] & ~(15u << 27)) | (res[s] << 27);
            }
            continue;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {  // W1 = f(W2) / g(W2, c2) (q1 / q2)
            const uint32_t w2 = x[s][1] & 0xffffu;
            const uint32_t w1 = sub ? g_pair(cur.t1, (x[s][1] >> 25) & 3u, w2) : f_pair(cur.t1, 0u, w2);
            x[s][1] = (x[s][1] & ~(0xffu << 16)) | (w1 << 16);
        }
#ifdef QPD_BXE
        if (QPD_BXE & 4) continue;
#endif
        if (t2 == BX_PLAIN) {
            bot_pair<true, 8, false>(st, x, cur.tf, 0, cur.tg, cur.V, 0, fr >> (2 * k), gl, gbase, L, lane, sel, sstride, c);
        } else {
            bx_spec_multi(st, x, t2, 2, 16, cur.V, gl, gbase, lane, sel, sstride, c);
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (!sub) {
                x[s][1] = (x[s][1] & ~(3u << 25)) | (c[s] << 25);
            } else {
                const uint32_t c2 = (x[s][1] >> 25) & 3u;
                const uint32_t c3 = (c2 ^ c[s]) | (c[s] << 2);  // combine at depth n-2
                if (h) c3r[s] = c3;
                else x[s][1] = (x[s][1] & ~(15u << 27)) | (c3 << 27);
            }
        }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {  // as the end of bot3_op
        const uint32_t c3l = (x[s][1] >> 27) & 15u;
        uint32_t res = (c3l ^ c3r[s]) | (c3r[s] << 4);  // combine at depth n-3
        if (op.flags & MF_BCOMB)
            res = ((M[s].ld(op.flags & MF_U_LDS, op.u_row, gbase + pfield(st[s].U(), op.sh_u)) & 0xFFu) ^ res) | (res << 8);
        if (op.flags & MF_BC2) {
            const int e = op.pad1;
            res = ((M[s].ld(op.flags & MF_BC2_ULDS, op.r_row, gbase + pfield(st[s].U(), e & 255)) & 0xFFFFu) ^ res) |
                  (res << 16);
            M[s].st(op.flags & MF_BC2_DLDS, e >> 16, lane, res);
            if (!(op.flags & MF_BC2_TOR)) st[s].U() = pset(st[s].U(), (e >> 8) & 255, gl);
            continue;
        }
        M[s].st(op.flags & MF_DST_LDS, op.dst_row, lane, res);
        if (!(op.flags & MF_TO_R)) st[s].U() = pset(st[s].U(), op.sh_dst, gl);
    }
}

// ---------------------------------------------------------------------------
// Special nodes of the Fast decoders (FastSCLUT.cpp:46-107,
// FastSCLLUTDecoder.cpp:82-213).  The node's symbols are read a word (8
// symbols) at a time and their quanta vcl[d-1][pos][sym] (H3) fetched 8 at a
// time, so a node costs one memory round trip per 8 elements; sums still run
// in the reference's sequential element order (H5).
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t lomask(int x) { return x >= 32 ? 0xffffffffu : ((1u << x) - 1u); }
__device__ __forceinline__ uint32_t hibit(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }  // x != 0

// stl::partition_prefix on an R1 array of 17..32 entries (keys < 16, MF_R1_RK),
// each Hoare partition driven by bit masks instead of its scans' dependent
// LDS reads: per round one pass over the array gives the positions whose key
// is >= / <= the pivot's; a partition's i-th left stop is then the next such
// position after the previous stop, or the previous right stop (whose
// swapped-in entry stops the scan there), the right stops likewise, and only
// the swaps touch LDS.  Returns `end` (partition_prefix); heap-sort fallbacks
// (the depth limit, never on the bench code) run stl::heap_sort as the
// reference does.
template <class Seq>
__device__ __forceinline__ int partition_prefix_masked(Seq &s, int temp, int m) {
    int f = 0, l = temp, dl = 0, end = temp;
    for (int t = temp; t > 1; t >>= 1) dl += 2;  // 2 * lg(temp)
    bool live = l - f > stl::kThreshold;
#pragma unroll 1
    while (__builtin_amdgcn_ballot_w64(live)) {
        if (live) {
            if (dl == 0) {
                stl::heap_sort(s, f, l);
                live = false;
            } else {
                --dl;
                stl::move_median_to_first(s, f, f + 1, f + (l - f) / 2, l - 1);
            }
        }
        // ranks >= / <= the pivot's over the 32 positions (one read pass)
        const uint32_t pv = (uint32_t)s.get(live ? f : 0) >> 5;
        uint32_t GE = 0u, LE = 0u;
#pragma unroll 4
        for (int i = 0; i < 16; ++i) {
            const uint32_t d = 2 * i < temp ? s.pair(i) : 0u;
            const uint32_t k0 = (d & 0xffffu) >> 5, k1 = d >> 21;
            GE |= ((uint32_t)(k0 >= pv) << (2 * i)) | ((uint32_t)(k1 >= pv) << (2 * i + 1));
            LE |= ((uint32_t)(k0 <= pv) << (2 * i)) | ((uint32_t)(k1 <= pv) << (2 * i + 1));
        }
        const uint32_t g0 = GE & lomask(l) & ~lomask(f + 1), e0 = LE & lomask(l) & ~lomask(f);
        uint32_t a = g0 ? (uint32_t)__builtin_ctz(g0) : 32u, b = e0 ? hibit(e0) : 0u;
        bool act = live && a < b;
#pragma unroll 1
        while (__builtin_amdgcn_ballot_w64(act)) {
            if (act) {
                const int ea = s.get((int)a), eb = s.get((int)b);
                s.set((int)a, eb);
                s.set((int)b, ea);
                const uint32_t in = lomask((int)b) & ~lomask((int)a + 1);
                const uint32_t g = GE & in, e = LE & in;
                const uint32_t na = g ? (uint32_t)__builtin_ctz(g) : b, nb = e ? hibit(e) : a;
                a = na;
                b = nb;
                act = a < b;
            }
        }
        if (live) {
            const int cut = (int)a;
            if (cut >= m && cut < end) end = cut;
            if (l - cut > stl::kThreshold) {
                if (cut >= end) live = false;
                else f = cut;
            } else {
                l = cut;
            }
            live = live && l - f > stl::kThreshold;
        }
    }
    return end;
}

// LDS view of the R1 argsort array: 16-bit entries (rank << 5 | element),
// entry p of this lane at row base + p/2, half p%2 of the lane's dword (rows
// `hs` halfwords apart: the set-interleaved row stride, see Mem).
struct LdsSeq16 {
    uint16_t *lane0;  // &row[base][lane] as 16-bit
    int hs;
    // entries 2i, 2i + 1 as one dword: a read that may alias the 16-bit stores
    // of set() (a plain uint32_t read may be moved above them: strict aliasing)
    __device__ __forceinline__ uint32_t pair(int i) const {
        typedef uint32_t __attribute__((may_alias)) u32a;
        return *(const u32a *)(lane0 + i * hs);
    }
    __device__ __forceinline__ int get(int p) const { return lane0[(p >> 1) * hs + (p & 1)]; }
    __device__ __forceinline__ void set(int p, int e) const { lane0[(p >> 1) * hs + (p & 1)] = (uint16_t)e; }
    __device__ __forceinline__ bool less(int a, int b) const { return (a >> 5) < (b >> 5); }  // keys only, as std::sort
};

// Survivor layers of an R1 node (FastSCLLUTDecoder.cpp:118-166) after its
// argsort: ord[q] = element of the q-th smallest |llr| (5 bits each in
// ordp0 / ordp1) and its symbol (4 bits each in symp), hw = hard decisions
// (l < 0).  Each of the m layers forks on flipping the next element; the flip
// position is the slot's own pre-selection ord (H2).  The arrays never move: a
// slot's lineage holds the arrays its `origin` lane computed (read per layer
// by shuffles; each lane re-derives its own entry's magnitude, a quanta-row
// lookup or a vcl read), and its flips are one bit mask (temp <= 32) shuffled
// with the survivors.  Returns the node's bits.
template <bool L8, class Path>
__device__ __forceinline__ uint32_t r1_layers(Path &st, int *sel, int sj, int gl, int gbase, int lane, int L, int m,
                                                     uint32_t ordp0, uint32_t ordp1, uint32_t symp, bool uni,
                                                     double vrow, const double *vq, int v, uint32_t hw, int temp) {
    uint32_t flips = 0;
    int origin = gl;
#if QPD_R1_UNROLL
#pragma unroll
#else
#pragma unroll 1  // (one copy of the fork code)
#endif
    for (int layer = 0; layer < kMaxM; ++layer) {
        if (layer < m) {
            const int o = gbase + origin;
            const int own = (int)(layer < 6 ? __builtin_amdgcn_ubfe(ordp0, 5 * layer, 5) : ordp1);
            const uint32_t sym = __builtin_amdgcn_ubfe(symp, 4 * layer, 4);
            const double own_ms = fabs(uni ? shfld(vrow, (int)sym) : vq[(size_t)own * v + sym]);
            const double kf = st.pm + shfld(own_ms, o);
            // Identity selection in every group: no flip survives and no
            // lineage moves, and since each slot's magnitudes ascend with the
            // layer (argsort order) and pm + a is monotone in a, every later
            // layer's flips are at least as large -- all remaining layers are
            // the identity too, so the node is decided.
            if constexpr (L8)
                if (keep_all8(__builtin_bit_cast(uint64_t, st.pm), __builtin_bit_cast(uint64_t, kf), gl)) break;
            const int pos_old = lane_read(own, o);  // H2
            const Sel sl = L8 ? select_survivors8(st.pm, kf, gl, gbase, lane, sel, sj)
                              : select_survivors(st.pm, kf, gl, gbase, L, sel);
            const int p = gbase + sl.parent;
            st.pm = pick(sl.upper, shfld(kf, p), shfld(st.pm, p));
            st.move(p);
            origin = lane_read(origin, p);
            flips = (uint32_t)lane_read((int)flips, p) ^ (sl.upper ? 1u << (pos_old & 31) : 0u);
        }
    }
    const uint32_t word = (uint32_t)lane_read((int)hw, gbase + origin) ^ flips;
    return temp < 32 ? word & ((1u << temp) - 1u) : word;
}

// Word w of a special node's symbols: its S[d] row, or (MF_SFG, size-8 nodes)
// f / g (MF_SGG, u = the left sibling's U[d] through usrc) of its depth d-1
// parent's two words, with the parent's table T2 (staged as bytes at tb: LT).
template <bool LT>
__device__ __forceinline__ uint32_t spec_in(const Mem &M, const MOp &op, int src, int usrc, int w, uint32_t T2,
                                            const uint8_t *tb) {
    const bool sl = op.flags & MF_SRC_LDS;
    if (!(op.flags & MF_SFG)) return M.ld(sl, op.src_row + w, src);
    const uint32_t a = M.ld(sl, op.src_row, src), b = M.ld(sl, op.src_row + 1, src);
    const uint32_t ub = (op.flags & MF_SGG) ? M.ld(op.flags & MF_U_LDS, op.u_row, usrc) : 0u;
    return LT ? lut_lds<8, true>(a, b, ub) : lut_vec<8>(T2, a, b, ub);  // (f: ub = 0, entries < 256)
}

// A special node's result word(s) `res` to its destination; MF_SCOMB (size 8):
// the parent's combine with the left sibling's U[d] (through the path's
// pointer after the node's forks, as the COMB op would read it) instead, to
// the parent's destination (utils.cpp:62-67).
template <class Path>
__device__ __forceinline__ void spec_out(const Mem &M, const MOp &op, Path &st, int gbase, int gl, int lane, int w,
                                         uint32_t res) {
    if (op.flags & MF_SCOMB)
        res = ((M.ld(op.flags & MF_U_LDS, op.u_row, gbase + pfield(st.U(), op.sh_u)) & 0xFFu) ^ res) | (res << 8);
    M.st(op.flags & MF_DST_LDS, op.dst_row + w, lane, res);
}

// The argsort half of an R1 node of <= 32 elements (:100-116) for one set:
// the m smallest |l| in std::sort's order, packed for r1_layers.
struct R1Prep {
    uint32_t ordp0, ordp1, symp, hw;
};

// GEN = false (the FastSCL-LUT kernels without R1L): every R1 node has its ranks in
// the op record (MF_R1_RK, one quanta row) -- the host takes the R1L instantiation
// otherwise -- so the rank-table and std::sort paths are not compiled.
template <bool LT = false, bool GEN = true, class Path>
__device__ __forceinline__ R1Prep r1_prep(const FastPlan &P, const Mem &M, const MOp &op, Path st, int gbase, int L,
                                          int lane, int temp, uint32_t *lds_wave, uint32_t T2 = 0u,
                                          const uint8_t *tb = nullptr) {
    const int src = gbase + pfield(st.ps, op.sh_src);
    const int v = P.v;
    const int m = (L - 1) < temp ? (L - 1) : temp;
    const uint16_t *rk = P.r1_rank + op.tab;
    const double *vq = P.vcl + (size_t)op.vrow * v;
    // MF_VUNI: one quanta row and one rank row for all elements, in registers
    const bool uni = !GEN || (op.flags & MF_VUNI), rku = !GEN || (op.flags & MF_R1_RK);
    const int s16 = lane & 15;
    const uint32_t rrow = GEN && uni && !rku && s16 < v ? (uint32_t)rk[s16] : 0u;
    (void)vq;
    // rank << 1 | sign of element j's symbol: from the op record's words (MF_R1_RK), the node's
    // one rank row in a register (MF_VUNI), or the per-element rank table
    const uint64_t RK = ((uint64_t)(uint32_t)op.tab2 << 32) | (uint32_t)op.r_row;
    auto rank_of = [&](int j, uint32_t sym) -> uint32_t {
        if (rku) return ((uint32_t)(RK >> (4 * sym)) & 15u) << 1 | (((uint32_t)op.pad1 >> sym) & 1u);
        return uni ? (uint32_t)lane_read((int)rrow, (int)sym) : (uint32_t)rk[j * v + sym];
    };
    uint32_t W[4], hw = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w)
        W[w] = (8 * w < temp) ? spec_in<LT>(M, op, src, gbase + pfield(st.U(), op.sh_u), w, T2, tb) : 0u;
    int ord[kMaxM];
#pragma unroll
    for (int q = 0; q < kMaxM; ++q) ord[q] = 0;
    if ((QPD_EXP_FSCL & 8) || temp <= stl::kThreshold) {
        // entries rank << 5 | j (< 2^14) two per register; the m smallest by
        // packed 16-bit min trees (v_pk_min_u16), the taken one set to 0xFFFF
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        u16x2 ep[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t lo = 0xffffu, hi = 0xffffu;
            if (2 * i < temp) {
                const uint32_t e = rank_of(2 * i, (W[i >> 2] >> (8 * (i & 3))) & 15u);
                hw |= (e & 1u) << (2 * i);
                lo = ((e >> 1) << 5) | (uint32_t)(2 * i);
            }
            if (2 * i + 1 < temp) {
                const uint32_t e = rank_of(2 * i + 1, (W[i >> 2] >> (8 * (i & 3) + 4)) & 15u);
                hw |= (e & 1u) << (2 * i + 1);
                hi = ((e >> 1) << 5) | (uint32_t)(2 * i + 1);
            }
            ep[i] = __builtin_bit_cast(u16x2, lo | (hi << 16));
        }
#pragma unroll
        for (int q = 0; q < kMaxM; ++q) {
            if (q < m) {
                u16x2 a = __builtin_elementwise_min(__builtin_elementwise_min(ep[0], ep[1]),
                                                    __builtin_elementwise_min(ep[2], ep[3]));
                u16x2 b = __builtin_elementwise_min(__builtin_elementwise_min(ep[4], ep[5]),
                                                    __builtin_elementwise_min(ep[6], ep[7]));
                a = __builtin_elementwise_min(a, b);
                const uint32_t mn = a.x < a.y ? a.x : a.y;
                ord[q] = (int)(mn & 31u);
                const u16x2 mm = {(unsigned short)mn, (unsigned short)mn};
                const u16x2 one = {1, 1}, zero = {0, 0};
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const u16x2 d = ep[i] - mm;                                // 0 where taken (all entries >= mn)
                    const u16x2 t = __builtin_elementwise_min(d, one) ^ one;   // 1 where taken
                    ep[i] = ep[i] | (zero - t);                               // taken -> 0xFFFF
                }
            }
        }
    } else {
        // the wave's whole LDS tail from the sets' row u_row on (the rows of depths > d and the
        // selection scratch of every set: free while this node runs; the sets run one after the
        // other), one 64-lane row per two entries
        const LdsSeq16 seq{(uint16_t *)(lds_wave + M.rw(op.u_row) + lane), 128};
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if (j < temp) {
                const uint32_t e = rank_of(j, (W[j >> 3] >> (4 * (j & 7))) & 15u);
                hw |= (e & 1u) << j;
                seq.set(j, (int)(((e >> 1) << 5) | (uint32_t)j));
            }
        }
        if (rku) {
            // the partitions in LDS, then the m smallest of the block [0, end) by (rank, position):
            // what the final insertion sort's first m outputs are (stl::partition_prefix), by
            // packed 16-bit min trees over rank << 10 | position << 5 | element (ranks < 16)
            const int end = QPD_EXP_FSCL & 128 ? stl::partition_prefix(seq, 0, temp, m) : partition_prefix_masked(seq, temp, m);
            typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
            u16x2 ep[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t d = 2 * i < temp ? seq.pair(i) : 0u;  // entries 2i, 2i + 1
                const uint32_t e0 = d & 0xffffu, e1 = d >> 16;
                const uint32_t lo = 2 * i < end ? ((e0 >> 5) << 10) | ((uint32_t)(2 * i) << 5) | (e0 & 31u) : 0xffffu;
                const uint32_t hi = 2 * i + 1 < end ? ((e1 >> 5) << 10) | ((uint32_t)(2 * i + 1) << 5) | (e1 & 31u) : 0xffffu;
                ep[i] = __builtin_bit_cast(u16x2, lo | (hi << 16));
            }
#pragma unroll
            for (int q = 0; q < kMaxM; ++q) {
                if (q < m) {
                    u16x2 a[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) a[i] = __builtin_elementwise_min(ep[2 * i], ep[2 * i + 1]);
#pragma unroll
                    for (int w = 4; w >= 1; w >>= 1)
#pragma unroll
                        for (int i = 0; i < w; ++i) a[i] = __builtin_elementwise_min(a[i], a[i + w]);
                    const uint32_t mn = a[0].x < a[0].y ? a[0].x : a[0].y;
                    ord[q] = (int)(mn & 31u);
                    const u16x2 mm = {(unsigned short)mn, (unsigned short)mn};
                    const u16x2 one = {1, 1}, zero = {0, 0};
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const u16x2 dd = ep[i] - mm;
                        ep[i] = ep[i] | (zero - (__builtin_elementwise_min(dd, one) ^ one));  // taken -> 0xFFFF
                    }
                }
            }
        } else if constexpr (GEN) {
            stl::sort_small_prefix(seq, 0, temp, m);  // only ord[0, m) is read
#pragma unroll
            for (int q = 0; q < kMaxM; ++q)
                if (q < m) ord[q] = seq.get(q) & 31;
        }
    }
    R1Prep r{0u, 0u, 0u, hw};
#pragma unroll
    for (int q = 0; q < kMaxM; ++q) {
        if (q < m) {
            const int k = ord[q] >> 3;
            const uint32_t w = k == 0 ? W[0] : k == 1 ? W[1] : k == 2 ? W[2] : W[3];
            r.symp |= ((w >> (4 * (ord[q] & 7))) & 15u) << (4 * q);
            if (q < 6)
                r.ordp0 |= (uint32_t)ord[q] << (5 * q);
            else
                r.ordp1 = (uint32_t)ord[q];
        }
    }
    return r;
}

template <bool L8, class Path>
__device__ __forceinline__ void r1_small(const FastPlan &P, const Mem &M, const MOp &op, Path &st, int *sel, int sj,
                                         int gl, int gbase, int L, int lane, int temp, uint32_t *lds_wave) {
    const int v = P.v;
    const int m = (L - 1) < temp ? (L - 1) : temp;
    const double *vq = P.vcl + (size_t)op.vrow * v;
    const bool uni = op.flags & MF_VUNI;
    const double vrow = uni && (lane & 15) < v ? vq[lane & 15] : 0.0;
    const R1Prep r = r1_prep(P, M, op, st, gbase, L, lane, temp, lds_wave);
    const uint32_t word =
        r1_layers<L8>(st, sel, sj, gl, gbase, lane, L, m, r.ordp0, r.ordp1, r.symp, uni, vrow, vq, v, r.hw, temp);
    M.st(op.flags & MF_DST_LDS, op.dst_row, lane, word);
}

// R1 nodes of <= 32 elements with L = 8 for all the wave's frame sets: the
// argsorts set by set, then the layers of the sets interleaved (their fork
// chains overlap), each set stopping at its first identity layer (r1_layers).
template <bool LT, bool GEN, int NS, class Path>
__device__ __forceinline__ void r1_multi(const FastPlan &P, const Mem (&Mv)[NS], const MOp &op, Path (&st)[NS], int *sel_all,
                                         int sstride, int gl, int gbase, int lane, uint32_t *lds_wave, uint32_t T2,
                                         uint8_t *tb) {
    const int temp = op.cnt, v = P.v;
    const int m = kMaxM < temp ? kMaxM : temp;  // L = 8
    const double *vq = P.vcl + (size_t)op.vrow * v;
    const bool uni = !GEN || (op.flags & MF_VUNI);
    const double vrow = uni && (lane & 15) < v ? vq[lane & 15] : 0.0;
    if constexpr (LT)
        if (op.flags & MF_SFG) stage_tab(tb, T2, (op.flags & MF_SGG) ? gtab_dw(lane) : (lane & 31));
    R1Prep pr[NS];
#pragma unroll 1
    for (int s = 0; s < NS; ++s) {  // set s in slot 0 (rotate_sets)
        if ((QPD_EXP_FSCL & 64) && temp > 16) pr[0] = R1Prep{0x1a418820u, 6u, 0u, 0u};  // (ord 0..6)
        else
        pr[0] = r1_prep<LT, GEN>(P, Mv[0].set(s), op, st[0], gbase, 8, lane, temp, lds_wave, T2, tb);
        rotate_sets(st);
        rotate_sets(pr);
    }
    uint32_t flips[NS];
    int origin[NS];
    bool done[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        flips[s] = 0;
        origin[s] = gl;
        done[s] = false;
    }
#pragma unroll 1
    for (int layer = 0; layer < ((QPD_EXP_FSCL & 32) && temp > 16 ? 0 : m); ++layer) {
        double kf[NS];
        int own[NS];
        bool all = true;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (done[s]) continue;
            const int o = gbase + origin[s];
            own[s] = (int)(layer < 6 ? __builtin_amdgcn_ubfe(pr[s].ordp0, 5 * layer, 5) : pr[s].ordp1);
            const uint32_t sym = __builtin_amdgcn_ubfe(pr[s].symp, 4 * layer, 4);
            const double own_ms = fabs(!GEN || uni ? shfld(vrow, (int)sym) : vq[(size_t)own[s] * v + sym]);
            kf[s] = st[s].pm + shfld(own_ms, o);
            done[s] = keep_all8(__builtin_bit_cast(uint64_t, st[s].pm), __builtin_bit_cast(uint64_t, kf[s]), gl);
            all = all && done[s];
        }
        if (all) break;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (done[s]) continue;
            const int o = gbase + origin[s];
            const int pos_old = lane_read(own[s], o);  // H2
            const Sel sl = select_survivors8(st[s].pm, kf[s], gl, gbase, lane, sel_all + sstride * s, NS * sstride);
            const int p = gbase + sl.parent;
            st[s].pm = pick(sl.upper, shfld(kf[s], p), shfld(st[s].pm, p));
            st[s].move(p);
            origin[s] = lane_read(origin[s], p);
            flips[s] = (uint32_t)lane_read((int)flips[s], p) ^ (sl.upper ? 1u << (pos_old & 31) : 0u);
        }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        uint32_t word = (uint32_t)lane_read((int)pr[s].hw, gbase + origin[s]) ^ flips[s];
        if (temp < 32) word &= (1u << temp) - 1u;
        spec_out(Mv[s], op, st[s], gbase, gl, lane, 0, word);
        if (!(op.flags & MF_TO_R)) st[s].U() = pset(st[s].U(), op.sh_dst, gl);
    }
}

// R0 / REP nodes with L = 8 for all the wave's frame sets, interleaved element
// by element (their sums are dependent fp64 chains in the reference's order,
// H5; the sets' chains overlap).
// GEN = false (the FastSCL-LUT kernels without R1L): every R0 / REP node has one quanta
// row (MF_VUNI; the host takes the R1L instantiation otherwise).  With the byte-table
// slot (LT) the two sums' terms of each symbol, (l < 0)|l| and (l >= 0)|l|, are staged
// in it once per node and each element reads both with one ds_read_b128 (the same
// doubles as the selects on the quanta: the sums are unchanged).
template <bool LT, bool GEN, int NS, class Path>
__device__ __forceinline__ void r0rep_multi(const FastPlan &P, const Mem (&Mv)[NS], const MOp &op, Path (&st)[NS], int *sel_all,
                                            int sstride, int gl, int gbase, int lane, uint32_t T2, uint8_t *tb) {
    const int fl = op.flags, temp = op.cnt, v = P.v;
    const bool rep = op.type == OP_REP, sl = fl & MF_SRC_LDS, dl = fl & MF_DST_LDS;
    const double *vq = P.vcl + (size_t)op.vrow * v;  // row d-1, position temp*node
    const bool uni = !GEN || (fl & MF_VUNI);
    const double vr = uni && (lane & 15) < v ? vq[lane & 15] : 0.0;
    int src[NS];
    double kk[NS], kf[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        src[s] = gbase + pfield(st[s].ps, op.sh_src);
        kk[s] = kf[s] = st[s].pm;
    }
    const int n8 = (temp + 7) >> 3;
    if constexpr (LT)
        if (fl & MF_SFG) stage_tab(tb, T2, (fl & MF_SGG) ? gtab_dw(lane) : (lane & 31));
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 *const qt = (d2 *)(tb + 512);  // (LT, !GEN) the symbols' terms, after the f / g tables' 512 B
    if constexpr (LT && !GEN) {
        if (lane < 16) qt[lane] = d2{vr < 0 ? fabs(vr) : 0.0, vr >= 0 ? fabs(vr) : 0.0};
        lds_order();
    }
#pragma unroll 1
    for (int w = 0; w < n8; ++w) {
        uint32_t word[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) word[s] = spec_in<LT>(Mv[s], op, src[s], gbase + pfield(st[s].U(), op.sh_u), w, T2, tb);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (8 * w + i >= temp) break;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const uint32_t sym = (word[s] >> (4 * i)) & 15u;
                if constexpr (LT && !GEN) {
                    const d2 t = qt[sym];
                    kk[s] += t.x;
                    if (rep) kf[s] += t.y;
                    continue;
                }
                const double l = uni ? shfld(vr, (int)sym) : vq[(size_t)(8 * w + i) * v + sym];
                kk[s] += l < 0 ? fabs(l) : 0.0;  // :88-95 / :176-180, (l<0)·|l|, (l>=0)·|l| as selects
                if (rep) kf[s] += l >= 0 ? fabs(l) : 0.0;
            }
        }
    }
    if constexpr (LT && !GEN) lds_order();  // (the slot's next writer comes after these reads)
    const int nwo = (temp + 31) >> 5;
    const uint32_t m = temp < 32 ? ((1u << temp) - 1u) : 0xffffffffu;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        uint32_t fill = 0;
        if (!rep || keep_all8(__builtin_bit_cast(uint64_t, kk[s]), __builtin_bit_cast(uint64_t, kf[s]), gl)) {
            st[s].pm = kk[s];  // R0; REP: the identity selection, every path keeps its all-zeros codeword
        } else {
            const Sel sx = select_survivors8(kk[s], kf[s], gl, gbase, lane, sel_all + sstride * s, NS * sstride);
            const int p = gbase + sx.parent;
            st[s].pm = pick(sx.upper, shfld(kf[s], p), shfld(kk[s], p));
            st[s].move(p);
            fill = sx.upper ? 0xffffffffu : 0u;
        }
        for (int w = 0; w < nwo; ++w) spec_out(Mv[s], op, st[s], gbase, gl, lane, w, fill & m);
        if (!(fl & MF_TO_R)) st[s].U() = pset(st[s].U(), op.sh_dst, gl);
    }
}

// R1 nodes above 32 elements (N >= 2048 codes) or without LDS room: the
// argsort arrays live in the wave's global slab (H / K / I rows).
template <class Path>
__device__ __forceinline__ void r1_large(const FastPlan &P, const Mem &M, const MOp &op, Path &st, int *sel, int gl,
                                      int gbase, int L, int lane, int temp) {
    const int src = gbase + pfield(st.ps, op.sh_src);
    const bool sl = op.flags & MF_SRC_LDS, dl = op.flags & MF_DST_LDS;
    const int nwo = (temp + 31) >> 5;
    const double *vq = P.vcl + (size_t)op.vrow * P.v;
    auto llr = [&](int j) -> double {
        const uint32_t w = M.ld(sl, op.src_row + (j >> 3), src);
        return vq[(size_t)j * P.v + ((w >> ((j & 7) << 2)) & 15u)];
    };
    const int m = (L - 1) < temp ? (L - 1) : temp;
    uint32_t *g = M.gp;
    for (int w = 0; w < nwo; ++w) {
        uint32_t word = 0;
        for (int i = 0; i < 32 && 32 * w + i < temp; ++i) {
            const int j = 32 * w + i;
            const double l = llr(j);
            word |= (uint32_t)(l < 0) << i;
            const uint64_t b = __builtin_bit_cast(uint64_t, fabs(l));
            g[(size_t)M.rw(P.K_row + 2 * j) + lane] = (uint32_t)b;
            g[(size_t)M.rw(P.K_row + 2 * j + 1) + lane] = (uint32_t)(b >> 32);
        }
        g[(size_t)M.rw(P.H_row + w) + lane] = word;
    }
    int ord[kMaxM];
    double ms[kMaxM];
    int flip[kMaxM];
    for (int q = 0; q < kMaxM; ++q) {
        ord[q] = 0;
        ms[q] = 0;
        flip[q] = -1;
    }
    FastSortSeq seq{g, P.I_row, P.K_row, lane, M.ns * 64};
    for (int p = 0; p < temp; ++p) seq.set(p, p);
    stl::sort(seq, 0, temp);
    for (int q = 0; q < kMaxM; ++q) {
        if (q < m) {
            ord[q] = seq.get(q);
            ms[q] = seq.key(ord[q]);
        }
    }
    wave_sync();  // H rows visible to the whole wave
    int origin = gl;
    for (int layer = 0; layer < kMaxM; ++layer) {
        if (layer < m) {
            const double kf = st.pm + ms[layer];
            const Sel sx = select_survivors(st.pm, kf, gl, gbase, L, sel);
            const int p = gbase + sx.parent;
            const int pos_old = ord[layer];  // H2
            st.pm = pick(sx.upper, shfld(kf, p), shfld(st.pm, p));
            st.move(p);
            origin = lane_read(origin, p);
            for (int q = 0; q < kMaxM; ++q) {
                ord[q] = lane_read(ord[q], p);
                ms[q] = shfld(ms[q], p);
                if (q < layer) flip[q] = lane_read(flip[q], p);
            }
            flip[layer] = sx.upper ? pos_old : -1;
        }
    }
    for (int w = 0; w < nwo; ++w) {
        uint32_t word = g[(size_t)M.rw(P.H_row + w) + gbase + origin];
        for (int q = 0; q < kMaxM; ++q)
            if (q < m && flip[q] >= 0 && (flip[q] >> 5) == w) word ^= 1u << (flip[q] & 31);
        if (temp < 32) word &= (1u << temp) - 1u;
        M.st(dl, op.dst_row + w, lane, word);
    }
}

// R1L: the schedule has an R1 node that needs r1_large (> 32 elements, or > 16
// without LDS room; N >= 2048 codes).  Only those plans get it compiled in:
// its argsort stack and arrays cost the other instantiations registers and
// scratch (+3 % FastSCL-LUT at N = 1024 without it).
template <bool kList, bool L8, bool R1L, class Path>
__device__ __forceinline__ void special_op(const FastPlan &P, const Mem &M, const MOp &op, Path &st, int *sel, int sj,
                                           int gl, int gbase, int L, int lane, uint32_t *lds_wave) {
    const int fl = op.flags;
    const int temp = op.cnt;
    const int src = gbase + pfield(st.ps, op.sh_src);
    const bool dl = fl & MF_DST_LDS, sl = fl & MF_SRC_LDS;
    const int nwo = (temp + 31) >> 5;
    const int v = P.v;
    const double *vq = P.vcl + (size_t)op.vrow * v;  // row d-1, position temp*node
    // MF_VUNI: the node's one quanta row, entry s in lanes s, s+16, s+32, s+48
    const bool uni = fl & MF_VUNI;
    const double vr = uni && (lane & 15) < v ? vq[lane & 15] : 0.0;
    // elements [8w, 8w + 8) of the node: quanta of its symbols
    auto llr8 = [&](int w, double (&l)[8], uint32_t &word) {
        word = M.ld(sl, op.src_row + w, src);
        if (uni) {
#pragma unroll
            for (int i = 0; i < 8; ++i) l[i] = shfld(vr, (int)((word >> (4 * i)) & 15u));
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                l[i] = (8 * w + i < temp) ? vq[(size_t)(8 * w + i) * v + ((word >> (4 * i)) & 15u)] : 0.0;
        }
    };
    const int n8 = (temp + 7) >> 3;
    if (QPD_EXP_FSCL & 2) return;
    if (op.type == OP_R0) {
        if (kList) {
            for (int w = 0; w < n8; ++w) {
                double l[8];
                uint32_t word;
                llr8(w, l, word);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (8 * w + i < temp) st.pm += l[i] < 0 ? fabs(l[i]) : 0.0;  // H5; (float)(l<0)·|l| as a select
            }
        }
        for (int w = 0; w < nwo; ++w) M.st(dl, op.dst_row + w, lane, 0u);
    } else if (op.type == OP_REP && !(QPD_EXP_FSCL & 16)) {
        uint32_t fill = 0;
        if (!kList) {
            double S = 0;
            for (int w = 0; w < n8; ++w) {
                double l[8];
                uint32_t word;
                llr8(w, l, word);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (8 * w + i < temp) S += l[i];
            }
            fill = S <= 0 ? 0xffffffffu : 0u;  // H4
        } else {
            double kk = st.pm, kf = st.pm;
            for (int w = 0; w < n8; ++w) {
                double l[8];
                uint32_t word;
                llr8(w, l, word);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (8 * w + i < temp) {
                        kk += l[i] < 0 ? fabs(l[i]) : 0.0;  // (l<0)·|l|, (l>=0)·|l| as selects
                        kf += l[i] >= 0 ? fabs(l[i]) : 0.0;
                    }
            }
            if (L8 && keep_all8(__builtin_bit_cast(uint64_t, kk), __builtin_bit_cast(uint64_t, kf), gl)) {
                st.pm = kk;  // identity selection: every path keeps its all-zeros codeword
            } else {
                const Sel sx = L8 ? select_survivors8(kk, kf, gl, gbase, lane, sel, sj) : select_survivors(kk, kf, gl, gbase, L, sel);
                const int p = gbase + sx.parent;
                st.pm = pick(sx.upper, shfld(kf, p), shfld(kk, p));
                st.move(p);
                fill = sx.upper ? 0xffffffffu : 0u;
            }
        }
        const uint32_t m = temp < 32 ? ((1u << temp) - 1u) : 0xffffffffu;
        for (int w = 0; w < nwo; ++w) M.st(dl, op.dst_row + w, lane, fill & m);
    } else if (op.type == OP_SPC) {  // FastSC only
        uint32_t parity = 0, word = 0;
        double best = 0;
        int bi = 0;
        for (int w = 0; w < n8; ++w) {
            double l[8];
            uint32_t sw;
            llr8(w, l, sw);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int j = 8 * w + i;
                if (j < temp) {
                    const uint32_t h = l[i] <= 0;
                    word |= h << (j & 31);
                    parity ^= h;
                    const double a = fabs(l[i]);
                    if (j == 0 || a < best) {  // first minimum (H6)
                        best = a;
                        bi = j;
                    }
                }
            }
            if ((w & 3) == 3 || w == n8 - 1) {
                M.st(dl, op.dst_row + (w >> 2), lane, word);
                word = 0;
            }
        }
        if (parity) {
            const int row = op.dst_row + (bi >> 5);
            M.stv(dl, row, lane, M.ldv(dl, row, lane) ^ (1u << (bi & 31)));  // bi: per lane
        }
    } else if (!kList) {  // OP_R1, FastSC: `<= 0`
        uint32_t word = 0;
        for (int w = 0; w < n8; ++w) {
            double l[8];
            uint32_t sw;
            llr8(w, l, sw);
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (8 * w + i < temp) word |= (uint32_t)(l[i] <= 0) << ((8 * w + i) & 31);
            if ((w & 3) == 3 || w == n8 - 1) {
                M.st(dl, op.dst_row + (w >> 2), lane, word);
                word = 0;
            }
        }
    } else if (QPD_EXP_FSCL & 4) {
    } else if (temp <= stl::kThreshold || (fl & MF_R1_LDS)) {
        r1_small<L8>(P, M, op, st, sel, sj, gl, gbase, L, lane, temp, lds_wave);
    } else if constexpr (R1L) {
        r1_large(P, M, op, st, sel, gl, gbase, L, lane, temp);
    }
    if (!(fl & MF_TO_R)) st.U() = pset(st.U(), op.sh_dst, gl);
}

// QPD_STAMPS (diagnostic builds only): wave cycles per op class (lane k of
// each wave accumulates class k; flushed into FastPlan::stamps once per task).
// Class = 2*type + (op syncs), or by depth with QPD_STAMPS_DEPTH.

// Waves per SIMD the register allocation targets: 6 (80 VGPRs) for one
// frame set, 4 (128 VGPRs) for two (5 for SCL-LUT, below), 6 for FastSCL's one set too (its special
// ops spill ~136 B at 80 VGPRs, yet with the task queue 6 waves beat 5 by 4%)
// -- the measured optima on MI355X.
#ifndef QPD_WPE1
#define QPD_WPE1 6
#endif
#ifndef QPD_WPE_FSCL
#define QPD_WPE_FSCL 6
#endif
#ifndef QPD_WPE2
#define QPD_WPE2 4
#endif
// SCL-LUT's two-set decode kernel: 5 waves per SIMD (96 VGPRs) since its path
// state takes one pointer word (PW1) and its BOT3 stages its loads (r04h:
// 44.3 vs 41.7 M frames/s at 4 waves)
#ifndef QPD_WPE2_SCL
#define QPD_WPE2_SCL 5
#endif
// FastSCL-LUT's two-set kernel: 4 waves per SIMD (128 VGPRs): its special-node
// and mixed-subtree code cost the whole kernel's allocation at 96 (the SCL-LUT op
// list on the FastSCL-LUT instantiation: 32.7 M frames/s at 5 waves, 37.7 M at 4,
// against 45.2 M on the SCL-LUT one; FastSCL-LUT 31.7 -> 37.7 M)
#ifndef QPD_WPE2_FSCL
#define QPD_WPE2_FSCL 4
#endif
#ifndef QPD_BX_PIPE
#define QPD_BX_PIPE 0  // BOTX slot operands loaded one slot ahead
#endif
#ifndef QPD_SPEC_ROT
#define QPD_SPEC_ROT 1  // special ops: one code copy, the sets rotated through slot 0 (else unrolled)
#endif
#ifndef QPD_R1_UNROLL
#define QPD_R1_UNROLL 0  // R1 layers unrolled
#endif
#ifndef QPD_WPE3
#define QPD_WPE3 3
#endif
#ifndef QPD_WPE_W16
#define QPD_WPE_W16 4  // SCL-LUT at 9 <= L <= 16 (W16): with the all-at-once swaps 5.27 M frames/s at L = 16
                       // vs 5.09 for one swap per round at 4 or 5 waves (r06o; the swaps at 5: 4.52, spills)
#endif
// NS frame sets per wave (see above); L8: list decoders with L = 8; W16: SCL-LUT with
// 9 <= L <= 16 (lane groups of 16, select_survivors16).
// LDS: NS * (lds_rows + 2) rows, set-interleaved (see Mem): a set's rows
// 0..lds_rows-1 (grouped by depth, see FastLayout), then its selection scratch
// as rows lds_rows (64 slots) and lds_rows + 1 (junk slots).
// Global slab: NS * glb_rows rows per workgroup, set-interleaved.
// PFX: the frozen-prefix kernel (lut_prefix_kernel below; one set, gs = 1, no
// tail, `out` unused).  A template argument rather than a wrapper around a
// shared body: the wrapper moved the decode kernels' register allocation
// (FastSCL-LUT 63 -> 71 ms per 2^21 frames, profiles/r03ac_ab.txt).
//
// `ops` is its own __restrict__ argument (= P.ops) so that the compiler can
// prove the op records are never written and fetch them with scalar loads
// instead of vector loads + readfirstlane, which drain vmcnt at every op.
// PW1: one pointer word per path (PathT; the host packed the op list's fields).
template <int KIND, int NS, bool L8, bool R1L = false, bool PFX = false, bool PW1 = false, bool W16 = false>
__global__ __launch_bounds__(64, NS == 3 ? QPD_WPE3
                                : W16 ? QPD_WPE_W16
                                : NS == 2 ? (KIND == K_SCL_LUT && !PFX ? QPD_WPE2_SCL : KIND == K_FASTSCL_LUT ? QPD_WPE2_FSCL : QPD_WPE2)
                                : KIND == K_FASTSCL_LUT ? QPD_WPE_FSCL : QPD_WPE1) void lut_fast_kernel(FastPlan P, const int32_t *__restrict__ in, int64_t B,
                                                               uint8_t *__restrict__ out,
                                                               const MOp *__restrict__ ops) {
    constexpr bool kList = (KIND == K_SCL_LUT || KIND == K_FASTSCL_LUT);
    static_assert(!W16 || (KIND == K_SCL_LUT && !L8), "W16: SCL-LUT list sizes 9..16");
    constexpr int LM = L8 ? 8 : W16 ? 16 : 0;  // list mode of the leaf forks (leaf_fork)
    // staged BOT3 loads: the list kinds (SCL-LUT, FastSCL-LUT)
    constexpr bool kLazy = QPD_BOT3_LAZY && kList;
    constexpr bool kFast = (KIND == K_FASTSC_LUT || KIND == K_FASTSCL_LUT) && !(QPD_EXP_FSCL & 256);
    // channel reads inside the decode (MF_CHAN: codes without the root pre-pass); the
    // one-pointer-word SCL-LUT instantiations run only op lists with the pre-pass
    // (build_fast; +1.1 % SCL-LUT, -1.3 % when FastSCL-LUT's dropped them too, r05z5)
    constexpr bool kChan = !(PW1 && KIND == K_SCL_LUT);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
    // list kinds at two frame sets: the f / g ops' byte tables (stage_tab) and the
    // folded descents (MF_FF), 768 B at the start of the wave's LDS -- a constant
    // address, so that every byte-table lookup is a ds_read_u8 of its index with the
    // table's place in the instruction's offset field (one VALU add per lookup less
    // than from a base in a register); then the rows of all sets, interleaved, and
    // each set's selection scratch as its next two rows (set s's slots at sel_all +
    // s * 64, its junk slots NS * 64 words on)
#ifndef QPD_EXP_NO_LDSTAB
#define QPD_EXP_NO_LDSTAB 0  // A/B: the f / g lookups by ds_bpermute from the table register (no byte tables)
#endif
    constexpr bool kLdsTab = kList && NS >= 2 && !QPD_EXP_NO_LDSTAB;
    constexpr int kTabWords = kLdsTab ? 192 : 0;  // (qpd_capi.hip: lds_tab_bytes)
    uint8_t *const tb = (uint8_t *)lds_dyn;
    uint32_t *const lds_rows = lds_dyn + kTabWords;
    const int sstride = 64;
    int *const sel_all = (int *)(lds_rows + NS * P.lds_rows * 64);
    Mem Mv[NS];
    {
        uint32_t *const slab = P.scratch + (size_t)blockIdx.x * NS * P.glb_rows * 64;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(slab, 0, NS * P.glb_rows * 256 * QPD_EXP_SLABMUL, 0x00020000);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            Mv[s].lds = lds_rows + s * 64;
            Mv[s].gp = slab + s * 64;
            Mv[s].rs = rs;
            Mv[s].so = s * 256;
            Mv[s].ns = NS;
        }
    }
    const int gs = P.gs;
    const int L = kList ? P.L : 1;
    const int N = P.N;
    const int64_t fpw = P.fpw;  // frames per set
    const int64_t ntasks = (B + NS * fpw - 1) / (NS * fpw);
    const double kInf = __builtin_huge_val();

    // Tasks: the first blockIdx.x, then (QPD_DYN) the next untaken one from
    // the queue -- every SIMD stays busy to the end whatever the residency --
    // or the grid-stride successor.
    for (int64_t task = blockIdx.x; task < ntasks;
         task = QPD_DYN ? (int64_t)gridDim.x + wave_take(P.task_ctr, P.task_base) : task + gridDim.x) {
#ifdef QPD_POISON
        // Diagnosis builds only: every LDS word and slab row of this wave set to
        // QPD_POISON at the start of each task, so that a read of a row no op of
        // this task wrote shows up as a parity difference.
        for (int i = threadIdx.x; i < NS * (P.lds_rows * 64 + kSelInts); i += 64) lds_rows[i] = (uint32_t)QPD_POISON;
        for (int r = 0; r < NS * P.glb_rows; ++r) Mv[0].gp[r * 64 + threadIdx.x] = (uint32_t)QPD_POISON;
        wave_sync();
#endif
        PathT<PW1> stv[NS];
        {
            const int lane = threadIdx.x, gl = lane & (gs - 1);
            uint64_t self = 0;
            for (int d = 0; d < kMaxDepth; ++d) self |= (uint64_t)gl << (4 * d);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                stv[s].pm = (gl == 0) ? 0.0 : kInf;
                stv[s].ps = self;
                stv[s].U() = self;  // (PW1: the same word)
            }
        }
#ifdef QPD_STAMPS
        uint64_t stamp_acc = 0, stamp_cnt = 0;
#endif
        MOp nxt = ops[0];
        Pre pre = fetch_pre(P, nxt, threadIdx.x, threadIdx.x < P.v ? threadIdx.x : 0);
        for (int oi = 0; oi < P.nops; ++oi) {
            // Re-derive the lane constants every op: without this the compiler
            // hoists dozens of lane-derived addresses out of the op loop and
            // pins them in VGPRs for the whole kernel (spills, low occupancy).
            int lane = threadIdx.x;
            asm volatile("" : "+v"(lane));
            const int gl = lane & (gs - 1);
            const int gbase = lane & ~(gs - 1);
            const int vlane = lane < P.v ? lane : 0;
            const int32_t *yv[NS];  // frame rows of `in` (read by MF_CHAN / MF_PRE ops only)
            const int gsh = __builtin_ctz(gs);
            if (nxt.flags & (MF_CHAN | MF_PRE)) {  // wave-uniform: no per-lane address math on other ops
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    int64_t f = (task * NS + s) * fpw + (lane >> gsh);
                    if (f >= B) f = B - 1;
                    yv[s] = in + (f << P.in_shift);
                }
            } else {
#pragma unroll
                for (int s = 0; s < NS; ++s) yv[s] = in;
            }
            if (nxt.flags & MF_SYNC) wave_sync();  // before the next prefetch is issued
            const MOp op = nxt;
            const Pre cur = pre;
#ifdef QPD_STAMPS
            __builtin_amdgcn_s_waitcnt(0);
            const uint64_t stamp_t0 = __builtin_amdgcn_s_memtime();
#endif
            // the next op's operands; a BOT3 issues them itself, late (see bot3_op)
            if (oi + 1 < P.nops) {
                nxt = ops[oi + 1];
                if (!kLazy || op.type != OP_BOT3) pre = fetch_pre(P, nxt, lane, vlane);
            }
            const int fl = op.flags;
            // special nodes, FastSCLUT.cpp:46-107 / FastSCLLUTDecoder.cpp:82-213
            auto run_special = [&]() {
              if constexpr (kFast) {
                  // the sets one after the other, one copy of the code: set s runs in
                  // stv[0] (the sets' states rotate; back in place after NS steps) --
                  // the special nodes' code is not in the instruction cache twice
                  if constexpr (KIND == K_FASTSCL_LUT && L8) {
                    if ((op.type == OP_R0 || op.type == OP_REP) && !(QPD_EXP_FSCL & 512)) {
                        r0rep_multi<kLdsTab, R1L>(P, Mv, op, stv, sel_all, sstride, gl, gbase, lane, cur.T2, tb);
                        return;
                    }
                    if (op.type == OP_R1 && (op.cnt <= stl::kThreshold || (fl & MF_R1_LDS)) && !(QPD_EXP_FSCL & 1024)) {
                        r1_multi<kLdsTab, R1L>(P, Mv, op, stv, sel_all, sstride, gl, gbase, lane, lds_rows, cur.T2, tb);
                        return;
                    }
                    // without R1L every R1 node of > 16 elements has its LDS tail (the host
                    // takes the R1L instantiation otherwise) and FastSCL-LUT has no SPC ops
                    // (H7): nothing is left for the generic special_op
                    if constexpr (!R1L) return;
                  }
#if QPD_SPEC_ROT
#pragma unroll 1
                  for (int s = 0; s < NS; ++s) {
                    special_op<kList, L8, R1L>(P, Mv[0].set(s), op, stv[0], sel_all + sstride * s, NS * sstride, gl, gbase,
                                               L, lane, lds_rows);
                    rotate_sets(stv);
                  }
#else
#pragma unroll
                  for (int s = 0; s < NS; ++s)
                    special_op<kList, L8, R1L>(P, Mv[s], op, stv[s], sel_all + sstride * s, NS * sstride, gl, gbase, L, lane,
                                               lds_rows);
#endif
              }
            };
            switch (op.type) {
                case OP_BOT3:
                    if constexpr (KIND == K_FASTSCL_LUT && L8 && !QPD_EXP_NO_BOTX) {
                        if (fl & MF_BOTX) {
                            if (kLazy && oi + 1 < P.nops) pre = fetch_pre(P, nxt, lane, vlane);
                            botx_op<kLdsTab, kChan>(P, Mv, op, yv, stv, cur.T, cur.T2, gl, gbase, L, sel_all, sstride, lane, tb);
                            break;
                        }
                    }
                    bot3_op<kList, LM, kLazy, kLdsTab, kChan>(P, Mv, op, yv, stv, cur.T, cur.T2, gl, gbase, L, sel_all, sstride, lane, [&]() {
                        if (oi + 1 < P.nops) pre = fetch_pre(P, nxt, lane, vlane);
                    }, tb);
                    break;
                case OP_F:
                case OP_G: {
                    int src[NS], usrc[NS];
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        src[s] = gbase + pfield(stv[s].ps, op.sh_src);
                        usrc[s] = gbase + pfield(stv[s].U(), op.sh_u);
                    }
                    if constexpr (kLdsTab) {
                        if (fl & MF_FF) {  // + the left child's f (fuse_descent)
                            const int key = ((fl & MF_DST_LDS) ? 1 : 0) | ((fl & MF_FF_DL) ? 2 : 0);
                            stage_tab(tb, cur.T, op.type == OP_F ? (lane & 31) : gtab_dw(lane));
                            stage_tab(tb + 512, cur.T2, lane & 31);
#define QPD_FF(G, D_, C_) ff_op<G, D_, C_, NS>(Mv, op, src, usrc, tb, lane)
                            if (op.type == OP_F) {
                                if (key == 0) QPD_FF(false, 0, 0);
                                else if (key == 2) QPD_FF(false, 0, 1);
                                else QPD_FF(false, 1, 1);
                            } else {
                                if (key == 0) QPD_FF(true, 0, 0);
                                else if (key == 2) QPD_FF(true, 0, 1);
                                else QPD_FF(true, 1, 1);
                            }
#undef QPD_FF
#pragma unroll
                            for (int s = 0; s < NS; ++s) stv[s].ps = pset(pset(stv[s].ps, op.sh_dst, gl), op.pad1, gl);
                            break;
                        }
                    }
                    if (fl & MF_GSEL)
                        gsel_op(Mv, op, yv, usrc, lane);
                    else if (NS >= 2 && !(fl & (MF_CHAN | MF_PRE))) {  // (one-set FastSCL: smaller code measured faster)
                        // row spaces of source and destination fixed per instantiation
                        const int key = ((fl & MF_SRC_LDS) ? 1 : 0) | ((fl & MF_DST_LDS) ? 2 : 0);
                        if constexpr (kLdsTab)
                            if (op.cnt >= 8) stage_tab(tb, cur.T, op.type == OP_F ? (lane & 31) : gtab_dw(lane));
#define QPD_FG(G, S_, D_) fg_op<G, true, NS, S_, D_, kLdsTab>(P, Mv, op, yv, src, usrc, cur.T, lane, tb)
                        // (S[d] in LDS puts S[d + 1] in LDS too: no key 1 variant)
                        if (op.type == OP_F) {
                            if (key == 0) QPD_FG(false, 0, 0);
                            else if (key == 2) QPD_FG(false, 0, 1);
                            else QPD_FG(false, 1, 1);
                        } else {
                            if (key == 0) QPD_FG(true, 0, 0);
                            else if (key == 2) QPD_FG(true, 0, 1);
                            else QPD_FG(true, 1, 1);
                        }
#undef QPD_FG
                    } else if (kChan && (fl & MF_CHAN)) {
                        if (op.type == OP_F) fg_chan_op<false>(P, Mv, op, yv, usrc, cur.T, lane);
                        else fg_chan_op<true>(P, Mv, op, yv, usrc, cur.T, lane);
                    } else if (op.type == OP_F)
                        fg_op<false, false>(P, Mv, op, yv, src, usrc, cur.T, lane);
                    else
                        fg_op<true, false>(P, Mv, op, yv, src, usrc, cur.T, lane);
#pragma unroll
                    for (int s = 0; s < NS; ++s) stv[s].ps = pset(stv[s].ps, op.sh_dst, gl);
                    break;
                }
                case OP_LEAF_L:
                case OP_LEAF_R: {
                    const bool right = op.type == OP_LEAF_R;
                    const bool frozen = op.cnt != 0;
                    double dm[NS];
                    uint32_t none[NS][1], dec[NS];
                    bool moved[NS];
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        dm[s] = 0;
                        none[s][0] = 0;
                        if (kList || !frozen) {
                            const uint32_t W = sym_word<kChan>(P, Mv[s], op, yv[s], gbase + pfield(stv[s].ps, op.sh_src), 0, 2);
                            uint32_t idx = QPD_LEAF_T ? (W & 0xFFu) : (((W & 15u) << 4) | ((W >> 4) & 15u));  // (leaf_idx)
                            if (right)
                                idx |= (Mv[s].ld(fl & MF_U_LDS, op.u_row, gbase + pfield(stv[s].U(), op.sh_u)) & 1u) << 8;
                            dm[s] = shfld(cur.V, (int)lut4(cur.T, idx));  // vcl[n-1][k][s] (H3)
                        }
                    }
                    leaf_decide<kList, LM>(stv, dm, frozen, gl, gbase, L, lane, sel_all, sstride, none, dec, moved);
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        Mv[s].st(fl & MF_DST_LDS, op.dst_row, lane, dec[s]);
                        if (!right) stv[s].U() = pset(stv[s].U(), op.sh_dst, gl);
                    }
                    break;
                }
                case OP_COMB: {
                    const int ctemp = op.cnt;
                    const bool ul = fl & MF_U_LDS, rl = fl & MF_R_LDS, dl = fl & MF_DST_LDS;
                    if (ctemp < 32) {
                        const uint32_t m = (1u << ctemp) - 1u;
                        uint32_t u[NS], r[NS];
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            u[s] = Mv[s].ld(ul, op.u_row, gbase + pfield(stv[s].U(), op.sh_u)) & m;
                            r[s] = Mv[s].ld(rl, op.r_row, lane) & m;
                        }
#pragma unroll
                        for (int s = 0; s < NS; ++s) Mv[s].st(dl, op.dst_row, lane, (u[s] ^ r[s]) | (r[s] << ctemp));
                    } else {
                        const int cw = ctemp >> 5;  // 1, 2 or a multiple of 4
                        int usrc[NS];
#pragma unroll
                        for (int s = 0; s < NS; ++s) usrc[s] = gbase + pfield(stv[s].U(), op.sh_u);
                        // 4 words of every set per round: all their loads in flight together
                        for (int w0 = 0; w0 < cw; w0 += 4) {
                            uint32_t u[NS][4], r[NS][4];
#pragma unroll
                            for (int s = 0; s < NS; ++s)
#pragma unroll
                                for (int k = 0; k < 4; ++k) {
                                    u[s][k] = r[s][k] = 0u;
                                    if (k == 0 || w0 + k < cw) {
                                        u[s][k] = Mv[s].ld(ul, op.u_row + w0 + k, usrc[s]);
                                        r[s][k] = Mv[s].ld(rl, op.r_row + w0 + k, lane);
                                    }
                                }
#pragma unroll
                            for (int s = 0; s < NS; ++s)
#pragma unroll
                                for (int k = 0; k < 4; ++k)
                                    if (k == 0 || w0 + k < cw) {
                                        Mv[s].st(dl, op.dst_row + w0 + k, lane, u[s][k] ^ r[s][k]);
                                        Mv[s].st(dl, op.dst_row + cw + w0 + k, lane, r[s][k]);
                                    }
                        }
                    }
                    if (!(fl & MF_TO_R)) {
#pragma unroll
                        for (int s = 0; s < NS; ++s) stv[s].U() = pset(stv[s].U(), op.sh_dst, gl);
                    }
                    break;
                }
                case OP_IMPORT:
                    if constexpr (KIND == K_SCL_LUT) {  // a frozen-prefix stage's records (lut_prefix_kernel)
                        const int live = op.tab2;
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            const bool dl = fl & MF_DST_LDS;
                            if (fl & MF_ZERO) {  // the prefix's partial sums: frozen zeros
                                for (int w = 0; w < op.cnt; ++w) Mv[s].st(dl, op.dst_row + w, lane, 0u);
                                continue;
                            }
                            int64_t f = (task * NS + s) * fpw + (lane >> gsh);
                            if (f >= B) f = B - 1;
                            const int G = op.vrow & 255;
                            // the record of this lane's path (dead paths: path 0's)
                            const uint32_t *src = (const uint32_t *)(((uint64_t)(uint32_t)op.r_row << 32) | (uint32_t)op.u_row) +
                                                  (((f >> G) * op.tab) << 6) + ((f & ((1 << G) - 1)) << (op.vrow >> 8)) +
                                                  (gl < live ? gl : 0);
                            if (fl & MF_PM) {
                                const uint64_t b = (uint64_t)src[op.src_row << 6] | ((uint64_t)src[(op.src_row + 1) << 6] << 32);
                                stv[s].pm = gl < live ? __builtin_bit_cast(double, b) : kInf;
                                            } else {  // live rows into every path's own column
                                for (int w = 0; w < op.cnt; ++w) Mv[s].st(dl, op.dst_row + w, lane, src[(op.src_row + w) << 6]);
                            }
                        }
                    }
                    break;
                case OP_EXPORT:
                    if constexpr (KIND == K_SCL_LUT && PFX) {  // the row of this path's lineage
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            const int64_t f = (task * NS + s) * fpw + (lane >> gsh);
                            const int at = (fl & MF_VIA_PS)   ? gbase + pfield(stv[s].ps, op.sh_src)
                                           : (fl & MF_VIA_PU) ? gbase + pfield(stv[s].U(), op.sh_src)
                                                              : lane;
                            const int G = P.pfx_geo & 255;
                            uint32_t *dst = P.pfx + (((f >> G) * P.pfx_rec) << 6) + ((f & ((1 << G) - 1)) << (P.pfx_geo >> 8)) + gl;
                            for (int w = 0; w < op.cnt; ++w) {
                                const uint32_t x = Mv[s].ld(fl & MF_SRC_LDS, op.src_row + w, at);
                                if (f < B) dst[(op.dst_row + w) << 6] = x;
                            }
                        }
                    }
                    break;
                default:
                    if constexpr (kFast) run_special();
                    break;
            }
#ifdef QPD_STAMPS
            __builtin_amdgcn_s_waitcnt(0);
            {
                const uint64_t dt = __builtin_amdgcn_s_memtime() - stamp_t0;
#ifdef QPD_STAMPS_DEPTH  // F / G / COMB by depth: 0-7 / 8-15 / 16-23; BOT3 24; leaves 25; specials 26-29
                const int dd = op.d < 7 ? op.d : 7;
                const int cls = op.type == OP_F ? dd : op.type == OP_G ? 8 + dd : op.type == OP_COMB ? 16 + dd
                              : op.type == OP_BOT3 ? ((fl & MF_BOTX) ? 30 : 24) : (op.type == OP_LEAF_L || op.type == OP_LEAF_R) ? 25
                              : 26 + (op.type - OP_R0) % 4;
#else
                const int cls = op.type == OP_R1 ? 24 + (op.cnt > 16) + (op.cnt > 8) : 2 * op.type + ((fl & MF_SYNC) ? 1 : 0);
#endif
                if ((int)(threadIdx.x & 31) == cls) stamp_acc += dt;
                if ((int)(threadIdx.x & 31) == cls) stamp_cnt += 1;
            }
#endif
        }
        if constexpr (PFX) {  // the stage's path metrics next to its rows; no decisions to output
            const int gl = threadIdx.x & (gs - 1);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int64_t f = (task * NS + s) * fpw + (threadIdx.x >> __builtin_ctz(gs));
                const int G = P.pfx_geo & 255;
                uint32_t *dst = P.pfx + (((f >> G) * P.pfx_rec) << 6) + ((f & ((1 << G) - 1)) << (P.pfx_geo >> 8)) + gl;
                const uint64_t b = __builtin_bit_cast(uint64_t, stv[s].pm);
                if (f < B) {
                    dst[P.pm_off << 6] = (uint32_t)b;
                    dst[(P.pm_off + 1) << 6] = (uint32_t)(b >> 32);
                }
            }
            wave_sync();  // the rows are reused by the next task, as after the tail below
            continue;
        }
#ifdef QPD_STAMPS
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t stamp_t2 = __builtin_amdgcn_s_memtime();
#endif

        // Root partial sums -> u = x F^{(x)n} (FastSCLUT.cpp:186-198), R[0] rows;
        // output u[info] of the winning path (SCLLUTDecoder.cpp:244-252).
        // FastSCL-LUT: the lane constants re-derived here too -- otherwise the compiler
        // computes the tail's lane-dependent addresses once before the task loop and
        // keeps them across the whole op loop in scratch (140 -> 80 B per lane, speed
        // unchanged).  Not for SCL-LUT: there the same change raised the SGPR spills
        // 148 -> 210 and cost 1.1 % (profiles/r06d_ab.txt); its scratch (112 B) is
        // written once before the task loop and read once per task, in the tail.
        int lane = threadIdx.x;
        if constexpr (KIND == K_FASTSCL_LUT) asm volatile("" : "+v"(lane));
        const int gl = lane & (gs - 1);
        const int gbase = lane & ~(gs - 1);
        const bool rl = P.R0_lds;
        const int r0 = P.R0_row;
        const int nwr = (N + 31) >> 5;
        const bool dword_out = (P.out_k & 3) == 0 && ((uintptr_t)out & 3) == 0;
        // Split tail (list decoders without CRC): the winner follows from the
        // path metrics alone, so only its root row is re-encoded, spread over
        // the frame's gs lanes (wpl words each; the cross-lane butterfly stages
        // by shuffles) and staged in this set's LDS rows for the output gather.
        const int wpl = nwr / gs;
        const bool split = kList && P.crc_n == 0 && nwr >= gs && wpl <= 8 && wpl <= P.lds_rows;
        if (!split) {  // every path re-encodes its own row (CRC-aided: each path's CRC is checked)
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const Mem &M = Mv[s];
                for (int w = 0; w < nwr; ++w) {
                    uint32_t x = M.ld(rl, r0 + w, lane);
                    if (N < 32) x &= (1u << N) - 1u;
                    M.st(rl, r0 + w, lane, polar_word(x));
                }
                for (int mw = 1; mw < nwr; mw *= 2)
                    for (int i = 0; i < nwr; i += 2 * mw)
                        for (int j = 0; j < mw; ++j)
                            M.st(rl, r0 + i + j, lane, M.ld(rl, r0 + i + j, lane) ^ M.ld(rl, r0 + i + mw + j, lane));
            }
            wave_sync();
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const Mem &M = Mv[s];
            int best = 0;
            if (kList && P.crc_n > 0) {
                best = ca_winner(stv[s].pm, gl, gbase, L, N, P.info_mask, P.ca_A, P.K - P.ca_A, P.crc_n, P.crc_q,
                                 [&](int w) { return M.ld(rl, r0 + w, lane); });
            } else if (kList) {
                double bpm = shfld(stv[s].pm, gbase);
                for (int j = 1; j < L; ++j) {
                    const double pj = shfld(stv[s].pm, gbase + j);
                    if (pj < bpm) {  // first minimum (H6)
                        bpm = pj;
                        best = j;
                    }
                }
            }
            const int src = gbase + best;
            const int wsh = __builtin_ctz(wpl > 0 ? wpl : 1);
            if (split) {
                uint32_t x[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) x[k] = k < wpl ? polar_word(M.ldv(rl, r0 + gl * wpl + k, src)) : 0u;
#pragma unroll
                for (int mw = 1; mw < 8; mw *= 2)  // word stages inside the lane
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (!(k & mw) && k + mw < wpl) x[k] ^= x[k + mw];
                for (int lm = 1; lm < gs; lm <<= 1)  // word stages across the frame's lanes
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (k < wpl) {
                            const uint32_t o = (uint32_t)lane_read((int)x[k], lane ^ lm);
                            if (!(gl & lm)) x[k] ^= o;
                        }
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k < wpl) M.lds[M.rw(k) + lane] = x[k];  // word gl*wpl + k at row k, column lane
                wave_sync();
            }
            const int64_t frame = (task * NS + s) * fpw + lane / gs;
            if (frame < B) {
                auto bit = [&](int pos) {
                    const int w = pos >> 5;
                    const uint32_t x = split ? M.lds[M.rw(w & (wpl - 1)) + gbase + (w >> wsh)] : M.ldv(rl, r0 + w, src);
                    return (x >> (pos & 31)) & 1u;
                };
                if (dword_out) {
                    // Four output bytes per store; 4 stores' loads issued together.
                    uint32_t *o32 = (uint32_t *)(out + frame * P.out_k);
                    const int nc = P.out_k >> 2;
                    for (int c0 = gl; c0 < nc; c0 += 4 * gs) {
                        uint32_t wv[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const int c = c0 + k * gs;
                            wv[k] = 0;
                            if (c < nc) {
                                const int4 pp = *(const int4 *)(P.info_pos + 4 * c);
                                wv[k] = bit(pp.x) | (bit(pp.y) << 8) | (bit(pp.z) << 16) | (bit(pp.w) << 24);
                            }
                        }
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            if (c0 + k * gs < nc) o32[c0 + k * gs] = wv[k];
                    }
                } else {
                    for (int t = gl; t < P.out_k; t += gs) out[frame * P.out_k + t] = (uint8_t)bit(P.info_pos[t]);
                }
            }
            if (split) wave_sync();  // the LDS rows are reused by the next set / task
        }
        wave_sync();
#ifdef QPD_STAMPS
        __builtin_amdgcn_s_waitcnt(0);
        if (threadIdx.x == 31) stamp_acc += __builtin_amdgcn_s_memtime() - stamp_t2;  // class 31: frame tail
        if (threadIdx.x == 31) stamp_cnt += 1;
        if (threadIdx.x < 32) {
            atomicAdd(&P.stamps[threadIdx.x], (unsigned long long)stamp_acc);
            atomicAdd(&P.stamps[32 + threadIdx.x], (unsigned long long)stamp_cnt);
        }
#endif
    }
}

// ---------------------------------------------------------------------------
// Frozen prefix (SCL-LUT in pre-mode): lut_fast_kernel<KIND, NS, false, false, true>.  Up to the first information leaf
// every path of a frame holds the same rows -- path 0 is the only one with a
// finite metric and all decisions are frozen zeros -- and until the third one
// at most 4 paths are live, yet the decode kernel would compute all of it L
// times (SCLLUTDecoder.cpp:62-144).  Two launches of this instantiation run
// that part of the schedule on the same op code and row layout:
//  * stage 1 -- the ops before the first forking op, one lane per frame (gs = 1,
//    64 frames per set);
//  * stage 2 -- from there to the op of the third information leaf at L = 4
//    (gs = 4), starting from stage 1's records (OP_IMPORT, MF_XBUF).
// Each stage ends with OP_EXPORT ops that write the rows the rest of the
// schedule reads before writing, through each path's lineage pointers, plus
// every path's metric, into the stage's own record buffer (d->pfx1_buf /
// pfx2_buf), interleaved across the frames of a 64-word block (FastPlan::pfx:
// address, record length and geometry).  The next stage or the decode kernel
// starts at the op after the split with OP_IMPORT ops (record address and
// layout in the op record) that copy each live path's record into its own
// column, zero the prefix's partial-sum rows (MF_ZERO) and load the metrics
// (MF_PM); dead slots start from path 0's rows with +inf.  The metrics are
// accumulated by the same code in the same leaf order, so the doubles are
// identical.
// ---------------------------------------------------------------------------
#define lut_prefix_kernel(KIND, NS, PW1) lut_fast_kernel<KIND, NS, false, false, true, PW1>

#ifndef QPD_FAST_TEMPLATES_ONLY  // qpd_fast_fscl.hip: the decode kernel templates only
// ---------------------------------------------------------------------------
// Root pre-pass (pre-mode: N >= 16, the root's left child a plain node).
// The root's f and both g variants depend on the channel symbols only, yet
// every path of a frame computes them (SCLLUTDecoder.cpp:83-89 / :157-164 at
// depth 0: L x N lookups per frame), and the decode kernel would read the
// frame's 4 KB of int32 symbols twice, half a decode apart.  Here one thread
// per output word computes them once per frame from one coalesced read of the
// channel, into a row of N/4 words per frame: [f(y) | g(y, 0) | g(y, 1) | -],
// N/16 words each, 8 nibble symbols per word as S[1].  The decode kernel then
// reads the left child's S[1] from the row (MF_PRE) and builds the root g by
// nibble selects (MF_GSEL, gsel_op).  Out-of-range symbols raise the error
// flag here, as chan_word8 does in the decode kernel.
// ---------------------------------------------------------------------------
// The root's f and g tables as bytes in LDS once per block (stage_tab): an
// element's 8-bit index addresses all three results (f, g with u = 0 at +0,
// u = 1 at +256) -- one field extract and three ds_read_u8 per element.
__global__ __launch_bounds__(256) void root_pre_kernel(FastPlan P, const int32_t *__restrict__ in, int64_t B,
                                                       uint32_t *__restrict__ pre) {
    __shared__ __attribute__((aligned(16))) uint8_t tf[256], tg[512];
    if (threadIdx.x < 64) {  // node 0 (posi 0)
        stage_tab(tg, P.g_tab[threadIdx.x], threadIdx.x);
        if (threadIdx.x < 32) stage_tab(tf, P.f_tab[threadIdx.x], threadIdx.x);
    }
    __syncthreads();
    const int wsh = P.n - 4;  // log2 words per segment
    const int half = P.N >> 1;
    const int64_t total = B << wsh;
    for (int64_t base = (int64_t)blockIdx.x * 256; base < total; base += (int64_t)gridDim.x * 256) {
        const int64_t t0 = base + threadIdx.x;
        const int64_t t = t0 < total ? t0 : total - 1;
        const int64_t f = t >> wsh;
        const int w = (int)(t & ((1 << wsh) - 1));
        const int32_t *y = in + (f << P.n);
        const uint32_t a = chan_word8(y, 8 * w, P.in_vec, P.v, P.err);
        const uint32_t b = chan_word8(y, half + 8 * w, P.in_vec, P.v, P.err);
        const uint32_t X = ((a << 4) & 0xF0F0F0F0u) | (b & 0x0F0F0F0Fu);  // byte j: index of element 2j
        const uint32_t Y = (a & 0xF0F0F0F0u) | ((b >> 4) & 0x0F0F0F0Fu);  // ... of element 2j + 1
        uint32_t fw = 0, g0 = 0, g1 = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t idx = __builtin_amdgcn_ubfe((k & 1) ? Y : X, 8 * (k >> 1), 8);
            fw |= (uint32_t)tf[idx] << (4 * k);
            g0 |= (uint32_t)tg[idx] << (4 * k);
            g1 |= (uint32_t)tg[256 + idx] << (4 * k);
        }
        if (t0 < total) {
            uint32_t *row = pre + (f << (P.n - 2));
            row[w] = fw;
            row[(1 << wsh) + w] = g0;
            row[(2 << wsh) + w] = g1;
        }
    }
}
#endif  // QPD_FAST_TEMPLATES_ONLY

}  // namespace qpd
