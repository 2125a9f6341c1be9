/*
 * qpd.h -- C-ABI of the MI355X quantized polar decoder (libqpd.so).
 *
 * The drop-in boundary for the reference's L1 decoders.  Each entry point
 * replaces one piece of the reference's pybind11 surface
 * (/root/reference/PolarDecoder/PolarDecoder/_cpp):
 *
 *   qpd_create    <- the decoder constructors, which copy every table into the
 *                    object:  SCLUT::SCLUT        src/SCLUTDecoder.cpp:10-19
 *                             SCLLUT::SCLLUT      src/SCLLUTDecoder.cpp:33-44
 *                             FastSCLUT::FastSCLUT src/FastSCLUT.cpp:13-24
 *                             FastSCLLUT::FastSCLLUT src/FastSCLLUTDecoder.cpp:42-55
 *                             SC::SC              src/SCDecoder.cpp:7-12
 *                             CASCLLUT::CASCLLUT  src/CASCLLUTDecoder.cpp:43-62
 *                             CAFastSCLLUT::CAFastSCLLUT src/CAFastSCLLUTDecoder.cpp:43-56
 *                             SCL::SCL            src/SCLDecoder.cpp:30-36
 *                             CASCL::CASCL        src/CASCLDecoder.cpp:42-54
 *                             FastSC::FastSC      src/FastSCDecoder.cpp:13-19
 *                             FastSCL::FastSCL    src/FastSCLDecoder.cpp:40-47
 *                             SCUniformQuantizedDecoder  src/SCUniformQuantizedDecoder.cpp:9-18
 *                             SCLUniformQuantizedDecoder src/SCLUniformQuantizedDecoder.cpp:31-41
 *                             SCLloydQuantizedDecoder    src/SCLloydQuantizedDecoder.cpp:6-20
 *                             SCLLloydQuantizedDecoder   src/SCLLloydQuantizedDecoder.cpp:29-44
 *                   bound at py_interface/py_*.cpp (all 15 classes of
 *                   _libPolarDecoder.cpp:29-50)
 *   qpd_decode    <- SCLUT::decode   src/SCLUTDecoder.cpp:21-124
 *                    SCLLUT::decode  src/SCLLUTDecoder.cpp:47-253
 *                    FastSCLUT::decode src/FastSCLUT.cpp:27-206
 *                    FastSCLLUT::decode src/FastSCLLUTDecoder.cpp:57-408
 *                    CASCLLUT::decode src/CASCLLUTDecoder.cpp:64-303
 *                    CAFastSCLLUT::decode src/CAFastSCLLUTDecoder.cpp:58-454
 *                   (batched: B frames per call instead of one)
 *   qpd_decode_f64 <- SC::decode     src/SCDecoder.cpp:14-89 (float64 LLR input)
 *                    SCL::decode    src/SCLDecoder.cpp:38-176
 *                    CASCL::decode  src/CASCLDecoder.cpp:74-249
 *                    FastSC::decode src/FastSCDecoder.cpp:21-174
 *                    FastSCL::decode src/FastSCLDecoder.cpp:49-423
 *                    SC{,L}UniformQuantizedDecoder::decode src/SCUniformQuantizedDecoder.cpp:20-99,
 *                        src/SCLUniformQuantizedDecoder.cpp:43-184
 *                    SC{l,L}loydQuantizedDecoder::decode src/SCLloydQuantizedDecoder.cpp:22-101,
 *                        src/SCLLloydQuantizedDecoder.cpp:46-187
 *   qpd_decode_host / qpd_decode_f64_host: the same from host buffers
 *                   (copy in, decode, copy out, synchronous) -- what a
 *                   per-frame `decode(symbols)` call needs.
 *   qpd_destroy   <- the pybind11 object's destructor
 *
 * Plain pointers and sizes only; no torch or HIP types in the signatures
 * (streams are passed as `void*` = hipStream_t, NULL = default stream).
 *
 * Errors: every function returns QPD_OK (0) or a negative QPD_E* code and
 * records a message retrievable with qpd_last_error() (thread-local).  The
 * reference performs no validation (out-of-range symbols are UB there); this
 * library rejects bad configurations at create time and flags out-of-range
 * channel symbols on the device (reported by the host entry points and by
 * qpd_check_input_error()).
 */
#ifndef QPD_H
#define QPD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QPD_ABI_VERSION 6

/* Decoder kinds (the reference's class names). */
enum qpd_kind {
    QPD_SC_FLOAT = 0,    /* SCDecoder       (min-sum on float64 LLRs)        */
    QPD_SC_LUT = 1,      /* SCLUTDecoder                                      */
    QPD_SCL_LUT = 2,     /* SCLLUTDecoder                                     */
    QPD_FASTSC_LUT = 3,  /* FastSCLUTDecoder  (R0/R1/REP/SPC shortcuts)       */
    QPD_FASTSCL_LUT = 4, /* FastSCLLUTDecoder (R0/R1/REP shortcuts; no SPC)   */
    QPD_CASCL_LUT = 5,   /* CASCLLUTDecoder     (SCL-LUT + CRC-aided output)   */
    QPD_CAFASTSCL_LUT = 6, /* CAFastSCLLUTDecoder (FastSCL-LUT + CRC-aided output) */
    /* float64-LLR decoders (qpd_decode_f64) */
    QPD_SCL_FLOAT = 7,   /* SCLDecoder        (min-sum list; PM init 1e300)    */
    QPD_CASCL_FLOAT = 8, /* CASCLDecoder      (SCL + CRC from crc_n/crc_loc)   */
    QPD_FASTSC_FLOAT = 9,   /* FastSCDecoder  (R0/R1/REP/SPC shortcuts)        */
    QPD_FASTSCL_FLOAT = 10, /* FastSCLDecoder (R0/R1/REP shortcuts; no SPC)    */
    QPD_SC_UNIFORM = 11,  /* SCUniformQuantizedDecoder  (Q after every f/g)   */
    QPD_SCL_UNIFORM = 12, /* SCLUniformQuantizedDecoder                       */
    QPD_SC_LLOYD = 13,    /* SCLloydQuantizedDecoder    (bisect after f/g)    */
    QPD_SCL_LLOYD = 14    /* SCLLloydQuantizedDecoder                         */
};

enum qpd_status {
    QPD_OK = 0,
    QPD_E_INVALID = -1,     /* bad argument / configuration                  */
    QPD_E_UNSUPPORTED = -2, /* valid for the reference, not supported here   */
    QPD_E_DEVICE = -3,      /* HIP runtime failure                           */
    QPD_E_INPUT = -4        /* input the reference cannot decode defined-ly,
                               seen on device: a channel symbol outside
                               [0, v); a Lloyd index outside the
                               reconstruction list; a NaN path metric       */
};

/*
 * Decoder description.  All arrays are host pointers, copied at create time
 * (the reference's ctors copy too).
 *
 * Tables use the packed layout (quantized_decoder_polar_codes_amd/lut.py):
 *   f table t : lut_f[t*v*v + a*v + b]              a = first-half symbol
 *   g table t : lut_g[(t*2 + u)*v*v + a*v + b]      u = left partial sum
 *   node p = 2^depth + node - 1, element j of that node uses table
 *            f_base[p] + j*f_step  (f_step = 0: one table per node)
 *   vcl[((row*N) + pos)*v + sym], row in [0, vcl_rows)
 */
typedef struct qpd_config {
    int32_t kind;               /* enum qpd_kind                                  */
    int32_t N;                  /* code length, power of two, 2..65536            */
    int32_t K;                  /* output bits = number of 0 entries in frozen    */
    int32_t L;                  /* list size (SCL kinds), 1..32 (> 8: generic engine); ignored otherwise */
    int32_t v;                  /* symbol alphabet size, 2..256 (LUT kinds); the
                                   re-quantizer's v (uniform kinds: M = (v/2 - 0.5) r_f,
                                   (v/2 - 1) r_g, integer v/2)                    */
    const int32_t *frozen_bits; /* [N], 1 = frozen, 0 = information               */
    const int32_t *node_type;   /* [2N-1] node labels (Fast kinds), else NULL     */
    const uint8_t *lut_f;       /* [lut_f_count][v][v]                            */
    int32_t lut_f_count;
    const int32_t *f_base;      /* [N-1]                                          */
    int32_t f_step;             /* 0 or 1                                         */
    const uint8_t *lut_g;       /* [lut_g_count][2][v][v]                         */
    int32_t lut_g_count;
    const int32_t *g_base;      /* [N-1]                                          */
    int32_t g_step;             /* 0 or 1                                         */
    const double *vcl;          /* [vcl_rows][N][v], finite                       */
    int32_t vcl_rows;           /* >= log2(N)                                     */
    int32_t device;             /* HIP device ordinal (-1 = current device)       */
    int32_t max_waves;          /* persistent-grid size cap (0 = default)         */
    int32_t engine;             /* enum qpd_engine (0 = auto)                     */
    /* CRC-aided kinds only (ignored otherwise).  Output = the first A info bits
     * of the first path, in stable path-metric order, whose info bits [0, A)
     * reproduce bits [A, K) under the CRC (CRC::encoding, utils.cpp:77-92;
     * coefficient j of the divisor is 1 for j in crc_loc).  The reference's CA
     * decoders always check CRC-24 with loc {24,23,21,20,17,15,13,12,8,4,2,1,0}
     * (CASCLLUTDecoder.h:33-34) whatever crc_n/crc_p their ctor received; the
     * Python shim passes exactly that.  Requires 1 <= A <= K, K - A <= crc_n. */
    int32_t A;                  /* message bits before the CRC                    */
    int32_t crc_n;              /* CRC length, 1..32                              */
    const int32_t *crc_loc;     /* [crc_loc_count] coefficient indices in [0, crc_n] */
    int32_t crc_loc_count;
    /* QPD_CASCL_FLOAT honours crc_n/crc_loc as given (CASCLDecoder.cpp:49-53)
     * and compares exactly crc_n bits after the A info bits: requires
     * 1 <= A, A + crc_n <= K. */
    /* Uniform kinds: step r per node_posi (decoder_r_f / decoder_r_g). */
    const double *r_f;          /* [N-1] */
    const double *r_g;          /* [N-1] */
    /* Lloyd kinds: table t (0 = f, 1 = g) of node p is
     * q_bnd[bnd_off[t*(N-1)+p] ... + bnd_len[...]) (boundaries) and
     * q_rec[rec_off[...] ... + rec_len[...]) (reconstruction values). */
    const double *q_bnd;
    int32_t q_bnd_count;
    const double *q_rec;
    int32_t q_rec_count;
    const int32_t *bnd_off;     /* [2*(N-1)] */
    const int32_t *bnd_len;     /* [2*(N-1)], >= 1 */
    const int32_t *rec_off;     /* [2*(N-1)] */
    const int32_t *rec_len;     /* [2*(N-1)], >= 1 */
} qpd_config;

/* Kernel selection.  AUTO picks FAST when the tables allow it (one table per
 * node, v <= 16) and GENERIC otherwise; the env var QPD_ENGINE overrides. */
enum qpd_engine { QPD_ENGINE_AUTO = 0, QPD_ENGINE_GENERIC = 1, QPD_ENGINE_FAST = 2 };

typedef struct qpd_decoder qpd_decoder;

int qpd_abi_version(void);
/* Hash of the sources and flags the library was built from (build.py
 * source_hash): the Python loader refuses a library built from other sources. */
const char *qpd_build_id(void);
const char *qpd_last_error(void);

int qpd_create(const qpd_config *cfg, qpd_decoder **out);
void qpd_destroy(qpd_decoder *dec);

/* LUT kinds.  d_symbols: device int32 [B][N]; d_out: device uint8 [B][K]
 * ([B][A] for the CRC-aided kinds; qpd_info.out_bits).  Asynchronous on
 * `stream`.
 * A decoder owns its work buffers (slab, pre-pass rows, task queue, error
 * word, staging), so the library orders its calls: a call on a stream other
 * than the one the decoder's previous work ran on first makes that stream wait
 * for it (hipStreamWaitEvent), and host threads are serialized per handle.
 * Any mix of streams and host threads on one decoder therefore decodes as if
 * the calls ran one after another (the reference's synchronous contract,
 * py_SCLLUTDecoder.cpp:15); concurrent streams on ONE decoder do not overlap
 * -- use one decoder per stream for that. */
int qpd_decode(qpd_decoder *dec, const int32_t *d_symbols, int64_t B, uint8_t *d_out, void *stream);
/* float64-LLR kinds (QPD_SC_FLOAT, 7..14).  d_llr: device float64 [B][N];
 * d_out: device uint8 [B][K] ([B][A] for QPD_CASCL_FLOAT). */
int qpd_decode_f64(qpd_decoder *dec, const double *d_llr, int64_t B, uint8_t *d_out, void *stream);

/* Host-buffer variants (synchronous) -- what the reference's per-frame
 * decode(symbols) call needs.  Small batches (qpd_info.host_max_frames; one
 * frame per call in the reference drivers) run on the host engine, a C++
 * decoder of this library for a few frames (no launch, copy or stream
 * synchronization: SCLUTDecoder.cpp:21-124 costs ~10 us per frame on one core,
 * a GPU call ~0.1 ms); larger batches on the GPU kernels.  Both decode the
 * same bits (the reference's). */
int qpd_decode_host(qpd_decoder *dec, const int32_t *h_symbols, int64_t B, uint8_t *h_out);
int qpd_decode_f64_host(qpd_decoder *dec, const double *h_llr, int64_t B, uint8_t *h_out);

/* Where the host-buffer calls run: AUTO (the default; the host engine up to
 * qpd_info.host_max_frames frames, the GPU above), GPU (always), CPU (the host
 * engine for every batch; QPD_E_UNSUPPORTED for the re-quantized float kinds,
 * which the host engine does not decode).  The environment variable
 * QPD_HOST_ENGINE=gpu|cpu sets it at create time. */
enum qpd_host_mode { QPD_HOST_AUTO = 0, QPD_HOST_GPU = 1, QPD_HOST_CPU = 2 };
int qpd_set_host_engine(qpd_decoder *dec, int32_t mode);

/* Returns QPD_E_INPUT (and clears the flags) if any decode since the last
 * check saw a channel symbol outside [0, v), a Lloyd bisect index outside
 * the reconstruction list, or a NaN path metric reaching a list selection
 * (each undefined behaviour in the reference); waits for the decoder's
 * previous work (not the whole device). */
int qpd_check_input_error(qpd_decoder *dec);

/*
 * GPU-resident Monte-Carlo frames (replaces the driver loop
 * mainQuantizedDecoder_LLRDomain.py:151-176): for global frame ids
 * [frame0, frame0+B): message bits, polar encoding (x = u F^{(x)n}, natural
 * order), BPSK, AWGN (std sigma), LLR = 2y/sigma^2 and the driver's channel
 * quantizer (<= edges[0] -> 0, >= edges[M] -> q-1, else
 * lut[bisect_left(edges[:M], llr) - 1]).  Random numbers are Philox4x32-10 of
 * (seed, global frame id), so frames do not depend on batching or sharding.
 * d_msg: device uint8 [B][K]; d_symbols: device int32 [B][N].  For the
 * CRC-aided kinds the message is A random bits followed by the first K-A bits
 * of their CRC (the driver's CRCEnc, mainQuantizedDecoder_LLRDomain.py:153-156),
 * and d_msg holds the A message bits ([B][A]).
 */
typedef struct qpd_mc_channel {
    double sigma;           /* AWGN standard deviation                 */
    int32_t q;              /* number of channel symbols               */
    int32_t n_edges;        /* M+1, 2..257                             */
    const double *edges;    /* host [n_edges], ascending               */
    const int32_t *lut;     /* host [n_edges-1], values in [0, q)      */
} qpd_mc_channel;
int qpd_mc_frames(qpd_decoder *dec, const qpd_mc_channel *ch, uint64_t seed, int64_t frame0, int64_t B,
                  uint8_t *d_msg, int32_t *d_symbols, void *stream);
/* The same frames, decoded: d_out = what qpd_decode returns for the symbols
 * qpd_mc_frames generates with the same arguments (d_msg as there), without
 * materializing the int32 symbols -- on a fast-engine decoder in pre-mode the
 * generator writes the root pre-pass rows the decode kernel reads (LUT kinds;
 * q <= v).  d_counts (device int64[2], or NULL): bit errors and block errors of
 * the B frames (d_out against d_msg) are ADDED to it, the driver's counters
 * (:181-183).  The driver's loop body (mainQuantizedDecoder_LLRDomain.py:151-183)
 * in one call. */
int qpd_mc_decode(qpd_decoder *dec, const qpd_mc_channel *ch, uint64_t seed, int64_t frame0, int64_t B,
                  uint8_t *d_msg, uint8_t *d_out, int64_t *d_counts, void *stream);

/*
 * Offline table design (host code, no device needed) -- the reference's
 * MinDistortion LUT generator without OpenCV.
 *
 * qpd_optls_quantizer  <- LLRQuantizer::find_OptLS_quantizer
 *                         Quantizers/quantizers/_cpp/LLRQuantizer/LLRQuantizer.cpp:67-165
 *                         (Python twin QuantizeDensityEvolution/MinDistortionQuantizer.py:28-99):
 *   merge M LLR quanta (any order; density-weighted) into K groups of
 *   consecutive sorted quanta with minimum squared error.  Outputs
 *   density[K], quanta[K] (density-weighted means), lut[M] (symbol -> group)
 *   and the minimum distortion.
 * qpd_lutgen_mindistortion <- LLRQuantizerSC.run
 *                         QuantizeDensityEvolution/QLLRDensityEvolution_MinDistortion.py:73-126:
 *   density evolution of the v-level channel (density/quanta [v]) down the
 *   code tree; per node p = 2^depth + node - 1 one f table lut_f[p][a][b] and
 *   one g table lut_g[p][u][a][b] (uint8, [N-1][v][v] / [N-1][2][v][v]), and
 *   the evolved llr_density / llr_quanta [log2(N)+1][N][v] (llr_quanta is
 *   the decoders' virtual_channel_llr).  threads <= 0: all host cores.
 * sum_order: QPD_SUM_SEQUENTIAL = the C++ quantizer the reference generator
 * calls; QPD_SUM_NUMPY = its numpy twin (pairwise sums).  Returns 0, -1 on bad
 * arguments, -2 if a node has fewer than v distinct values (the reference
 * aborts there: CV_Assert(M >= K)).
 */
enum qpd_sum_order { QPD_SUM_SEQUENTIAL = 0, QPD_SUM_NUMPY = 1 };
int qpd_optls_quantizer(const double *density, const double *quanta, int32_t M, int32_t K, int32_t sum_order,
                        double *out_density, double *out_quanta, int32_t *out_lut, double *out_distortion);
int qpd_lutgen_mindistortion(int32_t N, int32_t v, const double *ch_density, const double *ch_quanta,
                             int32_t sum_order, int32_t threads, uint8_t *lut_f, uint8_t *lut_g,
                             double *llr_density, double *llr_quanta);

/* Introspection for tests / benchmarks. */
typedef struct qpd_info {
    int32_t kind, N, K, L, v;
    int32_t num_ops;          /* length of the static traversal schedule     */
    int32_t frames_per_wave;  /* frames decoded by one 64-lane wavefront     */
    int32_t lanes_per_frame;  /* lane stride of one frame (pow2 >= L)        */
    int32_t max_waves;        /* persistent grid cap                         */
    int64_t scratch_bytes_per_wave;
    int32_t engine;           /* enum qpd_engine actually used               */
    int32_t lds_bytes_per_wave;
    int32_t lds_from_depth;   /* fast engine: tree depths >= this live in LDS */
    int32_t out_bits;         /* bits per decoded frame: K, or A (CRC-aided)  */
    int64_t host_max_frames;  /* host-buffer calls of up to this many frames run
                                 on the host engine (qpd_set_host_engine); 0: none */
    int32_t prefix_ops;       /* fast engine, list kinds: ops of the frozen prefix run
                                 once per frame by lut_prefix_kernel (0: no split);
                                 num_ops counts both parts */
    int32_t last_engine;      /* enum qpd_ran: what decoded the handle's last decode
                                 call (tests assert that a "GPU" case ran the kernels) */
    int64_t lookups_per_path; /* f/g table lookups one path of one frame makes in the
                                 reference's traversal of this code (N log2 N for the
                                 SC/SCL kinds; fewer where special nodes skip subtrees):
                                 the algorithmic unit of the roofline (bench.py) */
    int32_t fast_variant;     /* fast engine: which decode kernel instantiation the plan
                                 runs -- bit 0: one pointer word per path (PW1); bit 1:
                                 the general special-node instantiation (R1L: R1 nodes
                                 beyond the LDS tail or without op-record ranks, R0 / REP
                                 nodes without one quanta row); 0 otherwise */
    int32_t reserved0;
} qpd_info;
/* qpd_info.last_engine: no decode yet, the GPU kernels (qpd_decode*, the GPU
 * branch of the host-buffer calls, qpd_mc_decode), or the host engine. */
enum qpd_ran { QPD_RAN_NONE = 0, QPD_RAN_GPU = 1, QPD_RAN_HOST = 2 };
int qpd_get_info(const qpd_decoder *dec, qpd_info *info);

/*
 * Kernel timing for benchmarks (no reference counterpart).  While enabled,
 * every kernel launch of this handle is bracketed by HIP events recorded on
 * the launch stream; qpd_kernel_times waits for them and returns, per kernel
 * class, the summed durations (ms) and the number of launches since the last
 * call, then forgets them.  Arrays have QPD_KC_COUNT entries.
 */
enum qpd_kernel_class {
    QPD_KC_PRE = 0,    /* root_pre_kernel (fast engine, root pre-pass)              */
    QPD_KC_DECODE = 1, /* lut_fast_kernel / generic_decode_kernel                   */
    QPD_KC_MC = 2,     /* mc_frames_kernel (qpd_mc_frames)                          */
    QPD_KC_PFX = 3,    /* lut_prefix_kernel (fast engine, frozen prefix of list kinds) */
    QPD_KC_COUNT = 4
};
int qpd_profile(qpd_decoder *dec, int32_t enable);
int qpd_kernel_times(qpd_decoder *dec, double *ms, int64_t *launches);

/*
 * On-chip peak probe (no reference counterpart): the LDS-path rate of one
 * instruction with every CU busy, measured on `device` by a streaming
 * microbenchmark (independent chains, 16 wave-instructions in flight per
 * wave, 8 waves per CU).  op: QPD_PROBE_BPERMUTE (ds_bpermute_b32, the
 * decoder's table lookups and fork copies), QPD_PROBE_READ_B32 (ds_read_b32,
 * its LDS rows), QPD_PROBE_READ_B64.  *gbps = bytes moved (64 lanes x width
 * per wave-instruction) / s.
 */
enum qpd_probe_op { QPD_PROBE_BPERMUTE = 0, QPD_PROBE_READ_B32 = 1, QPD_PROBE_READ_B64 = 2 };
int qpd_probe_lds(int32_t device, int32_t op, double *gbps);

#ifdef __cplusplus
}
#endif
#endif /* QPD_H */
