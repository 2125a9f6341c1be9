// qpd_probe.hip -- on-chip peak probe for the roofline of the decode kernel
// (bench.py `roofline`): the chip-wide rate of the LDS-path
// instructions lut_fast_kernel issues, measured on the box it runs on.
//
// Each wave keeps 16 independent chains in flight; every wave-instruction
// moves 64 lanes x width bytes.  Addresses are conflict-free (lane-distinct
// banks), so the result is the instruction's streaming peak, not a pattern.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace qpd {

constexpr int kProbeChains = 16;
constexpr int kProbeThreads = 256;                 // 4 waves per workgroup
constexpr int kProbeLdsWords = kProbeThreads * 32;  // 32 KB: 8 waves/CU fit twice over

template <int OP>
__global__ __launch_bounds__(kProbeThreads) void lds_probe_kernel(int iters, uint32_t *sink) {
    __shared__ uint32_t buf[kProbeLdsWords];
    const int t = threadIdx.x, lane = t & 63;
    for (int i = t; i < kProbeLdsWords; i += kProbeThreads) buf[i] = (uint32_t)i;  // identity: x = buf[x] stays put
    __syncthreads();
    uint32_t x[kProbeChains];
#pragma unroll
    for (int k = 0; k < kProbeChains; ++k) {
        if (OP == 0) x[k] = (uint32_t)(((lane + 5 * k + 1) & 63) * 4);  // a byte address into the wave's lanes
        else if (OP == 1) x[k] = (uint32_t)(k * kProbeThreads + t);    // dword index, 64 distinct banks per wave
        else x[k] = (uint32_t)(2 * (k * 64 + lane) + (t >> 6) * 2 * kProbeChains * 64) % kProbeLdsWords;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < kProbeChains; ++k) {
            if (OP == 0) {
                // the value read is lane (addr >> 2)'s address: another valid address
                x[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)x[k], (int)x[k]);
            } else if (OP == 1) {
                x[k] = buf[x[k]];
            } else {
                const uint2 w = *reinterpret_cast<const uint2 *>(&buf[x[k] & ~1u]);
                x[k] = (w.x + w.y) >> 1;  // (x + x + 1) / 2 = x; both dwords used
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < kProbeChains; ++k) acc ^= x[k];
    if (acc == 0xFFFFFFFFu) sink[blockIdx.x] = acc;  // never true; keeps the chains live
}

// Runs the probe on the current device; returns bytes/s through *gbps (GB/s).
inline hipError_t probe_lds_run(int op, double *gbps) {
    int dev = 0, ncu = 256;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = ncu * 4;  // 16 waves per CU (4 per SIMD), 128 KB of LDS
    const int iters = 2048;
    uint32_t *sink = nullptr;
    if ((e = hipMalloc(&sink, sizeof(uint32_t) * blocks)) != hipSuccess) return e;
    const void *k = op == 0 ? reinterpret_cast<const void *>(&lds_probe_kernel<0>)
                  : op == 1 ? reinterpret_cast<const void *>(&lds_probe_kernel<1>)
                            : reinterpret_cast<const void *>(&lds_probe_kernel<2>);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    double best = 0.0;
    int it_arg = iters;
    void *args[] = {&it_arg, &sink};
    for (int rep = 0; rep < 4 && e == hipSuccess; ++rep) {
        (void)hipEventRecord(e0, nullptr);
        e = hipLaunchKernel(k, dim3(blocks), dim3(kProbeThreads), args, 0, nullptr);
        (void)hipEventRecord(e1, nullptr);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms > 0.f) {  // rep 0 is the warm-up
            const double width = op == 2 ? 8.0 : 4.0;
            const double bytes = (double)blocks * (kProbeThreads / 64) * iters * kProbeChains * 64.0 * width;
            const double r = bytes / (ms * 1e-3) / 1e9;
            if (r > best) best = r;
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(sink);
    *gbps = best;
    return e;
}

}  // namespace qpd
