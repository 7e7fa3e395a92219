// Shared helpers for the libfgreg kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/fgreg.h"

namespace fgr {

// Per-thread last-error string (the only mutable global state of the library).
void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Opt-in launch timing (fgr_time_next_call): a TimedCall placed right before an entry
// point's first launch records the armed start event there and the end event when the
// entry point returns, on the launch stream, then disarms -- so the measured interval
// holds this call's kernels only, not the caller's host time before the call.
void timing_arm_take(hipEvent_t* start, hipEvent_t* end);
struct TimedCall {
    hipStream_t st;
    hipEvent_t end = nullptr;
    explicit TimedCall(hipStream_t s) : st(s) {
        hipEvent_t start = nullptr;
        timing_arm_take(&start, &end);
        if (start) (void)hipEventRecord(start, st);
    }
    ~TimedCall() {
        if (end) (void)hipEventRecord(end, st);
    }
};

// Checks a kernel launch / runtime call; on failure records a message and returns.
#define FGR_CHECK_LAUNCH(what)                                                        \
    do {                                                                              \
        hipError_t e_ = hipGetLastError();                                            \
        if (e_ != hipSuccess) {                                                       \
            ::fgr::set_error("%s: %s", what, hipGetErrorString(e_));                  \
            return FGR_E_LAUNCH;                                                      \
        }                                                                             \
    } while (0)

#define FGR_CHECK_HIP(call)                                                           \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) {                                                       \
            ::fgr::set_error("%s: %s", #call, hipGetErrorString(e_));                 \
            return FGR_E_LAUNCH;                                                      \
        }                                                                             \
    } while (0)

#define FGR_REQUIRE(cond, ...)                                                        \
    do {                                                                              \
        if (!(cond)) {                                                                \
            ::fgr::set_error(__VA_ARGS__);                                            \
            return FGR_E_ARG;                                                         \
        }                                                                             \
    } while (0)

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}

// Reductions over the 16 lanes of a DPP row (lanes 16k..16k+15) on the VALU (no LDS
// crossbar): xor 1, xor 2 (quad_perm), then half-row and row mirrors.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
    v = fmaxf(v, dpp<0xB1>(v));    // quad_perm [1,0,3,2]
    v = fmaxf(v, dpp<0x4E>(v));    // quad_perm [2,3,0,1]
    v = fmaxf(v, dpp<0x141>(v));   // row_half_mirror
    v = fmaxf(v, dpp<0x140>(v));   // row_mirror
    return v;
}
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return v;
}
// Sum over all 64 lanes without the LDS crossbar: DPP within each 16-lane row, then
// v_permlane16/32_swap across the four rows; every lane gets the total.
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v = row16_sum(v);
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Index of the segment containing row r, given sorted offsets off[0..n] (off[0] = 0).
__device__ __forceinline__ int find_segment(const int64_t* off, int n, int64_t r) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Two-term fp16 splits and 3-way max by single VALU instructions (gfx950), shared by the
// f16x3 GEMM and attention loops.
// max(|a|, |b|, |c|) in one v_max3_f32 (no NaN canonicalisation: finite activations)
__device__ __forceinline__ float max3_abs(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// packed f16 (hi terms) of a sc, b sc: v_fma_mixlo / mixhi (round to nearest even, as a
// v_cvt_f16_f32 of the exact product)
__device__ __forceinline__ unsigned split_hi2(float a, float b, float sc) {
    unsigned d;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(d) : "v"(a), "v"(sc));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(d) : "v"(b), "v"(sc));
    return d;
}
// packed f16 (lo terms) of a sc - hi_a, b sc - hi_b (hi from split_hi2: f16 halves of h)
__device__ __forceinline__ unsigned split_lo2(float a, float b, float sc, unsigned h) {
    unsigned d;
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(d) : "v"(a), "v"(sc), "v"(h));
    asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "+v"(d) : "v"(b), "v"(sc), "v"(h));
    return d;
}

}  // namespace fgr
