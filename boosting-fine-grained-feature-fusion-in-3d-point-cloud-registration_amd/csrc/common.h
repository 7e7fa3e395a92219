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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Two-term fp16 splits and 3-way max by single VALU instructions (gfx950), shared by the
// f16x3 GEMM and attention loops.
// max(|a|, |b|, |c|) in one v_max3_f32 (no NaN canonicalisation: finite activations)
__device__ __forceinline__ float max3_abs(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// Eight values x[0..7] times a power of two sc, split into packed fp16 hi terms
// h = f16(x sc) and lo terms l = f16(x sc - h): 16 v_fma_mix{lo,hi}_f16 (one per term and
// element; x sc is exact and so is x sc - h in fp32, so the bits equal the two-step split)
// in ONE asm statement that ends with `s_nop 1`: hipcc pads nothing inside asm and only one
// state after it, while a VGPR written by VALU and read as an MFMA operand needs two
// (cdna_hip_programming.md 5.7 item 2) -- without the pad an MFMA issued right after can
// read stale fragments. Outputs are early-clobber (written while inputs are still read).
__device__ __forceinline__ void split8_f16(const float (&x)[8], float sc, u32x4& h, u32x4& l) {
    unsigned h0, h1, h2, h3, l0, l1, l2, l3;
    asm("v_fma_mixlo_f16 %0, %8, %16, 0\n\t"
        "v_fma_mixlo_f16 %1, %10, %16, 0\n\t"
        "v_fma_mixlo_f16 %2, %12, %16, 0\n\t"
        "v_fma_mixlo_f16 %3, %14, %16, 0\n\t"
        "v_fma_mixhi_f16 %0, %9, %16, 0\n\t"
        "v_fma_mixhi_f16 %1, %11, %16, 0\n\t"
        "v_fma_mixhi_f16 %2, %13, %16, 0\n\t"
        "v_fma_mixhi_f16 %3, %15, %16, 0\n\t"
        "v_fma_mixlo_f16 %4, %8, %16, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %5, %10, %16, -%1 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %6, %12, %16, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %7, %14, %16, -%3 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %4, %9, %16, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %5, %11, %16, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %6, %13, %16, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %7, %15, %16, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "s_nop 1"
        : "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]),
          "v"(sc));
    h = u32x4{h0, h1, h2, h3};
    l = u32x4{l0, l1, l2, l3};
}

// Attention-weight dropout in training (nn.MultiheadAttention(dropout = p), transformers.py:
// 95-96): entry (head, query row, key row) of the softmax weights is dropped iff
// attn_drop_hash(seed, head, q, k) < thresh = p * 2^32 (rows are the packed token rows). A
// counter-based hash, so the forward and the two backward kernels draw the same mask without
// storing it (fgreg/autograd.py restates it for the tests). Not torch's Philox stream: masks
// differ from the reference's draw-for-draw, the distribution is the same (Bernoulli(1 - p)
// per entry, kept entries scaled by 1 / (1 - p)).
__device__ __forceinline__ uint32_t attn_drop_hash(uint32_t seed, int head, int64_t q, int64_t k) {
    uint32_t x = seed ^ ((uint32_t)head * 0x9E3779B9u);
    x ^= (uint32_t)q * 0x85EBCA6Bu;
    x = (x ^ (x >> 16)) * 0x7FEB352Du;
    x ^= (uint32_t)k * 0xC2B2AE35u;
    x = (x ^ (x >> 15)) * 0x846CA68Bu;
    return x ^ (x >> 16);
}

// attention16.hip: the training attention backward on the f16 matrix cores (fgr_attention_bwd_train)
size_t attn_bwd_f16x3_bytes(int64_t n_rows, int32_t n_seg, int32_t n_head, int32_t dh);
int attn_bwd_f16x3(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                   int64_t ldv, const float* o, int64_t ldo, const float* dout, int64_t lddo,
                   float* dq, int64_t lddq, float* dk, int64_t lddk, float* dv, int64_t lddv,
                   const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                   int32_t n_seg, int32_t n_kv_seg, int64_t n_rows, int64_t max_q_len,
                   int64_t max_kv_len, int32_t nhead, int32_t dh, float scale, const float* lse_in,
                   float* lse_out, float* dsum_out, bool dkdv, void* ws, uint32_t drop_seed,
                   uint32_t drop_thresh, float inv_keep, hipStream_t st);

// gemm_ws.hip: the weight-split row-stationary f16x3 GEMM (K = 256, N = 256 / 768, many rows);
// `ln` (optional): LayerNorm prologue (+ add, + side output out2, + K / V attention images)
struct WsLn {
    const float* g; const float* b; const float* add; int64_t ld_add; float eps;
    const float* g2; const float* b2; float* out2; int64_t ld_out2;
    char* kv_img; int2* kv_sc; int n_head; int kv_col0;
};
bool gemm_ws_supported(int m, int n, int k);
bool gemm_ws_ln_supported(int m, int n, int k);   // the LayerNorm-prologue forms (N 256 / 768)
bool gemm_ws_f16x3(const float* A, int64_t lda, const void* W, const float* wsc, float* C,
                   int64_t ldc, const float* bias, const float* R, int64_t ldr, int M, int N,
                   int K, int act, hipStream_t st, const WsLn* ln);

}  // namespace fgr
