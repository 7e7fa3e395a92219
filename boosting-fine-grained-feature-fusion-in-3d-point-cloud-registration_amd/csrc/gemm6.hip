// "g6": f16x3 GEMM with BOTH operands pre-split into fragment images.
//
//   C[M, N] = act( sum_s sA[s][m] * (A_s[m, :] . W[n, :]) * wsc[n] + bias[n] (+ R[m, n]) )
//
// The activation operand arrives as an "A image" in the same fragment order as the weight
// images ([m16 panel][k32 step][term 2][g 4][16 rows] x 16 B) with one inverse scale per
// (row, k32 step): sA[s][m] = 2^-e, where 2^e brought that 32-wide chunk of the row into
// fp16's range before the hi / lo split (fgr_split_rows_h3, or a producer kernel's
// epilogue). The split -- 40-60 VALU per 16 x 32 fragment, the cost that kept the in-loop
// split kernels (gemm16.hip, gemm5.hip) at ~20-30 % of the pipe -- is thus paid ONCE per
// element, by whoever produces the activation, instead of once per consuming block.
//
// Structure: 256-thread blocks, 2 x 2 waves over (m, n), each wave a (BM/2 x BN/2) tile of
// TM x TN 16 x 16 fragments; per k32 step the A slice, the W slice and the step's A scales
// travel global -> LDS by LDS-DMA (global_load_lds, S stages in flight, counted vmcnt, raw
// s_barrier, all LDS in one array); per (i, j) fragment the three significant products
// accumulate into a zeroed temporary that is added to the accumulator with the lane's row
// scale (4 FMAs per 3 MFMAs). Swapped orientation (W fragments = MFMA A operand) as in the
// other f16x3 kernels: each lane's 4 accumulators belong to one activation row.
#include "common.h"

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm_lgkm0_6() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}

__device__ __forceinline__ float finish6(float y, float b, float r, int act) {
    if (act == FGR_ACT_RELU_RES_LEAKY) {
        const float t = fmaxf(y + b, 0.f) + r;
        return t > 0.f ? t : 0.1f * t;
    }
    const float t = y + b + r;
    return act == FGR_ACT_RELU ? fmaxf(t, 0.f) : t;
}

struct G6Args {
    const u32x4* A; int a_ksteps;      // A image; k32 steps per A panel
    const float* sA; int64_t ld_sA;     // inverse scales [kstep][ld_sA] (ld_sA >= M padded)
    const u32x4* W; int w_ksteps;      // W image (fgr_split_weights_h3)
    const float* wsc;                   // per n: 2^-e_n
    float* C; int64_t ldc;
    const float* bias;
    const float* R; int64_t ldr;
    int M, N, K, act, vec_out;
};

// RS: one scale per ROW for the whole K (fgr_split_rows_h3_rs, or a producer that sees full
// rows): the three products accumulate straight into acc (no per-step temporaries, no
// scale DMA) and the row scale is applied once in the epilogue.
template <int BM, int BN, int S, bool PROBE = false, int REP = 1, int KS = 1, bool RS = false>
__global__ void __launch_bounds__(256) gemm_g6(G6Args p) {
    constexpr int TM = BM / 32, TN = BN / 32;          // 16 x 16 fragments per wave
    constexpr int A_UNITS = (BM / 16) * 128;           // [panel][term][g][16] of one k32 step
    constexpr int W_UNITS = (BN / 16) * 128;
    constexpr int S_UNITS = RS ? 0 : 64;               // 4 pieces x 256 B of scales (BM <= 256)
    constexpr int ST1 = A_UNITS + W_UNITS + S_UNITS;   // one k32 step
    constexpr int ST = KS * ST1;                       // one stage = KS k32 steps
    constexpr int A_PIECES = A_UNITS / 64, W_PIECES = W_UNITS / 64;
    constexpr int NP1 = A_PIECES + W_PIECES + (RS ? 0 : 4);
    static_assert(NP1 % 4 == 0 && BM <= 256, "tile");
    constexpr int P1 = NP1 / 4, P = P1 * KS;           // DMA pieces per wave per k-step / stage
    __shared__ u32x4 lds[S * ST];

    const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int t = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int bm = t / nbn, bn = t % nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = (wv & 1) * (BM / 2), wn = (wv >> 1) * (BN / 2);
    const int g = lane >> 4, c = lane & 15;
    const int npanel_w = (p.N + 15) / 16;
    const int nst = (p.K + 32 * KS - 1) / (32 * KS);  // stages (images padded to even k32 steps)

    // DMA sources of one k32 step: piece q = wv + 4 j. A panels are padded to whole blocks
    // (fgr_split_rows_h3 allocates ceil(M / 256) * 16 panels), W panels are clamped.
    // (A_PIECES, W_PIECES multiples of 4: piece j's kind is the same in every wave)
    static_assert(A_PIECES % 4 == 0 && W_PIECES % 4 == 0, "pieces");
    constexpr int JA = A_PIECES / 4, JW = (A_PIECES + W_PIECES) / 4;
    const u32x4* src0[P1];
#pragma unroll
    for (int j = 0; j < P1; ++j) {
        const int q = wv + 4 * j;
        if (j < JA) {
            const int panel = q / 2, term = q % 2;
            src0[j] = p.A + ((int64_t)(m0 / 16 + panel) * p.a_ksteps) * 128 + term * 64 + lane;
        } else if (j < JW) {
            const int w = q - A_PIECES;
            const int panel = w / 2, term = w % 2;
            const int pg = min(n0 / 16 + panel, npanel_w - 1);
            src0[j] = p.W + ((int64_t)pg * p.w_ksteps) * 128 + term * 64 + lane;
        } else {
            const int sp = q - A_PIECES - W_PIECES;             // 256-B piece of the scales
            src0[j] = reinterpret_cast<const u32x4*>(p.sA + m0 + sp * 64 + lane);
        }
    }
    auto issue = [&](int s) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int k = s * KS + ks;                                  // k32 step
            __attribute__((address_space(3))) char* base =
                (__attribute__((address_space(3))) char*)(lds + (s % S) * ST + ks * ST1);
#pragma unroll
            for (int j = 0; j < P1; ++j) {
                const int q = wv + 4 * j;
                if (j >= JW) {
                    const float* src = reinterpret_cast<const float*>(src0[j]) + (int64_t)k * p.ld_sA;
                    __builtin_amdgcn_global_load_lds((const void*)src,
                                                     (lds_void*)(base + (A_UNITS + W_UNITS) * 16 +
                                                                 (q - A_PIECES - W_PIECES) * 256),
                                                     4, 0, 0);
                } else {
                    const u32x4* src = src0[j] + (int64_t)k * 128;
                    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + q * 1024),
                                                     16, 0, 0);
                }
            }
        }
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nst) issue(s);

    for (int s = 0; s < nst; ++s) {
        const int ahead = min(S - 2, nst - 1 - s);
        if constexpr (S >= 4) {
            if (ahead >= 2) wait_vm_lgkm0_6<2 * P>();
            else if (ahead == 1) wait_vm_lgkm0_6<P>();
            else wait_vm_lgkm0_6<0>();
        } else if constexpr (S == 3) {
            if (ahead >= 1) wait_vm_lgkm0_6<P>();
            else wait_vm_lgkm0_6<0>();
        } else {
            wait_vm_lgkm0_6<0>();
        }
        __builtin_amdgcn_s_barrier();
        // PROBE (timing experiment only, wrong results): no DMA after the prologue, so the
        // loop's cost without any global traffic is measured
        if (!PROBE && s + S - 1 < nst) issue(s + S - 1);
#pragma unroll 1
        for (int rep = 0; rep < REP; ++rep) {       // REP > 1: timing probe only
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
        const u32x4* st = lds + (PROBE ? 0 : (s % S) * ST) + ks * ST1;
        const float* sc = reinterpret_cast<const float*>(st + A_UNITS + W_UNITS);
        u32x4 af[TM][2], wf[TN][2];
        float sa[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int panel = (wm >> 4) + i;
            af[i][0] = st[panel * 128 + lane];
            af[i][1] = st[panel * 128 + 64 + lane];
            if constexpr (!RS) sa[i] = sc[wm + 16 * i + c];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int panel = (wn >> 4) + j;
            wf[j][0] = st[A_UNITS + panel * 128 + lane];
            wf[j][1] = st[A_UNITS + panel * 128 + 64 + lane];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const f16x8 wh = __builtin_bit_cast(f16x8, wf[j][0]);
            const f16x8 wl = __builtin_bit_cast(f16x8, wf[j][1]);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const f16x8 ah = __builtin_bit_cast(f16x8, af[i][0]);
                const f16x8 al = __builtin_bit_cast(f16x8, af[i][1]);
                if constexpr (RS) {
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, al, acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, acc[j][i], 0, 0, 0);
                } else {
                    f32x4 tt = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, f32x4{0.f, 0.f, 0.f, 0.f},
                                                                      0, 0, 0);
                    tt = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, al, tt, 0, 0, 0);
                    tt = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, tt, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[j][i][r] = __builtin_fmaf(tt[r], sa[i], acc[j][i][r]);
                }
            }
        }
        }
        }
    }

    // epilogue: lane holds C[m = m0 + wm + 16i + c][n = n0 + wn + 16j + 4g + r]
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm + 16 * i + c;
        if (m >= p.M) continue;
        const float rsc = RS ? p.sA[m] : 1.f;
        float* crow = p.C + (int64_t)m * p.ldc;
        const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn + 16 * j + 4 * g;
            if (n >= p.N) continue;
            const float4 ws = *reinterpret_cast<const float4*>(p.wsc + n);
            const float y[4] = {acc[j][i][0] * rsc * ws.x, acc[j][i][1] * rsc * ws.y,
                                acc[j][i][2] * rsc * ws.z, acc[j][i][3] * rsc * ws.w};
            if (p.vec_out && n + 3 < p.N) {
                float4 bb = make_float4(0.f, 0.f, 0.f, 0.f), rr = bb;
                if (p.bias) bb = *reinterpret_cast<const float4*>(p.bias + n);
                if (rrow) rr = *reinterpret_cast<const float4*>(rrow + n);
                *reinterpret_cast<float4*>(crow + n) =
                    make_float4(finish6(y[0], bb.x, rr.x, p.act), finish6(y[1], bb.y, rr.y, p.act),
                                finish6(y[2], bb.z, rr.z, p.act), finish6(y[3], bb.w, rr.w, p.act));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (n + e >= p.N) break;
                    crow[n + e] = finish6(y[e], p.bias ? p.bias[n + e] : 0.f,
                                          rrow ? rrow[n + e] : 0.f, p.act);
                }
            }
        }
    }
}

// fp32 rows -> A image + per-(row, k32 step) inverse scales. One wave per (16-row panel,
// k32 step) unit: lane (g, c) splits row c's 8 values k = 32 s + 8 g .. + 7 with the chunk's
// exponent (chunk max over the 4 g-lanes into [2^7, 2^8); all-zero chunk: scale 1, zeros).
__global__ void __launch_bounds__(256) split_rows_h3_kernel(const float* __restrict__ x,
                                                            int64_t ldx, int M, int K,
                                                            int ksteps, int64_t ld_s,
                                                            u32x4* __restrict__ img,
                                                            float* __restrict__ sA,
                                                            int64_t n_units) {
    const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u >= n_units) return;
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int s = (int)(u % ksteps);
    const int64_t panel = u / ksteps;
    const int64_t m = panel * 16 + c;
    const int k0 = s * 32 + 8 * g;
    float v[8];
    if (m < M && k0 + 8 <= K && (K % 4) == 0) {
        const float4 a = *reinterpret_cast<const float4*>(x + m * ldx + k0);
        const float4 b = *reinterpret_cast<const float4*>(x + m * ldx + k0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (m < M && k0 + e < K) ? x[m * ldx + k0 + e] : 0.f;
    }
    float cm = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) cm = fmaxf(cm, fabsf(v[e]));
    {
        auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
        auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
    }
    const int e = cm > 0.f ? min(8 - __builtin_amdgcn_frexp_expf(cm), 127) : 0;
    const float sc = __builtin_ldexpf(1.f, e);
    f16x8 h, lo;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float xs = v[q] * sc;
        const _Float16 hv = (_Float16)xs;
        h[q] = hv;
        lo[q] = (_Float16)(xs - (float)hv);
    }
    u32x4* dst = img + u * 128;
    dst[lane] = __builtin_bit_cast(u32x4, h);
    dst[64 + lane] = __builtin_bit_cast(u32x4, lo);
    if (g == 0) sA[(int64_t)s * ld_s + m] = __builtin_ldexpf(1.f, -e);
}

// fp32 rows -> A image with ONE exponent per row (the row's max over all of K into
// [2^14, 2^15); all-zero row: 0): one wave per 16-row panel; lane (g, c) walks row c's
// k-steps (8 values each), first for the max, then splitting with v_fma_mix. sA[m] = 2^-e.
__global__ void __launch_bounds__(256) split_rows_rs_kernel(const float* __restrict__ x,
                                                            int64_t ldx, int M, int K, int ksteps,
                                                            u32x4* __restrict__ img,
                                                            float* __restrict__ sA, int64_t n_panels) {
    const int64_t panel = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (panel >= n_panels) return;
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int64_t m = panel * 16 + c;
    const bool vec = (K % 4) == 0;
    auto load8 = [&](int s, float (&v)[8]) {
        const int k0 = s * 32 + 8 * g;
        if (m < M && k0 + 8 <= K && vec) {
            const float4 a = *reinterpret_cast<const float4*>(x + m * ldx + k0);
            const float4 b = *reinterpret_cast<const float4*>(x + m * ldx + k0 + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (m < M && k0 + e < K) ? x[m * ldx + k0 + e] : 0.f;
        }
    };
    float cm = 0.f;
    for (int s = 0; s < ksteps; ++s) {
        float v[8];
        load8(s, v);
        cm = fmaxf(cm, max3_abs(v[0], v[1], v[2]));
        cm = fmaxf(cm, max3_abs(v[3], v[4], v[5]));
        cm = fmaxf(cm, fmaxf(fabsf(v[6]), fabsf(v[7])));
    }
    {
        auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
        auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
    }
    const int e = cm > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(cm), 127) : 0;
    const float sc = __builtin_ldexpf(1.f, e);
    for (int s = 0; s < ksteps; ++s) {
        float v[8];
        load8(s, v);
        u32x4 hh, ll;
        split8_f16(v, sc, hh, ll);
        u32x4* dst = img + (panel * ksteps + s) * 128;
        dst[lane] = hh;
        dst[64 + lane] = ll;
    }
    if (g == 0 && m < M) sA[m] = __builtin_ldexpf(1.f, -e);
}

template <int BM, int BN, int S, bool PROBE = false, int REP = 1, int KS = 1, bool RS = false>
void launch_g6(const G6Args& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    hipLaunchKernelGGL((gemm_g6<BM, BN, S, PROBE, REP, KS, RS>), dim3((unsigned)(nbm * nbn)),
                       dim3(256), 0, st, a);
}

int ksteps6(int k) { return (k + 63) / 64 * 2; }
// A panels padded to whole 256-row blocks; scale rows padded by 256 for the 4-piece DMA
int64_t panels6(int m) { return (int64_t)(m + 255) / 256 * 16; }
int64_t ld_scales6(int m) { return panels6(m) * 16 + 256; }

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_split_rows_h3_bytes(int32_t m, int32_t k, size_t* bytes) {
    FGR_REQUIRE(bytes && m > 0 && k > 0, "fgr_split_rows_h3_bytes: bad arguments");
    *bytes = (size_t)panels6(m) * ksteps6(k) * 128 * 16 + (size_t)ksteps6(k) * ld_scales6(m) * 4;
    return FGR_OK;
}

extern "C" int fgr_split_rows_h3(const float* x, int64_t ldx, int32_t m, int32_t k, void* img,
                                 void* stream) {
    FGR_REQUIRE(x && img && m > 0 && k > 0 && ldx >= k && (reinterpret_cast<uintptr_t>(img) & 15) == 0,
                "fgr_split_rows_h3: bad arguments");
    FGR_REQUIRE(k % 4 != 0 || (ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0),
                "fgr_split_rows_h3: rows must be 16-B aligned when k %% 4 == 0");
    const int ks = ksteps6(k);
    const int64_t units = panels6(m) * ks;
    u32x4* im = static_cast<u32x4*>(img);
    float* sA = reinterpret_cast<float*>(im + units * 128);
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const char* rs = getenv("FGR_SPLIT_RS");     // experiment: one scale per row (RS GEMMs A..H)
    if (rs && rs[0] == '1')
        hipLaunchKernelGGL(split_rows_rs_kernel, dim3((unsigned)ceil_div(panels6(m), 4)), dim3(256), 0,
                           st, x, ldx, m, k, ks, im, sA, panels6(m));
    else
        hipLaunchKernelGGL(split_rows_h3_kernel, dim3((unsigned)ceil_div(units, 4)), dim3(256), 0, st, x,
                           ldx, m, k, ks, ld_scales6(m), im, sA, units);
    FGR_CHECK_LAUNCH("split_rows_h3_kernel");
    return FGR_OK;
}

extern "C" int fgr_gemm_h3_presplit(const void* a_img, const void* w_img, float* c, int64_t ldc,
                                    const float* bias, const float* r, int64_t ldr, int32_t m,
                                    int32_t n, int32_t k, int32_t act, void* stream) {
    FGR_REQUIRE(a_img && w_img && c && m > 0 && n > 0 && k > 0 && ldc >= n && (!r || ldr >= n),
                "fgr_gemm_h3_presplit: bad arguments (m %d n %d k %d)", m, n, k);
    FGR_REQUIRE(((reinterpret_cast<uintptr_t>(a_img) | reinterpret_cast<uintptr_t>(w_img)) & 15) == 0,
                "fgr_gemm_h3_presplit: images must be 16-B aligned");
    const int ks = ksteps6(k);
    const u32x4* A = static_cast<const u32x4*>(a_img);
    const float* sA = reinterpret_cast<const float*>(A + panels6(m) * ks * 128);
    const int npw = (n + 15) / 16;
    const float* wsc = reinterpret_cast<const float*>(static_cast<const char*>(w_img) +
                                                      (size_t)npw * ks * 128 * 16);
    const bool vo = (ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(c) & 15) == 0) &&
                    (!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0) &&
                    (!r || ((ldr % 4 == 0) && (reinterpret_cast<uintptr_t>(r) & 15) == 0));
    G6Args g{A, ks, sA, ld_scales6(m), (const u32x4*)w_img, ks, wsc, c, ldc, bias, r, ldr,
             m, n, k, act, vo ? 1 : 0};
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const char* force = getenv("FGR_GEMM_G6_TILE");
    const char cfg = force && force[0] ? force[0] : (n >= 512 ? 'b' : 'a');
    switch (cfg) {
        case 'a': launch_g6<64, 64, 4>(g, st); break;
        case 'b': launch_g6<128, 128, 3>(g, st); break;
        case 'c': launch_g6<64, 128, 4>(g, st); break;
        case 'd': launch_g6<128, 64, 4>(g, st); break;
        case 'e': launch_g6<128, 128, 4>(g, st); break;
        case 'f': launch_g6<64, 64, 3>(g, st); break;
        case 'g': launch_g6<128, 256, 2>(g, st); break;
        case 'h': launch_g6<256, 128, 2>(g, st); break;
        case 'y': launch_g6<64, 64, 3, true>(g, st); break;     // timing probes (wrong results)
        case 'z': launch_g6<128, 128, 3, true>(g, st); break;
        case 'w': launch_g6<64, 64, 3, true, 2>(g, st); break;
        case 'x': launch_g6<64, 64, 3, true, 4>(g, st); break;
        // two / four k32 steps per stage
        case 'i': launch_g6<64, 64, 2, false, 1, 2>(g, st); break;
        case 'j': launch_g6<64, 64, 3, false, 1, 2>(g, st); break;
        case 'k': launch_g6<64, 64, 2, false, 1, 4>(g, st); break;
        case 'l': launch_g6<128, 128, 2, false, 1, 2>(g, st); break;
        case 'm': launch_g6<64, 128, 2, false, 1, 2>(g, st); break;
        case 'n': launch_g6<128, 64, 2, false, 1, 2>(g, st); break;
        case 'o': launch_g6<64, 64, 3, true, 1, 2>(g, st); break;     // probe, 2 steps / stage
        // one scale per row (FGR_SPLIT_RS=1 images): A..H as a..h
        case 'A': launch_g6<64, 64, 4, false, 1, 1, true>(g, st); break;
        case 'B': launch_g6<128, 128, 3, false, 1, 1, true>(g, st); break;
        case 'C': launch_g6<64, 128, 4, false, 1, 1, true>(g, st); break;
        case 'D': launch_g6<128, 64, 4, false, 1, 1, true>(g, st); break;
        case 'E': launch_g6<128, 128, 4, false, 1, 1, true>(g, st); break;
        case 'F': launch_g6<64, 64, 3, false, 1, 1, true>(g, st); break;
        case 'G': launch_g6<128, 256, 2, false, 1, 1, true>(g, st); break;
        case 'H': launch_g6<256, 128, 2, false, 1, 1, true>(g, st); break;
        default: launch_g6<64, 64, 4>(g, st); break;
    }
    FGR_CHECK_LAUNCH("gemm_g6");
    return FGR_OK;
}
