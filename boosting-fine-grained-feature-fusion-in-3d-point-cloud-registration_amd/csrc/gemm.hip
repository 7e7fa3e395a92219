// Split-precision GEMM on the bf16 matrix cores: fp32-level accuracy at bf16 MFMA rate.
//
//   C[M, N] = act(A[M, K] . W[N, K]^T + bias[N] (+ R[M, N]))
//
// A (fp32 activations) is split on the fly, W (fp32 Linear weights, split once on the host)
// is given as bf16 pairs:  x = x_hi + x_lo,  x_hi = bf16(x),  x_lo = bf16(x - x_hi),
// and the product is accumulated in fp32 as  A_lo W_hi + A_hi W_lo + A_hi W_hi
// (v_mfma_f32_16x16x32_bf16, 3 MFMAs per tile step). The dropped A_lo W_lo term and the
// residual of the two-term split are ~2^-16 relative per product, far below the 1e-4
// parity bar, while the bf16 MFMA is 16x the fp32 MFMA rate on gfx950 (no xf32 exists).
//
// Block = 4 waves (2 x 2), tile BM x BN x 32; each wave owns (BM/2) x (BN/2) as
// (BM/32) x (BN/32) MFMA tiles. Per 32-deep k-step the next A / W tiles are loaded into
// registers while the current ones (in LDS, rows padded to 80 B so ds_read_b128 fragment
// loads are conflict-free) feed the MFMAs.
#include "common.h"

namespace fgr {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;
constexpr int PITCH = BK + 8;        // bf16 elements per LDS row (80 B)

struct GemmArgs {
    const float* A; int64_t lda;
    const __bf16* Whi; const __bf16* Wlo; int64_t ldw;   // (N, Kp) bf16, Kp % 32 == 0
    float* C; int64_t ldc;
    const float* bias;
    const float* R; int64_t ldr;
    int M, N, K, act;
};

template <int BM, int BN>
__global__ void __launch_bounds__(256) gemm_bf16x3_kernel(GemmArgs p) {
    constexpr int TM = BM / 32, TN = BN / 32;              // MFMA tiles per wave
    constexpr int AF4 = BM * BK / 4 / 256;                 // A float4 per thread per k-step
    constexpr int BV = BN * BK / 8 / 256;                  // W 16-B vectors (hi and lo) per thread
    static_assert(AF4 >= 1 && BV >= 1, "tile too small");
    __shared__ __attribute__((aligned(16))) __bf16 a_hi[BM * PITCH];
    __shared__ __attribute__((aligned(16))) __bf16 a_lo[BM * PITCH];
    __shared__ __attribute__((aligned(16))) __bf16 w_hi[BN * PITCH];
    __shared__ __attribute__((aligned(16))) __bf16 w_lo[BN * PITCH];

    // consecutive block ids walk the row panels of one W column panel
    const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
    const int bid = blockIdx.x;
    const int bm = bid % nbm, bn = bid / nbm;
    (void)nbn;
    const int m0 = bm * BM, n0 = bn * BN;

    const int tid = threadIdx.x, wv = tid / 64, lane = tid % 64;
    const int wm = (wv >> 1) * (BM / 2), wn = (wv & 1) * (BN / 2);
    const int fr = lane & 15, fk = (lane >> 4) * 8;

    float4 ar[AF4];
    uint4 whr[BV], wlr[BV];
    auto load = [&](int k0) {
#pragma unroll
        for (int j = 0; j < AF4; ++j) {
            const int f = tid + 256 * j;
            const int row = f / (BK / 4), kc = (f % (BK / 4)) * 4;
            const int m = m0 + row, k = k0 + kc;
            ar[j] = (m < p.M && k < p.K)
                        ? *reinterpret_cast<const float4*>(p.A + (int64_t)m * p.lda + k)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < BV; ++j) {
            const int f = tid + 256 * j;
            const int row = f / (BK / 8), kc = (f % (BK / 8)) * 8;
            const int n = n0 + row;
            if (n < p.N) {
                whr[j] = *reinterpret_cast<const uint4*>(p.Whi + (int64_t)n * p.ldw + k0 + kc);
                wlr[j] = *reinterpret_cast<const uint4*>(p.Wlo + (int64_t)n * p.ldw + k0 + kc);
            } else {
                whr[j] = make_uint4(0, 0, 0, 0);
                wlr[j] = make_uint4(0, 0, 0, 0);
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int j = 0; j < AF4; ++j) {
            const int f = tid + 256 * j;
            const int row = f / (BK / 4), kc = (f % (BK / 4)) * 4;
            const float4 a = ar[j];
            bf16x4 hi, lo;
            hi[0] = (__bf16)a.x; hi[1] = (__bf16)a.y; hi[2] = (__bf16)a.z; hi[3] = (__bf16)a.w;
            lo[0] = (__bf16)(a.x - (float)hi[0]);
            lo[1] = (__bf16)(a.y - (float)hi[1]);
            lo[2] = (__bf16)(a.z - (float)hi[2]);
            lo[3] = (__bf16)(a.w - (float)hi[3]);
            *reinterpret_cast<bf16x4*>(a_hi + row * PITCH + kc) = hi;
            *reinterpret_cast<bf16x4*>(a_lo + row * PITCH + kc) = lo;
        }
#pragma unroll
        for (int j = 0; j < BV; ++j) {
            const int f = tid + 256 * j;
            const int row = f / (BK / 8), kc = (f % (BK / 8)) * 8;
            *reinterpret_cast<uint4*>(w_hi + row * PITCH + kc) = whr[j];
            *reinterpret_cast<uint4*>(w_lo + row * PITCH + kc) = wlr[j];
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (p.K + BK - 1) / BK;
    load(0);
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();
        store();
        __syncthreads();
        if (kt + 1 < nk) load((kt + 1) * BK);
        bf16x8 ah[TM], al[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row = wm + i * 16 + fr;
            ah[i] = *reinterpret_cast<const bf16x8*>(a_hi + row * PITCH + fk);
            al[i] = *reinterpret_cast<const bf16x8*>(a_lo + row * PITCH + fk);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = wn + j * 16 + fr;
            const bf16x8 bh = *reinterpret_cast<const bf16x8*>(w_hi + col * PITCH + fk);
            const bf16x8 bl = *reinterpret_cast<const bf16x8*>(w_lo + col * PITCH + fk);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][j], 0, 0, 0);
            }
        }
    }

    // epilogue: C layout row = 4 * (lane >> 4) + r, col = lane & 15
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + j * 16 + fr;
        if (n >= p.N) continue;
        const float b = p.bias ? p.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
                if (m >= p.M) continue;
                float y = acc[i][j][r] + b;
                if (p.R) y += p.R[(int64_t)m * p.ldr + n];
                if (p.act == FGR_ACT_RELU) y = fmaxf(y, 0.f);
                p.C[(int64_t)m * p.ldc + n] = y;
            }
        }
    }
}

// fp32 weights -> (hi, lo) bf16 pairs, rows zero-padded to ldw (multiple of 32)
__global__ void split_weights_kernel(const float* __restrict__ w, int n, int k, int64_t ldw,
                                     __bf16* __restrict__ hi, __bf16* __restrict__ lo) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)n * ldw) return;
    const int64_t r = t / ldw;
    const int c = (int)(t - r * ldw);
    const float x = c < k ? w[r * k + c] : 0.f;
    const __bf16 h = (__bf16)x;
    hi[t] = h;
    lo[t] = (__bf16)(x - (float)h);
}

template <int BM, int BN>
void launch(const GemmArgs& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    hipLaunchKernelGGL((gemm_bf16x3_kernel<BM, BN>), dim3((unsigned)(nbm * nbn)), dim3(256), 0, st,
                       a);
}


// ------------------------------------------------------------------------------------
// bf16x6: fp32-accurate GEMM on the bf16 matrix cores.
//   x = h + m + l exactly-split bf16 terms (residual <= 2^-27 |x|); per 16x16x32 step the
//   six significant term products hh, hm, mh, hl, lh, mm accumulate in fp32 (dropped
//   ml, lm, ll ~ 2^-27 relative) -- fp32-level accuracy at 6 x 16 = 96 cycles per step
//   vs 8 x 32 = 256 on the fp32 MFMA.
// W (static) is pre-split by fgr_split_weights3 into an image laid out as the kernel's
// LDS tile: [n16 panel][k32 step][term 3][g 4][16 rows] x 16-B units (8 k each), so
// staging W is a flat copy. A (fp32 activations) is split in registers while staging:
// A LDS image [term 3][g 4][BM rows] units, row XOR (2g) so both the 16-B stores
// (8-lane groups: 2 rows x 4 g) and the ds_read_b128 fragment loads are conflict-free.
// 16x16x32 lane maps (lane l, g = l >> 4, c = l & 15): A[i = c][k = 8g + e],
// B[k = 8g + e][j = c], C[i = 4g + r][j = c].
// ------------------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

struct Gemm6Args {
    const float* A; int64_t lda;
    const u32x4* W; int ksteps;           // image, ksteps = ceil(K / 32)
    float* C; int64_t ldc;
    const float* bias;
    const float* R; int64_t ldr;
    int M, N, K, act;
};

template <int BM, int BN, bool KVEC>
__global__ void __launch_bounds__(256) gemm_bf16x6_kernel(Gemm6Args p) {
    constexpr int TM = BM / 32, TN = BN / 32;         // 16x16 subtiles per wave (2 x 2 waves)
    constexpr int UA = BM * 4 / 256;                   // A units (8 k of one row) per thread
    constexpr int UW = 12 * BN / 256;                  // W image units per thread
    static_assert(UA >= 1 && UW >= 1 && BM % 16 == 0 && BN % 16 == 0, "tile");
    __shared__ u32x4 a_lds[3 * 4 * BM];
    __shared__ u32x4 w_lds[12 * BN];

    const int nbm = (p.M + BM - 1) / BM;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int wm = (wv >> 1) * (BM / 2), wn = (wv & 1) * (BN / 2);
    const int g = lane >> 4, c = lane & 15;
    const int npanel = (p.N + 15) / 16;

    // Branch-free staging: rows past M and panels past N read a clamped (valid) address
    // -- their results are never stored; k past K is zeroed by a select.
    const float* arow[UA];
    int akk[UA];
#pragma unroll
    for (int j = 0; j < UA; ++j) {
        const int u = tid + 256 * j;
        arow[j] = p.A + (int64_t)min(m0 + (u >> 2), p.M - 1) * p.lda;
        akk[j] = 8 * (u & 3);
    }
    const u32x4* wsrc[UW];
#pragma unroll
    for (int j = 0; j < UW; ++j) {
        const int v = tid + 256 * j;
        const int panel = min(n0 / 16 + v / 192, npanel - 1);
        wsrc[j] = p.W + (int64_t)panel * p.ksteps * 192 + v % 192;
    }
    float4 ar[UA][2];
    u32x4 wr[UW];
    auto load = [&](int s) {
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int k = s * 32 + akk[j];
            if constexpr (KVEC) {
                const float* src = arow[j] + min(k, p.K - 8);
                float4 x0 = *reinterpret_cast<const float4*>(src);
                float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                const bool ok = k < p.K;
                ar[j][0] = ok ? x0 : make_float4(0.f, 0.f, 0.f, 0.f);
                ar[j][1] = ok ? x1 : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float t[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float xv = arow[j][min(k + e, p.K - 1)];
                    t[e] = k + e < p.K ? xv : 0.f;
                }
                ar[j][0] = make_float4(t[0], t[1], t[2], t[3]);
                ar[j][1] = make_float4(t[4], t[5], t[6], t[7]);
            }
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) wr[j] = wsrc[j][(int64_t)s * 192];
    };
    auto store = [&]() {
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int u = tid + 256 * j;
            const int row = u >> 2, gg = u & 3;
            const float x[8] = {ar[j][0].x, ar[j][0].y, ar[j][0].z, ar[j][0].w,
                                ar[j][1].x, ar[j][1].y, ar[j][1].z, ar[j][1].w};
            bf16x8 th, tm, tl;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                __bf16 h, m, l;
                split3(x[e], h, m, l);
                th[e] = h; tm[e] = m; tl[e] = l;
            }
            const int r = row ^ (2 * gg);
            a_lds[(0 * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, th);
            a_lds[(1 * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, tm);
            a_lds[(2 * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, tl);
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) w_lds[tid + 256 * j] = wr[j];
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (p.K + 31) / 32;
    load(0);
    for (int s = 0; s < nk; ++s) {
        __syncthreads();
        store();
        __syncthreads();
        if (s + 1 < nk) load(s + 1);
        bf16x8 bw[TN][3];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int pp = (wn + 16 * j) >> 4;
#pragma unroll
            for (int t = 0; t < 3; ++t)
                bw[j][t] = __builtin_bit_cast(bf16x8, w_lds[pp * 192 + (t * 4 + g) * 16 + c]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int r = (wm + 16 * i + c) ^ (2 * g);
            const bf16x8 ah = __builtin_bit_cast(bf16x8, a_lds[(0 * 4 + g) * BM + r]);
            const bf16x8 am = __builtin_bit_cast(bf16x8, a_lds[(1 * 4 + g) * BM + r]);
            const bf16x8 al = __builtin_bit_cast(bf16x8, a_lds[(2 * 4 + g) * BM + r]);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bw[j][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bw[j][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bw[j][2], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bw[j][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bw[j][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bw[j][0], acc[i][j], 0, 0, 0);
            }
        }
    }

#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + j * 16 + c;
        if (n >= p.N) continue;
        const float b = p.bias ? p.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + i * 16 + 4 * g + r;
                if (m >= p.M) continue;
                float y = acc[i][j][r] + b;
                if (p.R) y += p.R[(int64_t)m * p.ldr + n];
                if (p.act == FGR_ACT_RELU) y = fmaxf(y, 0.f);
                p.C[(int64_t)m * p.ldc + n] = y;
            }
        }
    }
}

// W (n x k, element (i, j) at w[i * sn + j * sk]) -> bf16x6 image (see above)
__global__ void split_weights3_kernel(const float* __restrict__ w, int n, int k, int64_t sn,
                                      int64_t sk, int ksteps, u32x4* __restrict__ img) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // image unit
    const int64_t total = (int64_t)((n + 15) / 16) * ksteps * 192;
    if (u >= total) return;
    const int i = (int)(u % 16);
    const int g = (int)((u / 16) % 4);
    const int t = (int)((u / 64) % 3);
    const int64_t ps = u / 192;
    const int s = (int)(ps % ksteps);
    const int panel = (int)(ps / ksteps);
    const int row = panel * 16 + i;
    bf16x8 out;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int col = s * 32 + 8 * g + e;
        const float x = (row < n && col < k) ? w[row * sn + col * sk] : 0.f;
        __bf16 h, m, l;
        split3(x, h, m, l);
        out[e] = t == 0 ? h : (t == 1 ? m : l);
    }
    img[u] = __builtin_bit_cast(u32x4, out);
}

template <int BM, int BN>
void launch6(const Gemm6Args& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    if (a.K % 8 == 0)
        hipLaunchKernelGGL((gemm_bf16x6_kernel<BM, BN, true>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((gemm_bf16x6_kernel<BM, BN, false>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_split_weights(const float* w, int32_t n, int32_t k, int64_t ldw, void* w_hi,
                                 void* w_lo, void* stream) {
    FGR_REQUIRE(w && w_hi && w_lo && n > 0 && k > 0 && ldw >= k && ldw % 32 == 0,
                "fgr_split_weights: bad arguments");
    const int64_t tot = (int64_t)n * ldw;
    hipLaunchKernelGGL(split_weights_kernel, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0,
                       as_stream(stream), w, n, k, ldw, (__bf16*)w_hi, (__bf16*)w_lo);
    FGR_CHECK_LAUNCH("split_weights_kernel");
    return FGR_OK;
}

extern "C" int fgr_gemm_bf16x3(const float* a, int64_t lda, const void* w_hi, const void* w_lo,
                               int64_t ldw, float* c, int64_t ldc, const float* bias,
                               const float* r, int64_t ldr, int32_t m, int32_t n, int32_t k,
                               int32_t act, void* stream) {
    FGR_REQUIRE(a && w_hi && w_lo && c && m >= 0 && n > 0 && k > 0 && k % 4 == 0 &&
                    lda >= k && lda % 4 == 0 && ldw >= k && ldw % 32 == 0 && ldc >= n &&
                    (!r || ldr >= n),
                "fgr_gemm_bf16x3: bad arguments (m %d n %d k %d lda %lld ldw %lld)", m, n, k,
                (long long)lda, (long long)ldw);
    FGR_REQUIRE((reinterpret_cast<uintptr_t>(a) & 15) == 0, "fgr_gemm_bf16x3: A not 16-B aligned");
    if (m == 0) return FGR_OK;
    GemmArgs g{a, lda, (const __bf16*)w_hi, (const __bf16*)w_lo, ldw, c, ldc, bias, r, ldr,
               m, n, k, act};
    hipStream_t st = as_stream(stream);
    // tile choice: big tiles when they still give >= 2 blocks per CU-ish, else 64 x 64
    const int64_t big = (int64_t)ceil_div(m, 128) * ceil_div(n, 128);
    if (big >= 512)
        launch<128, 128>(g, st);
    else if ((int64_t)ceil_div(m, 128) * ceil_div(n, 64) >= 384)
        launch<128, 64>(g, st);
    else
        launch<64, 64>(g, st);
    FGR_CHECK_LAUNCH("gemm_bf16x3_kernel");
    return FGR_OK;
}

extern "C" int fgr_split_weights3_bytes(int32_t n, int32_t k, size_t* bytes) {
    FGR_REQUIRE(bytes && n > 0 && k > 0, "fgr_split_weights3_bytes: bad arguments");
    *bytes = (size_t)((n + 15) / 16) * ((k + 31) / 32) * 192 * 16;
    return FGR_OK;
}

extern "C" int fgr_split_weights3(const float* w, int32_t n, int32_t k, int64_t stride_n,
                                  int64_t stride_k, void* img, void* stream) {
    FGR_REQUIRE(w && img && n > 0 && k > 0, "fgr_split_weights3: bad arguments");
    const int ksteps = (k + 31) / 32;
    const int64_t total = (int64_t)((n + 15) / 16) * ksteps * 192;
    hipLaunchKernelGGL(split_weights3_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0,
                       as_stream(stream), w, n, k, stride_n, stride_k, ksteps, (u32x4*)img);
    FGR_CHECK_LAUNCH("split_weights3_kernel");
    return FGR_OK;
}

extern "C" int fgr_gemm_bf16x6(const float* a, int64_t lda, const void* w_img, float* c,
                               int64_t ldc, const float* bias, const float* r, int64_t ldr,
                               int32_t m, int32_t n, int32_t k, int32_t act, void* stream) {
    FGR_REQUIRE(a && w_img && c && m >= 0 && n > 0 && k > 0 && lda >= k && ldc >= n &&
                    (!r || ldr >= n),
                "fgr_gemm_bf16x6: bad arguments (m %d n %d k %d lda %lld)", m, n, k,
                (long long)lda);
    const bool vec = (k % 8 == 0) && (lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(a) & 15) == 0);
    FGR_REQUIRE(vec || (k % 8 != 0), "fgr_gemm_bf16x6: A must be 16-B aligned with lda %% 4 == 0");
    if (m == 0) return FGR_OK;
    Gemm6Args g{a, lda, (const u32x4*)w_img, (k + 31) / 32, c, ldc, bias, r, ldr, m, n, k, act};
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    // tile choice (measured on the forward's shapes, microbench.py tiles): 64 x 128 for wide
    // outputs (N >= 512, N % 256 == 0), 64 x 64 otherwise -- small tiles at 4-5 blocks per
    // CU hide the 2-barrier staging better than 128 x 128 at 2. FGR_GEMM6_TILE overrides it
    // for tuning (a = 128x128, b = 128x64, c = 64x64, d = 64x128).
    const char* force = getenv("FGR_GEMM6_TILE");
    const char cfg = (force && force[0]) ? force[0] : (n >= 512 && n % 256 == 0) ? 'd' : 'c';
    if (cfg == 'a')
        launch6<128, 128>(g, st);
    else if (cfg == 'b')
        launch6<128, 64>(g, st);
    else if (cfg == 'd')
        launch6<64, 128>(g, st);
    else
        launch6<64, 64>(g, st);
    FGR_CHECK_LAUNCH("gemm_bf16x6_kernel");
    return FGR_OK;
}
