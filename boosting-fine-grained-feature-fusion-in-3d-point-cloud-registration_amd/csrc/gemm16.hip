// fp32-accurate GEMM on the fp16 matrix cores with scaled two-term splits ("f16x3").
//
//   C[M, N] = act(A[M, K] . W[N, K]^T + bias[N] (+ R[M, N]))
//
// Precision design. gfx950 has no xf32; its fp32 MFMA runs at 1/16 of the fp16/bf16 rate.
// An fp16 term carries 11 significant bits, so a two-term split x = h + m (h = f16(x),
// m = f16(x - h), both round-to-nearest) represents x to 2^-22 relative -- PROVIDED both
// terms stay in fp16's normal range. That is what the scales are for:
//   * W rows (output channels n) are scaled once, by a power of two, so that the row's
//     max |w| lies in [2^14, 2^15) (fgr_split_weights_h3, cached with the weight);
//   * A rows (activations) are scaled in flight by a power of two per row, chosen from the
//     first non-zero 32-wide k chunk so its max lands in [2^7, 2^8), and lowered (with the
//     row's partial sums rescaled by the same exact power of two) only when a later chunk
//     would pass 2^15 -- fp16 overflow is impossible and the common path costs one compare.
// Per 16x16x32 step the three significant products hh, hm, mh accumulate in fp32 on
// v_mfma_f32_16x16x32_f16; the dropped mm term is <= 2^-22 relative. Net: <= ~3 * 2^-22
// per product (below fp32 accumulation's own rounding for K >= 16), at 3 MFMAs per step
// where the bf16x6 split needs 6 -- half the matrix-core work, 2/3 of the operand bytes.
//
// Orientation ("swapped"): the MFMA computes C^T tiles, W fragments as the A operand and
// activation fragments as the B operand, so every lane's four accumulator values belong to
// ONE activation row (its column c): the per-row scale is lane-local and the epilogue
// stores 16-B float4s of C.
//
// Tiling: 256-thread blocks, 2 x 2 waves over (n, m), block tile BN x BM x 32. W images are
// flat-copied into LDS; A (fp32) is split in registers while staging into a
// [term][g][row ^ 2g] LDS image (conflict-free 16-B stores and ds_read_b128 fragment
// loads); the per-row scale exponents go through a small LDS array. Block ids are
// remapped so the blocks sharing an A row panel run on one XCD (its L2 keeps the panel).
// 16x16x32 f16 lane maps (lane l, g = l >> 4, c = l & 15): A[i = c][k = 8g + e],
// B[k = 8g + e][j = c], C[i = 4g + r][j = c].
#include "common.h"

namespace fgr {
bool gemm_g5_f16x3(char cfg, const float* A, int64_t lda, const void* W, int ksteps,
                   const float* wsc, float* C, int64_t ldc, const float* bias, const float* R,
                   int64_t ldr, int M, int N, int K, int act, int vec_out, hipStream_t st,
                   int ksplit, float* part);
bool g5_tile(char cfg, int* bm, int* bn);
bool gemm_g5_f16x3_qkv(const float* A, int64_t lda, const void* W, int ksteps, const float* wsc,
                       float* q, int64_t ld_q, const float* bias, int M, int d, int n_head,
                       char* kv_img, int2* kv_sc, hipStream_t st);
int g5_ksplit(int M, int N, int K, int BM, int BN);
char bf16_tile(int m, int n, int k);
int bf16_ksplit(char cfg, int m, int n, int k);
struct RsLn {
    const float* g; const float* b; const float* add; int64_t ld_add; float eps;
    const float* g2; const float* b2; float* out2; int64_t ld_out2;    // optional side output
    char* kv_img; int2* kv_sc; int n_head; int kv_col0;                // optional K / V images
};
struct RsHead {
    int n_act; float* c2;
    const float* w4; const float* b4; float* out3;
};
bool gemm_rs_f16x3(const float* A, int64_t lda, const void* W, int ksteps, const float* wsc,
                   float* C, int64_t ldc, const float* bias, const float* R, int64_t ldr, int M,
                   int N, int K, int act, hipStream_t st, const RsLn* ln = nullptr,
                   const RsHead* head = nullptr);
// few 64 x 64 tiles, narrow output, long contraction: split-K pays (measured)
inline bool splitk_shape(int m, int n, int k) {
    return k >= 1920 && n <= 256 && (int64_t)((m + 63) / 64) * ((n + 63) / 64) <= 160;
}
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int SH_UNSET = 0x3fff;     // "no non-zero chunk seen yet" (partial sums are 0)

struct GemmH3Args {
    const float* A; int64_t lda;
    const u32x4* W; int ksteps;       // image [panel][kstep][term 2][g 4][16] x 16 B
    const float* wsc;                 // per n: 2^-e_n (inverse of the W row scale)
    float* C; int64_t ldc;
    const float* bias;
    const float* R; int64_t ldr;
    int M, N, K, act, vec_out;
};

__device__ __forceinline__ float xg_max16(float v) {   // max over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float xg_sum16(float v) {   // sum over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// scale exponent for a chunk whose max |x| is cm: cm * 2^sh in [2^7, 2^8)
__device__ __forceinline__ int chunk_shift(float cm) {
    return min(8 - __builtin_amdgcn_frexp_expf(cm), 127);
}

// Epilogue of one output: act(y + b + r), or LeakyReLU_0.1(ReLU(y + b) + r) for
// FGR_ACT_RELU_RES_LEAKY (absent bias / residual come in as 0).
__device__ __forceinline__ float finish_out(float y, float b, float r, int act) {
    if (act == FGR_ACT_RELU_RES_LEAKY) {
        const float t = fmaxf(y + b, 0.f) + r;
        return t > 0.f ? t : 0.1f * t;
    }
    const float t = y + b + r;
    return act == FGR_ACT_RELU ? fmaxf(t, 0.f) : t;
}

// Stores one lane's 4 consecutive outputs n..n+3 of a row (16-B accesses when vec and the
// 4 columns are in range).
__device__ __forceinline__ void store_out4(const float (&y)[4], const float* bias,
                                           const float* rrow, float* crow, int n, int N, int act,
                                           bool vec) {
    if (vec && n + 3 < N) {
        float4 b = make_float4(0.f, 0.f, 0.f, 0.f), r = b;
        if (bias) b = *reinterpret_cast<const float4*>(bias + n);
        if (rrow) r = *reinterpret_cast<const float4*>(rrow + n);
        *reinterpret_cast<float4*>(crow + n) =
            make_float4(finish_out(y[0], b.x, r.x, act), finish_out(y[1], b.y, r.y, act),
                        finish_out(y[2], b.z, r.z, act), finish_out(y[3], b.w, r.w, act));
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (n + e >= N) break;
            crow[n + e] = finish_out(y[e], bias ? bias[n + e] : 0.f, rrow ? rrow[n + e] : 0.f, act);
        }
    }
}

// EPI: staged epilogue -- each wave's scaled (BM/2) x (BN/2) tile parked in LDS (sharing the
// A / W image space) and written row-major, 16 B per lane over whole row slices.
template <int BM, int BN, bool KVEC, bool EPI = false>
__global__ void __launch_bounds__(256) gemm_f16x3_kernel(GemmH3Args p) {
    constexpr int TM = BM / 32, TN = BN / 32;          // 16x16 subtiles per wave (m, n)
    constexpr int UA = BM * 4 / 256;                    // A units (8 k of one row) per thread
    constexpr int UW = 8 * BN / 256;                    // W image units per thread
    static_assert(UA >= 1 && UW >= 1, "tile");
    constexpr int ERS = BN / 2 + 4;                     // staged row stride (floats)
    constexpr int IMG_U = 2 * 4 * BM + 8 * BN;          // A + W images (16-B units)
    constexpr int EPI_U = EPI ? (4 * (BM / 2) * ERS * 4 + 15) / 16 : 0;
    __shared__ u32x4 img_lds[IMG_U > EPI_U ? IMG_U : EPI_U];
    u32x4* a_lds = img_lds;
    u32x4* w_lds = img_lds + 2 * 4 * BM;
    __shared__ int sh_lds[BM];

    // XCD-aware order: hardware dispatches block b to XCD b % 8; remap (bijectively) so that
    // each XCD gets a contiguous range of tiles, tiles ordered n-fastest within a row panel.
    const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int t = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int bm = t / nbn, bn = t % nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int wn = (wv >> 1) * (BN / 2), wm = (wv & 1) * (BM / 2);
    const int g = lane >> 4, c = lane & 15;
    const int npanel = (p.N + 15) / 16;

    const float* arow[UA];
    int akk[UA], sh[UA];
#pragma unroll
    for (int j = 0; j < UA; ++j) {
        const int u = tid + 256 * j;
        arow[j] = p.A + (int64_t)min(m0 + (u >> 2), p.M - 1) * p.lda;
        akk[j] = 8 * (u & 3);
        sh[j] = SH_UNSET;
    }
    const u32x4* wsrc[UW];
#pragma unroll
    for (int j = 0; j < UW; ++j) {
        const int v = tid + 256 * j;
        const int panel = min(n0 / 16 + v / 128, npanel - 1);
        wsrc[j] = p.W + (int64_t)panel * p.ksteps * 128 + v % 128;
    }
    float4 ar[UA][2];
    u32x4 wr[UW];
    auto load = [&](int s) {
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int k = s * 32 + akk[j];
            if constexpr (KVEC) {
                const float* src = arow[j] + min(k, p.K - 8);
                const float4 x0 = *reinterpret_cast<const float4*>(src);
                const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                const bool ok = k < p.K;
                ar[j][0] = ok ? x0 : make_float4(0.f, 0.f, 0.f, 0.f);
                ar[j][1] = ok ? x1 : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float tt[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float xv = arow[j][min(k + e, p.K - 1)];
                    tt[e] = k + e < p.K ? xv : 0.f;
                }
                ar[j][0] = make_float4(tt[0], tt[1], tt[2], tt[3]);
                ar[j][1] = make_float4(tt[4], tt[5], tt[6], tt[7]);
            }
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) wr[j] = wsrc[j][(int64_t)s * 128];
    };
    auto store = [&]() {
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int u = tid + 256 * j;
            const int row = u >> 2, gg = u & 3;
            const float x[8] = {ar[j][0].x, ar[j][0].y, ar[j][0].z, ar[j][0].w,
                                ar[j][1].x, ar[j][1].y, ar[j][1].z, ar[j][1].w};
            float cm = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
            cm = fmaxf(cm, fmaxf(fmaxf(fabsf(x[4]), fabsf(x[5])), fmaxf(fabsf(x[6]), fabsf(x[7]))));
            cm = fmaxf(cm, dppf<0xB1>(cm));              // the row's 4 lanes: quad xor 1, xor 2
            cm = fmaxf(cm, dppf<0x4E>(cm));
            if (cm > 0.f && __builtin_amdgcn_frexp_expf(cm) + sh[j] > 15) sh[j] = chunk_shift(cm);
            const float s = __builtin_ldexpf(1.f, sh[j] == SH_UNSET ? 0 : sh[j]);
            f16x8 th, tm;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float xs = x[e] * s;
                const _Float16 h = (_Float16)xs;
                th[e] = h;
                tm[e] = (_Float16)(xs - (float)h);
            }
            const int r = row ^ (2 * gg);
            a_lds[(0 * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, th);
            a_lds[(1 * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, tm);
            if (gg == 0) sh_lds[row] = sh[j];
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) w_lds[tid + 256 * j] = wr[j];
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int shr[TM];                                       // scale exponent of this lane's rows
#pragma unroll
    for (int i = 0; i < TM; ++i) shr[i] = SH_UNSET;

    const int nk = (p.K + 31) / 32;
    load(0);
    for (int s = 0; s < nk; ++s) {
        __syncthreads();
        store();
        __syncthreads();
        if (s + 1 < nk) load(s + 1);
        // rows whose scale was lowered this step: rescale their partial sums (exact, rare)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int shv = sh_lds[wm + 16 * i + c];
            if (__builtin_amdgcn_ballot_w64(shv != shr[i])) {
                const float f = (shr[i] == SH_UNSET || shv == shr[i])
                                    ? 1.f : __builtin_ldexpf(1.f, shv - shr[i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j][i] *= f;
                shr[i] = shv;
            }
        }
        f16x8 af[TM][2];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int r = (wm + 16 * i + c) ^ (2 * g);
            af[i][0] = __builtin_bit_cast(f16x8, a_lds[(0 * 4 + g) * BM + r]);
            af[i][1] = __builtin_bit_cast(f16x8, a_lds[(1 * 4 + g) * BM + r]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int pp = (wn + 16 * j) >> 4;
            const f16x8 wh = __builtin_bit_cast(f16x8, w_lds[pp * 128 + (0 * 4 + g) * 16 + c]);
            const f16x8 wl = __builtin_bit_cast(f16x8, w_lds[pp * 128 + (1 * 4 + g) * 16 + c]);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, af[i][0], acc[j][i], 0, 0, 0);
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][1], acc[j][i], 0, 0, 0);
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][0], acc[j][i], 0, 0, 0);
            }
        }
    }

    if constexpr (EPI) {
        if (p.vec_out) {
            __syncthreads();                                    // image reads retired
            float* buf = reinterpret_cast<float*>(img_lds) + wv * ((BM / 2) * ERS);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float rs = __builtin_ldexpf(1.f, -shr[i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = min(n0 + wn + 16 * j + 4 * g, ((p.N + 15) / 16) * 16 - 4);
                    const float4 ws = *reinterpret_cast<const float4*>(p.wsc + n);
                    *reinterpret_cast<float4*>(buf + (16 * i + c) * ERS + 16 * j + 4 * g) =
                        make_float4(acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                    acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w);
                }
            }
            __syncthreads();
            constexpr int LPRW = BN / 8, RPI = 64 / LPRW;       // lanes per row, rows per pass
            const int col = 4 * (lane % LPRW);
            const int n = n0 + wn + col;
#pragma unroll
            for (int it = 0; it < (BM / 2) / RPI; ++it) {
                const int row = it * RPI + lane / LPRW;
                const int m = m0 + wm + row;
                if (m >= p.M || n >= p.N) continue;
                const float4 yv = *reinterpret_cast<const float4*>(buf + row * ERS + col);
                const float y[4] = {yv.x, yv.y, yv.z, yv.w};
                store_out4(y, p.bias, p.R ? p.R + (int64_t)m * p.ldr : nullptr,
                           p.C + (int64_t)m * p.ldc, n, p.N, p.act, true);
            }
            return;
        }
    }
    // epilogue: lane holds C[m = m0 + wm + 16i + c][n = n0 + wn + 16j + 4g + r], r = 0..3
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm + 16 * i + c;
        if (m >= p.M) continue;
        const float rs = __builtin_ldexpf(1.f, -shr[i]);     // 0 for an all-zero row
        float* crow = p.C + (int64_t)m * p.ldc;
        const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn + 16 * j + 4 * g;
            if (n >= p.N) continue;
            const float4 ws = *reinterpret_cast<const float4*>(p.wsc + n);   // padded to 16
            const float y[4] = {acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w};
            store_out4(y, p.bias, rrow, crow, n, p.N, p.act, p.vec_out);
        }
    }
}

// ------------------------------------------------------------------------------------
// v2: KS k32-steps per staged tile (one row scale per KS*32 chunk, one barrier pair per
// stage instead of per k32-step) and optionally double-buffered LDS (DBUF: one barrier per
// stage; the next stage's split + LDS store overlaps other waves' MFMAs).
// LDS images per stage: A [ks][term 2][g 4][BM rows ^ 2g], W [panel][ks][term 2][g 4][16].
// ------------------------------------------------------------------------------------
template <int BM, int BN, int KS, bool DBUF, bool KVEC>
__global__ void __launch_bounds__(256) gemm_f16x3_v2(GemmH3Args p) {
    constexpr int TM = BM / 32, TN = BN / 32;
    constexpr int RU = 4 * KS;                          // units (8 k) of a row per stage
    constexpr int UA = BM * RU / 256;                   // A units per thread per stage
    constexpr int UW = 8 * BN * KS / 256;               // W units per thread per stage
    constexpr int ASZ = 8 * BM * KS, WSZ = 8 * BN * KS; // 16-B units per stage
    constexpr int NB = DBUF ? 2 : 1;
    static_assert(UA >= 1 && UW >= 1 && (RU == 4 || RU == 8), "tile");
    __shared__ u32x4 lds[NB * (ASZ + WSZ)];
    __shared__ int sh_lds[NB][BM];

    const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int t = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int bm = t / nbn, bn = t % nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int wn = (wv >> 1) * (BN / 2), wm = (wv & 1) * (BM / 2);
    const int g = lane >> 4, c = lane & 15;
    const int npanel = (p.N + 15) / 16;

    const float* arow[UA];
    int akk[UA], sh[UA];
#pragma unroll
    for (int j = 0; j < UA; ++j) {
        const int u = tid + 256 * j;
        arow[j] = p.A + (int64_t)min(m0 + u / RU, p.M - 1) * p.lda;
        akk[j] = 8 * (u % RU);
        sh[j] = SH_UNSET;
    }
    const u32x4* wsrc[UW];
#pragma unroll
    for (int j = 0; j < UW; ++j) {
        const int v = tid + 256 * j;
        const int panel = min(n0 / 16 + v / (128 * KS), npanel - 1);
        wsrc[j] = p.W + (int64_t)panel * p.ksteps * 128 + v % (128 * KS);
    }
    float4 ar[UA][2];
    u32x4 wr[UW];
    auto load = [&](int s) {
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int k = s * 32 * KS + akk[j];
            if constexpr (KVEC) {
                const float* src = arow[j] + min(k, p.K - 8);
                const float4 x0 = *reinterpret_cast<const float4*>(src);
                const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                const bool ok = k < p.K;
                ar[j][0] = ok ? x0 : make_float4(0.f, 0.f, 0.f, 0.f);
                ar[j][1] = ok ? x1 : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float tt[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float xv = arow[j][min(k + e, p.K - 1)];
                    tt[e] = k + e < p.K ? xv : 0.f;
                }
                ar[j][0] = make_float4(tt[0], tt[1], tt[2], tt[3]);
                ar[j][1] = make_float4(tt[4], tt[5], tt[6], tt[7]);
            }
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) wr[j] = wsrc[j][(int64_t)s * 128 * KS];
    };
    auto store = [&](int b) {
        u32x4* a_img = lds + b * (ASZ + WSZ);
        u32x4* w_img = a_img + ASZ;
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int u = tid + 256 * j;
            const int row = u / RU, q = u % RU, ks = q >> 2, gg = q & 3;
            const float x[8] = {ar[j][0].x, ar[j][0].y, ar[j][0].z, ar[j][0].w,
                                ar[j][1].x, ar[j][1].y, ar[j][1].z, ar[j][1].w};
            float cm = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
            cm = fmaxf(cm, fmaxf(fmaxf(fabsf(x[4]), fabsf(x[5])), fmaxf(fabsf(x[6]), fabsf(x[7]))));
            cm = fmaxf(cm, dppf<0xB1>(cm));              // the row's lanes: quad xor 1, xor 2,
            cm = fmaxf(cm, dppf<0x4E>(cm));
            if constexpr (RU == 8) cm = fmaxf(cm, dppf<0x141>(cm));   // + half-row mirror
            if (cm > 0.f && __builtin_amdgcn_frexp_expf(cm) + sh[j] > 15) sh[j] = chunk_shift(cm);
            const float s = __builtin_ldexpf(1.f, sh[j] == SH_UNSET ? 0 : sh[j]);
            f16x8 th, tm;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float xs = x[e] * s;
                const _Float16 h = (_Float16)xs;
                th[e] = h;
                tm[e] = (_Float16)(xs - (float)h);
            }
            const int r = row ^ (2 * gg);
            a_img[((ks * 2 + 0) * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, th);
            a_img[((ks * 2 + 1) * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, tm);
            if (q == 0) sh_lds[b][row] = sh[j];
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) w_img[tid + 256 * j] = wr[j];
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int shr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) shr[i] = SH_UNSET;

    auto compute = [&](int b) {
        const u32x4* a_img = lds + b * (ASZ + WSZ);
        const u32x4* w_img = a_img + ASZ;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int shv = sh_lds[b][wm + 16 * i + c];
            if (__builtin_amdgcn_ballot_w64(shv != shr[i])) {
                const float f = (shr[i] == SH_UNSET || shv == shr[i])
                                    ? 1.f : __builtin_ldexpf(1.f, shv - shr[i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j][i] *= f;
                shr[i] = shv;
            }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            f16x8 af[TM][2];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = (wm + 16 * i + c) ^ (2 * g);
                af[i][0] = __builtin_bit_cast(f16x8, a_img[((ks * 2 + 0) * 4 + g) * BM + r]);
                af[i][1] = __builtin_bit_cast(f16x8, a_img[((ks * 2 + 1) * 4 + g) * BM + r]);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int pp = (wn + 16 * j) >> 4;
                const u32x4* wb = w_img + pp * 128 * KS + ks * 128 + g * 16 + c;
                const f16x8 wh = __builtin_bit_cast(f16x8, wb[0]);
                const f16x8 wl = __builtin_bit_cast(f16x8, wb[64]);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, af[i][0], acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][1], acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][0], acc[j][i], 0, 0, 0);
                }
            }
        }
    };

    const int nst = (p.K + 32 * KS - 1) / (32 * KS);
    if constexpr (DBUF) {
        load(0);
        store(0);
        __syncthreads();
        if (nst > 1) load(1);
        for (int s = 0; s < nst; ++s) {
            compute(s & 1);
            if (s + 1 < nst) store((s + 1) & 1);
            if (s + 2 < nst) load(s + 2);
            __syncthreads();
        }
    } else {
        load(0);
        for (int s = 0; s < nst; ++s) {
            __syncthreads();
            store(0);
            __syncthreads();
            if (s + 1 < nst) load(s + 1);
            compute(0);
        }
    }

#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm + 16 * i + c;
        if (m >= p.M) continue;
        const float rs = __builtin_ldexpf(1.f, -shr[i]);
        float* crow = p.C + (int64_t)m * p.ldc;
        const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn + 16 * j + 4 * g;
            if (n >= p.N) continue;
            const float4 ws = *reinterpret_cast<const float4*>(p.wsc + n);
            const float y[4] = {acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w};
            store_out4(y, p.bias, rrow, crow, n, p.N, p.act, p.vec_out);
        }
    }
}

// ------------------------------------------------------------------------------------
// v3: the v2 stage layout (KS k32-steps per stage, double-buffered LDS, one barrier per
// stage) with a two-deep REGISTER ring: while stage s is multiplied, the global loads of
// stages s+1 and s+2 are in flight (v2 keeps only s+1 in flight, so every stage waits out
// most of an L2/HBM round trip). Stage s+1 is split and written to the idle LDS buffer after
// the MFMAs of stage s, then its registers are refilled with stage s+3. The loop is unrolled
// by two so every ring index is a compile-time constant (no scratch).
// ------------------------------------------------------------------------------------
template <int BM, int BN, int KS, bool KVEC>
__global__ void __launch_bounds__(256) gemm_f16x3_v3(GemmH3Args p) {
    constexpr int TM = BM / 32, TN = BN / 32;
    constexpr int RU = 4 * KS;                          // units (8 k) of a row per stage
    constexpr int UA = BM * RU / 256;                   // A units per thread per stage
    constexpr int UW = 8 * BN * KS / 256;               // W units per thread per stage
    constexpr int ASZ = 8 * BM * KS, WSZ = 8 * BN * KS; // 16-B units per stage
    static_assert(UA >= 1 && UW >= 1 && (RU == 4 || RU == 8), "tile");
    __shared__ u32x4 lds[2 * (ASZ + WSZ)];
    __shared__ int sh_lds[2][BM];

    const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int t = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int bm = t / nbn, bn = t % nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int wn = (wv >> 1) * (BN / 2), wm = (wv & 1) * (BM / 2);
    const int g = lane >> 4, c = lane & 15;
    const int npanel = (p.N + 15) / 16;

    const float* arow[UA];
    int akk[UA], sh[UA];
#pragma unroll
    for (int j = 0; j < UA; ++j) {
        const int u = tid + 256 * j;
        arow[j] = p.A + (int64_t)min(m0 + u / RU, p.M - 1) * p.lda;
        akk[j] = 8 * (u % RU);
        sh[j] = SH_UNSET;
    }
    const u32x4* wsrc[UW];
#pragma unroll
    for (int j = 0; j < UW; ++j) {
        const int v = tid + 256 * j;
        const int panel = min(n0 / 16 + v / (128 * KS), npanel - 1);
        wsrc[j] = p.W + (int64_t)panel * p.ksteps * 128 + v % (128 * KS);
    }
    float4 ar0[UA][2], ar1[UA][2];
    u32x4 wr0[UW], wr1[UW];
    auto load = [&](int s, float4 (&ar)[UA][2], u32x4 (&wr)[UW]) {
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int k = s * 32 * KS + akk[j];
            if constexpr (KVEC) {
                const float* src = arow[j] + min(k, p.K - 8);
                const float4 x0 = *reinterpret_cast<const float4*>(src);
                const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                const bool ok = k < p.K;
                ar[j][0] = ok ? x0 : make_float4(0.f, 0.f, 0.f, 0.f);
                ar[j][1] = ok ? x1 : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float tt[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float xv = arow[j][min(k + e, p.K - 1)];
                    tt[e] = k + e < p.K ? xv : 0.f;
                }
                ar[j][0] = make_float4(tt[0], tt[1], tt[2], tt[3]);
                ar[j][1] = make_float4(tt[4], tt[5], tt[6], tt[7]);
            }
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) wr[j] = wsrc[j][(int64_t)s * 128 * KS];
    };
    auto store = [&](int b, const float4 (&ar)[UA][2], const u32x4 (&wr)[UW]) {
        u32x4* a_img = lds + b * (ASZ + WSZ);
        u32x4* w_img = a_img + ASZ;
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int u = tid + 256 * j;
            const int row = u / RU, q = u % RU, ks = q >> 2, gg = q & 3;
            const float x[8] = {ar[j][0].x, ar[j][0].y, ar[j][0].z, ar[j][0].w,
                                ar[j][1].x, ar[j][1].y, ar[j][1].z, ar[j][1].w};
            float cm = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
            cm = fmaxf(cm, fmaxf(fmaxf(fabsf(x[4]), fabsf(x[5])), fmaxf(fabsf(x[6]), fabsf(x[7]))));
            cm = fmaxf(cm, dppf<0xB1>(cm));
            cm = fmaxf(cm, dppf<0x4E>(cm));
            if constexpr (RU == 8) cm = fmaxf(cm, dppf<0x141>(cm));
            if (cm > 0.f && __builtin_amdgcn_frexp_expf(cm) + sh[j] > 15) sh[j] = chunk_shift(cm);
            const float sc = __builtin_ldexpf(1.f, sh[j] == SH_UNSET ? 0 : sh[j]);
            f16x8 th, tm;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float xs = x[e] * sc;
                const _Float16 h = (_Float16)xs;
                th[e] = h;
                tm[e] = (_Float16)(xs - (float)h);
            }
            const int r = row ^ (2 * gg);
            a_img[((ks * 2 + 0) * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, th);
            a_img[((ks * 2 + 1) * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, tm);
            if (q == 0) sh_lds[b][row] = sh[j];
        }
#pragma unroll
        for (int j = 0; j < UW; ++j) w_img[tid + 256 * j] = wr[j];
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int shr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) shr[i] = SH_UNSET;

    auto compute = [&](int b) {
        const u32x4* a_img = lds + b * (ASZ + WSZ);
        const u32x4* w_img = a_img + ASZ;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int shv = sh_lds[b][wm + 16 * i + c];
            if (__builtin_amdgcn_ballot_w64(shv != shr[i])) {
                const float f = (shr[i] == SH_UNSET || shv == shr[i])
                                    ? 1.f : __builtin_ldexpf(1.f, shv - shr[i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j][i] *= f;
                shr[i] = shv;
            }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            f16x8 af[TM][2];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = (wm + 16 * i + c) ^ (2 * g);
                af[i][0] = __builtin_bit_cast(f16x8, a_img[((ks * 2 + 0) * 4 + g) * BM + r]);
                af[i][1] = __builtin_bit_cast(f16x8, a_img[((ks * 2 + 1) * 4 + g) * BM + r]);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int pp = (wn + 16 * j) >> 4;
                const u32x4* wb = w_img + pp * 128 * KS + ks * 128 + g * 16 + c;
                const f16x8 wh = __builtin_bit_cast(f16x8, wb[0]);
                const f16x8 wl = __builtin_bit_cast(f16x8, wb[64]);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, af[i][0], acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][1], acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][0], acc[j][i], 0, 0, 0);
                }
            }
        }
    };

    const int nst = (p.K + 32 * KS - 1) / (32 * KS);
    load(0, ar0, wr0);
    if (nst > 1) load(1, ar1, wr1);
    store(0, ar0, wr0);
    __syncthreads();
    if (nst > 2) load(2, ar0, wr0);
    // iteration s: multiply buffer s&1, stage s+1 from ring (s+1)&1, refill it with s+3
    for (int s = 0; s < nst; s += 2) {
        compute(0);
        if (s + 1 < nst) store(1, ar1, wr1);
        if (s + 3 < nst) load(s + 3, ar1, wr1);
        __syncthreads();
        if (s + 1 >= nst) break;
        compute(1);
        if (s + 2 < nst) store(0, ar0, wr0);
        if (s + 4 < nst) load(s + 4, ar0, wr0);
        __syncthreads();
    }

#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm + 16 * i + c;
        if (m >= p.M) continue;
        const float rs = __builtin_ldexpf(1.f, -shr[i]);
        float* crow = p.C + (int64_t)m * p.ldc;
        const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn + 16 * j + 4 * g;
            if (n >= p.N) continue;
            const float4 ws = *reinterpret_cast<const float4*>(p.wsc + n);
            const float y[4] = {acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w};
            store_out4(y, p.bias, rrow, crow, n, p.N, p.act, p.vec_out);
        }
    }
}

// ------------------------------------------------------------------------------------
// v4: W fragments straight from the image into registers. The f16x3 W image is stored in
// MFMA fragment order ([panel][kstep][term][g][16] x 16 B), so one wave-load of a panel's
// term is 1 KB contiguous in lane order -- no LDS round trip for W. The waves split the
// block's BN output channels (BN/4 each: TN = BN/64 16-column tiles) and each covers all
// BM activation rows, so no W byte is loaded twice per block; only A is staged (split in
// registers -> double-buffered LDS, one barrier per k32 step). W fragments of step s+1 are
// loaded while step s multiplies (register double buffer, loop unrolled by two).
// Motivation (VERDICT r1 / microbench): v1-v3 stage W through LDS with ds_write_b128, whose
// transfer cost (~13 cycles per wave-instruction) plus the fragment reads exceeds the
// MFMA time of a 64 x 128 step -- they are LDS-bound.
// ------------------------------------------------------------------------------------
template <int BM, int BN, bool KVEC>
__global__ void __launch_bounds__(256) gemm_f16x3_v4(GemmH3Args p) {
    constexpr int TM = BM / 16, TN = BN / 64;          // per wave: TM row tiles x TN col tiles
    constexpr int UA = BM * 4 / 256;                    // A units (8 k) per thread per step
    constexpr int ASZ = 8 * BM;                         // 16-B units of one A stage
    static_assert(UA >= 1 && TN >= 1, "tile");
    __shared__ u32x4 a_lds[2 * ASZ];
    __shared__ int sh_lds[2][BM];

    const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int t = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int bm = t / nbn, bn = t % nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const int npanel = (p.N + 15) / 16;
    const int wn = wv * (BN / 4);                       // this wave's first output channel

    const float* arow[UA];
    int akk[UA], sh[UA];
#pragma unroll
    for (int j = 0; j < UA; ++j) {
        const int u = tid + 256 * j;
        arow[j] = p.A + (int64_t)min(m0 + (u >> 2), p.M - 1) * p.lda;
        akk[j] = 8 * (u & 3);
        sh[j] = SH_UNSET;
    }
    // W fragment pointers: panel of tile j, lane's unit within a (kstep, term) block of 64
    const u32x4* wp[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int panel = min((n0 + wn) / 16 + j, npanel - 1);
        wp[j] = p.W + (int64_t)panel * p.ksteps * 128 + lane;
    }
    float4 ar[UA][2];
    auto load_a = [&](int s) {
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int k = s * 32 + akk[j];
            if constexpr (KVEC) {
                const float* src = arow[j] + min(k, p.K - 8);
                const float4 x0 = *reinterpret_cast<const float4*>(src);
                const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                const bool ok = k < p.K;
                ar[j][0] = ok ? x0 : make_float4(0.f, 0.f, 0.f, 0.f);
                ar[j][1] = ok ? x1 : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float tt[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float xv = arow[j][min(k + e, p.K - 1)];
                    tt[e] = k + e < p.K ? xv : 0.f;
                }
                ar[j][0] = make_float4(tt[0], tt[1], tt[2], tt[3]);
                ar[j][1] = make_float4(tt[4], tt[5], tt[6], tt[7]);
            }
        }
    };
    auto store_a = [&](int b) {
        u32x4* a_img = a_lds + b * ASZ;
#pragma unroll
        for (int j = 0; j < UA; ++j) {
            const int u = tid + 256 * j;
            const int row = u >> 2, gg = u & 3;
            const float x[8] = {ar[j][0].x, ar[j][0].y, ar[j][0].z, ar[j][0].w,
                                ar[j][1].x, ar[j][1].y, ar[j][1].z, ar[j][1].w};
            float cm = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
            cm = fmaxf(cm, fmaxf(fmaxf(fabsf(x[4]), fabsf(x[5])), fmaxf(fabsf(x[6]), fabsf(x[7]))));
            cm = fmaxf(cm, dppf<0xB1>(cm));
            cm = fmaxf(cm, dppf<0x4E>(cm));
            if (cm > 0.f && __builtin_amdgcn_frexp_expf(cm) + sh[j] > 15) sh[j] = chunk_shift(cm);
            const float sc = __builtin_ldexpf(1.f, sh[j] == SH_UNSET ? 0 : sh[j]);
            f16x8 th, tm;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float xs = x[e] * sc;
                const _Float16 h = (_Float16)xs;
                th[e] = h;
                tm[e] = (_Float16)(xs - (float)h);
            }
            const int r = row ^ (2 * gg);
            a_img[(0 * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, th);
            a_img[(1 * 4 + gg) * BM + r] = __builtin_bit_cast(u32x4, tm);
            if (gg == 0) sh_lds[b][row] = sh[j];
        }
    };
    u32x4 w0[TN][2], w1[TN][2];
    auto load_w = [&](int s, u32x4 (&w)[TN][2]) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            w[j][0] = wp[j][(int64_t)s * 128];
            w[j][1] = wp[j][(int64_t)s * 128 + 64];
        }
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int shr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) shr[i] = SH_UNSET;

    auto compute = [&](int b, const u32x4 (&w)[TN][2]) {
        const u32x4* a_img = a_lds + b * ASZ;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int shv = sh_lds[b][16 * i + c];
            if (__builtin_amdgcn_ballot_w64(shv != shr[i])) {
                const float f = (shr[i] == SH_UNSET || shv == shr[i])
                                    ? 1.f : __builtin_ldexpf(1.f, shv - shr[i]);
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j][i] *= f;
                shr[i] = shv;
            }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int r = (16 * i + c) ^ (2 * g);
            const f16x8 ah = __builtin_bit_cast(f16x8, a_img[(0 * 4 + g) * BM + r]);
            const f16x8 am = __builtin_bit_cast(f16x8, a_img[(1 * 4 + g) * BM + r]);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const f16x8 wh = __builtin_bit_cast(f16x8, w[j][0]);
                const f16x8 wl = __builtin_bit_cast(f16x8, w[j][1]);
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, acc[j][i], 0, 0, 0);
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, am, acc[j][i], 0, 0, 0);
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, acc[j][i], 0, 0, 0);
            }
        }
    };

    const int nk = (p.K + 31) / 32;
    load_a(0);
    load_w(0, w0);
    for (int s = 0; s < nk; s += 2) {
        store_a(0);
        __syncthreads();
        if (s + 1 < nk) {
            load_a(s + 1);
            load_w(s + 1, w1);
        }
        compute(0, w0);
        if (s + 1 >= nk) break;
        store_a(1);
        __syncthreads();
        if (s + 2 < nk) {
            load_a(s + 2);
            load_w(s + 2, w0);
        }
        compute(1, w1);
    }

#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + 16 * i + c;
        if (m >= p.M) continue;
        const float rs = __builtin_ldexpf(1.f, -shr[i]);
        float* crow = p.C + (int64_t)m * p.ldc;
        const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn + 16 * j + 4 * g;
            if (n >= p.N) continue;
            const float4 ws = *reinterpret_cast<const float4*>(p.wsc + n);
            const float y[4] = {acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w};
            store_out4(y, p.bias, rrow, crow, n, p.N, p.act, p.vec_out);
        }
    }
}

// Row max |w| of W (n x k, element (i, j) at w[i * sn + j * sk]) -> wsc[i] = 2^-e_i with
// e_i the row scale exponent (max * 2^e_i in [2^14, 2^15)); one wave per row, rows padded
// to a multiple of 16 get 0.
__global__ void weight_scale_kernel(const float* __restrict__ w, int n, int k, int64_t sn,
                                    int64_t sk, int npad, float* __restrict__ wsc) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= npad) return;
    float mx = 0.f;
    if (row < n) {
        const float* wr = w + (int64_t)row * sn;
        if (sk == 1 && k % 4 == 0 && (reinterpret_cast<uintptr_t>(wr) & 15) == 0) {
            // contiguous rows: 16-B loads, four in flight per lane (a row of the long-K KPConv
            // weights is 3840 floats: the scalar loop below waited on ~60 dependent trips)
            const float4* p = reinterpret_cast<const float4*>(wr);
            const int k4 = k / 4;
            float m1 = 0.f, m2 = 0.f, m3 = 0.f;
            int j = lane;
            for (; j + 192 < k4; j += 256) {
                const float4 a = p[j], b = p[j + 64], c = p[j + 128], d = p[j + 192];
                mx = fmaxf(mx, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
                m1 = fmaxf(m1, fmaxf(fmaxf(fabsf(b.x), fabsf(b.y)), fmaxf(fabsf(b.z), fabsf(b.w))));
                m2 = fmaxf(m2, fmaxf(fmaxf(fabsf(c.x), fabsf(c.y)), fmaxf(fabsf(c.z), fabsf(c.w))));
                m3 = fmaxf(m3, fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), fabsf(d.w))));
            }
            for (; j < k4; j += 64) {
                const float4 a = p[j];
                mx = fmaxf(mx, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
            }
            mx = fmaxf(fmaxf(mx, m1), fmaxf(m2, m3));
        } else {
            for (int j = lane; j < k; j += 64) mx = fmaxf(mx, fabsf(wr[(int64_t)j * sk]));
        }
    }
    mx = wave_max(mx);
    if (lane == 0) {
        const int e = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
        wsc[row] = row < n ? __builtin_ldexpf(1.f, -e) : 0.f;
    }
}

// The same row maxima for a W stored column-major (sn == 1: the transposed operand of the
// backward's dW = dY^T X, W = X^T): a block takes 64 consecutive rows (one 256-B load per
// wave and k index) over a chunk of k and folds its maxima into wsc with an unsigned-integer
// atomic max on the bit patterns (order-preserving for non-negative floats; max is exact, so
// the result is independent of the order). wsc must be zeroed first; weight_scale_finish
// turns the maxima into the scales.
__global__ void weight_scale_cols_kernel(const float* __restrict__ w, int n, int k, int64_t sk,
                                         int kchunk, unsigned* __restrict__ wmax) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int row = blockIdx.x * 64 + lane;
    const int j0 = blockIdx.y * kchunk, j1 = min(k, j0 + kchunk);
    float mx = 0.f;
    if (row < n) {
        int j = j0 + wv;
        for (; j + 12 < j1; j += 16) {
            const float a = w[(int64_t)j * sk + row], b = w[(int64_t)(j + 4) * sk + row];
            const float c = w[(int64_t)(j + 8) * sk + row], d = w[(int64_t)(j + 12) * sk + row];
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d))));
        }
        for (; j < j1; j += 4) mx = fmaxf(mx, fabsf(w[(int64_t)j * sk + row]));
    }
    __shared__ float red[4][64];
    red[wv][lane] = mx;
    __syncthreads();
    if (wv == 0 && row < n) {
        mx = fmaxf(fmaxf(red[0][lane], red[1][lane]), fmaxf(red[2][lane], red[3][lane]));
        if (mx > 0.f) atomicMax(wmax + row, __float_as_uint(mx));
    }
}

__global__ void weight_scale_finish(int n, int npad, float* __restrict__ wsc) {
    const int row = blockIdx.x * 256 + threadIdx.x;
    if (row >= npad) return;
    const float mx = __uint_as_float(reinterpret_cast<const unsigned*>(wsc)[row]);
    const int e = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
    wsc[row] = row < n ? __builtin_ldexpf(1.f, -e) : 0.f;
}

// W -> f16x3 image [panel][kstep][term 2][g 4][16 rows] x 16 B (8 k each), rows scaled by
// 1 / wsc[row] (exact powers of two), zero-padded past n and k.
__global__ void split_weights_h3_kernel(const float* __restrict__ w, int n, int k, int64_t sn,
                                        int64_t sk, int ksteps, const float* __restrict__ wsc,
                                        u32x4* __restrict__ img) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)((n + 15) / 16) * ksteps * 128;
    if (u >= total) return;
    const int i = (int)(u % 16);
    const int g = (int)((u / 16) % 4);
    const int t = (int)((u / 64) % 2);
    const int64_t ps = u / 128;
    const int s = (int)(ps % ksteps);
    const int panel = (int)(ps / ksteps);
    const int row = panel * 16 + i;
    const float sc = row < n ? 1.f / wsc[row] : 0.f;      // exact: a power of two
    f16x8 out;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int col = s * 32 + 8 * g + e;
        const float x = (row < n && col < k) ? w[(int64_t)row * sn + (int64_t)col * sk] * sc : 0.f;
        const _Float16 h = (_Float16)x;
        out[e] = t == 0 ? h : (_Float16)(x - (float)h);
    }
    img[u] = __builtin_bit_cast(u32x4, out);
}

// weight_scale_kernel + split_weights_h3_kernel in one launch for k <= kSplitFusedK: one block
// per 16-row panel takes the panel's row maxima (lanes along whichever stride is 1, so the
// reads coalesce for W and for W^T alike), then writes the panel's image units. Same scales,
// same image bits; training re-splits every weight twice per step (forward and transposed
// images), so this halves those launches.
constexpr int kSplitFusedK = 1024;

// one 16-row panel of fgr_split_weights_h3's image (the block's whole work in the fused and
// the batched kernels)
__device__ __forceinline__ void split_panel_h3(const float* __restrict__ w, int n, int k, int64_t sn,
                                               int64_t sk, int ksteps, float* __restrict__ wsc,
                                               u32x4* __restrict__ img, int panel) {
    const int tid = threadIdx.x;
    const int r0 = panel * 16;
    // phase 1: row maxima; (row, k-lane) = (tid % 16, tid / 16) when rows are contiguous in
    // memory (sn == 1), else (tid / 16, tid % 16)
    const bool rows_fast = sn == 1 && sk != 1;
    const int ri = rows_fast ? (tid & 15) : (tid >> 4), kl = rows_fast ? (tid >> 4) : (tid & 15);
    const int row = r0 + ri;
    float mx = 0.f;
    if (row < n) {
        const float* wr = w + (int64_t)row * sn;
        int j = kl;
        for (; j + 48 < k; j += 64) {
            const float a = wr[(int64_t)j * sk], b = wr[(int64_t)(j + 16) * sk];
            const float c = wr[(int64_t)(j + 32) * sk], d = wr[(int64_t)(j + 48) * sk];
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d))));
        }
        for (; j < k; j += 16) mx = fmaxf(mx, fabsf(wr[(int64_t)j * sk]));
    }
    __shared__ float red[16][17];
    __shared__ float scale_inv[16];
    red[ri][kl] = mx;
    __syncthreads();
    if (tid < 16) {
        float m = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) m = fmaxf(m, red[tid][q]);
        const int e = m > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(m), 127) : 0;
        const bool ok = r0 + tid < n;
        scale_inv[tid] = ok ? __builtin_ldexpf(1.f, e) : 0.f;
        wsc[r0 + tid] = ok ? __builtin_ldexpf(1.f, -e) : 0.f;
    }
    __syncthreads();
    // phase 2: the panel's units [kstep][term][g][i], as split_weights_h3_kernel; rows of
    // a row-major W with k % 8 == 0 read as two 16-B loads per unit
    const int units = ksteps * 128;
    const bool vec = sk == 1 && k % 8 == 0 && sn % 4 == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0;
    for (int u = tid; u < units; u += 256) {
        const int i = u & 15, g = (u >> 4) & 3, t = (u >> 6) & 1, s = u >> 7;
        const int rr = r0 + i;
        const float sc = scale_inv[i];
        const int c0 = s * 32 + 8 * g;
        float xv[8];
        if (vec) {
            const bool ok = rr < n && c0 < k;
            const float* src = w + (int64_t)min(rr, n - 1) * sn + min(c0, k - 8);
            const float4 a = *reinterpret_cast<const float4*>(src);
            const float4 b = *reinterpret_cast<const float4*>(src + 4);
            xv[0] = a.x; xv[1] = a.y; xv[2] = a.z; xv[3] = a.w;
            xv[4] = b.x; xv[5] = b.y; xv[6] = b.z; xv[7] = b.w;
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[e] = ok ? xv[e] * sc : 0.f;
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int col = c0 + e;
                xv[e] = (rr < n && col < k) ? w[(int64_t)rr * sn + (int64_t)col * sk] * sc : 0.f;
            }
        }
        f16x8 out;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const _Float16 h = (_Float16)xv[e];
            out[e] = t == 0 ? h : (_Float16)(xv[e] - (float)h);
        }
        img[(int64_t)panel * units + u] = __builtin_bit_cast(u32x4, out);
    }
}

__global__ void __launch_bounds__(256)
split_weights_h3_fused_kernel(const float* __restrict__ w, int n, int k, int64_t sn, int64_t sk,
                              int ksteps, float* __restrict__ wsc, u32x4* __restrict__ img) {
    split_panel_h3(w, n, k, sn, sk, ksteps, wsc, img, blockIdx.x);
}

// Many images in one launch (training re-splits every weight after each optimizer step):
// block b takes panel b of the concatenated panel list, its image found by binary search
// over the descriptors' first panels.
__global__ void __launch_bounds__(256)
split_weights_h3_batch_kernel(const fgr_split_desc* __restrict__ d, int count) {
    const int64_t b = blockIdx.x;
    int lo = 0, hi = count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (d[mid].panel0 <= b) lo = mid; else hi = mid - 1;
    }
    const fgr_split_desc e = d[lo];
    const int ksteps = (e.k + 63) / 64 * 2;
    u32x4* img = static_cast<u32x4*>(e.img);
    float* wsc = reinterpret_cast<float*>(static_cast<char*>(e.img) +
                                          (size_t)((e.n + 15) / 16) * ksteps * 128 * 16);
    split_panel_h3(e.w, e.n, e.k, e.stride_n, e.stride_k, ksteps, wsc, img, (int)(b - e.panel0));
}

template <int BM, int BN, bool EPI = false>
void launch_h3(const GemmH3Args& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    if (a.K % 8 == 0)
        hipLaunchKernelGGL((gemm_f16x3_kernel<BM, BN, true, EPI>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((gemm_f16x3_kernel<BM, BN, false, EPI>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
}

// k32-steps of the image, padded to an even count (v2 stages read 2 per stage)
int ksteps_h3(int k) { return (k + 63) / 64 * 2; }

size_t image_bytes_h3(int n, int k) {
    return (size_t)((n + 15) / 16) * ksteps_h3(k) * 128 * 16;
}

template <int BM, int BN>
void launch_h3v4(const GemmH3Args& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    if (a.K % 8 == 0)
        hipLaunchKernelGGL((gemm_f16x3_v4<BM, BN, true>), dim3((unsigned)(nbm * nbn)), dim3(256),
                           0, st, a);
    else
        hipLaunchKernelGGL((gemm_f16x3_v4<BM, BN, false>), dim3((unsigned)(nbm * nbn)), dim3(256),
                           0, st, a);
}

template <int BM, int BN, int KS>
void launch_h3v3(const GemmH3Args& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    if (a.K % 8 == 0)
        hipLaunchKernelGGL((gemm_f16x3_v3<BM, BN, KS, true>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((gemm_f16x3_v3<BM, BN, KS, false>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
}

template <int BM, int BN, int KS, bool DBUF>
void launch_h3v2(const GemmH3Args& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    if (a.K % 8 == 0)
        hipLaunchKernelGGL((gemm_f16x3_v2<BM, BN, KS, DBUF, true>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((gemm_f16x3_v2<BM, BN, KS, DBUF, false>), dim3((unsigned)(nbm * nbn)),
                           dim3(256), 0, st, a);
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_split_weights_h3_batch(const void* descs, int32_t count, int64_t total_panels,
                                          void* stream) {
    FGR_REQUIRE(count >= 0 && total_panels >= 0 && (count == 0 || descs),
                "fgr_split_weights_h3_batch: bad arguments");
    if (count == 0 || total_panels == 0) return FGR_OK;
    hipLaunchKernelGGL(split_weights_h3_batch_kernel, dim3((unsigned)total_panels), dim3(256), 0,
                       as_stream(stream), static_cast<const fgr_split_desc*>(descs), count);
    FGR_CHECK_LAUNCH("split_weights_h3_batch_kernel");
    return FGR_OK;
}

extern "C" int fgr_split_weights_h3_bytes(int32_t n, int32_t k, size_t* bytes) {
    FGR_REQUIRE(bytes && n > 0 && k > 0, "fgr_split_weights_h3_bytes: bad arguments");
    *bytes = image_bytes_h3(n, k) + (size_t)((n + 15) / 16) * 16 * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_split_weights_h3(const float* w, int32_t n, int32_t k, int64_t stride_n,
                                    int64_t stride_k, void* img, void* stream) {
    FGR_REQUIRE(w && img && n > 0 && k > 0, "fgr_split_weights_h3: bad arguments");
    FGR_REQUIRE((reinterpret_cast<uintptr_t>(img) & 15) == 0,
                "fgr_split_weights_h3: image not 16-B aligned");
    const int ksteps = ksteps_h3(k);
    const int npad = (n + 15) / 16 * 16;
    float* wsc = reinterpret_cast<float*>(static_cast<char*>(img) + image_bytes_h3(n, k));
    hipStream_t st = as_stream(stream);
    static const bool fused_on = [] { const char* e = getenv("FGR_SPLIT_FUSED"); return !(e && e[0] == '0'); }();
    if (k <= kSplitFusedK && fused_on) {
        hipLaunchKernelGGL(split_weights_h3_fused_kernel, dim3((unsigned)(npad / 16)), dim3(256), 0, st,
                           w, n, k, stride_n, stride_k, ksteps, wsc, (u32x4*)img);
        FGR_CHECK_LAUNCH("split_weights_h3_fused_kernel");
        return FGR_OK;
    }
    if (stride_n == 1 && k >= 1024) {
        // column-major W (the backward's transposed activations): coalesced chunked maxima;
        // >= 512 blocks of 64 rows x kchunk (a multiple of 64)
        const int nrb = ceil_div(n, 64);
        int nkc = ceil_div(512, nrb);
        if (nkc > ceil_div(k, 256)) nkc = ceil_div(k, 256);
        const int kchunk = ceil_div(ceil_div(k, nkc), 64) * 64;
        FGR_CHECK_HIP(hipMemsetAsync(wsc, 0, (size_t)npad * sizeof(float), st));
        hipLaunchKernelGGL(weight_scale_cols_kernel, dim3((unsigned)nrb, (unsigned)ceil_div(k, kchunk)),
                           dim3(256), 0, st, w, n, k, stride_k, kchunk, (unsigned*)wsc);
        FGR_CHECK_LAUNCH("weight_scale_cols_kernel");
        hipLaunchKernelGGL(weight_scale_finish, dim3((unsigned)ceil_div(npad, 256)), dim3(256), 0,
                           st, n, npad, wsc);
        FGR_CHECK_LAUNCH("weight_scale_finish");
    } else {
        hipLaunchKernelGGL(weight_scale_kernel, dim3((unsigned)ceil_div(npad, 4)), dim3(256), 0, st,
                           w, n, k, stride_n, stride_k, npad, wsc);
        FGR_CHECK_LAUNCH("weight_scale_kernel");
    }
    const int64_t total = (int64_t)(npad / 16) * ksteps * 128;
    hipLaunchKernelGGL(split_weights_h3_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0,
                       st, w, n, k, stride_n, stride_k, ksteps, wsc, (u32x4*)img);
    FGR_CHECK_LAUNCH("split_weights_h3_kernel");
    return FGR_OK;
}

namespace fgr {
// The tile variant the f16x3 dispatcher picks for a shape (FGR_GEMM16_TILE overrides it).
// Default per shape (measured on the forward's GEMMs with tools/gemm_tiles.py, device
// time from HIP-graph replays; profiles/r02_gemm_tiles*.txt): wide outputs take 64 x 128
// tiles (v4 -- W fragments straight to registers -- for K >= 1024, double-buffered v2
// for K >= 512), very tall ones 64 x 128; narrow outputs (N <= 256) and short row counts
// (M <= 4096, N <= 512) the 64 x 64 LDS-DMA g5 ('I') when K % 8 == 0, else the 64 x 64 v4.
// X / Y are I / B and y is b with the row-major staged epilogue (3-8 % faster;
// profiles/r02_gemm_tiles_epi.txt, r02_gemm_tiles_by.txt).
// Few tiles (<= 400 of 64 x 64, e.g. the 3DMatch transformer's 2 x 1060 tokens) with
// K >= 512: the two-k-group g5 ('W', 'T'; 8 waves per block) -- 1.1-1.45x there
// (profiles/r02_gemm_tiles_splitk*.txt).
char h3_tile_kloop(int m, int n, int k);
char h3_tile(int m, int n, int k) {
    const char* force = getenv("FGR_GEMM16_TILE");
    if (force && force[0]) return force[0];
    // short contractions over many rows: the row-stationary kernel (gemm_rs.hip) where it
    // measured faster than the k-looped choice (profiles/r03_gemm_rs_sweep3.txt: 9544 x 1792 x
    // 256 1.37x, x 1024 x 256 1.17x, x 768 x 256 1.10x, 57264 x 256 x 256 1.46x, K <= 128 with
    // N >= 224 1.0-1.41x; narrow outputs, short row counts and N = 256-512 at ~10k rows stay on
    // the k-looped kernels). FGR_GEMM_RS=0 disables.
    static const bool rs_on = [] { const char* e = getenv("FGR_GEMM_RS"); return !(e && e[0] == '0'); }();
    if (rs_on && k % 8 == 0 && k <= 256 && n % 16 == 0 && m >= 8000 &&
        (n >= 640 || (k <= 128 && n >= 224) || (m >= 25000 && n >= 224)))
        return 'z';
    return h3_tile_kloop(m, n, k);
}

// the k-looped kernels' choice
char h3_tile_kloop(int m, int n, int k) {
    const bool g5ok = k % 8 == 0;
    const int64_t tiles64 = (int64_t)ceil_div(m, 64) * ceil_div(n, 64);
    // very few tiles with a long K (3DMatch's 2120 x 256 x 3840, 2120 x 128 x 1920 KPConv
    // products): split-K over 64 x 64 tiles (h3_ksplit; profiles/r02_gemm_splitk_sweep.txt)
    if (g5ok && splitk_shape(m, n, k)) return k >= 2048 ? 'X' : 'W';
    // short row counts with a long contraction and wide outputs (3DMatch's 2120 x 1024 x 2048
    // KPConv product): the 64 x 64 staged g5 'X' -- 82.0 -> 51.4 us in the forward
    // (profiles/r05_gemm_longk_ab.txt; 'Y' before). FGR_GEMM_LONGK=0: the old choice (A/B)
    static const bool longk = [] { const char* e = getenv("FGR_GEMM_LONGK"); return !(e && e[0] == '0'); }();
    if (longk && g5ok && m <= 4096 && k >= 2048 && n >= 512) return 'X';
    // (K >= 2048 took 'S' until round 5; the training backward's 4753 x 256 x 4792 runs 1.4x
    // faster on 'W', profiles/r05_gemm_train_tiles.txt)
    if (g5ok && tiles64 <= 400 && k >= 512 && n >= 32)
        return n <= 64 ? 'S' : ((n <= 128 && k >= 1024 && tiles64 > 256) ? 'T' : 'W');
    if (g5ok && m <= 4096)
        return (n <= 512 || (n <= 1024 && k <= 512)) ? 'X' : 'Y';
    // (512 <= K < 1024 took the g5 'Y' until round 5: 'y' measured 1.2-1.3x faster on every
    // such shape, profiles/r05_gemm_tiles_k512.txt)
    if (n >= 512)
        return k >= 1024 ? 'u' : ((k >= 512 && !g5ok) ? 'k' : 'y');
    if (tiles64 >= 2048) return 'y';
    if (g5ok && (k >= 512 || m <= 16384)) return 'X';
    if (n <= 128 && k >= 1024) return 'f';
    return k <= 1024 ? 't' : 'e';
}

// split-K parts for a g5 variant (1 = none): by default only the measured shapes
// (splitk_shape; 4 parts at K >= 2048, else 2), FGR_GEMM_SPLITK=0 never, =1 the automatic
// factor (g5_ksplit) for any g5 variant; FGR_GEMM_KSPLIT forces one
int h3_ksplit(char cfg, int m, int n, int k) {
    int bm, bn;
    if (k % 8 != 0 || !g5_tile(cfg, &bm, &bn)) return 1;
    const char* on = getenv("FGR_GEMM_SPLITK");
    const char* f = getenv("FGR_GEMM_KSPLIT");
    if (f && f[0]) return g5_ksplit(m, n, k, bm, bn);
    if (on && on[0] == '0') return 1;
    if (on && on[0] == '1') return g5_ksplit(m, n, k, bm, bn);
    return splitk_shape(m, n, k) ? (k >= 2048 ? 4 : 2) : 1;
}
}  // namespace fgr

extern "C" int fgr_gemm_workspace(int32_t m, int32_t n, int32_t k, int32_t mode, size_t* bytes) {
    FGR_REQUIRE(bytes && m >= 0 && n > 0 && k > 0 && (mode == 0 || mode == 1),
                "fgr_gemm_workspace: bad arguments");
    const char cfg = mode == 0 ? h3_tile(m, n, k) : bf16_tile(m, n, k);
    const int ks = mode == 0 ? h3_ksplit(cfg, m, n, k) : bf16_ksplit(cfg, m, n, k);
    *bytes = ks > 1 ? (size_t)ks * m * n * sizeof(float) : 0;
    return FGR_OK;
}

static int gemm_f16x3_impl(const float* a, int64_t lda, const void* w_img, float* c,
                           int64_t ldc, const float* bias, const float* r, int64_t ldr,
                           int32_t m, int32_t n, int32_t k, int32_t act, void* ws,
                           size_t ws_bytes, void* stream) {
    FGR_REQUIRE(a && w_img && c && m >= 0 && n > 0 && k > 0 && lda >= k && ldc >= n &&
                    (!r || ldr >= n),
                "fgr_gemm_f16x3: bad arguments (m %d n %d k %d lda %lld)", m, n, k,
                (long long)lda);
    const bool vec = (k % 8 == 0) && (lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(a) & 15) == 0);
    FGR_REQUIRE(vec || (k % 8 != 0), "fgr_gemm_f16x3: A must be 16-B aligned with lda %% 4 == 0");
    FGR_REQUIRE((reinterpret_cast<uintptr_t>(w_img) & 15) == 0,
                "fgr_gemm_f16x3: image not 16-B aligned");
    if (m == 0) return FGR_OK;
    const bool vo = (ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(c) & 15) == 0) &&
                    (!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0) &&
                    (!r || ((ldr % 4 == 0) && (reinterpret_cast<uintptr_t>(r) & 15) == 0));
    const float* wsc = reinterpret_cast<const float*>(static_cast<const char*>(w_img) +
                                                      image_bytes_h3(n, k));
    GemmH3Args g{a, lda, (const u32x4*)w_img, ksteps_h3(k), wsc, c, ldc, bias, r, ldr,
                 m, n, k, act, vo ? 1 : 0};
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    // tile BM x BN (activation rows x output channels): h3_tile; FGR_GEMM16_TILE overrides it
    // for tuning (a = 128x128, b = 64x128, c = 64x64, d = 128x64, e..x: v2-v4 variants, A..Z,
    // 0..9: g5)
    char cfg = h3_tile(m, n, k);
    // ws (gemm_ws.hip): K = 256, N = 256 / 768 over many rows, 16-B aligned operands
    if (vec && vo && (!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0) &&
        getenv("FGR_GEMM16_TILE") == nullptr &&
        gemm_ws_f16x3(a, lda, w_img, wsc, c, ldc, bias, r, ldr, m, n, k, act, st, nullptr)) {
        FGR_CHECK_LAUNCH("gemm_ws");
        return FGR_OK;
    }
    // rs (gemm_rs.hip): K <= 256, 16-B aligned operands
    if (cfg == 'z') {
        if (vec && vo && gemm_rs_f16x3(a, lda, w_img, ksteps_h3(k), wsc, c, ldc, bias, r, ldr, m,
                                       n, k, act, st)) {
            FGR_CHECK_LAUNCH("gemm_rs");
            return FGR_OK;
        }
        cfg = h3_tile_kloop(m, n, k);                 // unaligned operands
    }
    // g5 (gemm5.hip: LDS-DMA pipeline, A split after the read): A..W, K % 8 == 0 only
    if (((cfg >= 'A' && cfg <= 'Z') || (cfg >= '0' && cfg <= '9')) && k % 8 == 0) {
        int ks = h3_ksplit(cfg, m, n, k);
        if (ks > 1 && (!ws || ws_bytes < (size_t)ks * m * n * sizeof(float) ||
                       (reinterpret_cast<uintptr_t>(ws) & 15) != 0))
            ks = 1;                                     // no room for the parts: no split
        FGR_REQUIRE(gemm_g5_f16x3(cfg, a, lda, w_img, ksteps_h3(k), wsc, c, ldc, bias, r, ldr, m, n, k, act,
                      vo ? 1 : 0, st, ks, static_cast<float*>(ws)),
                    "fgr_gemm_f16x3: g5 variant %c unavailable", cfg);
        FGR_CHECK_LAUNCH("gemm_g5");
        return FGR_OK;
    }
    // v2 variants (BM x BN, KS k32-steps per stage, DBUF) for tuning: e..m
    switch (cfg) {
        case 'e': launch_h3v2<64, 64, 2, false>(g, st); break;
        case 'f': launch_h3v2<64, 64, 2, true>(g, st); break;
        case 'g': launch_h3v2<64, 128, 2, false>(g, st); break;
        case 'h': launch_h3v2<64, 128, 2, true>(g, st); break;
        case 'i': launch_h3v2<128, 128, 2, false>(g, st); break;
        case 'j': launch_h3v2<128, 128, 1, true>(g, st); break;
        case 'k': launch_h3v2<64, 128, 1, true>(g, st); break;
        case 'l': launch_h3v2<64, 64, 1, true>(g, st); break;
        case 'm': launch_h3v2<128, 64, 2, false>(g, st); break;
        // v3 (two-deep register ring): n..s
        case 'n': launch_h3v3<64, 64, 2>(g, st); break;
        case 'o': launch_h3v3<64, 128, 1>(g, st); break;
        case 'p': launch_h3v3<64, 128, 2>(g, st); break;
        case 'q': launch_h3v3<128, 64, 1>(g, st); break;
        case 'r': launch_h3v3<128, 128, 1>(g, st); break;
        case 's': launch_h3v3<128, 64, 2>(g, st); break;
        // v4 (W fragments straight to registers): t..x
        case 't': launch_h3v4<64, 64>(g, st); break;
        case 'u': launch_h3v4<64, 128>(g, st); break;
        case 'v': launch_h3v4<128, 64>(g, st); break;
        case 'w': launch_h3v4<128, 128>(g, st); break;
        case 'x': launch_h3v4<64, 256>(g, st); break;
        default: break;
    }
    if (cfg >= 'e' && cfg <= 'x') {
        FGR_CHECK_LAUNCH("gemm_f16x3_v2");
        return FGR_OK;
    }
    if (cfg == 'a')
        launch_h3<128, 128>(g, st);
    else if (cfg == 'b')
        launch_h3<64, 128>(g, st);
    else if (cfg == 'y')                                   // 'b' with the staged epilogue
        launch_h3<64, 128, true>(g, st);
    else if (cfg == 'd')
        launch_h3<128, 64>(g, st);
    else
        launch_h3<64, 64>(g, st);
    FGR_CHECK_LAUNCH("gemm_f16x3_kernel");
    return FGR_OK;
}

extern "C" int fgr_gemm_f16x3(const float* a, int64_t lda, const void* w_img, float* c,
                              int64_t ldc, const float* bias, const float* r, int64_t ldr,
                              int32_t m, int32_t n, int32_t k, int32_t act, void* stream) {
    return gemm_f16x3_impl(a, lda, w_img, c, ldc, bias, r, ldr, m, n, k, act, nullptr, 0, stream);
}

extern "C" int fgr_gemm_f16x3_ws(const float* a, int64_t lda, const void* w_img, float* c,
                                 int64_t ldc, const float* bias, const float* r, int64_t ldr,
                                 int32_t m, int32_t n, int32_t k, int32_t act, void* ws,
                                 size_t ws_bytes, void* stream) {
    return gemm_f16x3_impl(a, lda, w_img, c, ldc, bias, r, ldr, m, n, k, act, ws, ws_bytes, stream);
}

// LayerNorm -> (+ add) -> Linear in one launch (the row-stationary kernel's LN prologue,
// gemm_rs.hip): supported where the dispatcher picks that kernel for (m, n, k).
extern "C" int fgr_gemm_f16x3_ln_supported(int32_t m, int32_t n, int32_t k) {
    return (m > 0 && n > 0 && k > 0 && (gemm_ws_ln_supported(m, n, k) || h3_tile(m, n, k) == 'z')) ? 1 : 0;
}

static int gemm_f16x3_ln_impl(const float* x, int64_t ldx, const float* gamma, const float* beta,
                              float eps, const float* add, int64_t ld_add, const void* w_img,
                              float* c, int64_t ldc, const float* bias, int32_t m, int32_t n,
                              int32_t k, int32_t act, const float* gamma2, const float* beta2,
                              float* out2, int64_t ld_out2, void* stream) {
    FGR_REQUIRE(x && gamma && beta && w_img && c && m >= 0 && n > 0 && k > 0 && ldx >= k &&
                    ldc >= n && (!add || ld_add >= k) && eps >= 0.f &&
                    (act == FGR_ACT_NONE || act == FGR_ACT_RELU),
                "fgr_gemm_f16x3_ln: bad arguments (m %d n %d k %d act %d)", m, n, k, act);
    FGR_REQUIRE(!out2 || (gamma2 && beta2 && add && ld_out2 >= k && ld_out2 % 4 == 0),
                "fgr_gemm_f16x3_ln_out2: the side output needs gamma2 / beta2, the add and ld_out2 >= k");
    FGR_REQUIRE(m == 0 || fgr_gemm_f16x3_ln_supported(m, n, k),
                "fgr_gemm_f16x3_ln: shape %d x %d x %d not supported (fgr_gemm_f16x3_ln_supported)",
                m, n, k);
    const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gamma) |
                         reinterpret_cast<uintptr_t>(beta) | reinterpret_cast<uintptr_t>(add) |
                         reinterpret_cast<uintptr_t>(w_img) | reinterpret_cast<uintptr_t>(c) |
                         reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(gamma2) |
                         reinterpret_cast<uintptr_t>(beta2) | reinterpret_cast<uintptr_t>(out2);
    FGR_REQUIRE((al & 15) == 0 && ldx % 4 == 0 && ldc % 4 == 0 && (!add || ld_add % 4 == 0),
                "fgr_gemm_f16x3_ln: operands must be 16-B aligned with row strides %% 4 == 0");
    if (m == 0) return FGR_OK;
    const float* wsc = reinterpret_cast<const float*>(static_cast<const char*>(w_img) +
                                                      image_bytes_h3(n, k));
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    if (act == FGR_ACT_NONE || act == FGR_ACT_RELU) {
        const WsLn wl{gamma, beta, add, ld_add, eps, gamma2, beta2, out2, ld_out2, nullptr, nullptr, 0, 0};
        if (gemm_ws_f16x3(x, ldx, w_img, wsc, c, ldc, bias, nullptr, 0, m, n, k, act, st, &wl)) {
            FGR_CHECK_LAUNCH("gemm_ws_ln");
            return FGR_OK;
        }
    }
    const RsLn ln{gamma, beta, add, ld_add, eps, gamma2, beta2, out2, ld_out2, nullptr, nullptr, 0, 0};
    FGR_REQUIRE(gemm_rs_f16x3(x, ldx, w_img, ksteps_h3(k), wsc, c, ldc, bias, nullptr, 0, m, n, k,
                              act, st, &ln),
                "fgr_gemm_f16x3_ln: row-stationary kernel rejected %d x %d x %d", m, n, k);
    FGR_CHECK_LAUNCH("gemm_rs_ln");
    return FGR_OK;
}

extern "C" int fgr_gemm_f16x3_ln(const float* x, int64_t ldx, const float* gamma, const float* beta,
                                 float eps, const float* add, int64_t ld_add, const void* w_img,
                                 float* c, int64_t ldc, const float* bias, int32_t m, int32_t n,
                                 int32_t k, int32_t act, void* stream) {
    return gemm_f16x3_ln_impl(x, ldx, gamma, beta, eps, add, ld_add, w_img, c, ldc, bias, m, n, k,
                              act, nullptr, nullptr, nullptr, 0, stream);
}

extern "C" int fgr_gemm_f16x3_ln_out2(const float* x, int64_t ldx, const float* gamma,
                                      const float* beta, float eps, const float* add, int64_t ld_add,
                                      const void* w_img, float* c, int64_t ldc, const float* bias,
                                      int32_t m, int32_t n, int32_t k, int32_t act,
                                      const float* gamma2, const float* beta2, float* out2,
                                      int64_t ld_out2, void* stream) {
    FGR_REQUIRE(out2, "fgr_gemm_f16x3_ln_out2: out2 is required");
    return gemm_f16x3_ln_impl(x, ldx, gamma, beta, eps, add, ld_add, w_img, c, ldc, bias, m, n, k,
                              act, gamma2, beta2, out2, ld_out2, stream);
}

// The CorrespondenceRegressor head (finegrained_regtr.py:411-455) in two row-stationary launches
// (gemm_rs.hip): [coor_mlp[0] | conf_logits_decoder] as one product over the stacked image of
// [W0; Wc; 0] (ReLU on the first d columns -> hidden, column d -> logits), then coor_mlp[2] ->
// ReLU -> coor_mlp[4] with the 3-wide output formed in the epilogue (hidden2 never written).
extern "C" int fgr_corr_head_supported(int32_t m, int32_t d) {
    return (m > 0 && d > 0 && d % 16 == 0 && d <= 256 && d / 16 + 1 <= 64) ? 1 : 0;
}

extern "C" int fgr_corr_head_f16x3(const float* f, int64_t ldf, int32_t m, int32_t d,
                                   const void* w0c_img, const float* b0c, const void* w2_img,
                                   const float* b2, const float* w4, const float* b4, float* hidden,
                                   float* corr, float* logits, void* stream) {
    FGR_REQUIRE(f && w0c_img && b0c && w2_img && b2 && w4 && b4 && hidden && corr && logits &&
                    m >= 0 && ldf >= d && ldf % 4 == 0,
                "fgr_corr_head_f16x3: bad arguments");
    FGR_REQUIRE(m == 0 || fgr_corr_head_supported(m, d),
                "fgr_corr_head_f16x3: d %d not supported (fgr_corr_head_supported)", d);
    const uintptr_t al = reinterpret_cast<uintptr_t>(f) | reinterpret_cast<uintptr_t>(w0c_img) |
                         reinterpret_cast<uintptr_t>(b0c) | reinterpret_cast<uintptr_t>(w2_img) |
                         reinterpret_cast<uintptr_t>(b2) | reinterpret_cast<uintptr_t>(w4) |
                         reinterpret_cast<uintptr_t>(hidden);
    FGR_REQUIRE((al & 15) == 0, "fgr_corr_head_f16x3: operands must be 16-B aligned");
    if (m == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const int ks = ksteps_h3(d);
    const float* wsc0 = reinterpret_cast<const float*>(static_cast<const char*>(w0c_img) +
                                                       image_bytes_h3(d + 16, d));
    const float* wsc2 = reinterpret_cast<const float*>(static_cast<const char*>(w2_img) +
                                                       image_bytes_h3(d, d));
    const RsHead h0{d, logits, nullptr, nullptr, nullptr};
    FGR_REQUIRE(gemm_rs_f16x3(f, ldf, w0c_img, ks, wsc0, hidden, d, b0c, nullptr, 0, m, d + 16, d,
                              FGR_ACT_RELU, st, nullptr, &h0),
                "fgr_corr_head_f16x3: row-stationary kernel rejected the first product");
    FGR_CHECK_LAUNCH("gemm_rs (corr head, coor_mlp[0] | conf_logits)");
    const RsHead h2{d, nullptr, w4, b4, corr};
    FGR_REQUIRE(gemm_rs_f16x3(hidden, d, w2_img, ks, wsc2, hidden, d, b2, nullptr, 0, m, d, d,
                              FGR_ACT_RELU, st, nullptr, &h2),
                "fgr_corr_head_f16x3: row-stationary kernel rejected the second product");
    FGR_CHECK_LAUNCH("gemm_rs (corr head, coor_mlp[2] -> coor_mlp[4])");
    return FGR_OK;
}

// ---- the pre-norm in_proj with the attention's K / V images in its epilogue ----------------
// Image geometry (attention16.hip, head dim 32): one 16 KB image per (global 64-row tile,
// head), then the int2 scale exponents of all of them.
extern "C" int fgr_kv_image_bytes(int64_t n_rows, int32_t n_head, int32_t head_dim, size_t* bytes) {
    FGR_REQUIRE(bytes && n_rows >= 0 && n_head > 0 && (head_dim == 32 || head_dim == 64),
                "fgr_kv_image_bytes: bad arguments (head_dim 32 or 64)");
    const int64_t nt = std::max<int64_t>(1, ceil_div(n_rows, 64)) * n_head;
    *bytes = (size_t)(nt * (head_dim == 32 ? 1024 : 2048) * 16 + nt * 8);
    return FGR_OK;
}

// the in_proj (no LayerNorm prologue) with the K / V images of head dim 64 in the staged g5
// epilogue (gemm5.hip gemm_g5_f16x3_qkv)
extern "C" int fgr_gemm_f16x3_qkv_supported(int32_t m, int32_t d, int32_t n_head) {
    return (m > 0 && n_head > 0 && d == 64 * n_head && d % 128 == 0) ? 1 : 0;
}

extern "C" int fgr_gemm_f16x3_qkv(const float* a, int64_t lda, const void* w_img, float* q,
                                  int64_t ld_q, const float* bias, int32_t m, int32_t d,
                                  int32_t n_head, void* kv_img, void* stream) {
    FGR_REQUIRE(a && w_img && q && bias && kv_img && m >= 0 && lda >= d && ld_q >= d,
                "fgr_gemm_f16x3_qkv: bad arguments");
    FGR_REQUIRE(m == 0 || fgr_gemm_f16x3_qkv_supported(m, d, n_head),
                "fgr_gemm_f16x3_qkv: d %d heads %d not supported (head dim 64, d %% 128 == 0)", d, n_head);
    const uintptr_t al = reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(w_img) |
                         reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(bias) |
                         reinterpret_cast<uintptr_t>(kv_img);
    FGR_REQUIRE((al & 15) == 0 && lda % 4 == 0 && ld_q % 4 == 0,
                "fgr_gemm_f16x3_qkv: operands must be 16-B aligned with row strides %% 4 == 0");
    if (m == 0) return FGR_OK;
    const int n = 3 * d;
    const float* wsc = reinterpret_cast<const float*>(static_cast<const char*>(w_img) +
                                                      image_bytes_h3(n, d));
    const int64_t nt = ceil_div(m, 64) * n_head;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    FGR_REQUIRE(gemm_g5_f16x3_qkv(a, lda, w_img, ksteps_h3(d), wsc, q, ld_q, bias, m, d, n_head,
                                  static_cast<char*>(kv_img),
                                  reinterpret_cast<int2*>(static_cast<char*>(kv_img) + nt * 2048 * 16), st),
                "fgr_gemm_f16x3_qkv: g5 variant unavailable");
    FGR_CHECK_LAUNCH("gemm_g5_qkv");
    return FGR_OK;
}

extern "C" int fgr_gemm_f16x3_ln_qkv_supported(int32_t m, int32_t d, int32_t n_head) {
    return (m > 0 && d == 32 * n_head && d == 256 && fgr_gemm_f16x3_ln_supported(m, 3 * d, d)) ? 1 : 0;
}

extern "C" int fgr_gemm_f16x3_ln_qkv(const float* x, int64_t ldx, const float* gamma,
                                     const float* beta, float eps, const float* add, int64_t ld_add,
                                     const void* w_img, float* q, int64_t ld_q, const float* bias,
                                     int32_t m, int32_t d, int32_t n_head, void* kv_img,
                                     const float* gamma2, const float* beta2, float* out2,
                                     int64_t ld_out2, void* stream) {
    FGR_REQUIRE(x && gamma && beta && add && w_img && q && bias && kv_img && m >= 0 && ldx >= d &&
                    ld_add >= d && ld_q >= d && eps >= 0.f && (!out2 || (gamma2 && beta2 && ld_out2 >= d)),
                "fgr_gemm_f16x3_ln_qkv: bad arguments");
    FGR_REQUIRE(m == 0 || fgr_gemm_f16x3_ln_qkv_supported(m, d, n_head),
                "fgr_gemm_f16x3_ln_qkv: m %d d %d heads %d not supported", m, d, n_head);
    const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gamma) |
                         reinterpret_cast<uintptr_t>(beta) | reinterpret_cast<uintptr_t>(add) |
                         reinterpret_cast<uintptr_t>(w_img) | reinterpret_cast<uintptr_t>(q) |
                         reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(kv_img) |
                         reinterpret_cast<uintptr_t>(gamma2) | reinterpret_cast<uintptr_t>(beta2) |
                         reinterpret_cast<uintptr_t>(out2);
    FGR_REQUIRE((al & 15) == 0 && ldx % 4 == 0 && ld_q % 4 == 0 && ld_add % 4 == 0 &&
                    (!out2 || ld_out2 % 4 == 0),
                "fgr_gemm_f16x3_ln_qkv: operands must be 16-B aligned with row strides %% 4 == 0");
    if (m == 0) return FGR_OK;
    const int n = 3 * d;
    const float* wsc = reinterpret_cast<const float*>(static_cast<const char*>(w_img) +
                                                      image_bytes_h3(n, d));
    const int64_t nt = ceil_div(m, 64) * n_head;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    {
        const WsLn wl{gamma, beta, add, ld_add, eps, gamma2, beta2, out2, ld_out2,
                      static_cast<char*>(kv_img),
                      reinterpret_cast<int2*>(static_cast<char*>(kv_img) + nt * 1024 * 16), n_head, d};
        if (gemm_ws_f16x3(x, ldx, w_img, wsc, q, ld_q, bias, nullptr, 0, m, n, d, FGR_ACT_NONE, st, &wl)) {
            FGR_CHECK_LAUNCH("gemm_ws_ln_qkv");
            return FGR_OK;
        }
    }
    const RsLn ln{gamma, beta, add, ld_add, eps, gamma2, beta2, out2, ld_out2,
                  static_cast<char*>(kv_img),
                  reinterpret_cast<int2*>(static_cast<char*>(kv_img) + nt * 1024 * 16), n_head, d};
    FGR_REQUIRE(gemm_rs_f16x3(x, ldx, w_img, ksteps_h3(d), wsc, q, ld_q, bias, nullptr, 0, m, n, d,
                              FGR_ACT_NONE, st, &ln),
                "fgr_gemm_f16x3_ln_qkv: row-stationary kernel rejected %d x %d x %d", m, n, d);
    FGR_CHECK_LAUNCH("gemm_rs_ln_qkv");
    return FGR_OK;
}
