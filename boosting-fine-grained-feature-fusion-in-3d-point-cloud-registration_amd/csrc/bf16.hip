// bf16 compute mode of the forward (BASELINE configs[4]: "3DLoMatch ... bf16 features with
// MFMA bf16 attention"): every dense product and the attention run ONE bf16 MFMA product per
// fp32 product (v_mfma_f32_16x16x32_bf16, fp32 accumulation), 3x fewer matrix-core cycles
// than the fp32-accurate f16x3 mode. Operands are rounded to bf16 (RNE) where they enter the
// MFMA; storage between kernels, accumulation, softmax, normalisation and the epilogues stay
// fp32. bf16 keeps fp32's exponent range, so no scaling is needed. Accuracy: ~2^-9 relative
// per product; the forward's tolerance against the fp32 oracle is stated in DESIGN.md and
// tests/test_gpu_bf16.py.
//
// * fgr_split_weights_bf16: W (n, k) -> image [n16 panel][k32 step][g 4][16 rows] x 16 B
//   (8 consecutive k of one row, bf16), i.e. the MFMA A-operand fragment order: one
//   wave-load of a (panel, step) is 1 KB contiguous in lane order.
// * fgr_gemm_bf16: C = act(A . W^T + bias (+ R)) with the f16x3 v4 structure (W fragments
//   straight from the image into registers, A rounded to bf16 while staging into a
//   double-buffered LDS image, one barrier per k32 step), swapped orientation (each lane
//   owns one activation row, 16-B epilogue stores).
// * fgr_attention_bf16: the flash attention of attention16.hip with single-term bf16 K / V
//   images ([k-step][g 4][key 64] / [key 64][DH] with the ds_read_b64_tr_b16 swizzle), Q and
//   P rounded to bf16 in registers, head_dim 32 or 64.
#include <type_traits>

#include "common.h"

namespace fgr {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float finish_bf(float y, float b, float r, int act) {
    if (act == FGR_ACT_RELU_RES_LEAKY) {
        const float t = fmaxf(y + b, 0.f) + r;
        return t > 0.f ? t : 0.1f * t;
    }
    const float t = y + b + r;
    return act == FGR_ACT_RELU ? fmaxf(t, 0.f) : t;
}

__global__ void split_weights_bf16_kernel(const float* __restrict__ w, int n, int k, int64_t sn,
                                          int64_t sk, int ksteps, u32x4* __restrict__ img) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)((n + 15) / 16) * ksteps * 64;
    if (u >= total) return;
    const int i = (int)(u % 16);
    const int g = (int)((u / 16) % 4);
    const int64_t ps = u / 64;
    const int s = (int)(ps % ksteps);
    const int panel = (int)(ps / ksteps);
    const int row = panel * 16 + i;
    bf16x8 out;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int col = s * 32 + 8 * g + e;
        out[e] = (__bf16)((row < n && col < k) ? w[(int64_t)row * sn + (int64_t)col * sk] : 0.f);
    }
    img[u] = __builtin_bit_cast(u32x4, out);
}

struct GemmBfArgs {
    const float* A; int64_t lda;
    const u32x4* W; int ksteps;
    float* C; int64_t ldc;
    const float* bias;
    const float* R; int64_t ldr;
    int M, N, K, act, vec_out;
    // K / V attention images (bf16, head dim 64; BM = 64, BN = 128): columns >= kv_col0 go to
    // the images of their GLOBAL 64-row tile and head (layout of attn_kv_image_bf16_kernel)
    char* kv_img; int n_head; int kv_col0;
};

// bf16 attention image of head dim 64 (bf_units<64>() below): 1024 16-B units per (tile, head),
// V from unit 512
constexpr int bf_units_kv() { return 64 * 8 + 2 * 256; }

template <int BM, int BN, bool KVEC>
__global__ void __launch_bounds__(256) gemm_bf16_kernel(GemmBfArgs p) {
    constexpr int TM = BM / 16, TN = BN / 64;
    constexpr int UA = BM * 4 / 256;
    constexpr int ASZ = 4 * BM;                          // 16-B units of one A stage
    static_assert(UA >= 1 && TN >= 1, "tile");
    __shared__ u32x4 a_lds[2 * ASZ];

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
    const int wn = wv * (BN / 4);

    const float* arow[UA];
    int akk[UA];
#pragma unroll
    for (int j = 0; j < UA; ++j) {
        const int u = tid + 256 * j;
        arow[j] = p.A + (int64_t)min(m0 + (u >> 2), p.M - 1) * p.lda;
        akk[j] = 8 * (u & 3);
    }
    const u32x4* wp[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int panel = min((n0 + wn) / 16 + j, npanel - 1);
        wp[j] = p.W + (int64_t)panel * p.ksteps * 64 + lane;
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
            bf16x8 v;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (__bf16)x[e];
            a_img[gg * BM + (row ^ (2 * gg))] = __builtin_bit_cast(u32x4, v);
        }
    };
    u32x4 w0[TN], w1[TN];
    auto load_w = [&](int s, u32x4 (&w)[TN]) {
#pragma unroll
        for (int j = 0; j < TN; ++j) w[j] = wp[j][(int64_t)s * 64];
    };
    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int b, const u32x4 (&w)[TN]) {
        const u32x4* a_img = a_lds + b * ASZ;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const bf16x8 av = __builtin_bit_cast(bf16x8, a_img[g * BM + ((16 * i + c) ^ (2 * g))]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, w[j]), av, acc[j][i], 0, 0, 0);
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
    if constexpr (BM == 64 && BN == 128) {
        if (p.kv_img && n0 >= p.kv_col0) {                 // block-uniform: K or V columns
            // bf16 has fp32's range: no scale, every lane converts its own 4 outputs; rows
            // past M are written as zeros (the attention's P is 0 there, V must be finite)
            const int rel0 = n0 + wn - p.kv_col0;
            const int isv = rel0 >= 64 * p.n_head ? 1 : 0;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int m = m0 + 16 * i + c;
                const int key = 16 * i + c;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = n0 + wn + 16 * j + 4 * g;
                    const int rel = n - p.kv_col0 - isv * 64 * p.n_head;
                    const int head = rel >> 6, d0 = rel & 63;
                    const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
                    const bool ok = m < p.M;
                    const __bf16 t[4] = {(__bf16)(ok ? acc[j][i][0] + bb.x : 0.f),
                                         (__bf16)(ok ? acc[j][i][1] + bb.y : 0.f),
                                         (__bf16)(ok ? acc[j][i][2] + bb.z : 0.f),
                                         (__bf16)(ok ? acc[j][i][3] + bb.w : 0.f)};
                    char* base = p.kv_img + ((int64_t)bm * p.n_head + head) * (int64_t)(bf_units_kv() * 16);
                    char* dst;
                    if (isv) {
                        const int vch = (d0 >> 3) ^ (((key >> 1) & 3) << 1);
                        dst = base + 512 * 16 + key * 128 + vch * 16 + ((d0 >> 2) & 1) * 8;
                    } else {
                        dst = base + (((d0 >> 5) * 4 + ((d0 & 31) >> 3)) * 64 + key) * 16 + ((d0 >> 2) & 1) * 8;
                    }
                    *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(t);
                }
            }
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + 16 * i + c;
        if (m >= p.M) continue;
        float* crow = p.C + (int64_t)m * p.ldc;
        const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn + 16 * j + 4 * g;
            if (n >= p.N) continue;
            if (p.vec_out && n + 3 < p.N) {
                float4 bb = make_float4(0.f, 0.f, 0.f, 0.f), rr = bb;
                if (p.bias) bb = *reinterpret_cast<const float4*>(p.bias + n);
                if (rrow) rr = *reinterpret_cast<const float4*>(rrow + n);
                *reinterpret_cast<float4*>(crow + n) = make_float4(
                    finish_bf(acc[j][i][0], bb.x, rr.x, p.act), finish_bf(acc[j][i][1], bb.y, rr.y, p.act),
                    finish_bf(acc[j][i][2], bb.z, rr.z, p.act), finish_bf(acc[j][i][3], bb.w, rr.w, p.act));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (n + e >= p.N) break;
                    crow[n + e] = finish_bf(acc[j][i][e], p.bias ? p.bias[n + e] : 0.f,
                                            rrow ? rrow[n + e] : 0.f, p.act);
                }
            }
        }
    }
}

// ---------------------------------- attention ------------------------------------------
__device__ __forceinline__ float xg_max16b(float v) {   // max over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float xg_sum16b(float v) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// 16-B units per (tile, head) image and the first V unit
template <int DH> constexpr int bf_units() { return DH * 8 + (DH / 32) * 256; }
template <int DH> constexpr int bf_unit_v() { return (DH / 32) * 256; }

// V image row swizzle (as attention16.hip v_swz): conflict-free transposed reads at DH 32 and 64
template <int DH>
__device__ __forceinline__ int bf_v_swz(int key) {
    if constexpr (DH == 64) return ((key >> 1) & 3) << 1;
    else return ((key >> 2) & 1) << 1;
}

template <int DH>
__global__ void __launch_bounds__(256)
attn_kv_image_bf16_kernel(const float* __restrict__ k, int64_t ld_k, const float* __restrict__ v,
                          int64_t ld_v, const int64_t* __restrict__ kv_off, int n_head,
                          uint4* __restrict__ img) {
    constexpr int NF = DH / 16, RU = DH / 4;
    const int s = blockIdx.z, h = blockIdx.y, tt = blockIdx.x;
    const int64_t kb = kv_off[s];
    const int nk = (int)(kv_off[s + 1] - kb);
    if (tt * 64 >= nk) return;
    const int64_t tile = (kb / 64 + s + tt) * n_head + h;
    char* base = reinterpret_cast<char*>(img + tile * bf_units<DH>());
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int e = threadIdx.x + 256 * i;
        const int key = e / RU, d0 = (e % RU) * 4;
        const bool ok = tt * 64 + key < nk;
        const int64_t row = kb + tt * 64 + key;
        const float4 kx = ok ? *reinterpret_cast<const float4*>(k + row * ld_k + h * DH + d0)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 vx = ok ? *reinterpret_cast<const float4*>(v + row * ld_v + h * DH + d0)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        const __bf16 kt[4] = {(__bf16)kx.x, (__bf16)kx.y, (__bf16)kx.z, (__bf16)kx.w};
        const __bf16 vt[4] = {(__bf16)vx.x, (__bf16)vx.y, (__bf16)vx.z, (__bf16)vx.w};
        const int ks = d0 >> 5, g = (d0 & 31) >> 3, half = (d0 >> 2) & 1;
        const int vch = (d0 >> 3) ^ bf_v_swz<DH>(key);
        *reinterpret_cast<uint2*>(base + ((ks * 4 + g) * 64 + key) * 16 + half * 8) =
            *reinterpret_cast<const uint2*>(kt);
        *reinterpret_cast<uint2*>(base + bf_unit_v<DH>() * 16 + key * (2 * DH) + vch * 16 +
                                  half * 8) = *reinterpret_cast<const uint2*>(vt);
    }
}

// v2 key-tile loop (as attention16.hip's attn_f16x3_v2_kernel): maxima by v_max3 without NaN
// canonicalisation, the tile loop unrolled by two so both LDS buffers' addresses are per-lane
// constants + instruction offsets, DMA pieces contiguous per wave; built -fno-slp-vectorize.
// The round-2 loop issued ~14 VALU per MFMA at head dim 32 (profiles/r03_pmc_attn_v1_before.json).
// (plain fmaxf: the file is built -fno-honor-nans; see attention16.hip)
__device__ __forceinline__ float vmax3b(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
__device__ __forceinline__ float vmax2b(float a, float b) { return fmaxf(a, b); }

template <int DH>
__global__ void __launch_bounds__(256, 4)
attn_bf16_v2_kernel(const float* __restrict__ q, int64_t ld_q, const uint4* __restrict__ img,
                    float* __restrict__ o, int64_t ld_o, const int64_t* __restrict__ q_off,
                    const int64_t* __restrict__ kv_off, const int32_t* __restrict__ kv_seg,
                    int n_head, int n_seg, int n_qblk, float scale_log2, int global_tiles) {
    constexpr int KD = DH / 32, TD = DH / 16;
    constexpr int UN = bf_units<DH>();
    constexpr int PW = UN / 64 / 4;
    // two LDS objects, pointer-addressed (see attn_f16x3_v2_kernel: the next tile's DMA then
    // does not hold the V reads of the current one)
    __shared__ u32x4 lds_b0[UN], lds_b1[UN];
    typedef __attribute__((address_space(3))) char lds_c;
    const int L = blockIdx.x, xcd = L & 7, j0 = L >> 3;
    const int pair = (j0 / n_qblk) * 8 + xcd, qblk = j0 % n_qblk;
    if (pair >= n_seg * n_head) return;
    const int seg = pair / n_head, head = pair % n_head;
    const int64_t qb = q_off[seg], qe = q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)qblk * 64;
    if (q0 >= qe) return;
    const int ks = kv_seg[seg];
    const int64_t kb = kv_off[ks];
    const int nk = (int)(kv_off[ks + 1] - kb);
    // per-segment images or images of GLOBAL 64-row tiles (written by the in_proj GEMM,
    // fgr_gemm_bf16_qkv): the segment's keys then start `lead` rows into its first tile
    const int lead = global_tiles ? (int)(kb & 63) : 0;
    const int ntile = (lead + nk + 63) / 64;
    const int64_t tile0 = (global_tiles ? kb / 64 : kb / 64 + ks) * n_head + head;
    const int64_t tile_stride = (int64_t)n_head * UN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const u32x4* src_lane = reinterpret_cast<const u32x4*>(img) + tile0 * UN + wv * PW * 64 + lane;

    const int64_t qrow = q0 + wv * 16 + c;
    bf16x8 qt[KD];
#pragma unroll
    for (int kd = 0; kd < KD; ++kd) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if (qrow < qe) {
            const float4* p = reinterpret_cast<const float4*>(q + qrow * ld_q + head * DH + 32 * kd + 8 * g);
            a = p[0];
            b = p[1];
        }
        const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) qt[kd][e] = (__bf16)(x[e] * scale_log2);
    }
    f32x4 acc[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    const uint32_t kaddr = (uint32_t)(g * 64 + c) * 16;
    const int qq = c >> 2, pp = c & 3;
    uint32_t vaddr[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t)
        vaddr[t] = bf_unit_v<DH>() * 16 + (4 * g + qq) * (2 * DH) +
                   (((2 * t + (pp >> 1)) ^ bf_v_swz<DH>(4 * g + qq)) * 16) + (pp & 1) * 8;
    auto dma = [&](int t, auto buf_tag) {
        constexpr int BUF = decltype(buf_tag)::value;
        const u32x4* src = src_lane + (int64_t)t * tile_stride;
        __attribute__((address_space(3))) char* dst =
            (lds_c*)(BUF == 0 ? lds_b0 : lds_b1) + wv * PW * 1024;
#pragma unroll
        for (int j = 0; j < PW; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(src + j * 64),
                                             (__attribute__((address_space(3))) void*)(dst + j * 1024),
                                             16, 0, 0);
    };
    // tile tt lives in LDS buffer (tt + shift) & 1 (a masked first tile takes buffer 1)
    const int shift = lead > 0 ? 1 : 0;
    if (ntile > 0) {
        if (shift) dma(0, std::integral_constant<int, 1>{});
        else dma(0, std::integral_constant<int, 0>{});
    }
    auto tile = [&](int tt, auto buf_tag, auto mask_tag) {
        constexpr int BUF = decltype(buf_tag)::value;
        constexpr bool MASK = decltype(mask_tag)::value;
        __builtin_amdgcn_s_waitcnt((7 << 4));                    // vmcnt(0) lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        if (tt + 1 < ntile) dma(tt + 1, std::integral_constant<int, 1 - BUF>{});
        lds_c* const bp = (lds_c*)(BUF == 0 ? lds_b0 : lds_b1);
        typedef __attribute__((address_space(3))) u32x4 lds_u4;
        typedef __attribute__((address_space(3))) s16x4 lds_s4;
        f32x4 s[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kd = 0; kd < KD; ++kd)
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, *(lds_u4*)(bp + kaddr + ((kd * 4) * 64 + 16 * n) * 16)),
                    qt[kd], a, 0, 0, 0);
            s[n] = a;
        }
        if constexpr (MASK) {
            const int lo = tt == 0 ? lead : 0, hi = lead + nk - tt * 64;   // valid keys [lo, hi)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int kl = 16 * n + 4 * g + r;
                    if (kl < lo || kl >= hi) s[n][r] = -INFINITY;
                }
        }
        float mx = vmax3b(s[0][0], s[0][1], s[0][2]);
        mx = vmax3b(mx, s[0][3], s[1][0]);
        mx = vmax3b(mx, s[1][1], s[1][2]);
        mx = vmax3b(mx, s[1][3], s[2][0]);
        mx = vmax3b(mx, s[2][1], s[2][2]);
        mx = vmax3b(mx, s[2][3], s[3][0]);
        mx = vmax3b(mx, s[3][1], s[3][2]);
        mx = vmax2b(mx, s[3][3]);
        {
            auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
            mx = vmax2b(__uint_as_float(a[0]), __uint_as_float(a[1]));
            auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
            mx = vmax2b(__uint_as_float(b[0]), __uint_as_float(b[1]));
        }
        const float m_new = vmax2b(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float rs = 0.f;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __builtin_amdgcn_exp2f(s[n][r] - m_new);
                s[n][r] = p;
                rs += p;
            }
        l_run = l_run * alpha + rs;
#pragma unroll
        for (int t = 0; t < TD; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[t][r] *= alpha;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            bf16x8 pt;
#pragma unroll
            for (int e = 0; e < 8; ++e) pt[e] = (__bf16)s[2 * j + (e >> 2)][e & 3];
#pragma unroll
            for (int t = 0; t < TD; ++t) {
                lds_c* const vb = bp + vaddr[t] + j * 32 * (2 * DH);
                const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)vb);
                const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vb + 16 * (2 * DH)));
                const s16x8 w8 = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w8), pt,
                                                                 acc[t], 0, 0, 0);
            }
        }
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    const int nfull = (lead + nk) / 64;              // tiles [shift, nfull) have 64 valid keys
    int tt = 0;
    if (shift) {                                     // the first tile, keys before the segment masked
        tile(0, B1{}, std::true_type{});
        tt = 1;
    }
    for (; tt + 2 <= nfull; tt += 2) {               // (tt + shift) even: buffer 0
        tile(tt, B0{}, std::false_type{});
        tile(tt + 1, B1{}, std::false_type{});
    }
    if (tt < nfull) {
        tile(tt, B0{}, std::false_type{});
        ++tt;
    }
    if (tt < ntile) {
        if ((tt + shift) & 1) tile(tt, B1{}, std::true_type{});
        else tile(tt, B0{}, std::true_type{});
    }
    const float inv = 1.0f / xg_sum16b(l_run);
    if (qrow < qe) {
#pragma unroll
        for (int t = 0; t < TD; ++t) {
            float4 y;
            y.x = acc[t][0] * inv; y.y = acc[t][1] * inv;
            y.z = acc[t][2] * inv; y.w = acc[t][3] * inv;
            *reinterpret_cast<float4*>(o + qrow * ld_o + head * DH + 16 * t + 4 * g) = y;
        }
    }
}

int ksteps_bf(int k) { return (k + 63) / 64 * 2; }     // even: g5 stages read 2 k32-steps
size_t image_bytes_bf(int n, int k) { return (size_t)((n + 15) / 16) * ksteps_bf(k) * 64 * 16; }
int64_t n_tiles_bf(int64_t n_kv_rows, int32_t n_kv_seg) { return n_kv_rows / 64 + n_kv_seg + 1; }

}  // namespace
bool gemm_g5_bf16(char cfg, const float* A, int64_t lda, const void* W, int ksteps, float* C,
                  int64_t ldc, const float* bias, const float* R, int64_t ldr, int M, int N, int K,
                  int act, int vec_out, hipStream_t st, int ksplit, float* part);
bool g5_tile(char cfg, int* bm, int* bn);
int g5_ksplit(int M, int N, int K, int BM, int BN);
inline bool splitk_shape(int m, int n, int k) {        // as gemm16.hip
    return k >= 1920 && n <= 256 && (int64_t)((m + 63) / 64) * ((n + 63) / 64) <= 160;
}

// narrow outputs with long contractions: the 64 x 64 LDS-DMA g5 ('X', gemm5.hip; measured
// 1.2-1.5x faster there); few tiles (<= 400 of 64 x 64) with K >= 512 and the short-M
// K >= 2048 layers: the two-k-group g5 ('S', 'T', 'W'); otherwise the register-staged
// kernel below ('z'; FGR_GEMM_BF16_TILE A..Z forces a g5 variant, anything else it)
char bf16_tile(int m, int n, int k) {
    const char* force = getenv("FGR_GEMM_BF16_TILE");
    if (force && force[0]) return force[0];
    const int64_t tiles64 = (int64_t)ceil_div(m, 64) * ceil_div(n, 64);
    if (k % 8 == 0 && splitk_shape(m, n, k)) return k >= 2048 ? 'X' : 'S';   // split-K
    if (tiles64 <= 400 && k >= 512 && n >= 32)
        return (k >= 2048 || n <= 64) ? 'S' : ((n <= 128 && k >= 1024 && tiles64 > 256) ? 'T' : 'W');
    if (m <= 4096 && k >= 2048) return 'W';
    return n <= 256 && k >= 1000 ? 'X' : 'z';
}

int bf16_ksplit(char cfg, int m, int n, int k) {
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

using namespace fgr;

extern "C" int fgr_split_weights_bf16_bytes(int32_t n, int32_t k, size_t* bytes) {
    FGR_REQUIRE(bytes && n > 0 && k > 0, "fgr_split_weights_bf16_bytes: bad arguments");
    *bytes = image_bytes_bf(n, k);
    return FGR_OK;
}

extern "C" int fgr_split_weights_bf16(const float* w, int32_t n, int32_t k, int64_t stride_n,
                                      int64_t stride_k, void* img, void* stream) {
    FGR_REQUIRE(w && img && n > 0 && k > 0 && (reinterpret_cast<uintptr_t>(img) & 15) == 0,
                "fgr_split_weights_bf16: bad arguments");
    const int64_t total = (int64_t)((n + 15) / 16) * ksteps_bf(k) * 64;
    hipLaunchKernelGGL(split_weights_bf16_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0,
                       as_stream(stream), w, n, k, stride_n, stride_k, ksteps_bf(k), (u32x4*)img);
    FGR_CHECK_LAUNCH("split_weights_bf16_kernel");
    return FGR_OK;
}

static int gemm_bf16_impl(const float* a, int64_t lda, const void* w_img, float* c, int64_t ldc,
                          const float* bias, const float* r, int64_t ldr, int32_t m, int32_t n,
                          int32_t k, int32_t act, void* ws, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(a && w_img && c && m >= 0 && n > 0 && k > 0 && lda >= k && ldc >= n &&
                    (!r || ldr >= n),
                "fgr_gemm_bf16: bad arguments (m %d n %d k %d)", m, n, k);
    const bool vec = (k % 8 == 0) && (lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(a) & 15) == 0);
    FGR_REQUIRE(vec || (k % 8 != 0), "fgr_gemm_bf16: A must be 16-B aligned with lda %% 4 == 0");
    FGR_REQUIRE((reinterpret_cast<uintptr_t>(w_img) & 15) == 0, "fgr_gemm_bf16: image not 16-B aligned");
    if (m == 0) return FGR_OK;
    const bool vo = (ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(c) & 15) == 0) &&
                    (!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0) &&
                    (!r || ((ldr % 4 == 0) && (reinterpret_cast<uintptr_t>(r) & 15) == 0));
    GemmBfArgs g{a, lda, (const u32x4*)w_img, ksteps_bf(k), c, ldc, bias, r, ldr, m, n, k, act,
                 vo ? 1 : 0, nullptr, 0, 0};
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const char cfg = bf16_tile(m, n, k);
    if (((cfg >= 'A' && cfg <= 'Z') || (cfg >= '0' && cfg <= '9')) && k % 8 == 0) {
        int ks = bf16_ksplit(cfg, m, n, k);
        if (ks > 1 && (!ws || ws_bytes < (size_t)ks * m * n * sizeof(float) ||
                       (reinterpret_cast<uintptr_t>(ws) & 15) != 0))
            ks = 1;                                     // no room for the parts: no split
        FGR_REQUIRE(gemm_g5_bf16(cfg, a, lda, w_img, ksteps_bf(k), c, ldc, bias, r, ldr, m, n, k, act,
                     vo ? 1 : 0, st, ks, static_cast<float*>(ws)),
                    "fgr_gemm_bf16: g5 variant %c unavailable", cfg);
        FGR_CHECK_LAUNCH("gemm_g5 (bf16)");
        return FGR_OK;
    }
    const int bm = 64, bn = n >= 128 ? 128 : 64;
    const unsigned nblk = (unsigned)(ceil_div(m, bm) * ceil_div(n, bn));
    if (bn == 128) {
        if (k % 8 == 0) hipLaunchKernelGGL((gemm_bf16_kernel<64, 128, true>), dim3(nblk), dim3(256), 0, st, g);
        else hipLaunchKernelGGL((gemm_bf16_kernel<64, 128, false>), dim3(nblk), dim3(256), 0, st, g);
    } else {
        if (k % 8 == 0) hipLaunchKernelGGL((gemm_bf16_kernel<64, 64, true>), dim3(nblk), dim3(256), 0, st, g);
        else hipLaunchKernelGGL((gemm_bf16_kernel<64, 64, false>), dim3(nblk), dim3(256), 0, st, g);
    }
    FGR_CHECK_LAUNCH("gemm_bf16_kernel");
    return FGR_OK;
}

extern "C" int fgr_gemm_bf16(const float* a, int64_t lda, const void* w_img, float* c, int64_t ldc,
                             const float* bias, const float* r, int64_t ldr, int32_t m, int32_t n,
                             int32_t k, int32_t act, void* stream) {
    return gemm_bf16_impl(a, lda, w_img, c, ldc, bias, r, ldr, m, n, k, act, nullptr, 0, stream);
}

extern "C" int fgr_gemm_bf16_ws(const float* a, int64_t lda, const void* w_img, float* c,
                                int64_t ldc, const float* bias, const float* r, int64_t ldr,
                                int32_t m, int32_t n, int32_t k, int32_t act, void* ws,
                                size_t ws_bytes, void* stream) {
    return gemm_bf16_impl(a, lda, w_img, c, ldc, bias, r, ldr, m, n, k, act, ws, ws_bytes, stream);
}

extern "C" int fgr_attention_bf16_workspace(int64_t n_kv_rows, int32_t n_kv_seg, int32_t n_head,
                                            size_t* bytes) {
    FGR_REQUIRE(bytes && n_kv_rows >= 0 && n_kv_seg >= 0 && n_head > 0,
                "fgr_attention_bf16_workspace: bad arguments");
    *bytes = (size_t)(n_tiles_bf(n_kv_rows, n_kv_seg) * n_head * bf_units<64>() * 16);
    return FGR_OK;
}

extern "C" int fgr_attention_bf16(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                  const float* v, int64_t ld_v, float* o, int64_t ld_o,
                                  const int64_t* q_off, const int64_t* kv_off,
                                  const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg,
                                  int64_t n_kv_rows, int32_t max_q_len, int32_t max_kv_len,
                                  int32_t n_head, int32_t head_dim, float scale, void* workspace,
                                  int64_t ws_bytes, void* stream) {
    FGR_REQUIRE(q && k && v && o && q_off && kv_off && kv_seg && workspace && n_seg > 0 &&
                    n_kv_seg > 0 && n_head > 0 && max_q_len >= 0 && max_kv_len >= 0,
                "fgr_attention_bf16: bad arguments");
    FGR_REQUIRE(head_dim == 32 || head_dim == 64, "fgr_attention_bf16: head_dim %d (32 or 64)",
                head_dim);
    const int dh = head_dim;
    FGR_REQUIRE(ld_q >= n_head * dh && ld_k >= n_head * dh && ld_v >= n_head * dh &&
                    ld_o >= n_head * dh && ld_q % 4 == 0 && ld_k % 4 == 0 && ld_v % 4 == 0 &&
                    ld_o % 4 == 0,
                "fgr_attention_bf16: row strides must be >= n_head*head_dim and multiples of 4");
    FGR_REQUIRE(((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
                  reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o) |
                  reinterpret_cast<uintptr_t>(workspace)) & 15) == 0,
                "fgr_attention_bf16: q/k/v/o/workspace must be 16-B aligned");
    const int un = dh == 32 ? bf_units<32>() : bf_units<64>();
    const int64_t need = n_tiles_bf(n_kv_rows, n_kv_seg) * n_head * un * 16;
    FGR_REQUIRE(ws_bytes >= need, "fgr_attention_bf16: workspace %lld < %lld bytes",
                (long long)ws_bytes, (long long)need);
    if (max_q_len == 0 || max_kv_len == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    uint4* img = static_cast<uint4*>(workspace);
    const dim3 kgrid((unsigned)ceil_div(max_kv_len, 64), (unsigned)n_head, (unsigned)n_kv_seg);
    const int n_qblk = (int)ceil_div(max_q_len, 64);
    const unsigned nb = (unsigned)(ceil_div((int64_t)n_seg * n_head, 8) * 8 * n_qblk);
    const float sl2 = scale * 1.4426950408889634f;
    if (dh == 32) {
        hipLaunchKernelGGL(attn_kv_image_bf16_kernel<32>, kgrid, dim3(256), 0, st, k, ld_k, v, ld_v,
                           kv_off, n_head, img);
        FGR_CHECK_LAUNCH("attn_kv_image_bf16_kernel");
        hipLaunchKernelGGL(attn_bf16_v2_kernel<32>, dim3(nb), dim3(256), 0, st, q, ld_q,
                               (const uint4*)img, o, ld_o, q_off, kv_off, kv_seg, n_head, n_seg, n_qblk, sl2, 0);
    } else {
        hipLaunchKernelGGL(attn_kv_image_bf16_kernel<64>, kgrid, dim3(256), 0, st, k, ld_k, v, ld_v,
                           kv_off, n_head, img);
        FGR_CHECK_LAUNCH("attn_kv_image_bf16_kernel");
        hipLaunchKernelGGL(attn_bf16_v2_kernel<64>, dim3(nb), dim3(256), 0, st, q, ld_q,
                               (const uint4*)img, o, ld_o, q_off, kv_off, kv_seg, n_head, n_seg, n_qblk, sl2, 0);
    }
    FGR_CHECK_LAUNCH("attn_bf16_v2_kernel");
    return FGR_OK;
}

// ---- the in_proj with the bf16 K / V attention images in its epilogue (head dim 64) ---------
extern "C" int fgr_kv_image_bf16_bytes(int64_t n_rows, int32_t n_head, int32_t head_dim, size_t* bytes) {
    FGR_REQUIRE(bytes && n_rows >= 0 && n_head > 0 && head_dim == 64,
                "fgr_kv_image_bf16_bytes: bad arguments (head_dim 64)");
    *bytes = (size_t)std::max<int64_t>(1, ceil_div(n_rows, 64)) * n_head * bf_units<64>() * 16;
    return FGR_OK;
}

extern "C" int fgr_gemm_bf16_qkv_supported(int32_t m, int32_t d, int32_t n_head) {
    return (m > 0 && n_head > 0 && d == 64 * n_head && d % 128 == 0) ? 1 : 0;
}

// q = (a W^T + bias)[:, :d] fp32; k / v columns as bf16 images of every GLOBAL 64-row tile and
// head (the register-staged 64 x 128 bf16 kernel's epilogue)
extern "C" int fgr_gemm_bf16_qkv(const float* a, int64_t lda, const void* w_img, float* q,
                                 int64_t ld_q, const float* bias, int32_t m, int32_t d,
                                 int32_t n_head, void* kv_img, void* stream) {
    FGR_REQUIRE(a && w_img && q && bias && kv_img && m >= 0 && lda >= d && ld_q >= d,
                "fgr_gemm_bf16_qkv: bad arguments");
    FGR_REQUIRE(m == 0 || fgr_gemm_bf16_qkv_supported(m, d, n_head),
                "fgr_gemm_bf16_qkv: d %d heads %d not supported (head dim 64, d %% 128 == 0)", d, n_head);
    const uintptr_t al = reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(w_img) |
                         reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(bias) |
                         reinterpret_cast<uintptr_t>(kv_img);
    FGR_REQUIRE((al & 15) == 0 && lda % 4 == 0 && ld_q % 4 == 0 && d % 8 == 0,
                "fgr_gemm_bf16_qkv: operands must be 16-B aligned with row strides %% 4 == 0");
    if (m == 0) return FGR_OK;
    const int n = 3 * d;
    GemmBfArgs g{a, lda, (const u32x4*)w_img, ksteps_bf(d), q, ld_q, bias, nullptr, 0, m, n, d,
                 FGR_ACT_NONE, 1, static_cast<char*>(kv_img), n_head, d};
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const unsigned nblk = (unsigned)(ceil_div(m, 64) * ceil_div(n, 128));
    hipLaunchKernelGGL((gemm_bf16_kernel<64, 128, true>), dim3(nblk), dim3(256), 0, st, g);
    FGR_CHECK_LAUNCH("gemm_bf16_kernel (qkv images)");
    return FGR_OK;
}

// the bf16 attention on those images (no image launch)
extern "C" int fgr_attention_bf16_img(const float* q, int64_t ld_q, const void* kv_img,
                                      int64_t n_kv_rows, float* o, int64_t ld_o,
                                      const int64_t* q_off, const int64_t* kv_off,
                                      const int32_t* kv_seg, int32_t n_seg, int32_t max_q_len,
                                      int32_t n_head, int32_t head_dim, float scale, void* stream) {
    FGR_REQUIRE(q && kv_img && o && q_off && kv_off && kv_seg && n_seg > 0 && n_head > 0 &&
                    max_q_len >= 0 && n_kv_rows >= 0 && head_dim == 64,
                "fgr_attention_bf16_img: bad arguments (head_dim 64)");
    FGR_REQUIRE(ld_q >= n_head * 64 && ld_o >= n_head * 64 && ld_q % 4 == 0 && ld_o % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(o) |
                      reinterpret_cast<uintptr_t>(kv_img)) & 15) == 0,
                "fgr_attention_bf16_img: strides / alignment");
    if (max_q_len == 0 || n_kv_rows == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const int n_qblk = (int)ceil_div(max_q_len, 64);
    const unsigned nb = (unsigned)(ceil_div((int64_t)n_seg * n_head, 8) * 8 * n_qblk);
    const float sl2 = scale * 1.4426950408889634f;
    hipLaunchKernelGGL(attn_bf16_v2_kernel<64>, dim3(nb), dim3(256), 0, st, q, ld_q,
                       static_cast<const uint4*>(kv_img), o, ld_o, q_off, kv_off, kv_seg, n_head,
                       n_seg, n_qblk, sl2, 1);
    FGR_CHECK_LAUNCH("attn_bf16_v2_kernel (global tiles)");
    return FGR_OK;
}
