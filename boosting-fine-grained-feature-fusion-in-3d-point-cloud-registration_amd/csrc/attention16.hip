// fp32-accurate attention (head_dim 32 or 64) on the fp16 matrix cores with scaled two-term splits
// ("f16x3") -- the same contract as fgr_attention_bf16x6, at half its matrix-core work.
//
// Replaces the core of nn.MultiheadAttention in the reference's cross encoder
// (transformers.py:95-96, 197-226): o = softmax((q * scale) k^T + key padding mask) v, with
// the mask expressed as the end of each packed key segment.
//
// Precision: every operand is brought into fp16's normal range by an exact power of two and
// split into two fp16 terms, x = h + m (2^-22 relative); per 16x16x32 step the three
// significant products hh, hm, mh accumulate in fp32 (dropped mm <= 2^-22):
//   * K and V: one scale per (64-key tile, head), max |x| of the tile in [2^14, 2^15)
//     (attn_kv_image16_kernel, which also writes the split images);
//   * Q: one scale per query (lane-local), max |q * scale * log2 e| in [2^14, 2^15);
//   * P = exp2(s - m) in [0, 1]: fixed scale 2^14.
// The S^T tile is unscaled inside the softmax FMA (s * f - m, f = 2^-(e_k + e_q) per lane);
// the PV partial of a tile goes to its own accumulator and is added as acc * alpha +
// tmp * 2^-(e_v + 14). Net per-product error <= ~3 * 2^-22 (fp32's own rounding 2^-24).
//
// Layout and data flow follow attn_bf16x6_kernel (attention.hip): swapped products
//   S^T[key][query] = K Q^T     A = K (LDS image), B = Q (registers, split once)
//   O^T[dh][query] += V^T P^T   A = V (LDS, ds_read_b64_tr_b16), B = P (registers)
// so every softmax row is lane-local; 16x16x32 f16 lane maps (lane l, g = l >> 4,
// c = l & 15): A[i = c][k = 8g + e], B[k = 8g + e][j = c], C[i = 4g + r][j = c].
// Per-(tile, head) image, 256 * DH B (16 KB at DH 32, 32 KB at DH 64), staged into LDS by a
// flat copy:
//   K: [k-step DH/32][term 2][g 4][key 64] x 16 B (8 dims)   ds_read_b128, conflict-free
//   V: [term 2][key 64][DH] f16, 16-B chunk index XOR v_swz<DH>(key)
// Tile t of kv segment s sits at tile index kv_off[s] / 64 + s + t; the (e_k, e_v) scale
// exponents of all tiles follow the images.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// 16-B units per (tile, head) image and the first V unit, by head dim
template <int DH> constexpr int units() { return DH * 16 + (DH / 32) * 512; }
template <int DH> constexpr int unit_v() { return (DH / 32) * 512; }

__device__ __forceinline__ float xg_max16(float v) {   // max over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float xg_sum16(float v) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// power-of-two exponent e with max * 2^e in [2^14, 2^15) (0 for an all-zero block)
__device__ __forceinline__ int range_exp(float mx) {
    return mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
}

__device__ __forceinline__ void split2(float x, _Float16& h, _Float16& m) {
    h = (_Float16)x;
    m = (_Float16)(x - (float)h);
}

// V image row swizzle: XOR applied to the 16-B chunk index of key row `key`, so that the
// ds_read_b64_tr_b16 of a 32-lane group (8 key rows x 32 B) hits 64 distinct banks. DH 32
// (64-B rows, 4 per 256-B bank period): rows r, r + 4 separated by 32 B (row bit 2); DH 64
// (128-B rows, 2 per period): rows r, r + 2, r + 4, r + 6 share banks and take four distinct
// 32-B chunk pairs (row bits 1-2) -- without it they read 2-way conflicted (round-3 PMC:
// 1.2 M conflict cycles per 0.9 M LDS instructions at DH 64, none at DH 32).
template <int DH>
__device__ __forceinline__ int v_swz(int key) {
    if constexpr (DH == 64) return ((key >> 1) & 3) << 1;
    else return ((key >> 2) & 1) << 1;
}

template <int DH>
__device__ __forceinline__ void kv_image16(const float* __restrict__ k, int64_t ld_k,
                                           const float* __restrict__ v, int64_t ld_v,
                                           const int64_t* __restrict__ kv_off, int n_head,
                                           uint4* __restrict__ img, int2* __restrict__ sc, int s,
                                           int h, int tt, bool v_part = true) {
    constexpr int NF = DH / 16;                                  // float4s per thread
    constexpr int RU = DH / 4;                                   // float4s per key row
    const int64_t kb = kv_off[s];
    const int nk = (int)(kv_off[s + 1] - kb);
    if (tt * 64 >= nk) return;                                   // block-uniform
    __shared__ float red[2][4];
    const int64_t tile = (kb / 64 + s + tt) * n_head + h;
    char* base = reinterpret_cast<char*>(img + tile * units<DH>());
    float kf[NF][4], vf[NF][4];
    float km = 0.f, vm = 0.f;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int e = threadIdx.x + 256 * i;                     // float4 of the 64 x DH tile
        const int key = e / RU, d0 = (e % RU) * 4;
        const bool ok = tt * 64 + key < nk;
        const int64_t row = kb + tt * 64 + key;
        const float4 kx = ok ? *reinterpret_cast<const float4*>(k + row * ld_k + h * DH + d0)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        // v == k (the backward's one-matrix images): one read
        const float4 vx = v == k ? kx
                          : ok   ? *reinterpret_cast<const float4*>(v + row * ld_v + h * DH + d0)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        kf[i][0] = kx.x; kf[i][1] = kx.y; kf[i][2] = kx.z; kf[i][3] = kx.w;
        vf[i][0] = vx.x; vf[i][1] = vx.y; vf[i][2] = vx.z; vf[i][3] = vx.w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            km = fmaxf(km, fabsf(kf[i][j]));
            vm = fmaxf(vm, fabsf(vf[i][j]));
        }
    }
    km = wave_max(km);
    vm = wave_max(vm);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wv] = km; red[1][wv] = vm; }
    __syncthreads();
    km = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    vm = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
    const int ek = range_exp(km), ev = range_exp(vm);
    if (threadIdx.x == 0) sc[tile] = make_int2(ek, ev);
    const float sk = __builtin_ldexpf(1.f, ek), sv = __builtin_ldexpf(1.f, ev);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int e = threadIdx.x + 256 * i;
        const int key = e / RU, d0 = (e % RU) * 4;
        _Float16 kt[2][4], vt[2][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            split2(kf[i][j] * sk, kt[0][j], kt[1][j]);
            split2(vf[i][j] * sv, vt[0][j], vt[1][j]);
        }
        const int ks = d0 >> 5, g = (d0 & 31) >> 3, half = (d0 >> 2) & 1;
        const int vch = (d0 >> 3) ^ v_swz<DH>(key);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            *reinterpret_cast<uint2*>(base + (((ks * 2 + t) * 4 + g) * 64 + key) * 16 + half * 8) =
                *reinterpret_cast<const uint2*>(kt[t]);
            if (v_part)
                *reinterpret_cast<uint2*>(base + unit_v<DH>() * 16 + t * (128 * DH) + key * (2 * DH) +
                                          vch * 16 + half * 8) =
                    *reinterpret_cast<const uint2*>(vt[t]);
        }
    }
}

template <int DH>
__global__ void __launch_bounds__(256)
attn_kv_image16_kernel(const float* __restrict__ k, int64_t ld_k, const float* __restrict__ v,
                       int64_t ld_v, const int64_t* __restrict__ kv_off, int n_head,
                       uint4* __restrict__ img, int2* __restrict__ sc) {
    kv_image16<DH>(k, ld_k, v, ld_v, kv_off, n_head, img, sc, blockIdx.z, blockIdx.y, blockIdx.x);
}

// the training backward's images of one matrix each (k = v = src: both parts), up to four
// matrices in one launch: blockIdx.z = job * max_seg + segment
struct ImgJobs {
    const float* src[4];
    int64_t ld[4];
    const int64_t* off[4];
    uint4* img[4];
    int2* sc[4];
    int n_seg[4];
    int v_part[4];                   // 0: only the K part is read (the dQ kernel's V image)
    int max_seg;
};

template <int DH>
__global__ void __launch_bounds__(256) attn_image16_jobs_kernel(ImgJobs j) {
    const int job = blockIdx.z / j.max_seg, s = blockIdx.z % j.max_seg;
    if (s >= j.n_seg[job]) return;
    kv_image16<DH>(j.src[job], j.ld[job], j.src[job], j.ld[job], j.off[job], (int)gridDim.y,
                   j.img[job], j.sc[job], s, blockIdx.y, blockIdx.x, j.v_part[job] != 0);
}

template <int N>
__device__ __forceinline__ void wait_vm_lgkm0_a() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}

// ---- key-tile loop: the K/V tile images go global -> LDS by LDS-DMA into two buffers (tile
// t + 1 in flight while tile t is computed; one barrier per tile, no staging registers, no
// ds_write pass); the per-tile scale exponents come by scalar loads (block-uniform address).
// Vector work per key tile is kept minimal (round 3; PMC in profiles/r03_pmc_attn_*.json):
// the round-2 loop issued ~8.6 VALU
// per MFMA at head dim 32 (154 VALU + 17 v_exp + 24 MFMA per wave and 64-key tile, 17 of the
// VALU packed fp32 ops); this loop issues ~100 VALU + 17 v_exp per tile (6.7 VALU per MFMA
// over the whole kernel), 50.6 -> 46.3 us on the ModelNet self-attention shape:
//   * the P scale 2^14 folded into the exponent (p14 = exp2(s f - (m - 14))): no multiply;
//   * P split with packed conversions: hi = v_cvt_pk_f16_f32 (2 per instruction), lo = one
//     v_fma_mix per element reading hi's half by op_sel (24 instructions per 16 values);
//   * row maxima by v_max3_f32 without NaN canonicalisation (scores are finite or -inf);
//   * the tile loop unrolled by two, so both LDS buffers' addresses are per-lane constants +
//     instruction offsets (no per-tile address arithmetic), K/V DMA pieces contiguous per
//     wave (one 64-bit add per tile, the pieces by instruction offsets);
//   * built with -fno-slp-vectorize (packed fp32 VALU costs ~22 extra cycles beside MFMAs).
// maxima of MFMA results: plain fmaxf (the file is built -fno-honor-nans, so no NaN
// canonicalisation of the inputs; inline asm cannot be used here: the compiler's hazard
// recognizer does not see an asm block's reads of MFMA results)
__device__ __forceinline__ float vmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
__device__ __forceinline__ float vmax2(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ float xg_max16_nc(float v) {   // max over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = vmax2(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return vmax2(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// x[0..7] (in fp16 range) -> h = f16(x) packed by v_cvt_pk_f16_f32 (RNE, the bits of split2's
// hi), l = f16(x - h) by v_fma_mix (x - h exact in fp32, one rounding). Ends with `s_nop 1`:
// the terms feed MFMAs (cdna_hip_programming.md 5.7 item 2).
__device__ __forceinline__ void split8_pk(const float (&x)[8], float one, u32x4& h, u32x4& l) {
    unsigned h0, h1, h2, h3, l0, l1, l2, l3;
    asm("v_cvt_pk_f16_f32 %0, %8, %9\n\t"
        "v_cvt_pk_f16_f32 %1, %10, %11\n\t"
        "v_cvt_pk_f16_f32 %2, %12, %13\n\t"
        "v_cvt_pk_f16_f32 %3, %14, %15\n\t"
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
          "v"(one));
    h = u32x4{h0, h1, h2, h3};
    l = u32x4{l0, l1, l2, l3};
}

// DROP (training only, fgr_attention_f16x3_drop): the softmax weights of the PV product are
// masked by attn_drop_hash (common.h) -- the row sum l keeps every weight, and the kept ones
// are scaled by 1 / (1 - p) with the final 1 / l (P stays <= 2^14 in fp16's range)
template <int DH, bool DROP = false>
__global__ void __launch_bounds__(256, DH == 64 ? 2 : 5)
attn_f16x3_v2_kernel(const float* __restrict__ q, int64_t ld_q, const uint4* __restrict__ img,
                     const int2* __restrict__ sc, float* __restrict__ o, int64_t ld_o,
                     const int64_t* __restrict__ q_off, const int64_t* __restrict__ kv_off,
                     const int32_t* __restrict__ kv_seg, int n_head, int n_seg, int n_qblk,
                     float scale_log2, int global_tiles, uint32_t drop_seed = 0,
                     uint32_t drop_thresh = 0, float inv_keep = 1.f, float* __restrict__ lse_out = nullptr) {
    constexpr int KD = DH / 32, TD = DH / 16;
    constexpr int UN = units<DH>();
    constexpr int PW = UN / 64 / 4;                              // DMA pieces per wave per tile
    // the two K/V tile buffers as two LDS objects, addressed by pointers derived from them:
    // the compiler's LDS-DMA tracking then knows that the DMA filling one buffer cannot alias
    // reads of the other (one array + integer addresses made it wait for the in-flight DMA of
    // the next tile -- vmcnt(0) -- before the first V read of every tile)
    __shared__ u32x4 lds_b0[UN], lds_b1[UN];
    typedef __attribute__((address_space(3))) char lds_c;
    const int L = blockIdx.x, xcd = L & 7, j0 = L >> 3;
    const int pair = (j0 / n_qblk) * 8 + xcd, qblk = j0 % n_qblk;
    if (pair >= n_seg * n_head) return;
    const int seg = pair / n_head, head = pair % n_head;
    const int64_t qb = q_off[seg], qe = q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)qblk * 64;
    if (q0 >= qe) return;                                        // block-uniform
    const int ks = kv_seg[seg];
    const int64_t kb = kv_off[ks];
    const int nk = (int)(kv_off[ks + 1] - kb);
    // per-segment images (attn_kv_image16_kernel: tile t of segment ks at kb / 64 + ks + t) or
    // images of GLOBAL 64-row tiles (written by the in_proj GEMM, fgr_gemm_f16x3_ln_qkv): the
    // segment's keys then start `lead` rows into its first tile
    const int lead = global_tiles ? (int)(kb & 63) : 0;
    const int ntile = (lead + nk + 63) / 64;
    const int64_t tile0 = (global_tiles ? kb / 64 : kb / 64 + ks) * n_head + head;
    const int64_t tile_stride = (int64_t)n_head * UN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    // this lane's DMA source within a tile: pieces wv * PW .. + PW - 1 (1 KiB each, contiguous)
    const u32x4* src_lane = reinterpret_cast<const u32x4*>(img) + tile0 * UN + wv * PW * 64 + lane;

    const int64_t qrow = q0 + wv * 16 + c;
    float x[KD][8];
#pragma unroll
    for (int kd = 0; kd < KD; ++kd) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if (qrow < qe) {
            const float4* p = reinterpret_cast<const float4*>(q + qrow * ld_q + head * DH + 32 * kd + 8 * g);
            a = p[0];
            b = p[1];
        }
        x[kd][0] = a.x; x[kd][1] = a.y; x[kd][2] = a.z; x[kd][3] = a.w;
        x[kd][4] = b.x; x[kd][5] = b.y; x[kd][6] = b.z; x[kd][7] = b.w;
    }
    float qm = 0.f;
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            x[kd][e] *= scale_log2;
            qm = fmaxf(qm, fabsf(x[kd][e]));
        }
    const int eq = range_exp(xg_max16(qm));
    const float sq = __builtin_ldexpf(1.f, eq);
    f16x8 qt[KD][2];
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            _Float16 h, m;
            split2(x[kd][e] * sq, h, m);
            qt[kd][0][e] = h; qt[kd][1][e] = m;
        }
    f32x4 acc[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    const float one = 1.0f;

    // per-lane LDS byte addresses (buffer 0); everything else is an instruction offset
    const uint32_t kaddr = (uint32_t)(g * 64 + c) * 16;            // K fragment reads (bytes)
    // V transposed reads: lane c = 4qq + p reads rows 4g + qq (+16 k, +32 j), columns
    // 16t + 4p .. +3: chunk 2t + (p >> 1) XOR the image's row swizzle (v_swz)
    const int qq = c >> 2, pp = c & 3;
    uint32_t vaddr[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t)
        vaddr[t] = unit_v<DH>() * 16 + (4 * g + qq) * (2 * DH) +
                   (((2 * t + (pp >> 1)) ^ v_swz<DH>(4 * g + qq)) * 16) + (pp & 1) * 8;

    auto dma = [&](int t, auto buf_tag) {                        // tile t -> buffer BUF
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
    // tile tt lives in LDS buffer (tt + shift) & 1: a masked first tile (lead > 0) takes buffer 1
    // so that the unrolled pairs of full tiles always start on buffer 0
    const int shift = lead > 0 ? 1 : 0;
    if (ntile > 0) {
        if (shift) dma(0, std::integral_constant<int, 1>{});
        else dma(0, std::integral_constant<int, 0>{});
    }

    auto tile = [&](int tt, auto buf_tag, auto mask_tag) {
        constexpr int BUF = decltype(buf_tag)::value;
        constexpr bool MASK = decltype(mask_tag)::value;
        wait_vm_lgkm0_a<0>();           // this wave's pieces of tile tt landed
        __builtin_amdgcn_s_barrier();   // everyone's landed; buffer 1 - BUF no longer read
        if (tt + 1 < ntile) dma(tt + 1, std::integral_constant<int, 1 - BUF>{});
        const int2 e2 = sc[tile0 + (int64_t)__builtin_amdgcn_readfirstlane(tt) * n_head];
        lds_c* const bp = (lds_c*)(BUF == 0 ? lds_b0 : lds_b1);
        typedef __attribute__((address_space(3))) u32x4 lds_u4;
        typedef __attribute__((address_space(3))) s16x4 lds_s4;

        f32x4 s[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kd = 0; kd < KD; ++kd) {
                const f16x8 kh = __builtin_bit_cast(
                    f16x8, *(lds_u4*)(bp + kaddr + (((kd * 2 + 0) * 4) * 64 + 16 * n) * 16));
                const f16x8 kl = __builtin_bit_cast(
                    f16x8, *(lds_u4*)(bp + kaddr + (((kd * 2 + 1) * 4) * 64 + 16 * n) * 16));
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kl, qt[kd][0], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qt[kd][1], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qt[kd][0], a, 0, 0, 0);
            }
            s[n] = a;
        }
        const float f = __builtin_ldexpf(1.f, -(e2.x + eq));
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
        float mx = vmax3(s[0][0], s[0][1], s[0][2]);
        mx = vmax3(mx, s[0][3], s[1][0]);
        mx = vmax3(mx, s[1][1], s[1][2]);
        mx = vmax3(mx, s[1][3], s[2][0]);
        mx = vmax3(mx, s[2][1], s[2][2]);
        mx = vmax3(mx, s[2][3], s[3][0]);
        mx = vmax3(mx, s[3][1], s[3][2]);
        mx = vmax2(mx, s[3][3]);
        mx = xg_max16_nc(mx) * f;
        const float m_new = vmax2(m_run, mx);           // finite: every tile has a valid key
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        const float m14 = m_new - 14.f;                 // p14 = 2^14 p, in fp16's range
        float rs = 0.f;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[n][r], f, -m14));
                s[n][r] = p;
                rs += p;
                if constexpr (DROP) {
                    // packed key row of this entry (tile-local key 16n + 4g + r)
                    const int64_t key = kb - lead + (int64_t)tt * 64 + 16 * n + 4 * g + r;
                    if (attn_drop_hash(drop_seed, head, qrow, key) < drop_thresh) s[n][r] = 0.f;
                }
            }
        l_run = l_run * alpha + rs;

        f32x4 tmp[TD];
#pragma unroll
        for (int t = 0; t < TD; ++t) tmp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // P^T operand of step j (keys 32j + 4g + {0..3}, 32j + 16 + 4g + {0..3})
            const float pv[8] = {s[2 * j][0], s[2 * j][1], s[2 * j][2], s[2 * j][3],
                                 s[2 * j + 1][0], s[2 * j + 1][1], s[2 * j + 1][2], s[2 * j + 1][3]};
            u32x4 ph, pl;
            split8_pk(pv, one, ph, pl);
            const f16x8 pt0 = __builtin_bit_cast(f16x8, ph), pt1 = __builtin_bit_cast(f16x8, pl);
#pragma unroll
            for (int t = 0; t < TD; ++t) {
                f16x8 vf[2];
#pragma unroll
                for (int tm = 0; tm < 2; ++tm) {
                    lds_c* const vb = bp + vaddr[t] + tm * (128 * DH) + j * 32 * (2 * DH);
                    const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)vb);
                    const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vb + 16 * (2 * DH)));
                    vf[tm] = __builtin_bit_cast(f16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
                }
                f32x4 a = tmp[t];
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf[1], pt0, a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf[0], pt1, a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf[0], pt0, a, 0, 0, 0);
                tmp[t] = a;
            }
        }
        const float fv = __builtin_ldexpf(1.f, -e2.y);   // p14's 2^14 cancels against l's
#pragma unroll
        for (int t = 0; t < TD; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[t][r] = __builtin_fmaf(tmp[t][r], fv, acc[t][r] * alpha);
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

    // O^T (dh 16t + 4g + r, query c) / l (both in 2^14 units)
    const float lsum = xg_sum16(l_run);
    const float inv = (DROP ? inv_keep : 1.0f) / lsum;
    // training: the row's log2-sum-exp of the scaled scores (l in 2^14 units) for the
    // backward, which then skips its own first pass (fgr_attention_bwd_train)
    if (lse_out && qrow < qe && g == 0)
        lse_out[qrow * n_head + head] = m_run + __builtin_amdgcn_logf(lsum) - 14.f;
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

int64_t n_tiles16(int64_t n_kv_rows, int32_t n_kv_seg) { return n_kv_rows / 64 + n_kv_seg + 1; }

// ---- training: dQ of the attention on the f16 matrix cores (f16x3), given the forward's
// log2-sum-exp (fgr_attention_bwd_train). The forward kernel's structure with three images per
// 64-key tile, built by attn_kv_image16_kernel (per-segment tiles):
//   imgK = (K as the K operand, K as the V operand), imgV = (V as the K operand, unused):
//   S^T[key][query]  = K Q^T        A = K (imgK, K part), B = Q (registers, split once)
//   dP^T[key][query] = V dO^T       A = V (imgV, K part), B = dO (registers, split once)
//   P = exp2(S - lse2) (no running max: the forward's lse), dS = P (dP - D), D = dO . O;
//   dQ^T[dh][query] += K^T dS^T     A = K (imgK, V part: transposed reads), B = dS (registers,
//                                   per query and tile scaled into fp16's range and split)
// dQ = scale * sum dS K. Same lane maps, DMA double buffer and barriers as the forward.
template <int DH, bool DROP>
__global__ void __launch_bounds__(256, DH == 64 ? 2 : 4)
attn_bwd_dq_f16x3_kernel(const float* __restrict__ q, int64_t ld_q, const float* __restrict__ dout,
                         int64_t ld_do, const float* __restrict__ o, int64_t ld_o,
                         const uint4* __restrict__ imgk, const int2* __restrict__ sck,
                         const uint4* __restrict__ imgv, const int2* __restrict__ scv,
                         float* __restrict__ dq, int64_t ld_dq, const int64_t* __restrict__ q_off,
                         const int64_t* __restrict__ kv_off, const int32_t* __restrict__ kv_seg,
                         int n_head, int n_seg, int n_qblk, float scale, float scale_log2,
                         const float* __restrict__ lse_in, float* __restrict__ lse_out,
                         float* __restrict__ dsum_out, float* __restrict__ lsed_t,
                         uint32_t drop_seed, uint32_t drop_thresh, float inv_keep) {
    constexpr int KD = DH / 32, TD = DH / 16;
    constexpr int UN = units<DH>();                              // imgK units per tile
    constexpr int UK = unit_v<DH>();                             // the K part (imgV)
    constexpr int PW = UN / 64 / 4, PWV = UK / 64 / 4;           // DMA pieces per wave per tile
    __shared__ u32x4 lk0[UN], lk1[UN], lv0[UK], lv1[UK];
    typedef __attribute__((address_space(3))) char lds_c;
    const int L = blockIdx.x, xcd = L & 7, j0 = L >> 3;
    const int pair = (j0 / n_qblk) * 8 + xcd, qblk = j0 % n_qblk;
    if (pair >= n_seg * n_head) return;
    const int seg = pair / n_head, head = pair % n_head;
    const int64_t qb = q_off[seg], qe = q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)qblk * 64;
    if (q0 >= qe) return;                                        // block-uniform
    const int ks = kv_seg[seg];
    const int64_t kb = kv_off[ks];
    const int nk = (int)(kv_off[ks + 1] - kb);
    const int ntile = (nk + 63) / 64;
    const int64_t tile0 = (kb / 64 + ks) * n_head + head;
    const int64_t tile_stride_k = (int64_t)n_head * UN, tile_stride_v = (int64_t)n_head * UN;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const u32x4* srck = reinterpret_cast<const u32x4*>(imgk) + tile0 * UN + wv * PW * 64 + lane;
    const u32x4* srcv = reinterpret_cast<const u32x4*>(imgv) + tile0 * UN + wv * PWV * 64 + lane;

    // this lane's query row: q (scaled into the log2 domain), dO, and D = dO . O
    const int64_t qrow = q0 + wv * 16 + c;
    const bool qok = qrow < qe;
    float x[KD][8], y[KD][8];
    float dpart = 0.f;
#pragma unroll
    for (int kd = 0; kd < KD; ++kd) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, da = a, db = a, oa = a, ob = a;
        if (qok) {
            const int64_t col = head * DH + 32 * kd + 8 * g;
            const float4* pq = reinterpret_cast<const float4*>(q + qrow * ld_q + col);
            const float4* pd = reinterpret_cast<const float4*>(dout + qrow * ld_do + col);
            const float4* po = reinterpret_cast<const float4*>(o + qrow * ld_o + col);
            a = pq[0]; b = pq[1]; da = pd[0]; db = pd[1]; oa = po[0]; ob = po[1];
        }
        x[kd][0] = a.x; x[kd][1] = a.y; x[kd][2] = a.z; x[kd][3] = a.w;
        x[kd][4] = b.x; x[kd][5] = b.y; x[kd][6] = b.z; x[kd][7] = b.w;
        y[kd][0] = da.x; y[kd][1] = da.y; y[kd][2] = da.z; y[kd][3] = da.w;
        y[kd][4] = db.x; y[kd][5] = db.y; y[kd][6] = db.z; y[kd][7] = db.w;
        dpart += ((da.x * oa.x + da.y * oa.y) + (da.z * oa.z + da.w * oa.w)) +
                 ((db.x * ob.x + db.y * ob.y) + (db.z * ob.z + db.w * ob.w));
    }
    const float D = xg_sum16(dpart);
    const float lse2 = qok ? lse_in[qrow * n_head + head] : 0.f;
    float qm = 0.f, dm = 0.f;
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            x[kd][e] *= scale_log2;
            qm = fmaxf(qm, fabsf(x[kd][e]));
            dm = fmaxf(dm, fabsf(y[kd][e]));
        }
    const int eq = range_exp(xg_max16(qm)), edo = range_exp(xg_max16(dm));
    const float sq = __builtin_ldexpf(1.f, eq), sdo = __builtin_ldexpf(1.f, edo);
    f16x8 qt[KD][2], dt[KD][2];
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            _Float16 h, m;
            split2(x[kd][e] * sq, h, m);
            qt[kd][0][e] = h; qt[kd][1][e] = m;
            split2(y[kd][e] * sdo, h, m);
            dt[kd][0][e] = h; dt[kd][1][e] = m;
        }
    f32x4 acc[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float one = 1.0f;
    const uint32_t kaddr = (uint32_t)(g * 64 + c) * 16;
    const int qq = c >> 2, pp = c & 3;
    uint32_t vaddr[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t)
        vaddr[t] = unit_v<DH>() * 16 + (4 * g + qq) * (2 * DH) +
                   (((2 * t + (pp >> 1)) ^ v_swz<DH>(4 * g + qq)) * 16) + (pp & 1) * 8;

    auto dma = [&](int t, auto buf_tag) {
        constexpr int BUF = decltype(buf_tag)::value;
        const u32x4* sk = srck + (int64_t)t * tile_stride_k;
        const u32x4* sv = srcv + (int64_t)t * tile_stride_v;
        lds_c* dk = (lds_c*)(BUF == 0 ? lk0 : lk1) + wv * PW * 1024;
        lds_c* dv = (lds_c*)(BUF == 0 ? lv0 : lv1) + wv * PWV * 1024;
#pragma unroll
        for (int j = 0; j < PW; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(sk + j * 64),
                                             (__attribute__((address_space(3))) void*)(dk + j * 1024), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < PWV; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(sv + j * 64),
                                             (__attribute__((address_space(3))) void*)(dv + j * 1024), 16, 0, 0);
    };
    if (ntile > 0) dma(0, std::integral_constant<int, 0>{});

    auto tile = [&](int tt, auto buf_tag) {
        constexpr int BUF = decltype(buf_tag)::value;
        wait_vm_lgkm0_a<0>();
        __builtin_amdgcn_s_barrier();
        if (tt + 1 < ntile) dma(tt + 1, std::integral_constant<int, 1 - BUF>{});
        const int2 ek2 = sck[tile0 + (int64_t)__builtin_amdgcn_readfirstlane(tt) * n_head];
        const int2 ev2 = scv[tile0 + (int64_t)__builtin_amdgcn_readfirstlane(tt) * n_head];
        lds_c* const bk = (lds_c*)(BUF == 0 ? lk0 : lk1);
        lds_c* const bv = (lds_c*)(BUF == 0 ? lv0 : lv1);
        typedef __attribute__((address_space(3))) u32x4 lds_u4;
        typedef __attribute__((address_space(3))) s16x4 lds_s4;
        f32x4 sc4[4], dp4[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
#pragma unroll
            for (int kd = 0; kd < KD; ++kd) {
                const int ko = (((kd * 2 + 0) * 4) * 64 + 16 * n) * 16, lo = (((kd * 2 + 1) * 4) * 64 + 16 * n) * 16;
                const f16x8 kh = __builtin_bit_cast(f16x8, *(lds_u4*)(bk + kaddr + ko));
                const f16x8 kl = __builtin_bit_cast(f16x8, *(lds_u4*)(bk + kaddr + lo));
                const f16x8 vh = __builtin_bit_cast(f16x8, *(lds_u4*)(bv + kaddr + ko));
                const f16x8 vl = __builtin_bit_cast(f16x8, *(lds_u4*)(bv + kaddr + lo));
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kl, qt[kd][0], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qt[kd][1], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qt[kd][0], a, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, dt[kd][0], b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, dt[kd][1], b, 0, 0, 0);
                b = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, dt[kd][0], b, 0, 0, 0);
            }
            sc4[n] = a;
            dp4[n] = b;
        }
        const float fs = __builtin_ldexpf(1.f, -(ek2.x + eq));
        const float fd = __builtin_ldexpf(1.f, -(ev2.x + edo));
        const int hi = nk - tt * 64;                             // valid keys [0, hi)
        float ds[16];
        float dmx = 0.f;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int kl = 16 * n + 4 * g + r;
                const float p = kl < hi ? __builtin_amdgcn_exp2f(__builtin_fmaf(sc4[n][r], fs, -lse2)) : 0.f;
                float dp = dp4[n][r] * fd;
                if constexpr (DROP) {
                    const int64_t key = kb + (int64_t)tt * 64 + kl;
                    dp = attn_drop_hash(drop_seed, head, qrow, key) < drop_thresh ? 0.f : dp * inv_keep;
                }
                const float v = p * (dp - D);
                ds[4 * n + r] = v;
                dmx = fmaxf(dmx, fabsf(v));
            }
        // per (query, tile) power of two bringing dS into fp16's range
        const int eds = range_exp(xg_max16(dmx));
        const float sds = __builtin_ldexpf(1.f, eds);
        f32x4 tmp[TD];
#pragma unroll
        for (int t = 0; t < TD; ++t) tmp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // dS^T operand of step j (keys 32j + 4g + {0..3}, 32j + 16 + 4g + {0..3})
            const float pv[8] = {ds[8 * j + 0] * sds, ds[8 * j + 1] * sds, ds[8 * j + 2] * sds, ds[8 * j + 3] * sds,
                                 ds[8 * j + 4] * sds, ds[8 * j + 5] * sds, ds[8 * j + 6] * sds, ds[8 * j + 7] * sds};
            u32x4 ph, pl;
            split8_pk(pv, one, ph, pl);
            const f16x8 pt0 = __builtin_bit_cast(f16x8, ph), pt1 = __builtin_bit_cast(f16x8, pl);
#pragma unroll
            for (int t = 0; t < TD; ++t) {
                f16x8 vf[2];
#pragma unroll
                for (int tm = 0; tm < 2; ++tm) {
                    lds_c* const vb = bk + vaddr[t] + tm * (128 * DH) + j * 32 * (2 * DH);
                    const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)vb);
                    const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vb + 16 * (2 * DH)));
                    vf[tm] = __builtin_bit_cast(f16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
                }
                f32x4 a = tmp[t];
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf[1], pt0, a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf[0], pt1, a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf[0], pt0, a, 0, 0, 0);
                tmp[t] = a;
            }
        }
        const float fv = __builtin_ldexpf(1.f, -(ek2.y + eds));
#pragma unroll
        for (int t = 0; t < TD; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[t][r] = __builtin_fmaf(tmp[t][r], fv, acc[t][r]);
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    int tt = 0;
    for (; tt + 2 <= ntile; tt += 2) {
        tile(tt, B0{});
        tile(tt + 1, B1{});
    }
    if (tt < ntile) tile(tt, B0{});

    if (qok) {
#pragma unroll
        for (int t = 0; t < TD; ++t) {
            float4 w;
            w.x = acc[t][0] * scale; w.y = acc[t][1] * scale;
            w.z = acc[t][2] * scale; w.w = acc[t][3] * scale;
            *reinterpret_cast<float4*>(dq + qrow * ld_dq + head * DH + 16 * t + 4 * g) = w;
        }
        if (g == 0 && lse_out) {
            lse_out[qrow * n_head + head] = lse2;
            dsum_out[qrow * n_head + head] = D;
        }
    }
    // lse2 / D of the block's 64 query rows by query tile for attn_bwd_dkdv_f16x3_kernel (rows
    // past the segment: lse +inf, D 0, so their P and dS vanish there without a mask)
    if (lsed_t && g == 0) {
        float* t = lsed_t + ((qb / 64 + seg + qblk) * n_head + head) * 128 + wv * 16 + c;
        t[0] = qok ? lse2 : INFINITY;
        t[64] = qok ? D : 0.f;
    }
}

// ---- training: dK / dV of the attention on the f16 matrix cores (f16x3). One block per (key
// segment, 64-key block, head), 4 waves x 16 keys; over the 64-query tiles of every query
// segment attending the key segment, with per-query-tile images of Q and dO
// (attn_kv_image16_kernel: K part for the row products, V part for the transposed ones):
//   S[query][key]  = Q K^T       A = Q (imgQ, K part), B = K (registers, scaled into the log2
//                                domain and split once)
//   dP[query][key] = dO V^T      A = dO (imgD, K part), B = V (registers)
//   P = exp2(S - lse2), dS = P (dP m - D)   (lse2 / D per query from the dQ kernel's tile array;
//                                m the dropout mask, 0 or 1 / (1 - p))
//   dV^T[dh][key] += dO^T (P k)  A = dO (imgD, V part, transposed reads), B = 2^14 P k, k the
//                                0 / 1 keep mask (1 / (1 - p) applied once at the end)
//   dK^T[dh][key] += Q^T dS      A = Q (imgQ, V part), B = dS scaled per (key, tile)
// dK = scale sum dS q, dV = sum P m dO. Per-key lanes: no atomics, each block owns its keys.
template <int DH, bool DROP>
__global__ void __launch_bounds__(256, DH == 64 ? 1 : 2)
attn_bwd_dkdv_f16x3_kernel(const float* __restrict__ k, int64_t ld_k, const float* __restrict__ v,
                           int64_t ld_v, const uint4* __restrict__ imgq, const int2* __restrict__ scq,
                           const uint4* __restrict__ imgd, const int2* __restrict__ scd,
                           const float* __restrict__ lsed_t, float* __restrict__ dk, int64_t ld_dk,
                           float* __restrict__ dv, int64_t ld_dv, const int64_t* __restrict__ q_off,
                           const int64_t* __restrict__ kv_off, const int32_t* __restrict__ kv_seg,
                           int n_head, int n_seg, int n_kv_seg, int n_kblk, float scale,
                           float scale_log2, uint32_t drop_seed, uint32_t drop_thresh, float inv_keep) {
    constexpr int KD = DH / 32, TD = DH / 16;
    constexpr int UN = units<DH>();
    constexpr int PW = UN / 64 / 4;
    __shared__ u32x4 lq0[UN], lq1[UN], ld0[UN], ld1[UN];
    __shared__ u32x4 ls0[32], ls1[32];                           // [lse2 64 | D 64] per tile
    typedef __attribute__((address_space(3))) char lds_c;
    const int L = blockIdx.x, xcd = L & 7, j0 = L >> 3;
    const int pair = (j0 / n_kblk) * 8 + xcd, kblk = j0 % n_kblk;
    if (pair >= n_kv_seg * n_head) return;
    const int ks = pair / n_head, head = pair % n_head;
    const int64_t kb = kv_off[ks], ke = kv_off[ks + 1];
    const int64_t k0 = kb + (int64_t)kblk * 64;
    if (k0 >= ke) return;                                        // block-uniform
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const int64_t krow = k0 + wv * 16 + c;
    const bool kok = krow < ke;
    float x[KD][8], y[KD][8];
    float km = 0.f, vm = 0.f;
#pragma unroll
    for (int kd = 0; kd < KD; ++kd) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, va = a, vb = a;
        if (kok) {
            const int64_t col = head * DH + 32 * kd + 8 * g;
            const float4* pk = reinterpret_cast<const float4*>(k + krow * ld_k + col);
            const float4* pv = reinterpret_cast<const float4*>(v + krow * ld_v + col);
            a = pk[0]; b = pk[1]; va = pv[0]; vb = pv[1];
        }
        x[kd][0] = a.x; x[kd][1] = a.y; x[kd][2] = a.z; x[kd][3] = a.w;
        x[kd][4] = b.x; x[kd][5] = b.y; x[kd][6] = b.z; x[kd][7] = b.w;
        y[kd][0] = va.x; y[kd][1] = va.y; y[kd][2] = va.z; y[kd][3] = va.w;
        y[kd][4] = vb.x; y[kd][5] = vb.y; y[kd][6] = vb.z; y[kd][7] = vb.w;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            x[kd][e] *= scale_log2;
            km = fmaxf(km, fabsf(x[kd][e]));
            vm = fmaxf(vm, fabsf(y[kd][e]));
        }
    }
    const int ek = range_exp(xg_max16(km)), ev = range_exp(xg_max16(vm));
    const float sk = __builtin_ldexpf(1.f, ek), sv = __builtin_ldexpf(1.f, ev);
    f16x8 kt[KD][2], vt[KD][2];
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            _Float16 h, m;
            split2(x[kd][e] * sk, h, m);
            kt[kd][0][e] = h; kt[kd][1][e] = m;
            split2(y[kd][e] * sv, h, m);
            vt[kd][0][e] = h; vt[kd][1][e] = m;
        }
    f32x4 adk[TD], adv[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t) adk[t] = adv[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float one = 1.0f;
    const uint32_t kaddr = (uint32_t)(g * 64 + c) * 16;
    const int qq = c >> 2, pp = c & 3;
    uint32_t vaddr[TD];
#pragma unroll
    for (int t = 0; t < TD; ++t)
        vaddr[t] = unit_v<DH>() * 16 + (4 * g + qq) * (2 * DH) +
                   (((2 * t + (pp >> 1)) ^ v_swz<DH>(4 * g + qq)) * 16) + (pp & 1) * 8;
    typedef __attribute__((address_space(3))) u32x4 lds_u4;
    typedef __attribute__((address_space(3))) s16x4 lds_s4;
    typedef __attribute__((address_space(3))) f32x4 lds_v4;

    for (int seg = 0; seg < n_seg; ++seg) {
        if (kv_seg[seg] != ks) continue;                         // block-uniform
        const int64_t qb = q_off[seg];
        const int nq = (int)(q_off[seg + 1] - qb);
        const int ntile = (nq + 63) / 64;
        if (ntile == 0) continue;
        const int64_t tile0 = (qb / 64 + seg) * n_head + head;
        const int64_t tstride = (int64_t)n_head * UN;
        const u32x4* srcq = reinterpret_cast<const u32x4*>(imgq) + tile0 * UN + wv * PW * 64 + lane;
        const u32x4* srcd = reinterpret_cast<const u32x4*>(imgd) + tile0 * UN + wv * PW * 64 + lane;
        const u32x4* srcl = reinterpret_cast<const u32x4*>(lsed_t) + tile0 * 32 + lane;
        auto dma = [&](int t, auto buf_tag) {
            constexpr int BUF = decltype(buf_tag)::value;
            lds_c* dq_ = (lds_c*)(BUF == 0 ? lq0 : lq1) + wv * PW * 1024;
            lds_c* dd_ = (lds_c*)(BUF == 0 ? ld0 : ld1) + wv * PW * 1024;
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                __builtin_amdgcn_global_load_lds((const void*)(srcq + t * tstride + j * 64),
                                                 (__attribute__((address_space(3))) void*)(dq_ + j * 1024), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(srcd + t * tstride + j * 64),
                                                 (__attribute__((address_space(3))) void*)(dd_ + j * 1024), 16, 0, 0);
            }
            if (wv == 0 && lane < 32)
                __builtin_amdgcn_global_load_lds((const void*)(srcl + (int64_t)t * n_head * 32),
                                                 (__attribute__((address_space(3))) void*)(BUF == 0 ? ls0 : ls1),
                                                 16, 0, 0);
        };
        __syncthreads();                                         // the previous segment's buffers
        dma(0, std::integral_constant<int, 0>{});

        auto tile = [&](int tt, auto buf_tag) {
            constexpr int BUF = decltype(buf_tag)::value;
            wait_vm_lgkm0_a<0>();
            __builtin_amdgcn_s_barrier();
            if (tt + 1 < ntile) dma(tt + 1, std::integral_constant<int, 1 - BUF>{});
            const int64_t ti = tile0 + (int64_t)__builtin_amdgcn_readfirstlane(tt) * n_head;
            const int2 eq2 = scq[ti], ed2 = scd[ti];
            lds_c* const bq = (lds_c*)(BUF == 0 ? lq0 : lq1);
            lds_c* const bd = (lds_c*)(BUF == 0 ? ld0 : ld1);
            lds_c* const bl = (lds_c*)(BUF == 0 ? ls0 : ls1);
            f32x4 s4[4], d4[4];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
#pragma unroll
                for (int kd = 0; kd < KD; ++kd) {
                    const int ko = (((kd * 2 + 0) * 4) * 64 + 16 * n) * 16, lo = (((kd * 2 + 1) * 4) * 64 + 16 * n) * 16;
                    const f16x8 qh = __builtin_bit_cast(f16x8, *(lds_u4*)(bq + kaddr + ko));
                    const f16x8 ql = __builtin_bit_cast(f16x8, *(lds_u4*)(bq + kaddr + lo));
                    const f16x8 dh_ = __builtin_bit_cast(f16x8, *(lds_u4*)(bd + kaddr + ko));
                    const f16x8 dl_ = __builtin_bit_cast(f16x8, *(lds_u4*)(bd + kaddr + lo));
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ql, kt[kd][0], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh, kt[kd][1], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh, kt[kd][0], a, 0, 0, 0);
                    b = __builtin_amdgcn_mfma_f32_16x16x32_f16(dl_, vt[kd][0], b, 0, 0, 0);
                    b = __builtin_amdgcn_mfma_f32_16x16x32_f16(dh_, vt[kd][1], b, 0, 0, 0);
                    b = __builtin_amdgcn_mfma_f32_16x16x32_f16(dh_, vt[kd][0], b, 0, 0, 0);
                }
                s4[n] = a;
                d4[n] = b;
            }
            const float fs = __builtin_ldexpf(1.f, -(eq2.x + ek));
            const float fd = __builtin_ldexpf(1.f, -(ed2.x + ev));
            float pk[16], ds[16];
            float dmx = 0.f;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const f32x4 lv = *(lds_v4*)(bl + (16 * n + 4 * g) * 4);
                const f32x4 Dv = *(lds_v4*)(bl + 256 + (16 * n + 4 * g) * 4);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s4[n][r], fs, -lv[r]));
                    float dp = d4[n][r] * fd, pkeep = p;
                    if constexpr (DROP) {
                        const int64_t qrow = qb + (int64_t)tt * 64 + 16 * n + 4 * g + r;
                        const bool drop = attn_drop_hash(drop_seed, head, qrow, krow) < drop_thresh;
                        dp = drop ? 0.f : dp * inv_keep;
                        pkeep = drop ? 0.f : p;
                    }
                    pk[4 * n + r] = pkeep * 16384.f;
                    const float d = p * (dp - Dv[r]);
                    ds[4 * n + r] = d;
                    dmx = fmaxf(dmx, fabsf(d));
                }
            }
            const int eds = range_exp(xg_max16(dmx));
            const float sds = __builtin_ldexpf(1.f, eds);
            f32x4 tv[TD], tk[TD];
#pragma unroll
            for (int t = 0; t < TD; ++t) tv[t] = tk[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float pv[8] = {pk[8 * j + 0], pk[8 * j + 1], pk[8 * j + 2], pk[8 * j + 3],
                                     pk[8 * j + 4], pk[8 * j + 5], pk[8 * j + 6], pk[8 * j + 7]};
                const float sv8[8] = {ds[8 * j + 0] * sds, ds[8 * j + 1] * sds, ds[8 * j + 2] * sds, ds[8 * j + 3] * sds,
                                      ds[8 * j + 4] * sds, ds[8 * j + 5] * sds, ds[8 * j + 6] * sds, ds[8 * j + 7] * sds};
                u32x4 ph, pl, sh, sl;
                split8_pk(pv, one, ph, pl);
                split8_pk(sv8, one, sh, sl);
                const f16x8 p0 = __builtin_bit_cast(f16x8, ph), p1 = __builtin_bit_cast(f16x8, pl);
                const f16x8 s0 = __builtin_bit_cast(f16x8, sh), s1 = __builtin_bit_cast(f16x8, sl);
#pragma unroll
                for (int t = 0; t < TD; ++t) {
                    f16x8 of[2], qf[2];
#pragma unroll
                    for (int tm = 0; tm < 2; ++tm) {
                        const uint32_t off = vaddr[t] + tm * (128 * DH) + j * 32 * (2 * DH);
                        const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(bd + off));
                        const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(bd + off + 16 * (2 * DH)));
                        of[tm] = __builtin_bit_cast(f16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
                        const s16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(bq + off));
                        const s16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(bq + off + 16 * (2 * DH)));
                        qf[tm] = __builtin_bit_cast(f16x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
                    }
                    f32x4 a = tv[t], b = tk[t];
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(of[1], p0, a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(of[0], p1, a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(of[0], p0, a, 0, 0, 0);
                    b = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[1], s0, b, 0, 0, 0);
                    b = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[0], s1, b, 0, 0, 0);
                    b = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[0], s0, b, 0, 0, 0);
                    tv[t] = a;
                    tk[t] = b;
                }
            }
            const float fv = __builtin_ldexpf(1.f, -(ed2.y + 14));
            const float fk = __builtin_ldexpf(1.f, -(eq2.y + eds));
#pragma unroll
            for (int t = 0; t < TD; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    adv[t][r] = __builtin_fmaf(tv[t][r], fv, adv[t][r]);
                    adk[t][r] = __builtin_fmaf(tk[t][r], fk, adk[t][r]);
                }
        };
        using B0 = std::integral_constant<int, 0>;
        using B1 = std::integral_constant<int, 1>;
        int tt = 0;
        for (; tt + 2 <= ntile; tt += 2) {
            tile(tt, B0{});
            tile(tt + 1, B1{});
        }
        if (tt < ntile) tile(tt, B0{});
    }
    if (!kok) return;
    const float fdv = DROP ? inv_keep : 1.f;
#pragma unroll
    for (int t = 0; t < TD; ++t) {
        *reinterpret_cast<float4*>(dk + krow * ld_dk + head * DH + 16 * t + 4 * g) =
            make_float4(adk[t][0] * scale, adk[t][1] * scale, adk[t][2] * scale, adk[t][3] * scale);
        *reinterpret_cast<float4*>(dv + krow * ld_dv + head * DH + 16 * t + 4 * g) =
            make_float4(adv[t][0] * fdv, adv[t][1] * fdv, adv[t][2] * fdv, adv[t][3] * fdv);
    }
}

}  // namespace

// fgr_attention_bwd_train on the f16 matrix cores (called from train.hip): the K / V / Q / dO
// per-tile images, then attn_bwd_dq_f16x3_kernel and (dkdv) attn_bwd_dkdv_f16x3_kernel; without
// dkdv, lse_out / dsum_out receive the rows' lse2 and D for train.hip's fp32-MFMA dK / dV
// kernel. q_off and kv_off index one packed row space of n_rows rows (q and kv segments of the
// same tensors, self- or cross-attention). ws: attn_bwd_f16x3_bytes.
size_t attn_bwd_f16x3_bytes(int64_t n_rows, int32_t n_seg, int32_t n_head, int32_t dh) {
    const int64_t nt = n_tiles16(n_rows, n_seg) * n_head;
    const int un = dh == 32 ? units<32>() : units<64>();
    return (size_t)4 * (nt * un * 16 + nt * 8) + (size_t)nt * 128 * 4;
}

int attn_bwd_f16x3(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                   int64_t ldv, const float* o, int64_t ldo, const float* dout, int64_t lddo,
                   float* dq, int64_t lddq, float* dk, int64_t lddk, float* dv, int64_t lddv,
                   const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                   int32_t n_seg, int32_t n_kv_seg, int64_t n_rows, int64_t max_q_len,
                   int64_t max_kv_len, int32_t nhead, int32_t dh, float scale, const float* lse_in,
                   float* lse_out, float* dsum_out, bool dkdv, void* ws, uint32_t drop_seed,
                   uint32_t drop_thresh, float inv_keep, hipStream_t st) {
    const int32_t nsm = std::max(n_seg, n_kv_seg);
    const int64_t nt = n_tiles16(n_rows, nsm) * nhead;
    const int un = dh == 32 ? units<32>() : units<64>();
    const int64_t ib = nt * un * 16 + nt * 8;                      // one image + its exponents
    char* base = static_cast<char*>(ws);
    auto img = [&](int i) { return reinterpret_cast<uint4*>(base + i * ib); };
    auto sc = [&](int i) { return reinterpret_cast<int2*>(base + i * ib + nt * un * 16); };
    float* lsed = reinterpret_cast<float*>(base + 4 * ib);
    const int n_qblk = (int)ceil_div(max_q_len, 64), n_kblk = (int)ceil_div(max_kv_len, 64);
    const int64_t n_blocks = ceil_div((int64_t)n_seg * nhead, 8) * 8 * n_qblk;
    const int64_t n_kblocks = ceil_div((int64_t)n_kv_seg * nhead, 8) * 8 * n_kblk;
    const float sl2 = scale * 1.4426950408889634f;
    const bool drop = drop_thresh != 0;
    ImgJobs jobs{{k, v, q, dout}, {ldk, ldv, ldq, lddo}, {kv_off, kv_off, q_off, q_off},
                 {img(0), img(1), img(2), img(3)}, {sc(0), sc(1), sc(2), sc(3)},
                 {n_kv_seg, n_kv_seg, n_seg, n_seg}, {1, 0, 1, 1}, nsm};
    const dim3 igrid((unsigned)ceil_div(std::max(max_q_len, max_kv_len), 64), (unsigned)nhead,
                     (unsigned)((dkdv ? 4 : 2) * nsm));
#define FGR_BWD16(D)                                                                                 \
    hipLaunchKernelGGL(attn_image16_jobs_kernel<D>, igrid, dim3(256), 0, st, jobs);                   \
    if (drop)                                                                                        \
        hipLaunchKernelGGL((attn_bwd_dq_f16x3_kernel<D, true>), dim3((unsigned)n_blocks), dim3(256), 0, st, \
                           q, ldq, dout, lddo, o, ldo, img(0), sc(0), img(1), sc(1), dq, lddq, q_off,   \
                           kv_off, kv_seg, nhead, n_seg, n_qblk, scale, sl2, lse_in,                  \
                           dkdv ? nullptr : lse_out, dsum_out, dkdv ? lsed : nullptr, drop_seed,      \
                           drop_thresh, inv_keep);                                                   \
    else                                                                                             \
        hipLaunchKernelGGL((attn_bwd_dq_f16x3_kernel<D, false>), dim3((unsigned)n_blocks), dim3(256), 0, st, \
                           q, ldq, dout, lddo, o, ldo, img(0), sc(0), img(1), sc(1), dq, lddq, q_off,   \
                           kv_off, kv_seg, nhead, n_seg, n_qblk, scale, sl2, lse_in,                  \
                           dkdv ? nullptr : lse_out, dsum_out, dkdv ? lsed : nullptr, drop_seed,      \
                           drop_thresh, inv_keep);                                                   \
    if (dkdv) {                                                                                      \
        if (drop)                                                                                    \
            hipLaunchKernelGGL((attn_bwd_dkdv_f16x3_kernel<D, true>), dim3((unsigned)n_kblocks), dim3(256), 0, \
                               st, k, ldk, v, ldv, img(2), sc(2), img(3), sc(3), lsed, dk, lddk, dv,  \
                               lddv, q_off, kv_off, kv_seg, nhead, n_seg, n_kv_seg, n_kblk, scale,   \
                               sl2, drop_seed, drop_thresh, inv_keep);                               \
        else                                                                                         \
            hipLaunchKernelGGL((attn_bwd_dkdv_f16x3_kernel<D, false>), dim3((unsigned)n_kblocks), dim3(256), 0, \
                               st, k, ldk, v, ldv, img(2), sc(2), img(3), sc(3), lsed, dk, lddk, dv,  \
                               lddv, q_off, kv_off, kv_seg, nhead, n_seg, n_kv_seg, n_kblk, scale,   \
                               sl2, drop_seed, drop_thresh, inv_keep);                               \
    }
    if (dh == 32) {
        FGR_BWD16(32)
    } else {
        FGR_BWD16(64)
    }
#undef FGR_BWD16
    FGR_CHECK_LAUNCH("attn_bwd_f16x3");
    return FGR_OK;
}

}  // namespace fgr

using namespace fgr;

extern "C" int fgr_attention_f16x3_workspace(int64_t n_kv_rows, int32_t n_kv_seg,
                                             int32_t n_head, size_t* bytes) {
    FGR_REQUIRE(bytes && n_kv_rows >= 0 && n_kv_seg >= 0 && n_head > 0,
                "fgr_attention_f16x3_workspace: bad arguments");
    // sized for the largest supported head dim (64)
    const int64_t nt = n_tiles16(n_kv_rows, n_kv_seg) * n_head;
    *bytes = (size_t)(nt * units<64>() * 16 + nt * 8);
    return FGR_OK;
}

static int attention_f16x3_impl(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                const float* v, int64_t ld_v, float* o, int64_t ld_o,
                                const int64_t* q_off, const int64_t* kv_off,
                                const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg,
                                int64_t n_kv_rows, int32_t max_q_len, int32_t max_kv_len,
                                int32_t n_head, int32_t head_dim, float scale, void* workspace,
                                int64_t ws_bytes, uint32_t drop_seed, float drop_p, void* stream,
                                float* lse_out = nullptr) {
    FGR_REQUIRE(q && k && v && o && q_off && kv_off && kv_seg && workspace && n_seg > 0 &&
                    n_kv_seg > 0 && n_head > 0 && max_q_len >= 0 && max_kv_len >= 0,
                "fgr_attention_f16x3: bad arguments");
    FGR_REQUIRE(head_dim == 32 || head_dim == 64, "fgr_attention_f16x3: head_dim %d (32 or 64)",
                head_dim);
    const int dh = head_dim;
    FGR_REQUIRE(ld_q >= n_head * dh && ld_k >= n_head * dh && ld_v >= n_head * dh &&
                    ld_o >= n_head * dh && ld_q % 4 == 0 && ld_k % 4 == 0 && ld_v % 4 == 0 &&
                    ld_o % 4 == 0,
                "fgr_attention_f16x3: row strides must be >= n_head*head_dim and multiples of 4");
    FGR_REQUIRE(((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
                  reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o) |
                  reinterpret_cast<uintptr_t>(workspace)) & 15) == 0,
                "fgr_attention_f16x3: q/k/v/o/workspace must be 16-B aligned");
    const int64_t nt = n_tiles16(n_kv_rows, n_kv_seg) * n_head;
    const int un = dh == 32 ? units<32>() : units<64>();
    const int64_t need = nt * un * 16 + nt * 8;
    FGR_REQUIRE(ws_bytes >= need, "fgr_attention_f16x3: workspace %lld < %lld bytes",
                (long long)ws_bytes, (long long)need);
    if (max_q_len == 0 || max_kv_len == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    uint4* img = static_cast<uint4*>(workspace);
    int2* sc = reinterpret_cast<int2*>(static_cast<char*>(workspace) + nt * un * 16);
    const dim3 kgrid((unsigned)ceil_div(max_kv_len, 64), (unsigned)n_head, (unsigned)n_kv_seg);
    if (dh == 32)
        hipLaunchKernelGGL(attn_kv_image16_kernel<32>, kgrid, dim3(256), 0, st, k, ld_k, v, ld_v,
                           kv_off, n_head, img, sc);
    else
        hipLaunchKernelGGL(attn_kv_image16_kernel<64>, kgrid, dim3(256), 0, st, k, ld_k, v, ld_v,
                           kv_off, n_head, img, sc);
    FGR_CHECK_LAUNCH("attn_kv_image16_kernel");
    const int n_qblk = (int)ceil_div(max_q_len, 64);
    const int64_t n_blocks = ceil_div((int64_t)n_seg * n_head, 8) * 8 * n_qblk;
    const float sl2 = scale * 1.4426950408889634f;
    if (drop_p > 0.f) {
        const uint32_t thresh = (uint32_t)std::min(4294967295.0, (double)drop_p * 4294967296.0);
        const float inv_keep = 1.0f / (1.0f - drop_p);
        if (dh == 32)
            hipLaunchKernelGGL((attn_f16x3_v2_kernel<32, true>), dim3((unsigned)n_blocks), dim3(256), 0,
                               st, q, ld_q, (const uint4*)img, (const int2*)sc, o, ld_o, q_off, kv_off,
                               kv_seg, n_head, n_seg, n_qblk, sl2, 0, drop_seed, thresh, inv_keep, lse_out);
        else
            hipLaunchKernelGGL((attn_f16x3_v2_kernel<64, true>), dim3((unsigned)n_blocks), dim3(256), 0,
                               st, q, ld_q, (const uint4*)img, (const int2*)sc, o, ld_o, q_off, kv_off,
                               kv_seg, n_head, n_seg, n_qblk, sl2, 0, drop_seed, thresh, inv_keep, lse_out);
    } else if (dh == 32) {
        hipLaunchKernelGGL((attn_f16x3_v2_kernel<32>), dim3((unsigned)n_blocks), dim3(256), 0, st, q,
                           ld_q, (const uint4*)img, (const int2*)sc, o, ld_o, q_off, kv_off, kv_seg,
                           n_head, n_seg, n_qblk, sl2, 0, 0u, 0u, 1.f, lse_out);
    } else {
        hipLaunchKernelGGL((attn_f16x3_v2_kernel<64>), dim3((unsigned)n_blocks), dim3(256), 0, st, q,
                           ld_q, (const uint4*)img, (const int2*)sc, o, ld_o, q_off, kv_off, kv_seg,
                           n_head, n_seg, n_qblk, sl2, 0, 0u, 0u, 1.f, lse_out);
    }
    FGR_CHECK_LAUNCH("attn_f16x3_v2_kernel");
    return FGR_OK;
}

extern "C" int fgr_attention_f16x3(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                   const float* v, int64_t ld_v, float* o, int64_t ld_o,
                                   const int64_t* q_off, const int64_t* kv_off,
                                   const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg,
                                   int64_t n_kv_rows, int32_t max_q_len, int32_t max_kv_len,
                                   int32_t n_head, int32_t head_dim, float scale,
                                   void* workspace, int64_t ws_bytes, void* stream) {
    return attention_f16x3_impl(q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, n_seg,
                                n_kv_seg, n_kv_rows, max_q_len, max_kv_len, n_head, head_dim,
                                scale, workspace, ws_bytes, 0u, 0.f, stream);
}

extern "C" int fgr_attention_f16x3_drop(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                        const float* v, int64_t ld_v, float* o, int64_t ld_o,
                                        const int64_t* q_off, const int64_t* kv_off,
                                        const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg,
                                        int64_t n_kv_rows, int32_t max_q_len, int32_t max_kv_len,
                                        int32_t n_head, int32_t head_dim, float scale,
                                        void* workspace, int64_t ws_bytes, uint32_t seed,
                                        float p, void* stream) {
    FGR_REQUIRE(p >= 0.f && p < 1.f, "fgr_attention_f16x3_drop: dropout p %f not in [0, 1)", p);
    return attention_f16x3_impl(q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, n_seg,
                                n_kv_seg, n_kv_rows, max_q_len, max_kv_len, n_head, head_dim,
                                scale, workspace, ws_bytes, seed, p, stream);
}

extern "C" int fgr_attention_f16x3_train(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                         const float* v, int64_t ld_v, float* o, int64_t ld_o,
                                         const int64_t* q_off, const int64_t* kv_off,
                                         const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg,
                                         int64_t n_kv_rows, int32_t max_q_len, int32_t max_kv_len,
                                         int32_t n_head, int32_t head_dim, float scale,
                                         void* workspace, int64_t ws_bytes, uint32_t seed, float p,
                                         float* lse, void* stream) {
    FGR_REQUIRE(p >= 0.f && p < 1.f, "fgr_attention_f16x3_train: dropout p %f not in [0, 1)", p);
    FGR_REQUIRE(lse, "fgr_attention_f16x3_train: null lse");
    return attention_f16x3_impl(q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, n_seg,
                                n_kv_seg, n_kv_rows, max_q_len, max_kv_len, n_head, head_dim,
                                scale, workspace, ws_bytes, seed, p, stream, lse);
}

// The attention on K / V images of GLOBAL 64-row tiles written by fgr_gemm_f16x3_ln_qkv (head
// dim 32) or fgr_gemm_f16x3_qkv (head dim 64): no image launch here.
extern "C" int fgr_attention_f16x3_img(const float* q, int64_t ld_q, const void* kv_img,
                                       int64_t n_kv_rows, float* o, int64_t ld_o,
                                       const int64_t* q_off, const int64_t* kv_off,
                                       const int32_t* kv_seg, int32_t n_seg, int32_t max_q_len,
                                       int32_t n_head, int32_t head_dim, float scale, void* stream) {
    FGR_REQUIRE(q && kv_img && o && q_off && kv_off && kv_seg && n_seg > 0 && n_head > 0 &&
                    max_q_len >= 0 && n_kv_rows >= 0,
                "fgr_attention_f16x3_img: bad arguments");
    FGR_REQUIRE(head_dim == 32 || head_dim == 64, "fgr_attention_f16x3_img: head_dim %d (32 or 64)",
                head_dim);
    FGR_REQUIRE(ld_q >= n_head * head_dim && ld_o >= n_head * head_dim && ld_q % 4 == 0 && ld_o % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(o) |
                      reinterpret_cast<uintptr_t>(kv_img)) & 15) == 0,
                "fgr_attention_f16x3_img: strides / alignment");
    if (max_q_len == 0 || n_kv_rows == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const int64_t nt = ceil_div(n_kv_rows, 64) * n_head;
    const int un = head_dim == 32 ? units<32>() : units<64>();
    const uint4* img = static_cast<const uint4*>(kv_img);
    const int2* sc = reinterpret_cast<const int2*>(static_cast<const char*>(kv_img) + nt * un * 16);
    const int n_qblk = (int)ceil_div(max_q_len, 64);
    const int64_t n_blocks = ceil_div((int64_t)n_seg * n_head, 8) * 8 * n_qblk;
    const float sl2 = scale * 1.4426950408889634f;
    if (head_dim == 32)
        hipLaunchKernelGGL((attn_f16x3_v2_kernel<32>), dim3((unsigned)n_blocks), dim3(256), 0, st, q, ld_q,
                           img, sc, o, ld_o, q_off, kv_off, kv_seg, n_head, n_seg, n_qblk, sl2, 1,
                           0u, 0u, 1.f);
    else
        hipLaunchKernelGGL((attn_f16x3_v2_kernel<64>), dim3((unsigned)n_blocks), dim3(256), 0, st, q, ld_q,
                           img, sc, o, ld_o, q_off, kv_off, kv_seg, n_head, n_seg, n_qblk, sl2, 1,
                           0u, 0u, 1.f);
    FGR_CHECK_LAUNCH("attn_f16x3_v2_kernel (global tiles)");
    return FGR_OK;
}
