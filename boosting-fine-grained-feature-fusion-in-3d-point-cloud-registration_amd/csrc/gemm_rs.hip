// "rs" (row-stationary) f16x3 GEMM for short contractions (K <= 256, K % 8 == 0):
//
//   C[M, N] = act(A[M, K] . W[N, K]^T + bias[N] (+ R[M, N]))
//
// Why. At K <= 256 a tile of the k-looped kernels (gemm16.hip, gemm5.hip) runs 4-8 k32-steps:
// every step waits an operand round trip, and every block that shares an A row panel loads
// and splits it again. Here a wave loads its activation rows ONCE, whole (16 * RT rows x K),
// splits them in registers into the two fp16 terms with ONE power-of-two scale per row (the
// row max over all of K into [2^14, 2^15): no in-flight rescaling, the scale goes to the
// epilogue), and keeps them resident; the block then streams its range of W panels (16
// output columns x K each, the fgr_split_weights_h3 image as it lies) global -> LDS by
// LDS-DMA into a three-panel ring shared by the 4 waves (two in flight), and per panel runs a
// pure MFMA loop (3 * RT * K/32 MFMAs per wave, no split VALU); the 16-B-per-lane epilogue of
// panel q - 1 is issued after panel q's MFMAs, so its VALU and stores fill the MFMA shadows
// (round 4: 1.09-1.17x on the LN-fused and 57264-row shapes).
//
// Precision: per product the three significant fp16 products hh, hm, mh in fp32
// accumulation as in gemm16.hip; one scale per row means elements far below the row max
// lose low bits of their lo term to fp16 subnormals, an ABSOLUTE error <= 2^-39 max|a_row|
// per element (2^-24 / 2 of the subnormal spacing over the 2^14 scale floor) -- relative to
// the dot product's own fp32 rounding (K 2^-24 sum|a w|) negligible.
//
// LayerNorm prologue (LN = true; fgr_gemm_f16x3_ln): A = LayerNorm(X) * gamma + beta (+ add),
// i.e. the pre-norm transformer's norm -> with_pos_embed -> Linear (transformers.py:193-196,
// :213-221, :231-232) in one launch. A wave holds whole rows (K = d) in registers anyway, so
// the row mean and the centred variance come from its own values (two passes over registers,
// the lane sums over the four k-groups by permlane swaps), gamma / beta are staged once per
// block in LDS, and the normalised row is split as above: the LayerNorm output never goes to
// memory and its launch disappears.
//
// Correspondence-head epilogues (fgr_corr_head_f16x3; CorrespondenceRegressor,
// finegrained_regtr.py:411-455): (a) `n_act` / `c2`: columns >= n_act take no activation and
// column n_act goes to c2[row] instead of C -- coor_mlp[0] (ReLU) and conf_logits_decoder
// (none) as ONE product over [W0; Wc; 0] (the 15 zero rows pad N to a panel); (b) HEAD: the
// block covers every panel of its rows and instead of storing the ReLU'd outputs it
// accumulates their dot products with the 3 rows of coor_mlp[4] (fp32 FMAs on the fp32
// outputs, no split), reduced over the 4 lane groups at the end: coor_mlp[2] -> ReLU ->
// coor_mlp[4] in one launch, the hidden (rows, d) tensor never written.
//
// K / V attention images (KV; fgr_gemm_f16x3_ln_qkv, head dim 32): the in_proj launch of the
// pre-norm layer writes the q columns as fp32 and the k / v columns straight into the f16x3
// attention images that attention16.hip reads (one per GLOBAL 64-row tile and head: the
// block's 64 rows, RT = 1), instead of fp32 k / v for a separate image launch. A head is two
// panels: its 8 values per lane stay in registers until both are done, each wave's max |.|
// goes to LDS, and after the next panel barrier every wave reads the four maxima, takes the
// tile's power-of-two exponent (max in [2^14, 2^15), as attn_kv_image16_kernel) and stores
// its split terms.
//
// Swapped orientation (gemm16.hip): W fragments are the MFMA A operand, activation fragments
// the B operand, so a lane's 4 accumulators are 4 consecutive output columns of ONE row.
// 16x16x32 f16 lane maps (lane l, g = l >> 4, c = l & 15): A[i = c][k = 8g + e],
// B[k = 8g + e][j = c], C[i = 4g + r][j = c].
#include <algorithm>
#include <cstdlib>

#include "common.h"

#ifdef FGR_RS_STAMP
// Diagnostic build only (tools/build_stamp.sh, tools/rs_stamp.py): per-block clock stamps of
// the rs kernel, read back by fgr_debug_rs_stamps. [0] s_memrealtime at entry, [1]
// s_memtime at entry, [2] after the prologue (rows loaded and split), [3] after panel 0's
// barrier, [4] after the last panel's barrier, [5] at exit, [6] s_memrealtime at exit, [7]
// panels of the block.
__device__ unsigned long long g_rs_stamp[1 << 14][8];
#endif

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct RsArgs {
    const float* A; int64_t lda;
    const u32x4* W;                   // image [panel][kstep KS][term 2][g 4][16] x 16 B
    const float* wsc;                 // per n: 2^-e_n (padded to 16)
    float* C; int64_t ldc;
    const float* bias;
    const float* R; int64_t ldr;
    int M, N, K, act;
    int nc;                           // W panels (16 columns) per block
    const float* ln_g; const float* ln_b;   // LN prologue: gamma, beta (K)
    const float* ln_add; int64_t ld_add;    //   optional row add (pos) after the affine
    float eps;
    const float* ln_g2; const float* ln_b2; //   side output (LNM 3): LN(x) * g2 + b2 -> out2
    float* ln_out2; int64_t ld_out2;
    int n_act;                        // columns >= n_act: no activation (n_act % 16 == 0)
    float* c2;                        //   and column n_act -> c2[row] (not stored in C)
    const float* w4; const float* b4; // HEAD: (3, N) fp32 rows and bias of the 3-wide output
    float* out3;                      //   -> out3 (M, 3)
    char* kv_img;                     // KV: attention K / V images per (global 64-row tile, head)
    int2* kv_sc;                      //   and their scale exponents (x: K, y: V)
    int n_head, kv_col0;              //   heads (head dim 32); first K column (V: + 32 n_head)
};

// s_waitcnt vmcnt(n) lgkmcnt(0) -- gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0_rs() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}

__device__ __forceinline__ float xg_max_rs(float v) {     // max over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float xg_sum_rs(float v) {     // sum over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// vmcnt(n) lgkmcnt(0) for a wave-uniform runtime n <= 15 (s_waitcnt takes an immediate)
__device__ __forceinline__ void wait_vm_lgkm0_dyn(int n) {
    switch (n) {
        case 0: wait_vm_lgkm0_rs<0>(); break;   case 1: wait_vm_lgkm0_rs<1>(); break;
        case 2: wait_vm_lgkm0_rs<2>(); break;   case 3: wait_vm_lgkm0_rs<3>(); break;
        case 4: wait_vm_lgkm0_rs<4>(); break;   case 5: wait_vm_lgkm0_rs<5>(); break;
        case 6: wait_vm_lgkm0_rs<6>(); break;   case 7: wait_vm_lgkm0_rs<7>(); break;
        case 8: wait_vm_lgkm0_rs<8>(); break;   case 9: wait_vm_lgkm0_rs<9>(); break;
        case 10: wait_vm_lgkm0_rs<10>(); break; case 11: wait_vm_lgkm0_rs<11>(); break;
        case 12: wait_vm_lgkm0_rs<12>(); break; case 13: wait_vm_lgkm0_rs<13>(); break;
        case 14: wait_vm_lgkm0_rs<14>(); break; default: wait_vm_lgkm0_rs<15>(); break;
    }
}

// W panels per pipeline stage: the panel loop waits for the stage's DMA, meets at one barrier
// and runs the MFMAs of all its panels; one stage is in flight while one computes (a ring of
// 2 * PPS panels). PPS = 1 is the round-4 loop (a 3-panel ring, two in flight). Round 5: a
// panel took ~0.3 us of MFMA plus ~0.7 us of wait / barrier latency, and doubling its MFMA
// work added the whole MFMA time (profiles/r05_rs_pps_ab.txt), so panels share the waits.
#ifndef FGR_RS_PPS
#define FGR_RS_PPS 2
#endif
constexpr int kRsPps = FGR_RS_PPS;
constexpr int kRsMaxNc = 32;       // panels per block (the per-block column scales / bias in LDS)
#ifndef FGR_RS_LA
#define FGR_RS_LA 4
#endif
constexpr int kRsLookahead = FGR_RS_LA;   // k-steps of W fragments read ahead of their MFMAs

// the epilogue of one output, the activation fixed at compile time
template <int ACT, bool RES>
__device__ __forceinline__ float finish_ct(float y, float b, float r) {
    if constexpr (ACT == FGR_ACT_RELU_RES_LEAKY) {
        float t = fmaxf(y + b, 0.f);
        if constexpr (RES) t += r;
        return t > 0.f ? t : 0.1f * t;
    } else {
        float t = y + b;
        if constexpr (RES) t += r;
        if constexpr (ACT == FGR_ACT_RELU) t = fmaxf(t, 0.f);
        return t;
    }
}

// LNM: 0 plain, 1 LayerNorm prologue, 2 LayerNorm prologue + row add, 3 as 2 plus a second
// LayerNorm output of the same rows (the encoder's per-layer output norm), written by the
// blocks of the first column group
// f16x3 attention image geometry for head dim 32 (attention16.hip units<32>, unit_v<32>,
// v_swz<32>): 1024 16-B units per (tile, head), V from unit 512
constexpr int kKvUnits = 1024;
constexpr int kKvUnitV = 512;

template <int RT, int KS, bool RES, int ACT, int LNM, bool HEAD = false, bool KV = false>
__global__ void __launch_bounds__(256, KV ? 2 : 1) gemm_rs_kernel(RsArgs p) {
    constexpr bool LN = LNM > 0;
    constexpr int PANEL_U = KS * 128;                  // 16-B units per W panel
    constexpr int PW = PANEL_U / 256;                  // DMA pieces (1 KiB) per wave per panel
    static_assert(PANEL_U % 256 == 0, "KS even");
    // panels per stage (the LN + K/V + side-output variant keeps one: with two its register
    // peak passes the 256 VGPRs of two waves per SIMD; so do K <= 128, sized for 4 blocks / CU;
    // the plain LN prologue (linear1) measured 30.8 us with one, 33.0 us with two)
    constexpr int PPS = ((KV && LNM == 3) || KS <= 4 || (LN && !KV)) ? 1 : kRsPps;
    constexpr int NB = PPS == 1 ? 3 : 2 * PPS;         // W panel ring
    constexpr int LA = PPS == 1 ? NB - 1 : PPS;        // DMA lookahead in panels
    static_assert(PPS == 1 || NB == 2 * PPS, "one stage in flight while one computes");
    __shared__ u32x4 ring[NB * PANEL_U];
    __shared__ float4 colw[kRsMaxNc * 4], colb[kRsMaxNc * 4];   // per (panel, g): wsc, bias
    __shared__ float4 lng[LN ? KS * 8 : 1], lnb[LN ? KS * 8 : 1];  // LN gamma / beta (K / 4)
    __shared__ float4 lng2[LNM == 3 ? KS * 8 : 1], lnb2[LNM == 3 ? KS * 8 : 1];
    __shared__ float4 colh[HEAD ? 3 * kRsMaxNc * 4 : 1];            // HEAD: w4 by (j, panel, g)
    __shared__ float kvred[KV ? 2 : 1][4];                          // KV: per-wave head maxima
    // KV: the head's 16 x 32 outputs of each wave as float4 dim quads [key][quad 8]
    __shared__ float4 kvbuf[KV ? 4 : 1][KV ? 16 : 1][8];
    static_assert(!KV || RT == 1, "KV images: one 64-row tile per block");

#ifdef FGR_RS_STAMP
    unsigned long long st_[8];
    st_[0] = __builtin_amdgcn_s_memrealtime();
    st_[1] = __builtin_amdgcn_s_memtime();
#endif
    const int nbm = (p.M + 64 * RT - 1) / (64 * RT);
    const int npanel = (p.N + 15) / 16;
    const int ngrp = (npanel + p.nc - 1) / p.nc;
    const int nwg = nbm * ngrp;
    int t = blockIdx.x;
    {   // XCD-aware order: each XCD a contiguous range, the column groups of a row block adjacent
        const int q = nwg / 8, r = nwg % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int bm = t / ngrp, grp = t % ngrp;
    const int p0 = grp * p.nc;
    const int np = min(p.nc, npanel - p0);             // block-uniform
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const int mw = bm * 64 * RT + wv * 16 * RT;        // this wave's first row

    // W panel DMA: wave wv moves pieces wv, wv + 4, ... (1 KiB each, contiguous in the image)
    const u32x4* wsrc = p.W + (int64_t)p0 * PANEL_U + wv * 64 + lane;
    auto dma = [&](int q) {
        __attribute__((address_space(3))) char* dst =
            (__attribute__((address_space(3))) char*)(ring + (q % NB) * PANEL_U) + wv * 1024;
#pragma unroll
        for (int j = 0; j < PW; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(wsrc + (int64_t)q * PANEL_U + j * 256),
                                             (__attribute__((address_space(3))) void*)(dst + j * 4096),
                                             16, 0, 0);
    };
#pragma unroll
    for (int d = 0; d < LA; ++d)
        if (d < np) dma(d);

    // activation rows -> registers, one scale per row, split once
    f16x8 af[RT][KS][2];
    float rs[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int64_t row = min(mw + 16 * i + c, p.M - 1);
        const float* ar = p.A + row * p.lda;
        float x[KS][8];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 32 * s + 8 * g;
            float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
            if constexpr (LN) {
                // LN: unconditional loads (a chunk past K re-reads the last one and is zeroed
                // below), so all 2 * KS are in flight before the row statistics. (Measured
                // slower for the plain kernel, which keeps the guarded loads:
                // profiles/r03_gemm_rs_sweep_ln.txt.)
                const int kl = min(k, p.K - 8);
                a0 = *reinterpret_cast<const float4*>(ar + kl);
                a1 = *reinterpret_cast<const float4*>(ar + kl + 4);
            } else if (k < p.K) {
                a0 = *reinterpret_cast<const float4*>(ar + k);
                a1 = *reinterpret_cast<const float4*>(ar + k + 4);
            }
            x[s][0] = a0.x; x[s][1] = a0.y; x[s][2] = a0.z; x[s][3] = a0.w;
            x[s][4] = a1.x; x[s][5] = a1.y; x[s][6] = a1.z; x[s][7] = a1.w;
        }
        if constexpr (LN) {
#pragma unroll
            for (int s = 0; s < KS; ++s)
                if (32 * s + 8 * g >= p.K)
#pragma unroll
                    for (int e = 0; e < 8; ++e) x[s][e] = 0.f;
        }
        if constexpr (LN) {
            if (i == 0) {          // gamma / beta -> LDS (K <= 32 * KS), the first rows in flight
                float4 gv = make_float4(0.f, 0.f, 0.f, 0.f), bv = gv;
                if (tid < p.K / 4) {
                    gv = reinterpret_cast<const float4*>(p.ln_g)[tid];
                    bv = reinterpret_cast<const float4*>(p.ln_b)[tid];
                }
                if (tid < KS * 8) { lng[tid] = gv; lnb[tid] = bv; }
                if constexpr (LNM == 3) {
                    float4 g2v = make_float4(0.f, 0.f, 0.f, 0.f), b2v = g2v;
                    if (tid < p.K / 4) {
                        g2v = reinterpret_cast<const float4*>(p.ln_g2)[tid];
                        b2v = reinterpret_cast<const float4*>(p.ln_b2)[tid];
                    }
                    if (tid < KS * 8) { lng2[tid] = g2v; lnb2[tid] = b2v; }
                }
                __syncthreads();
            }
            // row mean, then the centred variance (as the LayerNorm kernels: norm.hip), from
            // the row's K values held by lanes c, c + 16, c + 32, c + 48
            float sm = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s)
                sm += ((x[s][0] + x[s][1]) + (x[s][2] + x[s][3])) +
                      ((x[s][4] + x[s][5]) + (x[s][6] + x[s][7]));
            const float mean = xg_sum_rs(sm) / (float)p.K;
            float sq = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const bool in = 32 * s + 8 * g < p.K;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float d = in ? x[s][e] - mean : 0.f;
                    sq += d * d;
                }
            }
            const float rstd = 1.0f / sqrtf(xg_sum_rs(sq) / (float)p.K + p.eps);
            if constexpr (LNM == 3) {
                // the side output first, fenced off from the add loads below (scheduled
                // together they exceed the 256 registers of two waves per SIMD)
                if (grp == 0 && mw + 16 * i + c < p.M) {
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        const int k = 32 * s + 8 * g;
                        if (k < p.K) {
                            const float4 h0 = lng2[k / 4], h1 = lng2[k / 4 + 1];
                            const float4 c0 = lnb2[k / 4], c1 = lnb2[k / 4 + 1];
                            float* o2 = p.ln_out2 + row * p.ld_out2 + k;
                            *reinterpret_cast<float4*>(o2) = make_float4(
                                (x[s][0] - mean) * rstd * h0.x + c0.x, (x[s][1] - mean) * rstd * h0.y + c0.y,
                                (x[s][2] - mean) * rstd * h0.z + c0.z, (x[s][3] - mean) * rstd * h0.w + c0.w);
                            *reinterpret_cast<float4*>(o2 + 4) = make_float4(
                                (x[s][4] - mean) * rstd * h1.x + c1.x, (x[s][5] - mean) * rstd * h1.y + c1.y,
                                (x[s][6] - mean) * rstd * h1.z + c1.z, (x[s][7] - mean) * rstd * h1.w + c1.w);
                        }
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                // no branches around the loads (all in flight); chunks past K zeroed below
                const int kl = min(32 * s + 8 * g, p.K - 8);
                const float4 g0 = lng[kl / 4], g1 = lng[kl / 4 + 1];
                const float4 b0 = lnb[kl / 4], b1 = lnb[kl / 4 + 1];
                float4 d0 = make_float4(0.f, 0.f, 0.f, 0.f), d1 = d0;
                if constexpr (LNM >= 2) {
                    const float* dr = p.ln_add + row * p.ld_add + kl;
                    d0 = *reinterpret_cast<const float4*>(dr);
                    d1 = *reinterpret_cast<const float4*>(dr + 4);
                }
                const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
                const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
                const float dd[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) x[s][e] = (x[s][e] - mean) * rstd * gg[e] + bb[e] + dd[e];
            }
#pragma unroll
            for (int s = 0; s < KS; ++s)
                if (32 * s + 8 * g >= p.K)
#pragma unroll
                    for (int e = 0; e < 8; ++e) x[s][e] = 0.f;
        }
        float mx = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            mx = fmaxf(mx, max3_abs(x[s][0], x[s][1], x[s][2]));
            mx = fmaxf(mx, max3_abs(x[s][3], x[s][4], x[s][5]));
            mx = fmaxf(mx, max3_abs(x[s][6], x[s][7], 0.f));
        }
        mx = xg_max_rs(mx);
        // max * 2^e in [2^14, 2^15) (e = 0 for an all-zero row)
        const int e = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
        rs[i] = __builtin_ldexpf(1.f, -e);
        const float sc = __builtin_ldexpf(1.f, e);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            u32x4 h, l;
            split8_f16(x[s], sc, h, l);
            af[i][s][0] = __builtin_bit_cast(f16x8, h);
            af[i][s][1] = __builtin_bit_cast(f16x8, l);
        }
    }
    // the block's column scales and bias, by (panel, g) float4 (read by the epilogues)
    for (int u = tid; u < np * 4; u += 256) {
        const int n = p0 * 16 + 4 * u;
        colw[u] = *reinterpret_cast<const float4*>(p.wsc + n);
        float e[4] = {0.f, 0.f, 0.f, 0.f};
        if (p.bias)
            for (int j = 0; j < 4 && n + j < p.N; ++j) e[j] = p.bias[n + j];
        colb[u] = make_float4(e[0], e[1], e[2], e[3]);
        if constexpr (HEAD) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
                colh[j * kRsMaxNc * 4 + u] = *reinterpret_cast<const float4*>(p.w4 + (int64_t)j * p.N + n);
        }
    }
    // KV: the running max of the current head's 8 values per lane (two panels; the values in
    // kvbuf), and the head (+1) whose image is due after the next barrier (0: none)
    float kvm = 0.f;
    int kv_pend = 0;
    auto kv_finish = [&]() {
        const int hd = kv_pend - 1;
        kv_pend = 0;
        const float tm = fmaxf(fmaxf(kvred[hd & 1][0], kvred[hd & 1][1]),
                               fmaxf(kvred[hd & 1][2], kvred[hd & 1][3]));
        const int isv = hd >= p.n_head ? 1 : 0, head = hd - isv * p.n_head;
        const int e = tm > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(tm), 127) : 0;
        const float sc = __builtin_ldexpf(1.f, e);
        const int64_t tile = (int64_t)bm * p.n_head + head;
        if (tid == 0) reinterpret_cast<int*>(p.kv_sc + tile)[isv] = e;
        char* base = p.kv_img + tile * (kKvUnits * 16);
        // lane -> (key kl of the wave's 16, 8-dim group gq): one whole 16-B unit per term
        const int kl = lane >> 2, gq = lane & 3;
        const int key = wv * 16 + kl;
        const float4 a0 = kvbuf[wv][kl][2 * gq], a1 = kvbuf[wv][kl][2 * gq + 1];
        const float xv[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        _Float16 tv[2][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float x = xv[j] * sc;
            tv[0][j] = (_Float16)x;
            tv[1][j] = (_Float16)(x - (float)tv[0][j]);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            char* dst;
            if (isv)                                        // [term][key][32] f16, chunks ^ v_swz
                dst = base + kKvUnitV * 16 + t * (128 * 32) + key * 64 + (gq ^ (((key >> 2) & 1) << 1)) * 16;
            else                                            // [term][g'][key] x 8 dims
                dst = base + ((t * 4 + gq) * 64 + key) * 16;
            *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(tv[t]);
        }
    };
    float h3[RT][3];
    if constexpr (HEAD) {
#pragma unroll
        for (int i = 0; i < RT; ++i) h3[i][0] = h3[i][1] = h3[i][2] = 0.f;
    }

    // row tiles of this wave with at least one row < M (a tile past M is skipped by the wave)
    int nst = 0;
#pragma unroll
    for (int i = 0; i < RT; ++i) nst += (mw + 16 * i < p.M) ? 1 : 0;
    auto load_res = [&](int q, float4 (&rv)[RT]) {
        const int n = (p0 + q) * 16 + 4 * g;
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const int64_t row = min(mw + 16 * i + c, p.M - 1);
            rv[i] = *reinterpret_cast<const float4*>(p.R + row * p.ldr + n);
        }
    };
    // vector stores a wave issues in panel qq's epilogue (counted by the waits below; an
    // over-count would let a panel's DMA still be in flight when it is read)
    auto nstore = [&](int qq) -> int {
        if constexpr (HEAD) return 0;
        const int col = (p0 + qq) * 16;
        // KV panels store nothing in their epilogue (their image stores come after the next
        // barrier and are not counted: an under-count only makes a wait stricter)
        if constexpr (KV)
            if (col >= p.kv_col0) return 0;
        if (p.c2 && col >= p.n_act) return col == p.n_act ? nst : 0;
        return nst;
    };
    typedef __attribute__((address_space(3))) u32x4 lds_u4;
    // panel q's pure MFMA loop (W fragments from the LDS ring, A resident)
    auto panel_mfma = [&](int q, f32x4 (&acc)[RT]) {
        const uint32_t base = (uint32_t)(uintptr_t)(ring + (q % NB) * PANEL_U) +
                              (uint32_t)(g * 16 + c) * 16;
#pragma unroll
        for (int i = 0; i < RT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        // the fragments of RS_LA k-steps are read ahead of their MFMAs, pinned in that order by
        // sched_group_barrier (left to itself the scheduler issued each ds_read right before
        // its MFMA with an lgkmcnt(0) wait in between: one exposed LDS latency per k-step)
        // (K <= 128: none -- the extra registers cost occupancy there, 4 blocks per CU:
        // 11472 x 896 x 128 24.4 -> 27.9 us with it, profiles/r05_rs_lookahead_ab.txt)
        constexpr int LA_ = KS <= 4 ? 0 : (KS < kRsLookahead ? KS : kRsLookahead);
        if constexpr (LA_ == 0) {
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const f16x8 wh = __builtin_bit_cast(f16x8, *(lds_u4*)(uintptr_t)(base + (s * 2 + 0) * 64 * 16));
                const f16x8 wl = __builtin_bit_cast(f16x8, *(lds_u4*)(uintptr_t)(base + (s * 2 + 1) * 64 * 16));
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, af[i][s][0], acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][s][1], acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, af[i][s][0], acc[i], 0, 0, 0);
                }
            }
            return;
        }
        f16x8 wf[KS][2];
        auto rd = [&](int s) {
            wf[s][0] = __builtin_bit_cast(f16x8, *(lds_u4*)(uintptr_t)(base + (s * 2 + 0) * 64 * 16));
            wf[s][1] = __builtin_bit_cast(f16x8, *(lds_u4*)(uintptr_t)(base + (s * 2 + 1) * 64 * 16));
        };
#pragma unroll
        for (int s = 0; s < LA_; ++s) rd(s);
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * (LA_ > 0 ? LA_ : 1), 0);   // DS reads
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s + LA_ < KS) rd(s + LA_);
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][1], af[i][s][0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][0], af[i][s][1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][0], af[i][s][0], acc[i], 0, 0, 0);
            }
            if (s + LA_ < KS) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // next reads
            __builtin_amdgcn_sched_group_barrier(0x008, 3 * RT, 0);                // this step's MFMAs
        }
    };
    // panel q's epilogue: lane holds C[row = mw + 16i + c][n .. n + 3]
    auto epilogue = [&](int q, const f32x4 (&acc)[RT], const float4 (&rv)[RT]) {
        const int n = (p0 + q) * 16 + 4 * g;
        const float4 ws = colw[q * 4 + g], bv = colb[q * 4 + g];
        if constexpr (KV) {
            const int col = (p0 + q) * 16;
            if (col >= p.kv_col0) {                         // panel-uniform: a K or V panel
                const int rel = col - p.kv_col0;
                const int half = (rel >> 4) & 1;
                const float s0 = rs[0] * ws.x, s1 = rs[0] * ws.y, s2 = rs[0] * ws.z, s3 = rs[0] * ws.w;
                const bool ok = mw + c < p.M;               // rows past M: zeros, not in the max
                const float y0 = ok ? acc[0][0] * s0 + bv.x : 0.f, y1 = ok ? acc[0][1] * s1 + bv.y : 0.f;
                const float y2 = ok ? acc[0][2] * s2 + bv.z : 0.f, y3 = ok ? acc[0][3] * s3 + bv.w : 0.f;
                const float mx = max3_abs(y0, y1, fmaxf(fabsf(y2), fabsf(y3)));
                // parked in LDS (registers are at their limit in the LN prologue's kernel): dims
                // 16 half + 4g .. + 3 of key c are quad 4 half + g
                kvbuf[wv][c][4 * half + g] = make_float4(y0, y1, y2, y3);
                if (half == 0) {
                    kvm = mx;
                } else {
                    const float wm = xg_max_rs(row16_max(fmaxf(kvm, mx)));   // DPP + permlanes
                    const int hd = rel >> 5;                    // head index over [K heads | V heads]
                    if (lane == 0) kvred[hd & 1][wv] = wm;
                    kv_pend = 1 + hd;                           // finalised after the next barrier
                }
                return;
            }
        }
        if constexpr (HEAD) {
            // the ReLU'd outputs against coor_mlp[4]'s rows, fp32, not stored
            const float4 w0 = colh[q * 4 + g], w1 = colh[kRsMaxNc * 4 + q * 4 + g],
                         w2 = colh[2 * kRsMaxNc * 4 + q * 4 + g];
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const float s0 = rs[i] * ws.x, s1 = rs[i] * ws.y, s2 = rs[i] * ws.z, s3 = rs[i] * ws.w;
                const float y0 = finish_ct<ACT, false>(acc[i][0] * s0, bv.x, 0.f);
                const float y1 = finish_ct<ACT, false>(acc[i][1] * s1, bv.y, 0.f);
                const float y2 = finish_ct<ACT, false>(acc[i][2] * s2, bv.z, 0.f);
                const float y3 = finish_ct<ACT, false>(acc[i][3] * s3, bv.w, 0.f);
                h3[i][0] = fmaf(y3, w0.w, fmaf(y2, w0.z, fmaf(y1, w0.y, fmaf(y0, w0.x, h3[i][0]))));
                h3[i][1] = fmaf(y3, w1.w, fmaf(y2, w1.z, fmaf(y1, w1.y, fmaf(y0, w1.x, h3[i][1]))));
                h3[i][2] = fmaf(y3, w2.w, fmaf(y2, w2.z, fmaf(y1, w2.y, fmaf(y0, w2.x, h3[i][2]))));
            }
        } else if ((p0 + q) * 16 >= p.n_act) {            // panel-uniform: no activation
            if (p.c2 && (p0 + q) * 16 == p.n_act && g == 0) {
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    const int64_t row = mw + 16 * i + c;
                    if (row < p.M) p.c2[row] = acc[i][0] * (rs[i] * ws.x) + bv.x;
                }
            } else if (!p.c2) {
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    const int64_t row = mw + 16 * i + c;
                    const float s0 = rs[i] * ws.x, s1 = rs[i] * ws.y, s2 = rs[i] * ws.z, s3 = rs[i] * ws.w;
                    float4 r4 = make_float4(0.f, 0.f, 0.f, 0.f);
                    if constexpr (RES) r4 = rv[i];
                    const float4 y = make_float4(finish_ct<FGR_ACT_NONE, RES>(acc[i][0] * s0, bv.x, r4.x),
                                                 finish_ct<FGR_ACT_NONE, RES>(acc[i][1] * s1, bv.y, r4.y),
                                                 finish_ct<FGR_ACT_NONE, RES>(acc[i][2] * s2, bv.z, r4.z),
                                                 finish_ct<FGR_ACT_NONE, RES>(acc[i][3] * s3, bv.w, r4.w));
                    if (row < p.M) *reinterpret_cast<float4*>(p.C + row * p.ldc + n) = y;
                }
            }
        } else {                                           // N % 16 == 0: every panel in range
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const int64_t row = mw + 16 * i + c;
                const float s0 = rs[i] * ws.x, s1 = rs[i] * ws.y, s2 = rs[i] * ws.z, s3 = rs[i] * ws.w;
                float4 r4 = make_float4(0.f, 0.f, 0.f, 0.f);
                if constexpr (RES) r4 = rv[i];
                const float4 y = make_float4(finish_ct<ACT, RES>(acc[i][0] * s0, bv.x, r4.x),
                                             finish_ct<ACT, RES>(acc[i][1] * s1, bv.y, r4.y),
                                             finish_ct<ACT, RES>(acc[i][2] * s2, bv.z, r4.z),
                                             finish_ct<ACT, RES>(acc[i][3] * s3, bv.w, r4.w));
                if (row < p.M) *reinterpret_cast<float4*>(p.C + row * p.ldc + n) = y;
            }
        }
    };

#ifdef FGR_RS_STAMP
    st_[2] = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (PPS == 1) {
        float4 rcur[RT];
        f32x4 prev[RT];
        for (int q = 0; q < np; ++q) {
            // vector-memory ops issued after panel q's DMA (issued in iteration q - 2), counted so
            // that vmcnt guarantees that DMA has landed: the epilogue stores of iteration q - 2
            // (panel q - 3), then iteration q - 1's [residual loads, not counted: waiting for them
            // too is merely stricter], DMA of panel q + 1 if any, and its epilogue stores (panel
            // q - 2)
            static_assert(PPS > 1 || LA == 2, "the wait counts below assume two panels in flight");
    #if defined(FGR_RS_WAIT0)
            wait_vm_lgkm0_rs<0>();
    #else
            if (q == 0) wait_vm_lgkm0_dyn(np > 1 ? PW : 0);
            else wait_vm_lgkm0_dyn((q >= 3 ? nstore(q - 3) : 0) + (q >= 2 ? nstore(q - 2) : 0) +
                                   (q + 1 < np ? PW : 0));
    #endif
            __builtin_amdgcn_s_barrier();                    // every wave's pieces; buffer of q - 1 free
    #ifdef FGR_RS_STAMP
            if (q == 0) st_[3] = __builtin_amdgcn_s_memtime();
            if (q == np - 1) st_[4] = __builtin_amdgcn_s_memtime();
    #endif
            if constexpr (KV)
                if (kv_pend) kv_finish();                    // block-uniform
            if constexpr (RES)
                if (q >= 1) load_res(q - 1, rcur);
            if (q + LA < np) dma(q + LA);
            f32x4 acc[RT];
            panel_mfma(q, acc);
    #ifdef FGR_RS_MFMA2
            {   // diagnostic build only (timing probe, wrong results): the panel's MFMA work twice
                f32x4 acc2[RT];
                panel_mfma(q, acc2);
    #pragma unroll
                for (int i = 0; i < RT; ++i) acc[i] += acc2[i];
            }
    #endif
            // the previous panel's epilogue after this panel's MFMAs: its VALU and stores issue in
            // the MFMA shadows instead of between two panels' matrix work (measured 1.09-1.17x on
            // the LN-fused and 57264-row shapes, equal elsewhere: profiles/r04_rs_defer_ab.txt)
            if (q >= 1) epilogue(q - 1, prev, rcur);
    #pragma unroll
            for (int i = 0; i < RT; ++i) prev[i] = acc[i];
        }
        if constexpr (RES) load_res(np - 1, rcur);
        epilogue(np - 1, prev, rcur);
    } else {
        // stages of PPS panels: stage st = panels st * PPS .. + PPS - 1 (those < np), ring slots
        // (st & 1) * PPS + j. Iteration st issues: [wait: DMA of stage st landed] [barrier]
        // [K/V image stores of the previous head] [residual loads of stage st - 1] [DMA of stage
        // st + 1] [MFMAs of stage st] [epilogue stores of stage st - 1]; the ops younger than
        // stage st's DMA (issued in iteration st - 1) are that iteration's epilogue stores
        // (stage st - 2): the wait leaves exactly those outstanding
        const int nstage = (np + PPS - 1) / PPS;
        float4 rcur[PPS][RT];
        f32x4 prev[PPS][RT];
        for (int st = 0; st < nstage; ++st) {
            const int qa = st * PPS;
            {
                int cnt = 0;
                if (st >= 2)
#pragma unroll
                    for (int j = 0; j < PPS; ++j)
                        if (qa - 2 * PPS + j < np) cnt += nstore(qa - 2 * PPS + j);
                wait_vm_lgkm0_dyn(cnt);
            }
            __builtin_amdgcn_s_barrier();                    // every wave's pieces; stage st - 1's slots free
#ifdef FGR_RS_STAMP
            if (st == 0) st_[3] = __builtin_amdgcn_s_memtime();
            if (st == nstage - 1) st_[4] = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (KV)
                if (kv_pend) kv_finish();                    // block-uniform
            if constexpr (RES)
                if (st >= 1)
#pragma unroll
                    for (int j = 0; j < PPS; ++j) load_res(qa - PPS + j, rcur[j]);
#pragma unroll
            for (int j = 0; j < PPS; ++j)
                if (qa + PPS + j < np) dma(qa + PPS + j);
            f32x4 acc[PPS][RT];
#pragma unroll
            for (int j = 0; j < PPS; ++j)
                if (qa + j < np) panel_mfma(qa + j, acc[j]);     // block-uniform
#ifdef FGR_RS_MFMA2
#pragma unroll
            for (int j = 0; j < PPS; ++j)
                if (qa + j < np) {   // diagnostic build only (timing probe, wrong results)
                    f32x4 acc2[RT];
                    panel_mfma(qa + j, acc2);
#pragma unroll
                    for (int i = 0; i < RT; ++i) acc[j][i] += acc2[i];
                }
#endif
            if (st >= 1)
#pragma unroll
                for (int j = 0; j < PPS; ++j) epilogue(qa - PPS + j, prev[j], rcur[j]);
#pragma unroll
            for (int j = 0; j < PPS; ++j)
#pragma unroll
                for (int i = 0; i < RT; ++i) prev[j][i] = acc[j][i];
        }
        const int ql = (nstage - 1) * PPS;
        if constexpr (KV) {
            // the head completed by the loop's last epilogue (stage nstage - 2) before the last
            // stage's epilogue refills kvbuf
            if (kv_pend) {                                   // block-uniform
                __syncthreads();
                kv_finish();
                __syncthreads();
            }
        }
#pragma unroll
        for (int j = 0; j < PPS; ++j) {
            if (ql + j >= np) break;                         // block-uniform
            if constexpr (RES) load_res(ql + j, rcur[j]);
            epilogue(ql + j, prev[j], rcur[j]);
        }
    }
    if constexpr (KV) {
        if (kv_pend) {                                   // the last head of the block
            __syncthreads();
            kv_finish();
        }
    }
#ifdef FGR_RS_STAMP
    __syncthreads();
    st_[5] = __builtin_amdgcn_s_memtime();
    st_[6] = __builtin_amdgcn_s_memrealtime();
    st_[7] = (unsigned long long)np;
    if (tid < 8 && blockIdx.x < (1 << 14)) g_rs_stamp[blockIdx.x][tid] = st_[tid];
#endif
    if constexpr (HEAD) {
        // sum the lane groups' column quads: lanes c, c + 16, c + 32, c + 48 hold one row
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const int64_t row = mw + 16 * i + c;
            const float t0 = xg_sum_rs(h3[i][0]), t1 = xg_sum_rs(h3[i][1]), t2 = xg_sum_rs(h3[i][2]);
            if (g == 0 && row < p.M) {
                p.out3[row * 3 + 0] = t0 + p.b4[0];
                p.out3[row * 3 + 1] = t1 + p.b4[1];
                p.out3[row * 3 + 2] = t2 + p.b4[2];
            }
        }
    }
}

template <int RT, int KS, int ACT>
void launch_rs_act(const RsArgs& a, unsigned blocks, hipStream_t st) {
    if constexpr (RT == 1 && ACT == FGR_ACT_NONE && KS == 8) {
        if (a.ln_g && a.ln_add && a.kv_img) {
            if (a.ln_out2)
                hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, false, ACT, 3, false, true>), dim3(blocks), dim3(256), 0, st, a);
            else
                hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, false, ACT, 2, false, true>), dim3(blocks), dim3(256), 0, st, a);
            return;
        }
    }
    // LN prologue: one row tile per wave (at two, the row + add registers of the prologue
    // exceed the 256 VGPRs of two waves per SIMD and spill), no residual (checked by the caller)
    if constexpr (RT == 1 && ACT != FGR_ACT_RELU_RES_LEAKY) {
        if (a.ln_g && a.ln_add && a.ln_out2) {
            hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, false, ACT, 3>), dim3(blocks), dim3(256), 0, st, a);
            return;
        }
        if (a.ln_g && a.ln_add) {
            hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, false, ACT, 2>), dim3(blocks), dim3(256), 0, st, a);
            return;
        }
        if (a.ln_g) {
            hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, false, ACT, 1>), dim3(blocks), dim3(256), 0, st, a);
            return;
        }
    }
    if constexpr (ACT == FGR_ACT_RELU) {
        if (a.out3) {
            hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, false, ACT, 0, true>), dim3(blocks), dim3(256), 0, st, a);
            return;
        }
    }
    if (a.R)
        hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, true, ACT, 0>), dim3(blocks), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((gemm_rs_kernel<RT, KS, false, ACT, 0>), dim3(blocks), dim3(256), 0, st, a);
}

template <int RT, int KS>
bool launch_rs_k(const RsArgs& a, unsigned blocks, hipStream_t st) {
    switch (a.act) {
        case FGR_ACT_RELU: launch_rs_act<RT, KS, FGR_ACT_RELU>(a, blocks, st); return true;
        case FGR_ACT_RELU_RES_LEAKY: launch_rs_act<RT, KS, FGR_ACT_RELU_RES_LEAKY>(a, blocks, st); return true;
        default: launch_rs_act<RT, KS, FGR_ACT_NONE>(a, blocks, st); return true;
    }
}

}  // namespace

// The rs kernel applies to K <= 256, K % 8 == 0, N % 16 == 0 with 16-B aligned A / C / R / bias rows
// (checked by the caller). ksteps = the image's k32-steps (even, <= 8). `ln` (optional, no R):
// the LayerNorm prologue's gamma, beta, add (16-B aligned rows), ld_add and eps.
struct RsLn {
    const float* g; const float* b; const float* add; int64_t ld_add; float eps;
    const float* g2; const float* b2; float* out2; int64_t ld_out2;    // optional side output
    char* kv_img; int2* kv_sc; int n_head; int kv_col0;                // optional K / V images
};
// the correspondence-head epilogues (see the top of this file): n_act / c2, or out3 with w4 / b4
struct RsHead {
    int n_act; float* c2;
    const float* w4; const float* b4; float* out3;
};
bool gemm_rs_f16x3(const float* A, int64_t lda, const void* W, int ksteps, const float* wsc,
                   float* C, int64_t ldc, const float* bias, const float* R, int64_t ldr, int M,
                   int N, int K, int act, hipStream_t st, const RsLn* ln, const RsHead* head) {
    if (K % 8 != 0 || N % 16 != 0 || ksteps > 8 || ksteps % 2 != 0) return false;
    if (ln && (R || (ln->out2 && !ln->add))) return false;
    if (head && (ln || R || (head->out3 && (act != FGR_ACT_RELU || N / 16 > kRsMaxNc)) ||
                 head->n_act % 16 != 0))
        return false;
    // row tiles per wave: 2 (W fragments reused twice) unless that leaves too few blocks
    const char* rte = getenv("FGR_RS_RT");
    int RT = (rte && rte[0]) ? atoi(rte) : 2;
    if (RT != 1 && RT != 2) RT = 2;
    if (ln) RT = 1;
    const int npanel = (N + 15) / 16;
    const int nbm = (M + 64 * RT - 1) / (64 * RT);
    // panels per block: as few column groups as fill the resident-block slots once (a second,
    // partial round of blocks costs a whole block time; every group re-reads and re-splits its
    // rows): slots = 256 CUs x blocks per CU (2 at K > 128, 188 VGPRs; 4 below).
    // FGR_RS_NC overrides (0: ~3 blocks per CU regardless of occupancy)
    const char* nce = getenv("FGR_RS_NC");
    int nc;
    if (nce && nce[0]) {
        nc = atoi(nce);
        if (nc <= 0) {
            const int64_t target = 768;
            nc = (int)std::max<int64_t>(1, std::min<int64_t>(npanel, ((int64_t)nbm * npanel + target - 1) / target));
        }
    } else {
        // (the LN prologue at RT 1: 256 / 190 VGPRs at ksteps 8 / 6 -> 2 blocks per CU, 4 below)
        const int slots = ln ? 256 * (ksteps > 4 ? 2 : 4)
                             : 256 * (ksteps > 4 ? 2 : 4) * (RT == 1 ? 2 : 1);
        const int ngrp = std::max(1, slots / std::max(nbm, 1));
        nc = (npanel + ngrp - 1) / ngrp;
    }
    nc = std::min(std::min(nc, npanel), kRsMaxNc);
    if (head && head->out3) nc = npanel;              // the 3-wide head needs whole rows
    if (ln && ln->kv_img) {
        // K / V images: head dim 32 (two panels per head, never split between blocks), the
        // k | v columns the last 64 n_head, one 64-row tile per block (RT = 1, K = 256)
        if (ksteps != 8 || ln->n_head <= 0 || ln->kv_col0 % 32 != 0 ||
            N != ln->kv_col0 + 64 * ln->n_head)
            return false;
        nc += nc & 1;
    }
    const int ngrp = (npanel + nc - 1) / nc;
    const unsigned blocks = (unsigned)((int64_t)nbm * ngrp);
    RsArgs a{A, lda, (const u32x4*)W, wsc, C, ldc, bias, R, ldr, M, N, K, act, nc,
             ln ? ln->g : nullptr, ln ? ln->b : nullptr, ln ? ln->add : nullptr,
             ln ? ln->ld_add : 0, ln ? ln->eps : 0.f, ln ? ln->g2 : nullptr,
             ln ? ln->b2 : nullptr, ln ? ln->out2 : nullptr, ln ? ln->ld_out2 : 0,
             head ? head->n_act : N, head ? head->c2 : nullptr, head ? head->w4 : nullptr,
             head ? head->b4 : nullptr, head ? head->out3 : nullptr,
             ln ? ln->kv_img : nullptr, ln ? ln->kv_sc : nullptr, ln ? ln->n_head : 0,
             ln ? ln->kv_col0 : N};
#define RS_CASE(rt, ks) \
    if (RT == rt && ksteps == ks) return launch_rs_k<rt, ks>(a, blocks, st);
    RS_CASE(2, 2) RS_CASE(2, 4) RS_CASE(2, 6) RS_CASE(2, 8)
    RS_CASE(1, 2) RS_CASE(1, 4) RS_CASE(1, 6) RS_CASE(1, 8)
#undef RS_CASE
    return false;
}

}  // namespace fgr

#ifdef FGR_RS_STAMP
extern "C" int fgr_debug_rs_stamps(void* dst, int32_t nblocks) {
    if (nblocks > (1 << 14)) nblocks = 1 << 14;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rs_stamp), (size_t)nblocks * 64, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
