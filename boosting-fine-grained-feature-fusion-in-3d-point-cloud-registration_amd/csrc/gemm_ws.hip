// "ws" (weight-split row-stationary) f16x3 GEMM for K = 256 over many rows:
//
//   C[M, N] = act(A[M, 256] . W[N, 256]^T + bias[N] (+ R[M, N])),   N = 64 NPW
//
// with the row-stationary kernel's options (gemm_rs.hip): a LayerNorm prologue (+ row add,
// + a second LayerNorm output of the same rows) and the K / V attention images of head dim 32
// written by the epilogue (the pre-norm transformer's in_proj, transformers.py:193-196,
// :213-221).
//
// Why. The rs kernel gives each wave 16 rows and streams every W panel through LDS to all four
// waves of a block (LDS-DMA, a barrier per panel): per 16 KB panel a CU issues 16 DMA pieces,
// reads 64 KB of fragments and meets at a barrier for 96 MFMAs. Its panel time is ~1 us against
// 0.16 us of MFMA work (profiles/r04_rs_stamp_phases.txt), and the fused feed-forward kernel
// built that way measured the cost directly (ffn.hip, version 1: 446 cycles of DMA / read issue
// and 209 of DMA wait per 384-cycle unit). Here the WAVES SPLIT THE WEIGHTS: a block owns 64
// rows; they are loaded, (LayerNorm'd,) scaled by one power of two per row and split ONCE into
// an LDS image (4 row tiles x 8 k32 steps x 2 terms, 64 KB); wave w owns output panels
// w NPW .. (w + 1) NPW - 1 and reads their W fragments straight from global memory (L2) into
// registers -- every weight byte by one wave only, two 4-panel k32 groups ahead of the MFMAs --
// multiplying them against the 4 row tiles' fragments from LDS (read one k32 step ahead). No
// barrier after the prologue. Passes of 4 panels (64 accumulators per lane).
//
// K / V images (KV): each pass of a wave covers two whole heads (32 columns each) of all 64 rows
// of the block's global 64-row tile, so the tile's power-of-two exponent (max |.| in
// [2^14, 2^15), as attn_kv_image16_kernel) is a reduction inside the wave; the split terms go
// to the attention16.hip image layout (K [term][dim group][key], V [term][key][32] with the
// v_swz chunk swizzle) with 8-B stores (4 dims x fp16 per lane and term).
//
// Precision: as gemm_rs.hip (one scale per activation row, three fp16 products per product).
#include "common.h"

#ifdef FGR_WS_STAMP
// Diagnostic build only (tools/ws_bench.py): per (block, wave) s_memtime stamps: [0] entry,
// [1] after the prologue barrier, [2 + 2 p] pass p's MFMA loop done, [3 + 2 p] its epilogue done,
// [7] (one pass) the wave's stores complete
__device__ unsigned long long g_ws_stamp[2048][4][8];
#endif

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWsKS = 8;                 // k32 steps (K = 256)
constexpr int kWsPanelU = kWsKS * 128;   // 16-B units per W panel of the image
#ifndef FGR_WS_RING
#define FGR_WS_RING 3
#endif
constexpr int kWsRing = FGR_WS_RING;     // register ring of k32 groups (kWsRing - 1 in flight)
static_assert(kWsRing >= 2 && kWsRing <= 8, "vmcnt holds at most 63");
constexpr int kKvUnitsWs = 1024;         // attention16.hip units<32>: 16-B units per (tile, head)
constexpr int kKvUnitVWs = 512;          //   V from unit 512

struct WsArgs {
    const float* A; int64_t lda;
    const u32x4* W; const float* wsc; const float* bias;
    float* C; int64_t ldc;
    const float* R; int64_t ldr;
    int M, N;
    const float* ln_g; const float* ln_b; float eps;
    const float* add; int64_t ld_add;
    const float* g2; const float* b2; float* out2; int64_t ld_out2;
    char* kv_img; int2* kv_sc; int n_head, kv_col0;
};

__device__ __forceinline__ float xg_sum_w(float v) {      // sum over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float xg_max_w(float v) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// s_waitcnt vmcnt(N) only (lgkmcnt / expcnt untouched)
template <int N>
__device__ __forceinline__ void wait_vm_ws() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// vmcnt(8 n) for a (compile-time after unrolling) n in [0, 7]
__device__ __forceinline__ void wait_groups_ws(int n) {
    switch (n) {
        case 0: wait_vm_ws<0>(); break;   case 1: wait_vm_ws<8>(); break;
        case 2: wait_vm_ws<16>(); break;  case 3: wait_vm_ws<24>(); break;
        case 4: wait_vm_ws<32>(); break;  case 5: wait_vm_ws<40>(); break;
        case 6: wait_vm_ws<48>(); break;  default: wait_vm_ws<56>(); break;
    }
}

template <int ACT, bool RES>
__device__ __forceinline__ float finish_ws(float y, float b, float r) {
    float t = y + b;
    if constexpr (RES) t += r;
    if constexpr (ACT == FGR_ACT_RELU) t = fmaxf(t, 0.f);
    return t;
}

// LNM: 0 plain A, 1 LayerNorm(A), 2 LayerNorm(A) + add, 3 as 2 plus out2 = LayerNorm(A) g2 + b2
//
// Memory-order rule of the schedule: vmcnt counts loads AND stores in issue order, so a store
// issued before a weight group delays every later wait for weights until it has completed (the
// round-6 first form stored each pass's outputs between passes: ~6-8k cycles per pass, stamped).
// So every store of the block waits for the end: the finished values of all but the last pass
// stay in registers (64 per pass and lane), the side output (LNM 3) in LDS, and the stores go
// out after the last MFMA. The first weight groups are requested with the rows, and the column
// scales / bias sit in LDS.
// NPART > 1: the output columns split over NPART blocks per row tile (each NPW panels per
// wave), the row tile's blocks adjacent in the XCD order (one L2 serves their row loads)
template <int NPW, int LNM, bool KV, bool RES, int ACT, int RT, int NPART>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((NPART > 1 && !RES) ? 2 : 1)))
gemm_ws_kernel(WsArgs p) {
    static_assert(NPW % 4 == 0, "passes of 4 panels");
    static_assert(RT >= 1 && RT <= 4 && (!KV || RT == 4), "row tiles (K / V images: 64-row tiles)");
    constexpr int BR = 16 * RT;                           // rows per block
    static_assert(!KV || (LNM >= 2 && !RES && ACT == FGR_ACT_NONE), "K / V images: the in_proj");
    constexpr int NPASS = NPW / 4;
    constexpr int N = 64 * NPW;
    // RES, one pass: the residual is loaded with the weights and added before the activation;
    // several passes (registers): fin holds y + b and the store stage adds the residual
    constexpr bool kResEarly = RES && NPASS == 1;
    __shared__ u32x4 act[RT * kWsKS * 2 * 64];            // [row tile][k32 step][term][lane]
    __shared__ float rowrs[BR];                           // per row: 2^-e
    __shared__ float4 colw[N / 4], colb[N / 4];           // per column: 2^-e_n, bias
    __shared__ float4 lng[LNM ? 64 : 1], lnb[LNM ? 64 : 1];
    __shared__ float4 lng2[LNM == 3 ? 64 : 1], lnb2[LNM == 3 ? 64 : 1];
    // LNM 3, one block per row tile: the out2 rows staged in LDS, row-major; NPART > 1: the
    // parts recompute them at the end from re-read rows, a k range each (no 64 KB staging: two
    // blocks per CU)
    constexpr bool kSideLds = LNM == 3 && NPART == 1;
    __shared__ float4 side[kSideLds ? BR * 64 : 1];

#ifdef FGR_WS_STAMP
    unsigned long long st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    st_[0] = __builtin_amdgcn_s_memtime();
#endif
    const int nblk = (p.M + BR - 1) / BR * NPART;
    int t = blockIdx.x;
    {   // XCD-aware order: each XCD a contiguous range of (row block, part)
        const int q = nblk / 8, r = nblk % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int part = t % NPART;
    t /= NPART;                                           // the row block
    const int cb4 = part * (N / 4);                       // the part's first column / 4
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const int r0 = t * BR;
    const int rrow = r0 + 16 * min(wv, RT - 1) + c;       // the lane's prologue row (RT < 4: wave 3 idles)
    const int64_t row = min(rrow, p.M - 1);
    const int pw0 = part * 4 * NPW + wv * NPW;            // the wave's first panel

    // 1. loads, in this order (vmcnt is in order): LayerNorm parameters, column scales / bias,
    //    the wave's row tile and its row add, the first weight groups
    float4 lpg = make_float4(0.f, 0.f, 0.f, 0.f), lpb = lpg, lpg2 = lpg, lpb2 = lpg;
    if constexpr (LNM > 0) {
        const int t4 = tid & 63;
        lpg = reinterpret_cast<const float4*>(p.ln_g)[t4];
        lpb = reinterpret_cast<const float4*>(p.ln_b)[t4];
        if constexpr (LNM == 3) {
            lpg2 = reinterpret_cast<const float4*>(p.g2)[t4];
            lpb2 = reinterpret_cast<const float4*>(p.b2)[t4];
        }
    }
    constexpr int NC4 = (N / 4 + 255) / 256;              // column float4s per thread
    float4 pcw[NC4], pcb[NC4];
#pragma unroll
    for (int i = 0; i < NC4; ++i) {
        const int j = min(tid + 256 * i, N / 4 - 1);
        pcw[i] = reinterpret_cast<const float4*>(p.wsc)[cb4 + j];
        pcb[i] = p.bias ? reinterpret_cast<const float4*>(p.bias)[cb4 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __builtin_amdgcn_sched_barrier(0);
    float xr[kWsKS][8];
    float dr[LNM >= 2 ? kWsKS : 1][8];
    {
        const float* ar = p.A + row * p.lda;
#pragma unroll
        for (int s = 0; s < kWsKS; ++s) {
            const float4 a0 = *reinterpret_cast<const float4*>(ar + 32 * s + 8 * g);
            const float4 a1 = *reinterpret_cast<const float4*>(ar + 32 * s + 8 * g + 4);
            xr[s][0] = a0.x; xr[s][1] = a0.y; xr[s][2] = a0.z; xr[s][3] = a0.w;
            xr[s][4] = a1.x; xr[s][5] = a1.y; xr[s][6] = a1.z; xr[s][7] = a1.w;
        }
        if constexpr (LNM >= 2) {
            const float* dp = p.add + row * p.ld_add;
#pragma unroll
            for (int s = 0; s < kWsKS; ++s) {
                const float4 d0 = *reinterpret_cast<const float4*>(dp + 32 * s + 8 * g);
                const float4 d1 = *reinterpret_cast<const float4*>(dp + 32 * s + 8 * g + 4);
                dr[s][0] = d0.x; dr[s][1] = d0.y; dr[s][2] = d0.z; dr[s][3] = d0.w;
                dr[s][4] = d1.x; dr[s][5] = d1.y; dr[s][6] = d1.z; dr[s][7] = d1.w;
            }
        }
    }
    float4 rres[kResEarly ? RT : 1][4];                    // RES, one pass: the residual
    if constexpr (kResEarly) {
        const int col0 = pw0 * 16;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int64_t orow = min(r0 + 16 * rt + c, p.M - 1);
#pragma unroll
            for (int pp = 0; pp < 4; ++pp)
                rres[rt][pp] = *reinterpret_cast<const float4*>(p.R + orow * p.ldr + col0 + 16 * pp + 4 * g);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    auto issue = [&](int G, u32x4 (&slot)[8]) {
        const int pass = G / kWsKS, s = G % kWsKS;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int pp = e >> 1, tt = e & 1;
            slot[e] = p.W[(int64_t)(pw0 + 4 * pass + pp) * kWsPanelU + (s * 2 + tt) * 64 + lane];
        }
    };
    constexpr int NG = NPASS * kWsKS;
    u32x4 ring[kWsRing][8];
#pragma unroll
    for (int G = 0; G < kWsRing - 1; ++G) issue(G, ring[G]);
    __builtin_amdgcn_sched_barrier(0);

    // the parameters and rows landed; the weight groups stay in flight
#pragma unroll
    for (int i = 0; i < NC4; ++i) {
        const int j = tid + 256 * i;
        if (j < N / 4) { colw[j] = pcw[i]; colb[j] = pcb[i]; }
    }
    float ln_mean = 0.f, ln_rstd = 0.f;                   // the lane's row (LNM 3, NPART > 1)
    if constexpr (LNM > 0) {
        if (tid < 64) { lng[tid] = lpg; lnb[tid] = lpb; }
        if constexpr (LNM == 3)
            if (tid < 64) { lng2[tid] = lpg2; lnb2[tid] = lpb2; }
        __syncthreads();
        float sm = 0.f;
#pragma unroll
        for (int s = 0; s < kWsKS; ++s)
            sm += ((xr[s][0] + xr[s][1]) + (xr[s][2] + xr[s][3])) +
                  ((xr[s][4] + xr[s][5]) + (xr[s][6] + xr[s][7]));
        const float mean = xg_sum_w(sm) / 256.f;
        float sq = 0.f;
#pragma unroll
        for (int s = 0; s < kWsKS; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float d = xr[s][e] - mean;
                sq += d * d;
            }
        const float rstd = 1.0f / sqrtf(xg_sum_w(sq) / 256.f + p.eps);
        ln_mean = mean;
        ln_rstd = rstd;
        if (kSideLds && wv < RT) {                        // out2 rows -> LDS (stored at the end)
#pragma unroll
            for (int s = 0; s < kWsKS; ++s) {
                const int k = 32 * s + 8 * g;
                const float4 h0 = lng2[k / 4], h1 = lng2[k / 4 + 1];
                const float4 c0 = lnb2[k / 4], c1 = lnb2[k / 4 + 1];
                float4* o2 = side + (16 * wv + c) * 64 + k / 4;
                o2[0] = make_float4((xr[s][0] - mean) * rstd * h0.x + c0.x, (xr[s][1] - mean) * rstd * h0.y + c0.y,
                                    (xr[s][2] - mean) * rstd * h0.z + c0.z, (xr[s][3] - mean) * rstd * h0.w + c0.w);
                o2[1] = make_float4((xr[s][4] - mean) * rstd * h1.x + c1.x, (xr[s][5] - mean) * rstd * h1.y + c1.y,
                                    (xr[s][6] - mean) * rstd * h1.z + c1.z, (xr[s][7] - mean) * rstd * h1.w + c1.w);
            }
        }
#pragma unroll
        for (int s = 0; s < kWsKS; ++s) {
            const int k = 32 * s + 8 * g;
            const float4 g0 = lng[k / 4], g1 = lng[k / 4 + 1];
            const float4 b0 = lnb[k / 4], b1 = lnb[k / 4 + 1];
            const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
            const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                xr[s][e] = (xr[s][e] - mean) * rstd * gg[e] + bb[e];
                if constexpr (LNM >= 2) xr[s][e] += dr[s][e];
            }
        }
    }
    {   // one power-of-two scale per row (max in [2^14, 2^15)), the split into the row image
        float mx = 0.f;
#pragma unroll
        for (int s = 0; s < kWsKS; ++s) {
            mx = fmaxf(mx, max3_abs(xr[s][0], xr[s][1], xr[s][2]));
            mx = fmaxf(mx, max3_abs(xr[s][3], xr[s][4], xr[s][5]));
            mx = fmaxf(mx, max3_abs(xr[s][6], xr[s][7], 0.f));
        }
        mx = xg_max_w(mx);
        const int e = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
        const float sc = __builtin_ldexpf(1.f, e);
        if (wv < RT) {
#pragma unroll
            for (int s = 0; s < kWsKS; ++s) {
                u32x4 h, l;
                split8_f16(xr[s], sc, h, l);
                act[((wv * kWsKS + s) * 2 + 0) * 64 + lane] = h;
                act[((wv * kWsKS + s) * 2 + 1) * 64 + lane] = l;
            }
            if (g == 0) rowrs[16 * wv + c] = __builtin_ldexpf(1.f, -e);
        }
    }
    // LDS writes done, no vector-memory wait (the weight groups stay in flight)
    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));
    __builtin_amdgcn_s_barrier();
#ifdef FGR_WS_STAMP
    st_[1] = __builtin_amdgcn_s_memtime();
#endif

    // 2. the wave's panels, 4 per pass; k32 group G = pass * 8 + s loads W (panel, s, term)
    auto read_act = [&](int s, u32x4 (&f)[2 * RT]) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            f[2 * rt + 0] = act[((rt * kWsKS + s) * 2 + 0) * 64 + lane];
            f[2 * rt + 1] = act[((rt * kWsKS + s) * 2 + 1) * 64 + lane];
        }
    };
    u32x4 fa[2][2 * RT];
    // finished values of each pass (stored at the end): plain -> 4 floats, KV -> hi / lo
    // halves of 4 dims; [pass][row tile][panel]
    u32x4 fin[NPASS][RT][4];
    int kv_e[NPASS][2];                                   // KV: the pass's two head exponents
    float rs[RT];
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
        const int col0 = (pw0 + 4 * pass) * 16;
        const bool kvp = KV && col0 >= p.kv_col0;          // wave-uniform: two K or V heads
        f32x4 acc[RT][4];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int pp = 0; pp < 4; ++pp) acc[rt][pp] = f32x4{0.f, 0.f, 0.f, 0.f};
        read_act(0, fa[0]);
#pragma unroll
        for (int s = 0; s < kWsKS; ++s) {
            const int G = pass * kWsKS + s;
            if (G + kWsRing - 1 < NG) issue(G + kWsRing - 1, ring[(G + kWsRing - 1) % kWsRing]);
            // group G landed: the groups issued after it may still be in flight
            wait_groups_ws(NG - 1 - G < kWsRing - 1 ? NG - 1 - G : kWsRing - 1);
            u32x4 (&wf)[8] = ring[G % kWsRing];
            u32x4 (&cur)[2 * RT] = fa[s & 1];
            if (s + 1 < kWsKS) read_act(s + 1, fa[(s + 1) & 1]);
            __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);
            if (s + 1 < kWsKS) __builtin_amdgcn_sched_group_barrier(0x100, 2 * RT, 0);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const f16x8 ah = __builtin_bit_cast(f16x8, cur[2 * rt + 0]);
                const f16x8 al = __builtin_bit_cast(f16x8, cur[2 * rt + 1]);
#pragma unroll
                for (int pp = 0; pp < 4; ++pp) {
                    const f16x8 wh = __builtin_bit_cast(f16x8, wf[2 * pp]);
                    const f16x8 wl = __builtin_bit_cast(f16x8, wf[2 * pp + 1]);
                    acc[rt][pp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, acc[rt][pp], 0, 0, 0);
                    acc[rt][pp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, al, acc[rt][pp], 0, 0, 0);
                    acc[rt][pp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, acc[rt][pp], 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 12 * RT, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
#ifdef FGR_WS_STAMP
        if (pass < 3) st_[2 + 2 * pass] = __builtin_amdgcn_s_memtime();
#endif
        // 3. the pass's finished values (no stores): lane holds rows r0 + 16 rt + c, columns
        //    col0 + 16 pp + 4 g .. + 3
        if (pass == 0)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) rs[rt] = rowrs[16 * rt + c];
        if (kvp) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                float y[4][2][4];
                float mx = 0.f;
#pragma unroll
                for (int pp = 0; pp < 2; ++pp) {
                    const int n = col0 + 32 * hh + 16 * pp + 4 * g;
                    const float4 ws = colw[n / 4 - cb4], bv = colb[n / 4 - cb4];
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) {
                        const bool ok = r0 + 16 * rt + c < p.M;      // rows past M: zeros
                        const f32x4 a = acc[rt][2 * hh + pp];
                        y[rt][pp][0] = ok ? a[0] * (rs[rt] * ws.x) + bv.x : 0.f;
                        y[rt][pp][1] = ok ? a[1] * (rs[rt] * ws.y) + bv.y : 0.f;
                        y[rt][pp][2] = ok ? a[2] * (rs[rt] * ws.z) + bv.z : 0.f;
                        y[rt][pp][3] = ok ? a[3] * (rs[rt] * ws.w) + bv.w : 0.f;
                        mx = fmaxf(mx, max3_abs(y[rt][pp][0], y[rt][pp][1], fmaxf(fabsf(y[rt][pp][2]), fabsf(y[rt][pp][3]))));
                    }
                }
                mx = xg_max_w(row16_max(mx));
                const int e = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
                kv_e[pass][hh] = e;
                const float sc = __builtin_ldexpf(1.f, e);
                // the split of two row tiles' 4 dims at once: 16 v_fma_mix (split8_f16, the
                // bits of hi = f16(y sc), lo = f16(y sc - hi))
#pragma unroll
                for (int rt = 0; rt < RT; rt += 2)
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp) {
                        const float v8[8] = {y[rt][pp][0], y[rt][pp][1], y[rt][pp][2], y[rt][pp][3],
                                             y[rt + 1][pp][0], y[rt + 1][pp][1], y[rt + 1][pp][2], y[rt + 1][pp][3]};
                        u32x4 h, l;
                        split8_f16(v8, sc, h, l);
                        fin[pass][rt][2 * hh + pp] = u32x4{h[0], h[1], l[0], l[1]};
                        fin[pass][rt + 1][2 * hh + pp] = u32x4{h[2], h[3], l[2], l[3]};
                    }
            }
        } else {
#pragma unroll
            for (int pp = 0; pp < 4; ++pp) {
                const int n = col0 + 16 * pp + 4 * g;
                const float4 ws = colw[n / 4 - cb4], bv = colb[n / 4 - cb4];
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    float4 r4 = make_float4(0.f, 0.f, 0.f, 0.f);
                    if constexpr (kResEarly) r4 = rres[rt][pp];
                    const f32x4 a = acc[rt][pp];
                    constexpr int A1 = (RES && !kResEarly) ? FGR_ACT_NONE : ACT;
                    const float4 yv = make_float4(finish_ws<A1, kResEarly>(a[0] * (rs[rt] * ws.x), bv.x, r4.x),
                                                  finish_ws<A1, kResEarly>(a[1] * (rs[rt] * ws.y), bv.y, r4.y),
                                                  finish_ws<A1, kResEarly>(a[2] * (rs[rt] * ws.z), bv.z, r4.z),
                                                  finish_ws<A1, kResEarly>(a[3] * (rs[rt] * ws.w), bv.w, r4.w));
                    fin[pass][rt][pp] = __builtin_bit_cast(u32x4, yv);
                }
            }
        }
#ifdef FGR_WS_STAMP
        if (pass < 3) st_[3 + 2 * pass] = __builtin_amdgcn_s_memtime();
#endif
    }

    // 4. every store of the block
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
        const int col0 = (pw0 + 4 * pass) * 16;
        const bool kvp = KV && col0 >= p.kv_col0;
        if (kvp) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int hd = (col0 + 32 * hh - p.kv_col0) >> 5;     // over [K heads | V heads]
                const int isv = hd >= p.n_head ? 1 : 0, head = hd - isv * p.n_head;
                const int64_t tile = (int64_t)t * p.n_head + head;
                if (lane == 0) reinterpret_cast<int*>(p.kv_sc + tile)[isv] = kv_e[pass][hh];
                char* base = p.kv_img + tile * (kKvUnitsWs * 16);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    const int key = 16 * rt + c;
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp) {
                        // dims 16 pp + 4 g .. + 3: dim group gq = 2 pp + g / 2, half g & 1 of its unit
                        const int gq = 2 * pp + (g >> 1);
                        const u32x4 f = fin[pass][rt][2 * hh + pp];
#pragma unroll
                        for (int tt = 0; tt < 2; ++tt) {
                            char* dst;
                            if (isv)
                                dst = base + kKvUnitVWs * 16 + tt * (128 * 32) + key * 64 +
                                      (gq ^ (((key >> 2) & 1) << 1)) * 16 + 8 * (g & 1);
                            else
                                dst = base + ((tt * 4 + gq) * 64 + key) * 16 + 8 * (g & 1);
                            *reinterpret_cast<uint2*>(dst) = tt ? uint2{f[2], f[3]} : uint2{f[0], f[1]};
                        }
                    }
                }
            }
        } else {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const int rr = r0 + 16 * rt + c;
                if (rr < p.M) {
#pragma unroll
                    for (int pp = 0; pp < 4; ++pp) {
                        u32x4 v = fin[pass][rt][pp];
                        if constexpr (RES && !kResEarly) {
                            const float4 r4 = *reinterpret_cast<const float4*>(p.R + (int64_t)rr * p.ldr + col0 + 16 * pp + 4 * g);
                            const float4 y = __builtin_bit_cast(float4, v);
                            v = __builtin_bit_cast(u32x4, make_float4(finish_ws<ACT, true>(y.x, 0.f, r4.x),
                                                                      finish_ws<ACT, true>(y.y, 0.f, r4.y),
                                                                      finish_ws<ACT, true>(y.z, 0.f, r4.z),
                                                                      finish_ws<ACT, true>(y.w, 0.f, r4.w)));
                        }
                        *reinterpret_cast<u32x4*>(p.C + (int64_t)rr * p.ldc + col0 + 16 * pp + 4 * g) = v;
                    }
                }
            }
        }
    }
    if (LNM == 3 && !kSideLds && wv < RT) {
        // out2 = LN(x) g2 + b2 of the wave's rows from a second read of x (L2), after every
        // other store of the block; the row tile's NPART blocks take a k32-step range each
        // (part p: steps [8p / NPART, 8(p + 1) / NPART)), all loads issued before the stores
        const int s_lo = part * kWsKS / NPART, s_hi = (part + 1) * kWsKS / NPART;
        constexpr int SPP = (kWsKS + NPART - 1) / NPART;  // steps per part, at most
        const float* ar = p.A + row * p.lda;
        float4 a0[SPP], a1[SPP];
#pragma unroll
        for (int j = 0; j < SPP; ++j) {
            const int kk = 32 * min(s_lo + j, kWsKS - 1) + 8 * g;
            a0[j] = *reinterpret_cast<const float4*>(ar + kk);
            a1[j] = *reinterpret_cast<const float4*>(ar + kk + 4);
        }
#pragma unroll
        for (int j = 0; j < SPP; ++j) {
            const int k = 32 * (s_lo + j) + 8 * g;
            if (s_lo + j < s_hi && rrow < p.M) {
                const float4 h0 = lng2[k / 4], h1 = lng2[k / 4 + 1];
                const float4 c0 = lnb2[k / 4], c1 = lnb2[k / 4 + 1];
                float* o2 = p.out2 + (int64_t)rrow * p.ld_out2 + k;
                *reinterpret_cast<float4*>(o2) = make_float4(
                    (a0[j].x - ln_mean) * ln_rstd * h0.x + c0.x, (a0[j].y - ln_mean) * ln_rstd * h0.y + c0.y,
                    (a0[j].z - ln_mean) * ln_rstd * h0.z + c0.z, (a0[j].w - ln_mean) * ln_rstd * h0.w + c0.w);
                *reinterpret_cast<float4*>(o2 + 4) = make_float4(
                    (a1[j].x - ln_mean) * ln_rstd * h1.x + c1.x, (a1[j].y - ln_mean) * ln_rstd * h1.y + c1.y,
                    (a1[j].z - ln_mean) * ln_rstd * h1.z + c1.z, (a1[j].w - ln_mean) * ln_rstd * h1.w + c1.w);
            }
        }
    }
    if (kSideLds) {
        // out2: the block's rows x 256 from LDS, 16 B per lane, whole rows per instruction
#pragma unroll
        for (int i = 0; i < 4 * RT; ++i) {
            const int u = tid + 256 * i;                  // float4 index in [BR rows][64]
            const int rr = r0 + (u >> 6);
            if (rr < p.M) *reinterpret_cast<float4*>(p.out2 + (int64_t)rr * p.ld_out2 + 4 * (u & 63)) = side[u];
        }
    }
#ifdef FGR_WS_STAMP
    __builtin_amdgcn_s_waitcnt(0);
    if (NPASS == 1) st_[7] = __builtin_amdgcn_s_memtime();    // every store of the wave done
    if (lane < 8 && blockIdx.x < 2048) g_ws_stamp[blockIdx.x][wv][lane] = st_[lane];
#endif
}

// row tiles per block: 3 (48-row blocks) where they fit the CUs in one round and 64-row
// blocks leave CUs idle (ModelNet's 9544 rows: 199 blocks instead of 150), else 4; the K / V
// image epilogue writes whole 64-row tiles (4 only). FGR_WS_RT overrides (A/B).
constexpr int kCusWs = 256;
template <int NPW, int LNM, bool KV, bool RES, int ACT, int NPART = 1>
void launch_ws(const WsArgs& a, hipStream_t st) {
    static const int rt_env = [] { const char* e = getenv("FGR_WS_RT"); return e ? atoi(e) : 0; }();
    int rt = (rt_env >= 3 && rt_env <= 4) ? rt_env
             : ((a.M + 47) / 48 <= kCusWs && (a.M + 63) / 64 < kCusWs) ? 3 : 4;
    if (KV) rt = 4;
    if (rt == 3)
        hipLaunchKernelGGL((gemm_ws_kernel<NPW, LNM, KV, RES, ACT, KV ? 4 : 3, NPART>),
                           dim3((unsigned)((a.M + 47) / 48 * NPART)), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((gemm_ws_kernel<NPW, LNM, KV, RES, ACT, 4, NPART>),
                           dim3((unsigned)((a.M + 63) / 64 * NPART)), dim3(256), 0, st, a);
}

}  // namespace

// The ws kernel's shapes: K = 256, N = 256 (out_proj) or 768 (in_proj), many rows; operands
// 16-B aligned (checked by the caller). FGR_GEMM_WS=0 disables it (the rs kernel then).
bool gemm_ws_supported(int m, int n, int k) {
    static const bool on = [] { const char* e = getenv("FGR_GEMM_WS"); return !(e && e[0] == '0'); }();
    if (!on || k != 256 || m < 4096) return false;
    // N = 512 / 1024: the columns over N / 256 blocks per row tile (ModelNet's 9544 x 512 x 256:
    // 22.2-22.9 -> 19.4-19.6 us; 9544 x 1792 x 256 measured equal to the row-stationary kernel
    // and left there, profiles/r06_ws_wide_ab.txt); FGR_GEMM_WSN=0 keeps them off (A/B)
    static const bool wide = [] { const char* e = getenv("FGR_GEMM_WSN"); return !(e && e[0] == '0'); }();
    return n == 256 || n == 768 || (wide && (n == 512 || n == 1024));
}

bool gemm_ws_ln_supported(int m, int n, int k) {
    return (n == 256 || n == 768) && gemm_ws_supported(m, n, k);
}

bool gemm_ws_f16x3(const float* A, int64_t lda, const void* W, const float* wsc, float* C,
                   int64_t ldc, const float* bias, const float* R, int64_t ldr, int M, int N,
                   int K, int act, hipStream_t st, const WsLn* ln) {
    if (!gemm_ws_supported(M, N, K)) return false;
    if (ln && R) return false;
    if (act != FGR_ACT_NONE && act != FGR_ACT_RELU) return false;
    WsArgs a{A, lda, (const u32x4*)W, wsc, bias, C, ldc, R, ldr, M, N,
             ln ? ln->g : nullptr, ln ? ln->b : nullptr, ln ? ln->eps : 0.f,
             ln ? ln->add : nullptr, ln ? ln->ld_add : 0,
             ln ? ln->g2 : nullptr, ln ? ln->b2 : nullptr, ln ? ln->out2 : nullptr,
             ln ? ln->ld_out2 : 0, ln ? ln->kv_img : nullptr, ln ? ln->kv_sc : nullptr,
             ln ? ln->n_head : 0, ln ? ln->kv_col0 : N};
    const bool relu = act == FGR_ACT_RELU;
    if (N != 256 && N != 768) {                  // 512 / 1024: N / 256 blocks per row tile
        if (ln) return false;
#define FGR_WS_PARTS(P)                                                                         \
        if (R) { if (relu) launch_ws<4, 0, false, true, FGR_ACT_RELU, P>(a, st);                \
                 else launch_ws<4, 0, false, true, FGR_ACT_NONE, P>(a, st); }                   \
        else if (relu) launch_ws<4, 0, false, false, FGR_ACT_RELU, P>(a, st);                   \
        else launch_ws<4, 0, false, false, FGR_ACT_NONE, P>(a, st);
        if (N == 512) { FGR_WS_PARTS(2) }
        else { FGR_WS_PARTS(4) }
#undef FGR_WS_PARTS
        return true;
    }
    if (N == 768) {
        if (!ln) {
            if (R) launch_ws<12, 0, false, true, FGR_ACT_NONE>(a, st);
            else if (relu) launch_ws<12, 0, false, false, FGR_ACT_RELU>(a, st);
            else launch_ws<12, 0, false, false, FGR_ACT_NONE>(a, st);
            return true;
        }
        if (ln->kv_img) {
            if (relu || !ln->add || ln->n_head * 64 + ln->kv_col0 != N || ln->kv_col0 != 256) return false;
            // without the side output: q | k | v over three blocks per row tile (450 blocks at
            // ModelNet's 9544 rows, two resident per CU; 28.2 -> 25.3 us), unless FGR_WS_SPLIT=0.
            // With it (its 64 KB LDS staging: one block per CU) one block per row tile (31.3 us
            // vs 35.6 split; profiles/r06_ws_split_ab.txt)
            static const bool split = [] { const char* e = getenv("FGR_WS_SPLIT"); return !(e && e[0] == '0'); }();
            static const bool split3 = [] { const char* e = getenv("FGR_WS_SPLIT3"); return !(e && e[0] == '0'); }();
            if (ln->out2) {
                if (split && split3) launch_ws<4, 3, true, false, FGR_ACT_NONE, 3>(a, st);
                else launch_ws<12, 3, true, false, FGR_ACT_NONE>(a, st);
            } else if (split) launch_ws<4, 2, true, false, FGR_ACT_NONE, 3>(a, st);
            else launch_ws<12, 2, true, false, FGR_ACT_NONE>(a, st);
            return true;
        }
        if (relu) return false;
        if (ln->out2) launch_ws<12, 3, false, false, FGR_ACT_NONE>(a, st);
        else if (ln->add) launch_ws<12, 2, false, false, FGR_ACT_NONE>(a, st);
        else launch_ws<12, 1, false, false, FGR_ACT_NONE>(a, st);
        return true;
    }
    // N == 256
    if (ln) return false;
    if (R) {
        if (relu) launch_ws<4, 0, false, true, FGR_ACT_RELU>(a, st);
        else launch_ws<4, 0, false, true, FGR_ACT_NONE>(a, st);
    } else {
        if (relu) launch_ws<4, 0, false, false, FGR_ACT_RELU>(a, st);
        else launch_ws<4, 0, false, false, FGR_ACT_NONE>(a, st);
    }
    return true;
}

}  // namespace fgr

#ifdef FGR_WS_STAMP
extern "C" int fgr_debug_ws_stamps(void* dst, int32_t nblocks) {
    if (nblocks > 2048) nblocks = 2048;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ws_stamp), (size_t)nblocks * 4 * 8 * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
