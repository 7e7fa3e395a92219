// Fused KPConv: gather-weight stage + weight GEMM in one launch, the (Nq, K * Cin) wf tensor
// never leaves the chip (finegrained_kpconv_blocks.py:296-399 up to the normaliser division):
//
//   out[q, n] = sum_{k, c} wf[q, k, c] W[k, c, n],
//   wf[q, k, c] = sum_{valid h} max(0, 1 - |s[idx[q,h]] - q - kp[k]| / extent) x[idx[q,h], c],
//   nnorm[q]    = max(1, #{valid h : sum_c x[idx[q, h], c] > 0}).
//
// Structure (one 256-thread block = 64 queries x BN output channels; wave w owns queries
// 16w .. 16w + 15):
//   * the block's neighbour table goes to LDS once (int32 ids, -1 for shadows; per query the
//     last valid position and the normaliser count, from kpf_row_positive_kernel's per-row
//     flags), so the gather never waits on an index load;
//   * the contraction index runs over (16-channel chunk cc, k32-step t, lane group g,
//     element e) with kernel point k = g + 4 (e >> 1) and channel c = 16 cc + 2 t + (e & 1)
//     (kernel-point slot 15 is zero padding) -- the KPConv weight is stored once in THAT order
//     as an f16x3 / bf16 MFMA image (fgr_kpconv_fused_weights);
//   * so lane (g, c16) of a wave gathers, for ITS query c16 and ITS four kernel points
//     g, g + 4, g + 8, g + 12, the 16 channels of the chunk: 4 influences per neighbour (none
//     computed twice inside a chunk); each lane loads only its 16-B quarter of the neighbour's
//     64-B row chunk and the other quarters arrive from the column's sibling lanes by
//     permlane16 / permlane32 swaps; neighbours go in batches of 4 with the next batch's loads
//     in flight. When the chunk is done the lane's 64 registers ARE the MFMA B fragments of
//     the chunk's 8 k32-steps (B[k = 8g + e][j = c16]) -- no LDS pass, no HBM round trip;
//   * W fragments (the MFMA A operand) travel global -> LDS by LDS-DMA through an S-stage ring
//     shared by the 4 waves; the stages of the next chunk are in flight while it is gathered;
//   * f16x3: the query's row scale is set / lowered per chunk from the chunk's exact max over
//     the query's 4 lanes (the g5 policy, gemm5.hip), then each step's 8 values are split by
//     v_fma_mix (split8_f16); bf16: rounded once.
// Lane maps of v_mfma_f32_16x16x32_{f16,bf16} (lane l, g = l >> 4, c = l & 15): A[i = c][k =
// 8g + e], B[k = 8g + e][j = c], C[i = 4g + r][j = c].
#include "common.h"

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kKpMax = 15;          // kernel points of the fused path (slot 15 = padding)
constexpr int SH_UNSET = 0x3fff;

// k32-steps of the fused contraction (16 kernel-point slots x cin channels / 32)
__host__ __device__ inline int kf_ksteps(int cin) { return cin / 2; }
size_t kf_image_bytes(int cout, int cin, int terms) {
    return (size_t)((cout + 15) / 16) * kf_ksteps(cin) * terms * 64 * 16;
}

// per output channel n: 2^-e_n with max_k,c |W[k, c, n]| 2^e_n in [2^14, 2^15) (f16x3)
__global__ void kf_weight_scale_kernel(const float* __restrict__ w, int nk, int cin, int cout,
                                       int npad, float* __restrict__ wsc) {
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (n >= npad) return;
    float mx = 0.f;
    if (n < cout)
        for (int j = lane; j < nk * cin; j += 64) mx = fmaxf(mx, fabsf(w[(int64_t)j * cout + n]));
    mx = wave_max(mx);
    if (lane == 0) {
        const int e = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
        wsc[n] = n < cout ? __builtin_ldexpf(1.f, -e) : 0.f;
    }
}

// W (nk, cin, cout) -> image [panel][kstep][term][g 4][16 rows] x 16 B in the fused order
__global__ void kf_split_weights_kernel(const float* __restrict__ w, int nk, int cin, int cout,
                                        int terms, const float* __restrict__ wsc,
                                        u32x4* __restrict__ img) {
    const int ksteps = kf_ksteps(cin);
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)((cout + 15) / 16) * ksteps * terms * 64;
    if (u >= total) return;
    const int i = (int)(u % 16);
    const int g = (int)((u / 16) % 4);
    const int term = (int)((u / 64) % terms);
    const int64_t ps = u / (64 * terms);
    const int s = (int)(ps % ksteps);
    const int panel = (int)(ps / ksteps);
    const int n = panel * 16 + i;
    const int cc = s / 8, t = s % 8;
    const float sc = (terms == 2 && n < cout) ? 1.f / wsc[n] : 1.f;   // exact: a power of two
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = g + 4 * (e >> 1), c = 16 * cc + 2 * t + (e & 1);
        v[e] = (n < cout && k < nk) ? w[((int64_t)k * cin + c) * cout + n] * sc : 0.f;
    }
    if (terms == 2) {
        f16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const _Float16 h = (_Float16)v[e];
            o[e] = term == 0 ? h : (_Float16)(v[e] - (float)h);
        }
        img[u] = __builtin_bit_cast(u32x4, o);
    } else {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
        img[u] = __builtin_bit_cast(u32x4, o);
    }
}

// pos[r] = (sum_c x[r, c] > 0): 16 lanes per row (16-B loads, 64 channels per pass), DPP
// row sum; 4 rows per wave
__global__ void __launch_bounds__(256)
kpf_row_positive_kernel(const float* __restrict__ x, int64_t ns, int cin,
                        unsigned char* __restrict__ pos) {
    const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const int l = threadIdx.x & 15;
    const int64_t rc = r < ns ? r : ns - 1;
    float t = 0.f;
    for (int c = 4 * l; c < cin; c += 64) {
        const float4 v = *reinterpret_cast<const float4*>(x + rc * cin + c);
        t += (v.x + v.y) + (v.z + v.w);
    }
    t = row16_sum(t);
    if (r < ns && l == 0) pos[r] = t > 0.f ? 1 : 0;
}

template <int N>
__device__ __forceinline__ void kf_wait_vm() {        // s_waitcnt vmcnt(N) lgkmcnt(0)
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}

__device__ __forceinline__ float kf_xg_max(float v) {  // max over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

struct KFArgs {
    const float* q; const float* s; int64_t nq, ns;
    const int64_t* idx; int width, wpad;
    const float* x; int cin;
    const unsigned char* pos;
    const float* kp; int n_kp; float inv_ext;
    const u32x4* W; int ksteps; const float* wsc;
    float* out; int64_t ldo; float* nnorm; int N;
};

// lane (g, c) holds piece v of row g of its 16-lane column c; returns all four rows' pieces
// (r[j] = piece of row j) by one permlane16 and two permlane32 swaps (no LDS)
__device__ __forceinline__ void kf_col_gather(float v, float (&r)[4]) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    // a[0] = row (g & ~1), a[1] = row (g | 1)
    auto e = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);    // rows 0, 2
    auto o = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);    // rows 1, 3
    r[0] = __uint_as_float(e[0]); r[2] = __uint_as_float(e[1]);
    r[1] = __uint_as_float(o[0]); r[3] = __uint_as_float(o[1]);
}

// s_waitcnt vmcnt(ahead * P): the W stages issued after the one about to be read may stay
// in flight
template <int P, int S>
__device__ __forceinline__ void kf_wait_ahead(int ahead) {
    switch (S >= 8 ? ahead : min(ahead, S - 2)) {
        case 0: kf_wait_vm<0>(); break;
        case 1: kf_wait_vm<P>(); break;
        case 2: kf_wait_vm<(S >= 4 ? 2 : 1) * P>(); break;
        case 3: kf_wait_vm<(S >= 5 ? 3 : 1) * P>(); break;
        case 4: kf_wait_vm<(S >= 6 ? 4 : 1) * P>(); break;
        case 5: kf_wait_vm<(S >= 7 ? 5 : 1) * P>(); break;
        default: kf_wait_vm<(S >= 8 ? 6 : 1) * P>(); break;
    }
}

template <int BN, int TERMS, int S, int NB, int OCC>
__global__ void __launch_bounds__(256, OCC) kpconv_fused_kernel(KFArgs p) {
    constexpr int TN = BN / 16;                // W panels per block (every wave: all of them)
    constexpr int W_PANEL = TERMS * 64;        // 16-B units of one (panel, k32-step)
    constexpr int ST = TN * W_PANEL;           // units per stage (one k32-step)
    constexpr int NP = ST / 64;                // DMA wave-instructions per stage
    static_assert(NP % 4 == 0, "stage pieces per wave");
    constexpr int P = NP / 4;
    static_assert(S * P <= 63 && S <= 8, "vmcnt range");
    __shared__ u32x4 lds[S * ST];
    __shared__ int hlast[64], npos[64];
    extern __shared__ int ids[];               // [64 queries][wpad]: neighbour id or -1

    const int nbm = (int)((p.nq + 63) / 64), nbn = (p.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int tb = blockIdx.x;
    {   // XCD-aware bijective remap: the N tiles of one query block run on one XCD (its L2
        // serves their shared neighbour rows)
        const int qd = nwg / 8, rm = nwg % 8, xc = tb % 8, lo = tb / 8;
        tb = (xc < rm ? xc * (qd + 1) : rm * (qd + 1) + (xc - rm) * qd) + lo;
    }
    const int bm = tb / nbn, bn = tb % nbn;
    const int n0 = bn * BN;
    const int64_t m0 = (int64_t)bm * 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c = lane & 15;
    const int npanel = (p.N + 15) / 16;
    const int nk = p.ksteps;

    // ---- W DMA pieces of this wave (piece q = panel * TERMS + term)
    const u32x4* wsrc[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int qp = wv + 4 * j;
        const int panel = qp / TERMS, term = qp % TERMS;
        const int pg = min(n0 / 16 + panel, npanel - 1);
        wsrc[j] = p.W + (int64_t)pg * nk * W_PANEL + term * 64 + lane;
    }
    auto issue = [&](int st) {
        __attribute__((address_space(3))) char* base =
            (__attribute__((address_space(3))) char*)(lds + (st % S) * ST);
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int qp = wv + 4 * j;
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[j] + (int64_t)st * W_PANEL),
                                             (lds_void*)(base + qp * 1024), 16, 0, 0);
        }
    };
#pragma unroll
    for (int st = 0; st < S - 1; ++st)
        if (st < nk) issue(st);

    // ---- the block's neighbour table -> LDS (int32, -1 = shadow / past the row), the last
    // valid position and the normaliser count per query (every row read once per block)
    if (tid < 64) { hlast[tid] = 0; npos[tid] = 0; }
    __syncthreads();
    {
        const int64_t nrow = min((int64_t)64, p.nq - m0);
        const int64_t tot = 64 * (int64_t)p.wpad;
        for (int64_t e = tid; e < tot; e += 256) {
            const int qq = (int)(e / p.wpad), h = (int)(e % p.wpad);
            int id = -1;
            if (qq < nrow && h < p.width) {
                const int64_t v = p.idx[(m0 + qq) * p.width + h];
                if (v >= 0 && v < p.ns) id = (int)v;
            }
            ids[e] = id;
            if (id >= 0) {
                atomicMax(&hlast[qq], h + 1);
                if (p.pos[id]) atomicAdd(&npos[qq], 1);
            }
        }
    }
    __syncthreads();

    // ---- this lane's query and kernel points
    const int ql = wv * 16 + c;
    const int64_t qi = m0 + ql;
    const bool qok = qi < p.nq;
    const int64_t qs = qok ? qi : 0;
    const float qx = p.q[3 * qs], qy = p.q[3 * qs + 1], qz = p.q[3 * qs + 2];
    float kx[4], ky[4], kz[4];
    bool kv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = g + 4 * j;
        kv[j] = k < p.n_kp;
        const int kk = kv[j] ? k : 0;
        kx[j] = p.kp[3 * kk]; ky[j] = p.kp[3 * kk + 1]; kz[j] = p.kp[3 * kk + 2];
    }
    // neighbour positions to scan: the wave's largest last-valid position, in whole batches
    const int hmax = (int)row16_max((float)hlast[ql]);
    const int nbatch = (hmax + NB - 1) / NB;
    const int* myids = ids + ql * p.wpad;

    f32x4 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int sh = SH_UNSET;
    float scv = 1.f;

    // one batch of NB neighbours: ids (one 16-B LDS read), this lane's 16-B quarter of each
    // row chunk (16 channels), the neighbour positions
    struct Batch { int id[NB]; float4 xq[NB]; float sx[NB], sy[NB], sz[NB]; };
    auto load_batch = [&](int b, int cc, Batch& B) {
#pragma unroll
        for (int u = 0; u < NB; ++u) B.id[u] = myids[b * NB + u];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int64_t sid = B.id[u] >= 0 ? B.id[u] : 0;
            B.xq[u] = *reinterpret_cast<const float4*>(p.x + sid * p.cin + 16 * cc + 4 * g);
            B.sx[u] = p.s[3 * sid]; B.sy[u] = p.s[3 * sid + 1]; B.sz[u] = p.s[3 * sid + 2];
        }
    };

    const int nchunks = p.cin / 16;
    for (int cc = 0; cc < nchunks; ++cc) {
        // ---- gather: ga[j][ch] = wf[q, g + 4 j, 16 cc + ch]
        float ga[4][16];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) ga[j][e] = 0.f;
        Batch cur, nxt;
        if (nbatch > 0) load_batch(0, cc, cur);
        for (int b = 0; b < nbatch; ++b) {
            if (b + 1 < nbatch) load_batch(b + 1, cc, nxt);
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const bool valid = cur.id[u] >= 0;
                const float nx = cur.sx[u] - qx, ny = cur.sy[u] - qy, nz = cur.sz[u] - qz;
                float w[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    // neighbours are centred first, then compared with the kernel points
                    // (:302, :313)
                    const float dx = nx - kx[j], dy = ny - ky[j], dz = nz - kz[j];
                    const float d2 = dx * dx + dy * dy + dz * dz;
                    w[j] = (valid && kv[j]) ? fmaxf(1.0f - sqrtf(d2) * p.inv_ext, 0.0f) : 0.f;
                }
                // the row's 16 channels: quarter r of the chunk comes from row r of the column
                float xv[16];
                {
                    float t[4];
                    kf_col_gather(cur.xq[u].x, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) xv[4 * r] = t[r];
                    kf_col_gather(cur.xq[u].y, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) xv[4 * r + 1] = t[r];
                    kf_col_gather(cur.xq[u].z, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) xv[4 * r + 2] = t[r];
                    kf_col_gather(cur.xq[u].w, t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) xv[4 * r + 3] = t[r];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) ga[j][e] = fmaf(w[j], xv[e], ga[j][e]);
            }
            if (b + 1 < nbatch) cur = nxt;
        }
        // ---- f16x3 row scale: set by the first non-zero chunk (max into [2^7, 2^8)), lowered
        // with the partial sums rescaled when a chunk would pass 2^15
        if constexpr (TERMS == 2) {
            float cm = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) cm = fmaxf(cm, fabsf(ga[j][e]));
            cm = kf_xg_max(cm);
            const bool lower = cm > 0.f && (sh == SH_UNSET ||
                                            __builtin_amdgcn_frexp_expf(cm) + sh > 15);
            if (lower) {
                const int nsh = min(8 - __builtin_amdgcn_frexp_expf(cm), 127);
                const float f = sh == SH_UNSET ? 1.f : __builtin_ldexpf(1.f, nsh - sh);
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j] *= f;
                sh = nsh;
                scv = __builtin_ldexpf(1.f, sh);
            }
        }
        // ---- the chunk's 8 k32-steps: B fragments from ga, W fragments from the ring
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int st = cc * 8 + t;
            kf_wait_ahead<P, S>(min(S - 2, nk - 1 - st));
            __builtin_amdgcn_s_barrier();
            if (st + S - 1 < nk) issue(st + S - 1);
            const u32x4* sb = lds + (st % S) * ST;
            const float xb[8] = {ga[0][2 * t], ga[0][2 * t + 1], ga[1][2 * t], ga[1][2 * t + 1],
                                 ga[2][2 * t], ga[2][2 * t + 1], ga[3][2 * t], ga[3][2 * t + 1]};
            if constexpr (TERMS == 2) {
                u32x4 bh, bl;
                split8_f16(xb, scv, bh, bl);
                const f16x8 ah = __builtin_bit_cast(f16x8, bh);
                const f16x8 al = __builtin_bit_cast(f16x8, bl);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const f16x8 wh = __builtin_bit_cast(f16x8, sb[j * W_PANEL + lane]);
                    const f16x8 wl = __builtin_bit_cast(f16x8, sb[j * W_PANEL + 64 + lane]);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, al, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, acc[j], 0, 0, 0);
                }
            } else {
                bf16x8 hb;
#pragma unroll
                for (int e = 0; e < 8; ++e) hb[e] = (__bf16)xb[e];
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, sb[j * W_PANEL + lane]), hb, acc[j], 0, 0, 0);
            }
        }
    }

    // ---- epilogue: lane holds out[qi][n0 + 16 j + 4 g + r]
    if (qok) {
        const float rs = TERMS == 2 ? __builtin_ldexpf(1.f, -sh) : 1.f;   // 0: all-zero row
        float* orow = p.out + qi * p.ldo;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + 16 * j + 4 * g;
            if (n >= p.N) continue;
            float4 ws = make_float4(1.f, 1.f, 1.f, 1.f);
            if constexpr (TERMS == 2) ws = *reinterpret_cast<const float4*>(p.wsc + n);
            const float y[4] = {acc[j][0] * rs * ws.x, acc[j][1] * rs * ws.y,
                                acc[j][2] * rs * ws.z, acc[j][3] * rs * ws.w};
            if (n + 3 < p.N && (p.ldo & 3) == 0) {
                *reinterpret_cast<float4*>(orow + n) = make_float4(y[0], y[1], y[2], y[3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (n + e < p.N) orow[n + e] = y[e];
            }
        }
        if (bn == 0 && g == 0) p.nnorm[qi] = (float)(npos[ql] > 1 ? npos[ql] : 1);
    }
}

template <int BN, int TERMS, int S, int NB, int OCC>
void launch_kf(const KFArgs& a, hipStream_t st) {
    const int nbm = (int)((a.nq + 63) / 64), nbn = (a.N + BN - 1) / BN;
    hipLaunchKernelGGL((kpconv_fused_kernel<BN, TERMS, S, NB, OCC>), dim3((unsigned)(nbm * nbn)), dim3(256),
                       (size_t)64 * a.wpad * sizeof(int), st, a);
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_kpconv_fused_weights_bytes(int32_t n_kp, int32_t cin, int32_t cout,
                                              int32_t mode, size_t* bytes) {
    FGR_REQUIRE(bytes && n_kp > 0 && n_kp <= kKpMax && cin > 0 && cin % 16 == 0 && cout > 0 &&
                    (mode == FGR_KPF_F16X3 || mode == FGR_KPF_BF16),
                "fgr_kpconv_fused_weights_bytes: bad arguments (n_kp %d cin %d cout %d mode %d)",
                n_kp, cin, cout, mode);
    const int terms = mode == FGR_KPF_F16X3 ? 2 : 1;
    *bytes = kf_image_bytes(cout, cin, terms) + (size_t)((cout + 15) / 16) * 16 * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_kpconv_fused_weights(const float* w, int32_t n_kp, int32_t cin, int32_t cout,
                                        int32_t mode, void* img, void* stream) {
    size_t nb = 0;
    if (int e = fgr_kpconv_fused_weights_bytes(n_kp, cin, cout, mode, &nb)) return e;
    FGR_REQUIRE(w && img && (reinterpret_cast<uintptr_t>(img) & 15) == 0,
                "fgr_kpconv_fused_weights: null pointer or image not 16-B aligned");
    const int terms = mode == FGR_KPF_F16X3 ? 2 : 1;
    const int npad = (cout + 15) / 16 * 16;
    float* wsc = reinterpret_cast<float*>(static_cast<char*>(img) + kf_image_bytes(cout, cin, terms));
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(kf_weight_scale_kernel, dim3((unsigned)ceil_div(npad, 4)), dim3(256), 0, st,
                       w, n_kp, cin, cout, npad, wsc);
    FGR_CHECK_LAUNCH("kf_weight_scale_kernel");
    const int64_t total = (int64_t)(npad / 16) * kf_ksteps(cin) * terms * 64;
    hipLaunchKernelGGL(kf_split_weights_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0,
                       st, w, n_kp, cin, cout, terms, wsc, (u32x4*)img);
    FGR_CHECK_LAUNCH("kf_split_weights_kernel");
    return FGR_OK;
}

extern "C" int fgr_kpconv_fused_workspace(int64_t ns, size_t* bytes) {
    FGR_REQUIRE(bytes && ns >= 0, "fgr_kpconv_fused_workspace: bad arguments");
    *bytes = (size_t)(ns > 0 ? ns : 1);
    return FGR_OK;
}

extern "C" int fgr_kpconv_fused(const float* q, const float* s, int64_t nq, int64_t ns,
                                const int64_t* idx, int32_t width, const float* x, int32_t cin,
                                const float* kp, int32_t n_kp, float extent, const void* w_img,
                                int32_t cout, int32_t mode, float* out, int64_t ldo, float* nnorm,
                                void* workspace, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(nq >= 0 && ns >= 0 && width >= 0 && cin > 0 && cin % 16 == 0 && n_kp > 0 &&
                    n_kp <= kKpMax && extent > 0.f && cout > 0 && ldo >= cout &&
                    (mode == FGR_KPF_F16X3 || mode == FGR_KPF_BF16),
                "fgr_kpconv_fused: bad arguments (cin %d n_kp %d cout %d mode %d)", cin, n_kp,
                cout, mode);
    FGR_REQUIRE(nq == 0 || (q && s && x && kp && w_img && out && nnorm && (idx || width == 0)),
                "fgr_kpconv_fused: null pointer");
    FGR_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(w_img) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(out) & 15) == 0,
                "fgr_kpconv_fused: x, w_img and out must be 16-B aligned");
    if (nq == 0) return FGR_OK;
    FGR_REQUIRE(workspace && ws_bytes >= (size_t)(ns > 0 ? ns : 1),
                "fgr_kpconv_fused: workspace of %lld bytes needed", (long long)(ns > 0 ? ns : 1));
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    unsigned char* pos = static_cast<unsigned char*>(workspace);
    if (ns > 0) {
        hipLaunchKernelGGL(kpf_row_positive_kernel, dim3((unsigned)ceil_div(ns * 16, 256)), dim3(256),
                           0, st, x, ns, cin, pos);
        FGR_CHECK_LAUNCH("kpf_row_positive_kernel");
    }
    const int terms = mode == FGR_KPF_F16X3 ? 2 : 1;
    const float* wsc = reinterpret_cast<const float*>(static_cast<const char*>(w_img) +
                                                      kf_image_bytes(cout, cin, terms));
    const int wpad = (width + 3) / 4 * 4;
    KFArgs a{q, s, nq, ns, idx, width, wpad, x, cin, pos, kp, n_kp, 1.0f / extent,
             static_cast<const u32x4*>(w_img), kf_ksteps(cin), wsc, out, ldo, nnorm, cout};
    // variants (FGR_KPF_TILE): '1' 128 columns, 3 W stages, 2-neighbour batches, 2 blocks per
    // CU; '2' 128 / 8 stages / 4 / 1; '3' 64 / 8 / 4 / 1; '4' 128 / 6 / 8 / 1; '6' 64 / 4 / 2 / 2
    const char* force = getenv("FGR_KPF_TILE");
    const char v = force && force[0] ? force[0] : (cout > 64 ? '1' : '6');
    if (terms == 2) {
        switch (v) {
            case '2': launch_kf<128, 2, 8, 4, 1>(a, st); break;
            case '3': launch_kf<64, 2, 8, 4, 1>(a, st); break;
            case '4': launch_kf<128, 2, 6, 8, 1>(a, st); break;
            case '6': launch_kf<64, 2, 4, 2, 2>(a, st); break;
            default: launch_kf<128, 2, 3, 2, 2>(a, st); break;
        }
    } else {
        switch (v) {
            case '2': launch_kf<128, 1, 8, 4, 1>(a, st); break;
            case '3': launch_kf<64, 1, 8, 4, 1>(a, st); break;
            case '4': launch_kf<128, 1, 8, 8, 1>(a, st); break;
            case '6': launch_kf<64, 1, 4, 2, 2>(a, st); break;
            default: launch_kf<128, 1, 4, 2, 2>(a, st); break;
        }
    }
    FGR_CHECK_LAUNCH("kpconv_fused_kernel");
    return FGR_OK;
}
