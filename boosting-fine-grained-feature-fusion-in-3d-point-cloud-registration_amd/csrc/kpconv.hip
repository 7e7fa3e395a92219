// KPConv gather-weight stage and max-pool shortcut on gfx950.
//
// fgr_kpconv_gather computes, for every query q,
//   wf[q, k, c] = sum_{valid h} w(q, h, k) * x[idx[q, h], c],
//   w(q, h, k)  = max(0, 1 - sqrt(|(s[idx[q,h]] - q) - kp[k]|^2) / extent)
// (finegrained_kpconv_blocks.py:296-381) and the KPConv normaliser
//   nnorm[q] = max(1, #{valid h : sum_c x[idx[q, h], c] > 0})            (:395-399).
// Shadow entries (idx >= ns) carry zero weight and a zero feature row in the
// reference, so they are skipped here: only valid neighbours are read.
//
// HBM-bound. Per query the algorithmic traffic is
//   8*width (idx row) + 12 (q) + v*(12 + 4*cin) (valid neighbour xyz + feature row)
//   + 4*K*cin (wf row) + 4 (nnorm),
// dominated by the wf write. Wide-channel layers (cin % 64 == 0) run one wave per
// query with channels on lanes (VEC contiguous floats per lane -> 16-B loads/stores);
// narrow layers (cin < 64) run one thread per (query, kernel point).
#include "common.h"

namespace fgr {
namespace {

constexpr int kMaxKp = 32;         // kernel points supported (configs use 15)
constexpr int kGatherWaves = 4;    // waves (= queries) per block, wide kernel
#ifndef GATHER_U
#define GATHER_U 4                 // neighbour rows in flight per wave (8 measured 10 % slower)
#endif

template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, float (&v)[VEC]) {
    if constexpr (VEC == 1) {
        v[0] = p[0];
    } else if constexpr (VEC == 2) {
        float2 t = *reinterpret_cast<const float2*>(p);
        v[0] = t.x; v[1] = t.y;
    } else {
#pragma unroll
        for (int j = 0; j < VEC; j += 4) {
            float4 t = *reinterpret_cast<const float4*>(p + j);
            v[j] = t.x; v[j + 1] = t.y; v[j + 2] = t.z; v[j + 3] = t.w;
        }
    }
}

template <int VEC>
__device__ __forceinline__ void store_vec(float* p, const float (&v)[VEC]) {
    if constexpr (VEC == 1) {
        p[0] = v[0];
    } else if constexpr (VEC == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    } else {
#pragma unroll
        for (int j = 0; j < VEC; j += 4)
            *reinterpret_cast<float4*>(p + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
    }
}

typedef float wf4 __attribute__((ext_vector_type(4)));
typedef float wf2 __attribute__((ext_vector_type(2)));

// wf rows are written once and read once, later, by the weight GEMM: non-temporal stores
// (same-box A/B: gather 0.593 -> 0.655 of HBM peak and ModelNet step 3.76 -> 3.72 ms;
// 3DMatch 0.536 -> 0.556; the GEMM reading wf unchanged)
template <int VEC>
__device__ __forceinline__ void store_wf(float* p, const float (&v)[VEC]) {
    if constexpr (VEC == 1) {
        __builtin_nontemporal_store(v[0], p);
    } else if constexpr (VEC == 2) {
        __builtin_nontemporal_store(wf2{v[0], v[1]}, reinterpret_cast<wf2*>(p));
    } else {
#pragma unroll
        for (int j = 0; j < VEC; j += 4)
            __builtin_nontemporal_store(wf4{v[j], v[j + 1], v[j + 2], v[j + 3]},
                                        reinterpret_cast<wf4*>(p + j));
    }
}

__device__ __forceinline__ float kp_weight(float nx, float ny, float nz, const float* kp, int k,
                                           float inv_extent) {
    float dx = nx - kp[3 * k], dy = ny - kp[3 * k + 1], dz = nz - kp[3 * k + 2];
    float d2 = dx * dx + dy * dy + dz * dz;
    return fmaxf(1.0f - sqrtf(d2) * inv_extent, 0.0f);
}

// One wave per query, cin = 64 * VEC, K kernel points (runtime, <= kMaxKp, unrolled by KU).
// Valid neighbours of each 64-wide chunk are compacted by ballot; their feature rows are
// then streamed 4 at a time (4 x 16-B loads in flight per lane) into K accumulators.
// POSI: the normaliser's "row sum > 0" is taken from the rows as they stream by (a DPP /
// permlane wave sum per row, no LDS); otherwise from per-source-row flags `pos`.
template <int VEC, int KU, bool POSI>
__global__ void __launch_bounds__(64 * kGatherWaves)
kpconv_gather_wide(const float* __restrict__ q, const float* __restrict__ s, int64_t nq, int64_t ns,
                   const int64_t* __restrict__ idx, int width, const float* __restrict__ x,
                   const unsigned char* __restrict__ pos, const float* __restrict__ kp_g, int n_kp,
                   float inv_extent, float* __restrict__ wf, float* __restrict__ nnorm) {
    constexpr int CIN = 64 * VEC;
    constexpr int U = GATHER_U;                        // neighbour rows in flight
    __shared__ float w_lds[kGatherWaves][64 + U][KU];
    __shared__ int nb_lds[kGatherWaves][64 + U];
    __shared__ float3 p_lds[kGatherWaves][64];
    __shared__ float kp[3 * kMaxKp];
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (int i = threadIdx.x; i < 3 * n_kp; i += blockDim.x) kp[i] = kp_g[i];
    __syncthreads();
    const int64_t qi = (int64_t)blockIdx.x * kGatherWaves + wv;
    if (qi >= nq) return;
    const float qx = q[3 * qi], qy = q[3 * qi + 1], qz = q[3 * qi + 2];

    float acc[KU][VEC];
#pragma unroll
    for (int k = 0; k < KU; ++k)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[k][j] = 0.f;
    int n_pos = 0;
    const int64_t* row = idx + qi * width;

    for (int h0 = 0; h0 < width; h0 += 64) {
        const int h = h0 + lane;
        const int64_t id = h < width ? row[h] : ns;
        const bool valid = id >= 0 && id < ns;
        const unsigned long long m = __ballot(valid);
        const int v = __popcll(m);
        if (v == 0) continue;
        if constexpr (!POSI) n_pos += __popcll(__ballot(valid && pos[id] != 0));
        const int p = __popcll(m & ((1ull << lane) - 1ull));
        if (valid) {
            // the lane that holds a valid neighbour loads its position once (one memory round
            // trip for the whole chunk; the influence loop below then reads LDS only)
            nb_lds[wv][p] = (int)id;
            // neighbours are centred first, then compared with the kernel points (:302, :313)
            p_lds[wv][p] = make_float3(s[3 * id] - qx, s[3 * id + 1] - qy, s[3 * id + 2] - qz);
        }
        if (lane < U) nb_lds[wv][v + lane] = 0;       // pad rows: weight 0, row 0
        __builtin_amdgcn_wave_barrier();
        // the first U rows are requested before the influences are computed (both need only
        // the compacted ids), so their memory round trip overlaps the influence loop; with
        // VEC <= 2 every later batch is also requested one batch ahead
        constexpr bool DB = VEC <= 2;
        float xn[U][VEC];
#pragma unroll
        for (int u = 0; u < U; ++u)
            load_vec<VEC>(x + (int64_t)nb_lds[wv][u] * CIN + lane * VEC, xn[u]);
        // kernel-point influences of the valid neighbours -> LDS (pad rows get 0)
        for (int t = lane; t < (v + U) * KU; t += 64) {
            const int hh = t / KU, k = t - hh * KU;
            float w = 0.f;
            if (hh < v && k < n_kp) {
                const float3 d = p_lds[wv][hh];
                w = kp_weight(d.x, d.y, d.z, kp, k, inv_extent);
            }
            w_lds[wv][hh][k] = w;
        }
        __builtin_amdgcn_wave_barrier();
        for (int hh = 0; hh < v; hh += U) {
            float xv[U][VEC];
            if (hh == 0 || DB) {
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int j = 0; j < VEC; ++j) xv[u][j] = xn[u][j];
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    load_vec<VEC>(x + (int64_t)nb_lds[wv][hh + u] * CIN + lane * VEC, xv[u]);
            }
            if (DB && hh + U < v) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    // rows past v + U read pad entries (row 0) only when v + U > 64: clamp
                    const int e = min(hh + U + u, v + U - 1);
                    load_vec<VEC>(x + (int64_t)nb_lds[wv][e] * CIN + lane * VEC, xn[u]);
                }
            }
            if constexpr (POSI) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    float t = 0.f;
#pragma unroll
                    for (int j = 0; j < VEC; ++j) t += xv[u][j];
                    t = wave_sum_dpp(t);
                    n_pos += (hh + u < v && t > 0.f) ? 1 : 0;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < KU; ++k) {
                    const float w = w_lds[wv][hh + u][k];
#pragma unroll
                    for (int j = 0; j < VEC; ++j) acc[k][j] = fmaf(w, xv[u][j], acc[k][j]);
                }
        }
        __builtin_amdgcn_wave_barrier();
    }
    float* out = wf + qi * (int64_t)n_kp * CIN + lane * VEC;
#pragma unroll
    for (int k = 0; k < KU; ++k)
        if (k < n_kp) store_wf<VEC>(out + (int64_t)k * CIN, acc[k]);
    if (lane == 0) nnorm[qi] = (float)(n_pos > 1 ? n_pos : 1);
}

// cin = 16 / 32 (3DMatch's first bottleneck convs run at 128 / 4 = 32 channels): one wave per
// query, lanes = (kernel-point group kg, channel quad): every lane owns 4 channels (one 16-B
// load per neighbour row; the wave reads each row as one 64- / 128-B line) of KPL kernel
// points k = kg, kg + KG, .... Valid neighbours are compacted by ballot and their K kernel-
// point influences computed once into LDS (as kpconv_gather_wide); the row-sum positivity
// of the normaliser is a DPP reduction over the QUADS lanes that hold the row.
template <int QUADS, int KPL>
__global__ void __launch_bounds__(256)
kpconv_gather_quads(const float* __restrict__ q, const float* __restrict__ s, int64_t nq,
                    int64_t ns, const int64_t* __restrict__ idx, int width,
                    const float* __restrict__ x, const float* __restrict__ kp_g, int n_kp,
                    float inv_extent, float* __restrict__ wf, float* __restrict__ nnorm) {
    constexpr int CIN = 4 * QUADS, KG = 64 / QUADS, U = GATHER_U, KW = 16;
    static_assert(KG * KPL >= KW, "kernel points per lane");
    __shared__ float w_lds[4][64 + U][KW];
    __shared__ int nb_lds[4][64 + U];
    __shared__ float3 p_lds[4][64];
    __shared__ float kp[3 * kMaxKp];
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int quad = lane % QUADS, kg = lane / QUADS;
    for (int i = threadIdx.x; i < 3 * n_kp; i += blockDim.x) kp[i] = kp_g[i];
    __syncthreads();
    const int64_t qi = (int64_t)blockIdx.x * 4 + wv;
    if (qi >= nq) return;
    const float qx = q[3 * qi], qy = q[3 * qi + 1], qz = q[3 * qi + 2];
    float4 acc[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    int n_pos = 0;
    const int64_t* row = idx + qi * width;
    for (int h0 = 0; h0 < width; h0 += 64) {
        const int h = h0 + lane;
        const int64_t id = h < width ? row[h] : ns;
        const bool valid = id >= 0 && id < ns;
        const unsigned long long m = __ballot(valid);
        const int v = __popcll(m);
        if (v == 0) continue;
        if (valid) {
            const int p = __popcll(m & ((1ull << lane) - 1ull));
            nb_lds[wv][p] = (int)id;
            p_lds[wv][p] = make_float3(s[3 * id] - qx, s[3 * id + 1] - qy, s[3 * id + 2] - qz);
        }
        if (lane < U) nb_lds[wv][v + lane] = 0;        // pad rows: weight 0, row 0
        __builtin_amdgcn_wave_barrier();
        for (int t = lane; t < (v + U) * KW; t += 64) {
            const int hh = t / KW, k = t % KW;
            float w = 0.f;
            if (hh < v && k < n_kp) {
                const float3 d = p_lds[wv][hh];
                w = kp_weight(d.x, d.y, d.z, kp, k, inv_extent);
            }
            w_lds[wv][hh][k] = w;
        }
        __builtin_amdgcn_wave_barrier();
        for (int hh = 0; hh < v; hh += U) {
            float4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                xv[u] = *reinterpret_cast<const float4*>(x + (int64_t)nb_lds[wv][hh + u] * CIN + 4 * quad);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float rs = (xv[u].x + xv[u].y) + (xv[u].z + xv[u].w);
                rs += dpp<0xB1>(rs);                     // quad_perm xor 1
                rs += dpp<0x4E>(rs);                     // quad_perm xor 2
                if constexpr (QUADS == 8) rs += dpp<0x141>(rs);   // row_half_mirror: 8 lanes
                n_pos += (hh + u < v && rs > 0.f) ? 1 : 0;
#pragma unroll
                for (int j = 0; j < KPL; ++j) {
                    const float w = w_lds[wv][hh + u][kg + KG * j];
                    acc[j].x = fmaf(w, xv[u].x, acc[j].x);
                    acc[j].y = fmaf(w, xv[u].y, acc[j].y);
                    acc[j].z = fmaf(w, xv[u].z, acc[j].z);
                    acc[j].w = fmaf(w, xv[u].w, acc[j].w);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    float* out = wf + qi * (int64_t)n_kp * CIN + 4 * quad;
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = kg + KG * j;
        if (k < n_kp) {
            const float a4[4] = {acc[j].x, acc[j].y, acc[j].z, acc[j].w};
            store_wf<4>(out + (int64_t)k * CIN, a4);
        }
    }
    if (lane == 0) nnorm[qi] = (float)(n_pos > 1 ? n_pos : 1);
}

// One thread per (query, kernel point); cin <= 64 (narrow layers, incl. the cin = 1 stem).
template <int CMAX>
__global__ void __launch_bounds__(256)
kpconv_gather_narrow(const float* __restrict__ q, const float* __restrict__ s, int64_t nq,
                     int64_t ns, const int64_t* __restrict__ idx, int width,
                     const float* __restrict__ x, int cin, const float* __restrict__ kp_g,
                     int n_kp, float inv_extent, float* __restrict__ wf,
                     float* __restrict__ nnorm) {
    __shared__ float kp[3 * kMaxKp];
    for (int i = threadIdx.x; i < 3 * n_kp; i += blockDim.x) kp[i] = kp_g[i];
    __syncthreads();
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq * n_kp) return;
    const int64_t qi = t / n_kp;
    const int k = (int)(t - qi * n_kp);
    const float qx = q[3 * qi], qy = q[3 * qi + 1], qz = q[3 * qi + 2];
    float acc[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) acc[c] = 0.f;
    int n_pos = 0;
    const int64_t* row = idx + qi * width;
    for (int h = 0; h < width; ++h) {
        const int64_t id = row[h];
        if (id < 0 || id >= ns) continue;
        const float nx = s[3 * id] - qx, ny = s[3 * id + 1] - qy, nz = s[3 * id + 2] - qz;
        const float w = kp_weight(nx, ny, nz, kp, k, inv_extent);
        const float* xr = x + id * cin;
        float rs = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c) {
            if (c < cin) {
                const float xv = xr[c];
                rs += xv;
                acc[c] = fmaf(w, xv, acc[c]);
            }
        }
        n_pos += rs > 0.f ? 1 : 0;
    }
    float* out = wf + t * cin;
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
        if (c < cin) out[c] = acc[c];
    if (k == 0) nnorm[qi] = (float)(n_pos > 1 ? n_pos : 1);
}

// cin == 1 (the stem: feats0 = ones, finegrained_regtr.py:126): 16 lanes per query, 4
// queries per wave. Lane l of a query takes neighbours h = l, l + 16, ... (coalesced index
// reads), accumulates all K kernel-point sums, and the 16 lanes reduce them with DPP; lane
// k then writes wf[q, k] (and k + 16), so each neighbour is read once per query instead of
// once per (query, kernel point).
template <int KU>
__global__ void __launch_bounds__(256)
kpconv_gather_c1(const float* __restrict__ q, const float* __restrict__ s, int64_t nq, int64_t ns,
                 const int64_t* __restrict__ idx, int width, const float* __restrict__ x,
                 const float* __restrict__ kp_g, int n_kp, float inv_extent,
                 float* __restrict__ wf, float* __restrict__ nnorm) {
    __shared__ float kp[3 * kMaxKp];
    for (int i = threadIdx.x; i < 3 * n_kp; i += blockDim.x) kp[i] = kp_g[i];
    __syncthreads();
    const int64_t qi = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int l = threadIdx.x & 15;
    const int64_t qc = qi < nq ? qi : nq - 1;          // tail lanes still join the reductions
    const float qx = q[3 * qc], qy = q[3 * qc + 1], qz = q[3 * qc + 2];
    float acc[KU];
#pragma unroll
    for (int k = 0; k < KU; ++k) acc[k] = 0.f;
    float n_pos = 0.f;
    const int64_t* row = idx + qc * width;
    for (int h = l; h < width; h += 16) {
        const int64_t id = row[h];
        if (id < 0 || id >= ns) continue;
        const float nx = s[3 * id] - qx, ny = s[3 * id + 1] - qy, nz = s[3 * id + 2] - qz;
        const float xv = x[id];
        n_pos += xv > 0.f ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < KU; ++k)
            if (k < n_kp) acc[k] = fmaf(kp_weight(nx, ny, nz, kp, k, inv_extent), xv, acc[k]);
    }
    float mine0 = 0.f, mine1 = 0.f;
#pragma unroll
    for (int k = 0; k < KU; ++k) {
        const float t = row16_sum(acc[k]);
        if (k == l) mine0 = t;
        if (k == l + 16) mine1 = t;
    }
    n_pos = row16_sum(n_pos);
    if (qi < nq) {
        float* out = wf + qi * n_kp;
        if (l < n_kp) out[l] = mine0;
        if (KU > 16 && l + 16 < n_kp) out[l + 16] = mine1;
        if (l == 0) nnorm[qi] = n_pos > 1.f ? n_pos : 1.f;
    }
}

template <int CMAX>
void launch_narrow(const float* q, const float* s, int64_t nq, int64_t ns, const int64_t* idx,
                   int width, const float* x, int cin, const float* kp, int n_kp, float inv_ext,
                   float* wf, float* nnorm, hipStream_t st) {
    const int64_t n = nq * n_kp;
    hipLaunchKernelGGL(kpconv_gather_narrow<CMAX>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                       st, q, s, nq, ns, idx, width, x, cin, kp, n_kp, inv_ext, wf, nnorm);
}

template <int VEC>
void launch_wide_k(const float* q, const float* s, int64_t nq, int64_t ns, const int64_t* idx,
                   int width, const float* x, const float* kp, int n_kp, float inv_ext, float* wf,
                   float* nnorm, hipStream_t st) {
    dim3 grid((unsigned)ceil_div(nq, kGatherWaves));
    if (n_kp <= 16)
        hipLaunchKernelGGL((kpconv_gather_wide<VEC, 16, true>), grid, dim3(64 * kGatherWaves), 0,
                           st, q, s, nq, ns, idx, width, x, nullptr, kp, n_kp, inv_ext, wf, nnorm);
    else
        hipLaunchKernelGGL((kpconv_gather_wide<VEC, kMaxKp, true>), grid, dim3(64 * kGatherWaves),
                           0, st, q, s, nq, ns, idx, width, x, nullptr, kp, n_kp, inv_ext, wf,
                           nnorm);
}

// max_pool, one wave per query (c % 64 == 0, VEC floats per lane): valid neighbours are
// compacted by ballot, their feature rows read with 16-B loads; a shadow entry in the
// row contributes the appended zero row (blocks:134-140).
template <int VEC>
__global__ void __launch_bounds__(256)
max_pool_wave(const float* __restrict__ x, int64_t ns, const int64_t* __restrict__ idx,
              int64_t nq, int width, float* __restrict__ out) {
    constexpr int C = 64 * VEC;
    __shared__ int nb_lds[4][64];
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int64_t qi = (int64_t)blockIdx.x * 4 + wv;
    if (qi >= nq) return;
    const int64_t* row = idx + qi * width;
    float m[VEC];
    bool shadow = false;
#pragma unroll
    for (int j = 0; j < VEC; ++j) m[j] = -INFINITY;
    for (int h0 = 0; h0 < width; h0 += 64) {
        const int h = h0 + lane;
        const int64_t id = h < width ? row[h] : 0;
        const bool valid = h < width && id >= 0 && id < ns;
        shadow |= (h < width && !valid);
        const unsigned long long bm = __ballot(valid);
        const int v = __popcll(bm);
        if (valid) nb_lds[wv][__popcll(bm & ((1ull << lane) - 1ull))] = (int)id;
        __builtin_amdgcn_wave_barrier();
        for (int hh = 0; hh < v; ++hh) {
            float xv[VEC];
            load_vec<VEC>(x + (int64_t)nb_lds[wv][hh] * C + lane * VEC, xv);
#pragma unroll
            for (int j = 0; j < VEC; ++j) m[j] = fmaxf(m[j], xv[j]);
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (__ballot(shadow) != 0ull) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) m[j] = fmaxf(m[j], 0.f);
    }
    store_vec<VEC>(out + qi * C + lane * VEC, m);
}

// max_pool: one thread per (query, channel); shadows contribute the appended zero row.
__global__ void max_pool_kernel(const float* __restrict__ x, int64_t ns, int c,
                                const int64_t* __restrict__ idx, int64_t nq, int width,
                                float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq * c) return;
    const int64_t qi = t / c;
    const int ch = (int)(t - qi * c);
    const int64_t* row = idx + qi * width;
    float m = -INFINITY;
    for (int h = 0; h < width; ++h) {
        const int64_t id = row[h];
        const float v = (id >= 0 && id < ns) ? x[id * c + ch] : 0.f;
        m = fmaxf(m, v);
    }
    out[t] = m;
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_kpconv_gather_workspace(int64_t ns, int32_t cin, size_t* bytes) {
    FGR_REQUIRE(bytes && ns >= 0 && cin > 0, "fgr_kpconv_gather_workspace: bad arguments");
    *bytes = 0;       // kept in the ABI; the normaliser's positivity is taken inline now
    return FGR_OK;
}

extern "C" int fgr_kpconv_gather(const float* q, const float* s, int64_t nq, int64_t ns,
                                 const int64_t* idx, int32_t width, const float* x, int32_t cin,
                                 const float* kp, int32_t n_kp, float extent, float* wf,
                                 float* nnorm, void* workspace, size_t ws_bytes, void* stream) {
    (void)workspace; (void)ws_bytes;
    FGR_REQUIRE(nq >= 0 && ns >= 0 && width >= 0 && cin > 0 && n_kp > 0 && n_kp <= kMaxKp &&
                    extent > 0.f,
                "fgr_kpconv_gather: bad arguments (cin %d, n_kp %d, width %d)", cin, n_kp, width);
    FGR_REQUIRE(nq == 0 || (q && s && x && kp && wf && nnorm && (idx || width == 0)),
                "fgr_kpconv_gather: null pointer");
    if (nq == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const float inv_ext = 1.0f / extent;
    if (cin % 64 == 0 && cin <= 256) {
        switch (cin / 64) {
            case 1: launch_wide_k<1>(q, s, nq, ns, idx, width, x, kp, n_kp, inv_ext, wf, nnorm, st); break;
            case 2: launch_wide_k<2>(q, s, nq, ns, idx, width, x, kp, n_kp, inv_ext, wf, nnorm, st); break;
            default: launch_wide_k<4>(q, s, nq, ns, idx, width, x, kp, n_kp, inv_ext, wf, nnorm, st); break;
        }
    } else if (cin <= 64) {
        if (cin == 1) {
            const dim3 grid((unsigned)ceil_div(nq * 16, 256));
            if (n_kp <= 16)
                hipLaunchKernelGGL(kpconv_gather_c1<16>, grid, dim3(256), 0, st, q, s, nq, ns, idx,
                                   width, x, kp, n_kp, inv_ext, wf, nnorm);
            else
                hipLaunchKernelGGL(kpconv_gather_c1<kMaxKp>, grid, dim3(256), 0, st, q, s, nq, ns,
                                   idx, width, x, kp, n_kp, inv_ext, wf, nnorm);
        } else if ((cin == 16 || cin == 32) && n_kp <= 16 &&
                   (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(wf) & 15) == 0) {
            const dim3 grid((unsigned)ceil_div(nq, 4));
            if (cin == 32)
                hipLaunchKernelGGL((kpconv_gather_quads<8, 2>), grid, dim3(256), 0, st, q, s, nq, ns,
                                   idx, width, x, kp, n_kp, inv_ext, wf, nnorm);
            else
                hipLaunchKernelGGL((kpconv_gather_quads<4, 1>), grid, dim3(256), 0, st, q, s, nq, ns,
                                   idx, width, x, kp, n_kp, inv_ext, wf, nnorm);
        } else if (cin <= 8) launch_narrow<8>(q, s, nq, ns, idx, width, x, cin, kp, n_kp, inv_ext, wf, nnorm, st);
        else if (cin <= 16) launch_narrow<16>(q, s, nq, ns, idx, width, x, cin, kp, n_kp, inv_ext, wf, nnorm, st);
        else if (cin <= 32) launch_narrow<32>(q, s, nq, ns, idx, width, x, cin, kp, n_kp, inv_ext, wf, nnorm, st);
        else launch_narrow<64>(q, s, nq, ns, idx, width, x, cin, kp, n_kp, inv_ext, wf, nnorm, st);
    } else {
        set_error("fgr_kpconv_gather: cin %d unsupported (need <= 64 or a multiple of 64 <= 256)", cin);
        return FGR_E_ARG;
    }
    FGR_CHECK_LAUNCH("kpconv_gather");
    return FGR_OK;
}

extern "C" int fgr_max_pool(const float* x, int64_t ns, int32_t c, const int64_t* idx, int64_t nq,
                            int32_t width, float* out, void* stream) {
    FGR_REQUIRE(ns >= 0 && c > 0 && nq >= 0 && width > 0, "fgr_max_pool: bad arguments");
    FGR_REQUIRE(nq == 0 || (x && idx && out), "fgr_max_pool: null pointer");
    if (nq == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    if (c == 64 || c == 128 || c == 256 || c == 512) {
        dim3 grid((unsigned)ceil_div(nq, 4));
        if (c == 64) hipLaunchKernelGGL(max_pool_wave<1>, grid, dim3(256), 0, st, x, ns, idx, nq, width, out);
        else if (c == 128) hipLaunchKernelGGL(max_pool_wave<2>, grid, dim3(256), 0, st, x, ns, idx, nq, width, out);
        else if (c == 256) hipLaunchKernelGGL(max_pool_wave<4>, grid, dim3(256), 0, st, x, ns, idx, nq, width, out);
        else hipLaunchKernelGGL(max_pool_wave<8>, grid, dim3(256), 0, st, x, ns, idx, nq, width, out);
    } else {
        const int64_t n = nq * c;
        hipLaunchKernelGGL(max_pool_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, x,
                           ns, c, idx, nq, width, out);
    }
    FGR_CHECK_LAUNCH("max_pool_kernel");
    return FGR_OK;
}
