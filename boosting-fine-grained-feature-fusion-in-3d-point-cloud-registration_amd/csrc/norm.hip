// Normalisation / embedding kernels on gfx950: segmented instance norm (per cloud),
// row LayerNorm (+ positional add), sine coordinate embedding.
#include "common.h"

namespace fgr {
namespace {

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == FGR_ACT_LEAKY) return v > 0.f ? v : 0.1f * v;  // nn.LeakyReLU(0.1)
    if (act == FGR_ACT_RELU) return fmaxf(v, 0.f);
    return v;
}

// Segmented instance norm. Block = 16 waves x 64 channels (lane = channel); a block
// owns a chunk of up to kChunk rows of one segment and keeps it in registers
// (kRpw rows per wave), so x is read from HBM once. Segments longer than one chunk
// are reduced in two launches: per-chunk (n, mean, M2) partials, then a Chan merge
// fused with the normalising write.
constexpr int kInW = 16;               // waves per block
constexpr int kRpw = 48;               // rows per wave held in registers (no spills)
constexpr int kChunk = kInW * kRpw;    // rows per block

struct InArgs {
    const float* x;
    int c;
    const int64_t* seg_off;
    const float* row_div;
    float eps;
    int act;
    const float* residual;
    int post_act;
    float* out;
    float* part;      // [n_seg][n_chunks][3][c] partials (multi-chunk only)
    int n_chunks;
};

__device__ __forceinline__ float block_sum16(float v, float (*red)[64], int wv, int lane) {
    red[wv][lane] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kInW; ++w) t += red[w][lane];
    __syncthreads();
    return t;
}

// MODE 0: single chunk -> stats + normalise; MODE 1: write partials; MODE 2: merge + normalise.
template <int MODE>
__global__ void __launch_bounds__(64 * kInW) instnorm_chunk_kernel(InArgs a) {
    __shared__ float red[kInW][64];
    const int seg = blockIdx.y, chunk = blockIdx.z;
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int ch = blockIdx.x * 64 + lane;
    const bool cok = ch < a.c;
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    const int64_t cb = b + (int64_t)chunk * kChunk;
    if (cb >= e && !(MODE == 0 && chunk == 0)) return;      // block-uniform
    if (e <= b) return;
    const int64_t ce = min(e, cb + kChunk);
    float v[kRpw];
    float s = 0.f;
    const int nrow = (int)(ce - cb);                     // rows of this chunk (<= kChunk)
    const int step = kInW * a.c;
    {
        // loads first (clamped rows / channel, masked afterwards): all in flight together
        const int chc = cok ? ch : 0;
        float dv[kRpw];
#pragma unroll
        for (int j = 0; j < kRpw; ++j) {
            const int rr = min(wv + kInW * j, nrow - 1);
            v[j] = a.x[(cb + rr) * a.c + chc];
            dv[j] = a.row_div ? a.row_div[cb + rr] : 1.f;
        }
#pragma unroll
        for (int j = 0; j < kRpw; ++j) {
            const bool ok = wv + kInW * j < nrow && cok;
            v[j] = ok ? (a.row_div ? v[j] / dv[j] : v[j]) : 0.f;
            s += v[j];
        }
    }
    float mean, rstd;
    if (MODE == 2) {
        // merge the per-chunk partials of this segment (Chan et al.)
        float n = 0.f, m = 0.f, m2 = 0.f;
        const float* pp = a.part + (int64_t)seg * a.n_chunks * 3 * a.c;
        for (int k = 0; k < a.n_chunks; ++k) {
            const int64_t kb = b + (int64_t)k * kChunk;
            if (kb >= e || !cok) break;
            const float nb = pp[(k * 3 + 0) * a.c + ch];
            const float mb = pp[(k * 3 + 1) * a.c + ch];
            const float qb = pp[(k * 3 + 2) * a.c + ch];
            const float nn = n + nb;
            const float d = mb - m;
            m = m + d * (nb / nn);
            m2 = m2 + qb + d * d * (n * nb / nn);
            n = nn;
        }
        mean = m;
        rstd = 1.0f / sqrtf(m2 / (float)(e - b) + a.eps);
    } else {
        const float cnt = (float)(ce - cb);
        mean = block_sum16(s, red, wv, lane) / cnt;
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < kRpw; ++j) {
            const float d = (wv + kInW * j < nrow) ? v[j] - mean : 0.f;
            sq += d * d;
        }
        const float m2 = block_sum16(sq, red, wv, lane);
        if (MODE == 1) {
            if (wv == 0 && cok) {
                float* pp = a.part + ((int64_t)seg * a.n_chunks + chunk) * 3 * a.c;
                pp[0 * a.c + ch] = cnt;
                pp[1 * a.c + ch] = mean;
                pp[2 * a.c + ch] = m2;
            }
            return;
        }
        rstd = 1.0f / sqrtf(m2 / cnt + a.eps);
    }
    if (!cok) return;
    const int64_t o0 = (cb + wv) * a.c + ch;
    const float* rp = a.residual ? a.residual + o0 : nullptr;
    float* op = a.out + o0;
#pragma unroll
    for (int j = 0; j < kRpw; ++j) {
        if (wv + kInW * j < nrow) {
            float y = act_fn((v[j] - mean) * rstd, a.act);
            if (rp) y = act_fn(y + rp[j * step], a.post_act);
            op[j * step] = y;
        }
    }
}

// Segmented instance norm, one block per (16 channels, segment) for segments of up to
// kSegRows rows: 16 waves x 4 row-lanes x 16 channel-lanes, every value held in registers
// (x read from HBM once). 16 channels per block give C/16 x n_seg blocks -- 4x the blocks
// of the 64-channel chunk kernel, which left most CUs idle at 16 clouds x 256 channels.
constexpr int kSegRpl = 16;                        // rows per lane
constexpr int kSegRows = kSegRpl * 4 * kInW;       // 1024

__device__ __forceinline__ float xg16_32_sum(float v) {   // sum over lanes l, l^16, l^32, l^48
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
}

template <int VEC>
__global__ void __launch_bounds__(64 * kInW) instnorm_seg16_kernel(InArgs a) {
    // VEC consecutive channels per lane (VEC = 2: 8-B accesses, 128-B row segments per 16
    // lanes, for C >= 512 where C / 32 x n_seg blocks still fill the chip)
    __shared__ float red[kInW][16 * VEC];
    const int seg = blockIdx.y;
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int rl = lane >> 4, cc = lane & 15;
    const int ch = (blockIdx.x * 16 + cc) * VEC;
    const bool cok = ch < a.c;                           // C % VEC == 0 (checked by the caller)
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    const int nrow = (int)(e - b);
    if (nrow <= 0) return;
    const int r0 = wv * 4 + rl;                          // this lane's first row
    // every load issued before any use (clamped rows / channels, masked afterwards), so a
    // lane's 16 loads are in flight together instead of one round trip each
    const int chc = cok ? ch : 0;
    // segment-uniform bases + 32-bit lane offsets (one scalar base, no 64-bit address per row)
    const float* xs = a.x + b * a.c;
    float v[kSegRpl][VEC], dv[kSegRpl];
#pragma unroll
    for (int j = 0; j < kSegRpl; ++j) {
        const int rr = min(r0 + 64 * j, nrow - 1);
        const float* src = xs + (uint32_t)(rr * a.c + chc);
        if constexpr (VEC == 2) {
            const float2 t = *reinterpret_cast<const float2*>(src);
            v[j][0] = t.x; v[j][1] = t.y;
        } else {
            v[j][0] = *src;
        }
        dv[j] = a.row_div ? a.row_div[b + rr] : 1.f;
    }
    float s[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) s[u] = 0.f;
#pragma unroll
    for (int j = 0; j < kSegRpl; ++j) {
        const bool ok = r0 + 64 * j < nrow && cok;
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
            v[j][u] = ok ? (a.row_div ? v[j][u] / dv[j] : v[j][u]) : 0.f;
            s[u] += v[j][u];
        }
    }
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
        s[u] = xg16_32_sum(s[u]);
        if (rl == 0) red[wv][cc * VEC + u] = s[u];
    }
    __syncthreads();
    const float cnt = (float)nrow;
    float mean[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < kInW; ++w) tot += red[w][cc * VEC + u];
        mean[u] = tot / cnt;
    }
    __syncthreads();
    float sq[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) sq[u] = 0.f;
#pragma unroll
    for (int j = 0; j < kSegRpl; ++j)
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
            const float d = (r0 + 64 * j < nrow) ? v[j][u] - mean[u] : 0.f;
            sq[u] += d * d;
        }
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
        sq[u] = xg16_32_sum(sq[u]);
        if (rl == 0) red[wv][cc * VEC + u] = sq[u];
    }
    __syncthreads();
    float rstd[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
        float m2 = 0.f;
#pragma unroll
        for (int w = 0; w < kInW; ++w) m2 += red[w][cc * VEC + u];
        rstd[u] = 1.0f / sqrtf(m2 / cnt + a.eps);
    }
    if (!cok) return;
    float rv[kSegRpl][VEC];
    if (a.residual) {
#pragma unroll
        for (int j = 0; j < kSegRpl; ++j) {
            const float* src = a.residual + b * a.c + (uint32_t)(min(r0 + 64 * j, nrow - 1) * a.c + ch);
            if constexpr (VEC == 2) {
                const float2 t = *reinterpret_cast<const float2*>(src);
                rv[j][0] = t.x; rv[j][1] = t.y;
            } else {
                rv[j][0] = *src;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kSegRpl; ++j) {
        const int rr = r0 + 64 * j;
        if (rr < nrow) {
            float* const dst = a.out + b * a.c + (uint32_t)(rr * a.c + ch);
            float y[VEC];
#pragma unroll
            for (int u = 0; u < VEC; ++u) {
                y[u] = act_fn((v[j][u] - mean[u]) * rstd[u], a.act);
                if (a.residual) y[u] = act_fn(y[u] + rv[j][u], a.post_act);
            }
            if constexpr (VEC == 2) *reinterpret_cast<float2*>(dst) = make_float2(y[0], y[1]);
            else *dst = y[0];
        }
    }
}

// Segmented instance norm for long segments (> kSegRows rows, e.g. 3DMatch's 20k-row clouds),
// three launches that keep every CU busy (the register-resident chunk kernel above runs
// only C/64 x n_seg x rows/768 blocks -- ~100 at 2 x 20k x 64):
//   1. stats: one 256-thread block per (segment, chunk of kLsIter x kLsRpi rows), 16-B loads
//      (TPR = C/4 threads per row), shifted sums S = sum(v - K), Q = sum((v - K)^2) with the
//      segment's first row as the pivot K (no cancellation when |mean| >> std);
//   2. merge: per (segment, channel) the chunk partials in fp64 -> mean, rstd;
//   3. apply: the same chunks, (v - mean) * rstd -> act (-> + residual -> post_act), 16-B stores.
// v = x / row_div (when given) is recomputed identically in passes 1 and 3.
constexpr int kLsIter = 4;                 // row iterations per block (16 KB of x per block)

struct LsArgs {
    const float* x;
    int c, tpr, rpi, rows;                 // channels, threads per row (c/4), rows per iteration, rows per chunk
    const int64_t* seg_off;
    int n_chunks;
    const float* row_div;
    float eps;
    int act;
    const float* residual;
    int post_act;
    float* out;
    float* part;                           // [n_seg][n_chunks][2][c] (S, Q)
    float* stats;                          // [n_seg][2][c] (mean, rstd)
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__global__ void __launch_bounds__(256) instnorm_ls_stats_kernel(LsArgs a) {
    __shared__ float4 red[2][256];
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * a.rows;
    if (r0 >= e) return;                                   // block-uniform
    const int64_t r1 = min(e, r0 + a.rows);
    const int t = threadIdx.x, cg = t % a.tpr, rr = t / a.tpr;
    const int col = 4 * cg;
    float4 k = ld4(a.x + b * a.c + col);                   // pivot: the segment's first row
    if (a.row_div) {
        const float d = a.row_div[b];
        k.x = k.x / d; k.y = k.y / d; k.z = k.z / d; k.w = k.w / d;
    }
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
    // kLsIter rows per thread, loads issued together (clamped, masked afterwards)
    float4 xv[kLsIter];
    float dv[kLsIter];
#pragma unroll
    for (int it = 0; it < kLsIter; ++it) {
        const int64_t r = min(r0 + rr + (int64_t)it * a.rpi, r1 - 1);
        xv[it] = ld4(a.x + r * a.c + col);
        dv[it] = a.row_div ? a.row_div[r] : 1.f;
    }
#pragma unroll
    for (int it = 0; it < kLsIter; ++it) {
        if (r0 + rr + (int64_t)it * a.rpi >= r1) break;
        float4 v = xv[it];
        if (a.row_div) {
            const float d = dv[it];
            v.x = v.x / d; v.y = v.y / d; v.z = v.z / d; v.w = v.w / d;
        }
        const float dx = v.x - k.x, dy = v.y - k.y, dz = v.z - k.z, dw = v.w - k.w;
        s.x += dx; s.y += dy; s.z += dz; s.w += dw;
        q.x += dx * dx; q.y += dy * dy; q.z += dz * dz; q.w += dw * dw;
    }
    red[0][t] = s;
    red[1][t] = q;
    __syncthreads();
    if (rr != 0) return;
    for (int j = 1; j < a.rpi; ++j) {
        const float4 s2 = red[0][t + j * a.tpr], q2 = red[1][t + j * a.tpr];
        s.x += s2.x; s.y += s2.y; s.z += s2.z; s.w += s2.w;
        q.x += q2.x; q.y += q2.y; q.z += q2.z; q.w += q2.w;
    }
    float* pp = a.part + ((int64_t)seg * a.n_chunks + chunk) * 2 * a.c;
    *reinterpret_cast<float4*>(pp + col) = s;
    *reinterpret_cast<float4*>(pp + a.c + col) = q;
}

// one 1024-thread block per (64-channel group, segment): lane = channel, the 16 waves
// stride over the chunks (coalesced 256-B rows of partials), fp64 sums merged through LDS
__global__ void __launch_bounds__(1024) instnorm_ls_merge_kernel(LsArgs a) {
    __shared__ double red[2][16][64];
    const int seg = blockIdx.y;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ch = blockIdx.x * 64 + lane;
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    if (e <= b) return;                                    // block-uniform
    const int nch = (int)((e - b + a.rows - 1) / a.rows);
    double S = 0.0, Q = 0.0;
    if (ch < a.c) {
        const float* pp = a.part + (int64_t)seg * a.n_chunks * 2 * a.c + ch;
#pragma unroll 4
        for (int k = wv; k < nch; k += 16) {
            S += (double)pp[(int64_t)k * 2 * a.c];
            Q += (double)pp[(int64_t)k * 2 * a.c + a.c];
        }
    }
    red[0][wv][lane] = S;
    red[1][wv][lane] = Q;
    __syncthreads();
    if (wv != 0 || ch >= a.c) return;
    S = 0.0;
    Q = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        S += red[0][w][lane];
        Q += red[1][w][lane];
    }
    float kv = a.x[b * a.c + ch];
    if (a.row_div) kv = kv / a.row_div[b];
    const double n = (double)(e - b);
    const double m = S / n;
    const double var = fmax(Q / n - m * m, 0.0);          // biased, of the shifted values
    a.stats[((int64_t)seg * 2) * a.c + ch] = (float)((double)kv + m);
    a.stats[((int64_t)seg * 2 + 1) * a.c + ch] = 1.0f / sqrtf((float)var + a.eps);
}

__global__ void __launch_bounds__(256) instnorm_ls_apply_kernel(LsArgs a) {
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * a.rows;
    if (r0 >= e) return;
    const int64_t r1 = min(e, r0 + a.rows);
    const int t = threadIdx.x, cg = t % a.tpr, rr = t / a.tpr;
    const int col = 4 * cg;
    const float4 mean = ld4(a.stats + ((int64_t)seg * 2) * a.c + col);
    const float4 rstd = ld4(a.stats + ((int64_t)seg * 2 + 1) * a.c + col);
    float4 xv[kLsIter], rv[kLsIter];
    float dv[kLsIter];
#pragma unroll
    for (int it = 0; it < kLsIter; ++it) {
        const int64_t r = min(r0 + rr + (int64_t)it * a.rpi, r1 - 1);
        xv[it] = ld4(a.x + r * a.c + col);
        dv[it] = a.row_div ? a.row_div[r] : 1.f;
        if (a.residual) rv[it] = ld4(a.residual + r * a.c + col);
    }
#pragma unroll
    for (int it = 0; it < kLsIter; ++it) {
        const int64_t r = r0 + rr + (int64_t)it * a.rpi;
        if (r >= r1) break;
        float4 v = xv[it];
        if (a.row_div) {
            const float d = dv[it];
            v.x = v.x / d; v.y = v.y / d; v.z = v.z / d; v.w = v.w / d;
        }
        float4 y;
        y.x = act_fn((v.x - mean.x) * rstd.x, a.act);
        y.y = act_fn((v.y - mean.y) * rstd.y, a.act);
        y.z = act_fn((v.z - mean.z) * rstd.z, a.act);
        y.w = act_fn((v.w - mean.w) * rstd.w, a.act);
        if (a.residual) {
            y.x = act_fn(y.x + rv[it].x, a.post_act);
            y.y = act_fn(y.y + rv[it].y, a.post_act);
            y.z = act_fn(y.z + rv[it].z, a.post_act);
            y.w = act_fn(y.w + rv[it].w, a.post_act);
        }
        *reinterpret_cast<float4*>(a.out + r * a.c + col) = y;
    }
}

// the long-segment path applies when C/4 threads per row tile a 256-thread block
inline bool ls_ok(int c) { return c % 4 == 0 && c / 4 <= 256 && 256 % (c / 4) == 0; }
inline int ls_rows(int c) { return (256 / (c / 4)) * kLsIter; }

// LayerNorm, LPR lanes per row (16 / 32 / 64: 16 / 8 / 4 rows per 256-thread block), d % 64
// == 0 and d <= 4 * LPR * NV: each lane holds NV float4 (16-B loads / stores). Every load of
// the row (x, pre_bias, gamma, beta, add) is issued before the reductions, so a row costs
// one memory round trip; row sums on DPP within 16-lane rows, then permlane16 / 32 swaps.
// `pre_bias` as in layernorm_kernel below.
template <int LPR>
__device__ __forceinline__ float lpr_sum(float v) {
    v = row16_sum(v);
    if constexpr (LPR >= 32) {
        auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    }
    if constexpr (LPR >= 64) {
        auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    }
    return v;
}

// DUAL: a second affine output from the same statistics, out2 = xhat * g2 + b2 (+ add2) (the
// encoder's output norm of layer l and norm1 (+ pos) of layer l + 1 read the same rows)
template <int LPR, int NV, bool DUAL = false>
__global__ void __launch_bounds__(256)
layernorm_lpr_kernel(float* __restrict__ x, int64_t n, int d, const float* __restrict__ g,
                     const float* __restrict__ bta, float eps, const float* __restrict__ add,
                     const float* __restrict__ pre_bias, float* __restrict__ out,
                     const float* __restrict__ g2 = nullptr, const float* __restrict__ b2 = nullptr,
                     const float* __restrict__ add2 = nullptr, float* __restrict__ out2 = nullptr) {
    constexpr int RPB = 256 / LPR;
    const int64_t r = (int64_t)blockIdx.x * RPB + threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const bool ok = r < n;                               // keep all lanes for the DPP sums
    const int64_t rr = ok ? r : n - 1;
    float4 v[NV], gg[NV], bb[NV], ad[NV];
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    // every load unconditional (column clamped into the row, chunks past d zeroed after):
    // guarded loads had put these arrays in scratch (round 5)
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int col = min(4 * (l + LPR * j), d - 4);
        v[j] = *reinterpret_cast<const float4*>(x + rr * d + col);
        gg[j] = *reinterpret_cast<const float4*>(g + col);
        bb[j] = *reinterpret_cast<const float4*>(bta + col);
    }
    if (add) {
#pragma unroll
        for (int j = 0; j < NV; ++j)
            ad[j] = *reinterpret_cast<const float4*>(add + rr * d + min(4 * (l + LPR * j), d - 4));
    } else {
#pragma unroll
        for (int j = 0; j < NV; ++j) ad[j] = z;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
        if (4 * (l + LPR * j) >= d) v[j] = z;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int col = 4 * (l + LPR * j);
        if (pre_bias && col < d) {
            const float4 pb = *reinterpret_cast<const float4*>(pre_bias + col);
            v[j].x += pb.x; v[j].y += pb.y; v[j].z += pb.z; v[j].w += pb.w;
            if (ok) *reinterpret_cast<float4*>(x + rr * d + col) = v[j];
        }
        s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    }
    const float mean = lpr_sum<LPR>(s) / (float)d;
    float sq = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        if (4 * (l + LPR * j) < d) {
            const float a0 = v[j].x - mean, a1 = v[j].y - mean, a2 = v[j].z - mean, a3 = v[j].w - mean;
            sq += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
        }
    }
    const float rstd = 1.0f / sqrtf(lpr_sum<LPR>(sq) / (float)d + eps);
    if (!ok) return;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int col = 4 * (l + LPR * j);
        if (col < d) {
            float4 y;
            y.x = (v[j].x - mean) * rstd * gg[j].x + bb[j].x + ad[j].x;
            y.y = (v[j].y - mean) * rstd * gg[j].y + bb[j].y + ad[j].y;
            y.z = (v[j].z - mean) * rstd * gg[j].z + bb[j].z + ad[j].z;
            y.w = (v[j].w - mean) * rstd * gg[j].w + bb[j].w + ad[j].w;
            *reinterpret_cast<float4*>(out + r * d + col) = y;
            if constexpr (DUAL) {
                const float4 g4 = *reinterpret_cast<const float4*>(g2 + col);
                const float4 b4 = *reinterpret_cast<const float4*>(b2 + col);
                const float4 a4 = add2 ? *reinterpret_cast<const float4*>(add2 + r * d + col)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
                float4 z;
                z.x = (v[j].x - mean) * rstd * g4.x + b4.x + a4.x;
                z.y = (v[j].y - mean) * rstd * g4.y + b4.y + a4.y;
                z.z = (v[j].z - mean) * rstd * g4.z + b4.z + a4.z;
                z.w = (v[j].w - mean) * rstd * g4.w + b4.w + a4.w;
                *reinterpret_cast<float4*>(out2 + r * d + col) = z;
            }
        }
    }
}

// One wave per row; d <= 64 * 16.
// `pre_bias` (optional): x[r] += pre_bias is applied first and written back to x (the
// pending Linear bias of the residual branch that produced x), then normalised.
template <int PER>
__global__ void __launch_bounds__(256)
layernorm_kernel(float* __restrict__ x, int64_t n, int d, const float* __restrict__ g,
                 const float* __restrict__ bta, float eps, const float* __restrict__ add,
                 const float* __restrict__ pre_bias, float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const int lane = threadIdx.x % 64;
    if (r >= n) return;
    float* xr = x + r * d;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int col = lane + 64 * j;
        v[j] = col < d ? xr[col] : 0.f;
        if (pre_bias && col < d) {
            v[j] += pre_bias[col];
            xr[col] = v[j];
        }
        s += v[j];
    }
    const float mean = wave_sum(s) / (float)d;
    float sq = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int col = lane + 64 * j;
        const float dd = col < d ? v[j] - mean : 0.f;
        sq += dd * dd;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)d + eps);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int col = lane + 64 * j;
        if (col < d) {
            float y = (v[j] - mean) * rstd * g[col] + bta[col];
            if (add) y += add[r * d + col];
            out[r * d + col] = y;
        }
    }
}

// PositionEmbeddingCoordsSine, n_dim = 3 (position_embedding.py:29-49):
//   npf = d // 3 // 2 * 2; dim_t[i] = T ** (2 * (i // 2) / npf);
//   out[3 * ... ] interleaves sin (even i) / cos (odd i) of xyz_d * scale / dim_t,
//   grouped per coordinate, then zero padding to d.
// kPeRows rows per 256-thread block; the npf/2 distinct dim_t values are computed once per
// block into LDS (same powf expression, so the same bits as computing them per element).
constexpr int kPeRows = 8;
constexpr int kPeMaxPairs = 512;

__global__ void __launch_bounds__(256)
sine_pe_kernel(const float* __restrict__ xyz, int64_t n, int d, int npf, float temperature,
               float scale, float* __restrict__ out) {
    __shared__ float dim_t[kPeMaxPairs];
    for (int p = threadIdx.x; p < npf / 2; p += blockDim.x)
        dim_t[p] = powf(temperature, (float)(2 * p) / (float)npf);
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * kPeRows;
    const int rows = (int)min<int64_t>(kPeRows, n - r0);
    for (int e = threadIdx.x; e < rows * d; e += blockDim.x) {
        const int rr = e / d, col = e - rr * d;
        const int64_t r = r0 + rr;
        float y = 0.f;
        if (col < 3 * npf) {
            const int dim = col / npf, i = col - dim * npf;
            // torch: stack([sin(pd[..., 0::2]), cos(pd[..., 1::2])], -1).reshape -> (sin, cos)
            // pairs; sin uses even feature 2p, cos odd 2p+1, both with dim_t[p]
            const int pair = i >> 1, is_cos = i & 1;
            const float pd = (xyz[r * 3 + dim] * scale) / dim_t[pair];
            y = is_cos ? cosf(pd) : sinf(pd);
        }
        out[r * d + col] = y;
    }
}

// out = a + b elementwise (the post-norm layer's `with_pos_embed`, transformers.py:121-124):
// 16-B accesses, four per thread in flight.
__global__ void __launch_bounds__(256)
add4_kernel(const float4* __restrict__ a, const float4* __restrict__ b, int64_t n4,
            float4* __restrict__ out) {
    const int64_t i0 = ((int64_t)blockIdx.x * 256 * 4) + threadIdx.x;
    float4 va[4], vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + 256 * u;
        if (i < n4) { va[u] = a[i]; vb[u] = b[i]; }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + 256 * u;
        if (i < n4)
            out[i] = make_float4(va[u].x + vb[u].x, va[u].y + vb[u].y, va[u].z + vb[u].z,
                                 va[u].w + vb[u].w);
    }
}

__global__ void __launch_bounds__(256)
add1_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
            float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = a[i] + b[i];
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_add(const float* a, const float* b, int64_t n, float* out, void* stream) {
    FGR_REQUIRE(n >= 0, "fgr_add: bad arguments");
    FGR_REQUIRE(n == 0 || (a && b && out), "fgr_add: null pointer");
    if (n == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    const bool vec = n % 4 == 0 && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                                     reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    if (vec)
        hipLaunchKernelGGL(add4_kernel, dim3((unsigned)ceil_div(n / 4, 1024)), dim3(256), 0, st,
                           reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b),
                           n / 4, reinterpret_cast<float4*>(out));
    else
        hipLaunchKernelGGL(add1_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, a, b, n, out);
    FGR_CHECK_LAUNCH("add_kernel");
    return FGR_OK;
}

extern "C" int fgr_instnorm_workspace(int64_t max_seg_len, int32_t c, int32_t n_seg,
                                      size_t* bytes) {
    FGR_REQUIRE(bytes && max_seg_len >= 0 && c > 0 && n_seg > 0, "fgr_instnorm_workspace: bad arguments");
    if (max_seg_len > kSegRows && ls_ok(c)) {
        const int64_t chunks = ceil_div(max_seg_len, ls_rows(c));
        *bytes = (size_t)n_seg * (chunks + 1) * 2 * c * sizeof(float);
        return FGR_OK;
    }
    const int64_t chunks = ceil_div(max_seg_len, kChunk);
    *bytes = chunks > 1 ? (size_t)n_seg * chunks * 3 * c * sizeof(float) : 0;
    return FGR_OK;
}

extern "C" int fgr_instnorm(const float* x, int64_t n, int32_t c, const int64_t* seg_off,
                            int32_t n_seg, int64_t max_seg_len, const float* row_div, float eps,
                            int32_t act, const float* residual, int32_t post_act, float* out,
                            void* ws, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(n >= 0 && c > 0 && n_seg > 0 && seg_off && eps >= 0.f && max_seg_len >= 0,
                "fgr_instnorm: bad arguments");
    FGR_REQUIRE(n == 0 || (x && out), "fgr_instnorm: null pointer");
    if (n == 0 || max_seg_len == 0) return FGR_OK;
    const int64_t chunks = ceil_div(max_seg_len, kChunk);
    InArgs a{x, c, seg_off, row_div, eps, act, residual, post_act, out, (float*)ws, (int)chunks};
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const unsigned cx = (unsigned)ceil_div(c, 64);
    if (max_seg_len <= kSegRows) {
        // 2 channels per lane for wide features (C / 32 x n_seg blocks) when 8-B aligned
        const bool v2 = c >= 512 && c % 2 == 0 &&
                        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                          reinterpret_cast<uintptr_t>(residual)) & 7) == 0;
        if (v2)
            hipLaunchKernelGGL(instnorm_seg16_kernel<2>, dim3((unsigned)ceil_div(c, 32), n_seg, 1),
                               dim3(64 * kInW), 0, st, a);
        else
            hipLaunchKernelGGL(instnorm_seg16_kernel<1>, dim3((unsigned)ceil_div(c, 16), n_seg, 1),
                               dim3(64 * kInW), 0, st, a);
    } else if (ls_ok(c)) {
        const int rows = ls_rows(c);
        const int64_t lc = ceil_div(max_seg_len, rows);
        const size_t need = (size_t)n_seg * (lc + 1) * 2 * c * sizeof(float);
        FGR_REQUIRE(ws && ws_bytes >= need &&
                        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                          reinterpret_cast<uintptr_t>(residual) |
                          reinterpret_cast<uintptr_t>(ws)) & 15) == 0,
                    "fgr_instnorm: workspace %zu < %zu bytes or operands not 16-B aligned",
                    ws_bytes, need);
        float* part = (float*)ws;
        LsArgs la{x, c, c / 4, 256 / (c / 4), rows, seg_off, (int)lc, row_div, eps, act,
                  residual, post_act, out, part, part + (size_t)n_seg * lc * 2 * c};
        hipLaunchKernelGGL(instnorm_ls_stats_kernel, dim3((unsigned)lc, n_seg), dim3(256), 0, st, la);
        FGR_CHECK_LAUNCH("instnorm_ls_stats_kernel");
        hipLaunchKernelGGL(instnorm_ls_merge_kernel, dim3((unsigned)ceil_div(c, 64), n_seg), dim3(1024),
                           0, st, la);
        FGR_CHECK_LAUNCH("instnorm_ls_merge_kernel");
        hipLaunchKernelGGL(instnorm_ls_apply_kernel, dim3((unsigned)lc, n_seg), dim3(256), 0, st, la);
    } else if (chunks == 1) {
        hipLaunchKernelGGL(instnorm_chunk_kernel<0>, dim3(cx, n_seg, 1), dim3(64 * kInW), 0, st, a);
    } else {
        const size_t need = (size_t)n_seg * chunks * 3 * c * sizeof(float);
        if (!ws || ws_bytes < need) {
            set_error("fgr_instnorm: workspace %zu < %zu bytes", ws_bytes, need);
            return FGR_E_WORKSPACE;
        }
        hipLaunchKernelGGL(instnorm_chunk_kernel<1>, dim3(cx, n_seg, (unsigned)chunks), dim3(64 * kInW), 0, st, a);
        FGR_CHECK_LAUNCH("instnorm_partials");
        hipLaunchKernelGGL(instnorm_chunk_kernel<2>, dim3(cx, n_seg, (unsigned)chunks), dim3(64 * kInW), 0, st, a);
    }
    FGR_CHECK_LAUNCH("instnorm_kernel");
    return FGR_OK;
}

extern "C" int fgr_layernorm(float* x, int64_t n, int32_t d, const float* gamma,
                             const float* beta, float eps, const float* add,
                             const float* pre_bias, float* out, void* stream) {
    FGR_REQUIRE(n >= 0 && d > 0 && d <= 1024 && gamma && beta, "fgr_layernorm: bad arguments");
    FGR_REQUIRE(n == 0 || (x && out), "fgr_layernorm: null pointer");
    if (n == 0) return FGR_OK;
    dim3 grid((unsigned)ceil_div(n, 4));
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const bool vec = d % 64 == 0 && d <= 1024 &&
                     ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                       reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta) |
                       reinterpret_cast<uintptr_t>(add) | reinterpret_cast<uintptr_t>(pre_bias)) & 15) == 0;
    if (vec) {
        // lanes per row sized so each lane holds at most 4 float4 (rows stay in flight)
        // d <= 256: 32 lanes per row (2 float4 each; measured 6-7 % faster than 16 lanes x 4 at
        // 9544 x 256, tools/ln_bench.py); FGR_LN_LPR = 16 / 64 selects the others (A/B)
        const char* lp = getenv("FGR_LN_LPR");
        const int lpr = (lp && lp[0]) ? atoi(lp) : 32;
        if (d <= 128 && lpr == 32)
            hipLaunchKernelGGL((layernorm_lpr_kernel<32, 1>), dim3((unsigned)ceil_div(n, 8)),
                               dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
        else if (d <= 256 && lpr == 32)
            hipLaunchKernelGGL((layernorm_lpr_kernel<32, 2>), dim3((unsigned)ceil_div(n, 8)),
                               dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
        else if (d <= 256 && lpr == 64)
            hipLaunchKernelGGL((layernorm_lpr_kernel<64, 1>), dim3((unsigned)ceil_div(n, 4)),
                               dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
        else if (d <= 256)
            hipLaunchKernelGGL((layernorm_lpr_kernel<16, 4>), dim3((unsigned)ceil_div(n, 16)),
                               dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
        else if (d <= 512)
            hipLaunchKernelGGL((layernorm_lpr_kernel<32, 4>), dim3((unsigned)ceil_div(n, 8)),
                               dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
        else
            hipLaunchKernelGGL((layernorm_lpr_kernel<64, 4>), dim3((unsigned)ceil_div(n, 4)),
                               dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
    } else if (d <= 64)
        hipLaunchKernelGGL(layernorm_kernel<1>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
    else if (d <= 256)
        hipLaunchKernelGGL(layernorm_kernel<4>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
    else if (d <= 512)
        hipLaunchKernelGGL(layernorm_kernel<8>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
    else
        hipLaunchKernelGGL(layernorm_kernel<16>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, pre_bias, out);
    FGR_CHECK_LAUNCH("layernorm_kernel");
    return FGR_OK;
}

extern "C" int fgr_sine_pos_embed(const float* xyz, int64_t n, int32_t d_model, float temperature,
                                  float scale, float* out, void* stream) {
    FGR_REQUIRE(n >= 0 && d_model >= 6, "fgr_sine_pos_embed: bad arguments");
    FGR_REQUIRE(n == 0 || (xyz && out), "fgr_sine_pos_embed: null pointer");
    if (n == 0) return FGR_OK;
    const int npf = d_model / 3 / 2 * 2;
    FGR_REQUIRE(npf / 2 <= kPeMaxPairs, "fgr_sine_pos_embed: d_model %d too large", d_model);
    hipLaunchKernelGGL(sine_pe_kernel, dim3((unsigned)ceil_div(n, kPeRows)), dim3(256), 0,
                       as_stream(stream), xyz, n, d_model, npf, temperature, scale, out);
    FGR_CHECK_LAUNCH("sine_pe_kernel");
    return FGR_OK;
}

extern "C" int fgr_layernorm_dual(const float* x, int64_t n, int32_t d, const float* gamma,
                                  const float* beta, const float* add, float* out,
                                  const float* gamma2, const float* beta2, const float* add2,
                                  float* out2, float eps, void* stream) {
    FGR_REQUIRE(n >= 0 && d > 0 && d <= 1024 && gamma && beta && gamma2 && beta2,
                "fgr_layernorm_dual: bad arguments");
    FGR_REQUIRE(n == 0 || (x && out && out2), "fgr_layernorm_dual: null pointer");
    if (n == 0) return FGR_OK;
    const bool vec = d % 64 == 0 && d <= 512 &&
                     ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                       reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta) |
                       reinterpret_cast<uintptr_t>(add) | reinterpret_cast<uintptr_t>(out2) |
                       reinterpret_cast<uintptr_t>(gamma2) | reinterpret_cast<uintptr_t>(beta2) |
                       reinterpret_cast<uintptr_t>(add2)) & 15) == 0;
    if (!vec) {                       // two passes of fgr_layernorm
        const int r1 = fgr_layernorm(const_cast<float*>(x), n, d, gamma, beta, eps, add, nullptr, out, stream);
        if (r1 != FGR_OK) return r1;
        return fgr_layernorm(const_cast<float*>(x), n, d, gamma2, beta2, eps, add2, nullptr, out2, stream);
    }
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    float* xm = const_cast<float*>(x);                 // read only (no pre_bias)
    if (d <= 128)
        hipLaunchKernelGGL((layernorm_lpr_kernel<32, 1, true>), dim3((unsigned)ceil_div(n, 8)), dim3(256), 0,
                           st, xm, n, d, gamma, beta, eps, add, nullptr, out, gamma2, beta2, add2, out2);
    else if (d <= 256)
        hipLaunchKernelGGL((layernorm_lpr_kernel<32, 2, true>), dim3((unsigned)ceil_div(n, 8)), dim3(256), 0,
                           st, xm, n, d, gamma, beta, eps, add, nullptr, out, gamma2, beta2, add2, out2);
    else
        hipLaunchKernelGGL((layernorm_lpr_kernel<32, 4, true>), dim3((unsigned)ceil_div(n, 8)), dim3(256), 0,
                           st, xm, n, d, gamma, beta, eps, add, nullptr, out, gamma2, beta2, add2, out2);
    FGR_CHECK_LAUNCH("layernorm_dual_kernel");
    return FGR_OK;
}
