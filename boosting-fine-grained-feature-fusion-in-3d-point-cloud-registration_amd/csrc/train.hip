// Training backward of the forward's non-GEMM ops on gfx950 (train.py's
// `loss.backward()`, trainer.py:110-125). The dense products' backward (dX = dY W, dW = dY^T X)
// runs on the f16x3 / bf16 GEMMs with transposed weight images (fgreg/autograd.py); this file
// holds the rest:
//
//   fgr_kpconv_scatter      KPConv gather-weight backward: dx[idx[q,h], c] += sum_k w(q,h,k)
//                           dwf[q,k,c] -- the scatter-add that the reference's
//                           `gather(method=2)` exists for (finegrained_kpconv_blocks.py:66-97)
//   fgr_max_pool_bwd        max_pool (:125-141): the gradient goes to the row's first max entry
//   fgr_segnorm_stats/_apply/_bwd
//                           per-(segment, channel) normalisation with batch statistics: the
//                           InstanceNorm of BatchNormBlock (:462-518, segment = cloud) and the
//                           Res2Net BatchNorm1d in train() (res2net.py:126-159, one segment, affine)
//   fgr_layernorm_bwd       nn.LayerNorm backward (transformers.py:105-107) + gamma / beta grads
//   fgr_colsum              deterministic column sums (bias gradients)
//   fgr_attention_bwd       MHA core backward (transformers.py:197-226) over packed segments
//
// Reductions are deterministic (fixed-order partials in fp64, merged in order) except the two
// scatters (KPConv, max-pool), which add with fp32 global atomics: their sums are exact up to
// fp32 rounding in an order that can vary between runs (|err| ~ 1e-7 relative).
#include "common.h"

#include <algorithm>

namespace fgr {
namespace {

constexpr int kMaxKpT = 32;

__device__ __forceinline__ float kp_w(float nx, float ny, float nz, const float* kp, int k,
                                      float inv_extent) {
    float dx = nx - kp[3 * k], dy = ny - kp[3 * k + 1], dz = nz - kp[3 * k + 2];
    float d2 = dx * dx + dy * dy + dz * dz;
    return fmaxf(1.0f - sqrtf(d2) * inv_extent, 0.0f);
}

// One wave per query: the valid neighbours of each 64-wide chunk are compacted by ballot and
// their K influences computed once into LDS (the forward gather's recipe, kpconv.hip); then for
// every 64-channel slice the query's dwf rows (K x 64) are held in registers and each valid
// neighbour receives sum_k w_hk dwf[q, k, c] by one atomic add per channel.
__global__ void __launch_bounds__(256)
kpconv_scatter_kernel(const float* __restrict__ q, const float* __restrict__ s, int64_t nq, int64_t ns,
                      const int64_t* __restrict__ idx, int width, const float* __restrict__ dwf,
                      int cin, const float* __restrict__ kp_g, int n_kp, float inv_extent,
                      float* __restrict__ dx) {
    __shared__ float w_lds[4][64][kMaxKpT + 1];
    __shared__ int nb_lds[4][64];
    __shared__ float kp[3 * kMaxKpT];
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (int i = threadIdx.x; i < 3 * n_kp; i += blockDim.x) kp[i] = kp_g[i];
    __syncthreads();
    const int64_t qi = (int64_t)blockIdx.x * 4 + wv;
    if (qi >= nq) return;
    const float qx = q[3 * qi], qy = q[3 * qi + 1], qz = q[3 * qi + 2];
    const int64_t* row = idx + qi * width;
    const float* dq = dwf + qi * (int64_t)n_kp * cin;
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
            const float nx = s[3 * id] - qx, ny = s[3 * id + 1] - qy, nz = s[3 * id + 2] - qz;
            for (int k = 0; k < n_kp; ++k) w_lds[wv][p][k] = kp_w(nx, ny, nz, kp, k, inv_extent);
        }
        __builtin_amdgcn_wave_barrier();
        for (int c0 = 0; c0 < cin; c0 += 64) {
            const int c = c0 + lane;
            const bool act = c < cin;
            float dw[kMaxKpT];
#pragma unroll
            for (int k = 0; k < kMaxKpT; ++k)
                dw[k] = (act && k < n_kp) ? dq[(int64_t)k * cin + c] : 0.f;
            for (int hh = 0; hh < v; ++hh) {
                float g = 0.f;
#pragma unroll
                for (int k = 0; k < kMaxKpT; ++k)
                    if (k < n_kp) g = fmaf(w_lds[wv][hh][k], dw[k], g);
                if (act) unsafeAtomicAdd(dx + (int64_t)nb_lds[wv][hh] * cin + c, g);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Thread per (query, channel): the row's first maximum over x[idx[q, h], c] with shadow entries
// reading 0 (the appended zero row, finegrained_kpconv_blocks.py:134-140); a real winner
// receives dy[q, c].
__global__ void __launch_bounds__(256)
max_pool_bwd_kernel(const float* __restrict__ x, int64_t ns, int c, const int64_t* __restrict__ idx,
                    int64_t nq, int width, const float* __restrict__ dy, float* __restrict__ dx) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nq * c) return;
    const int64_t qi = t / c;
    const int ch = (int)(t - qi * c);
    const int64_t* row = idx + qi * width;
    int64_t arg = ns;
    float best = 0.f;
    for (int h = 0; h < width; ++h) {
        const int64_t id = row[h];
        const bool real = id >= 0 && id < ns;
        const float v = real ? x[id * c + ch] : 0.f;
        if (h == 0 || v > best) {
            best = v;
            arg = real ? id : ns;
        }
    }
    if (arg < ns) unsafeAtomicAdd(dx + arg * c + ch, dy[t]);
}

// ---- per-(segment, channel) normalisation --------------------------------------------------
// z = (v - mean) * rstd (* gamma + beta), v = x / row_div;  a = act(z);  y = post(a + residual)
// Partial sums per (segment, chunk of kRowsChunk rows, channel), in fp64 and shifted by the
// segment's first row (no cancellation for |mean| >> std), merged in chunk order.
constexpr int kRowsChunk = 256;

__device__ __forceinline__ float act_fwd(float z, int act) {
    if (act == FGR_ACT_RELU) return fmaxf(z, 0.f);
    if (act == FGR_ACT_LEAKY) return z > 0.f ? z : 0.1f * z;
    return z;
}
// derivative factor from the activation's INPUT sign (torch: relu' = (out > 0), leaky' =
// (in > 0 ? 1 : slope); out and in share their sign for both)
__device__ __forceinline__ float act_grad(float zin, int act) {
    if (act == FGR_ACT_RELU) return zin > 0.f ? 1.f : 0.f;
    if (act == FGR_ACT_LEAKY) return zin > 0.f ? 1.f : 0.1f;
    return 1.f;
}

struct SegArgs {
    const float* x;
    const float* row_div;
    const int64_t* seg_off;
    int n_seg;
    int c;
    int n_chunks;
};

__global__ void __launch_bounds__(256)
segnorm_stats_kernel(SegArgs a, double* __restrict__ part) {
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int ch = blockIdx.z * 64 + threadIdx.x % 64;
    const int rg = threadIdx.x / 64;
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * kRowsChunk;
    double s1 = 0.0, s2 = 0.0;
    int cnt = 0;
    if (ch < a.c && r0 < e) {
        const double piv = (double)(a.row_div ? a.x[b * a.c + ch] / a.row_div[b] : a.x[b * a.c + ch]);
        const int64_t r1 = min(e, r0 + kRowsChunk);
        for (int64_t r = r0 + rg; r < r1; r += 4) {
            const float v = a.row_div ? a.x[r * a.c + ch] / a.row_div[r] : a.x[r * a.c + ch];
            const double d = (double)v - piv;
            s1 += d;
            s2 += d * d;
            ++cnt;
        }
    }
    __shared__ double l1[4][64], l2[4][64];
    __shared__ int lc[4][64];
    l1[rg][threadIdx.x % 64] = s1;
    l2[rg][threadIdx.x % 64] = s2;
    lc[rg][threadIdx.x % 64] = cnt;
    __syncthreads();
    if (rg == 0 && ch < a.c) {
        const int l = threadIdx.x;
        s1 = ((l1[0][l] + l1[1][l]) + l1[2][l]) + l1[3][l];
        s2 = ((l2[0][l] + l2[1][l]) + l2[2][l]) + l2[3][l];
        cnt = lc[0][l] + lc[1][l] + lc[2][l] + lc[3][l];
        double* p = part + (((int64_t)seg * a.n_chunks + chunk) * a.c + ch) * 3;
        p[0] = s1;
        p[1] = s2;
        p[2] = (double)cnt;
    }
}

// Thread per (segment, channel): merge the chunk partials in order -> mean, rstd, biased var.
__global__ void __launch_bounds__(256)
segnorm_merge_kernel(SegArgs a, const double* __restrict__ part, float eps, float* __restrict__ mean,
                     float* __restrict__ rstd, float* __restrict__ var) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)a.n_seg * a.c) return;
    const int seg = (int)(t / a.c), ch = (int)(t % a.c);
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    if (e <= b) {
        mean[t] = 0.f; rstd[t] = 0.f; var[t] = 0.f;
        return;
    }
    double s1 = 0.0, s2 = 0.0, n = 0.0;
    for (int k = 0; k < a.n_chunks; ++k) {
        const double* p = part + (((int64_t)seg * a.n_chunks + k) * a.c + ch) * 3;
        s1 += p[0];
        s2 += p[1];
        n += p[2];
    }
    const double piv = (double)(a.row_div ? a.x[b * a.c + ch] / a.row_div[b] : a.x[b * a.c + ch]);
    const double m1 = s1 / n;
    const double vv = fmax(s2 / n - m1 * m1, 0.0);
    mean[t] = (float)(piv + m1);
    var[t] = (float)vv;
    rstd[t] = (float)(1.0 / sqrt(vv + (double)eps));
}

struct SegApply {
    SegArgs a;
    int64_t n;
    const float* mean;
    const float* rstd;
    const float* gamma;
    const float* beta;
    int act;
    const float* residual;
    int post_act;
};

__global__ void __launch_bounds__(256)
segnorm_apply_kernel(SegApply p, float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= p.n * p.a.c) return;
    const int64_t r = t / p.a.c;
    const int ch = (int)(t - r * p.a.c);
    const int seg = find_segment(p.a.seg_off, p.a.n_seg, r);
    const float v = p.a.row_div ? p.a.x[t] / p.a.row_div[r] : p.a.x[t];
    const int64_t sc = (int64_t)seg * p.a.c + ch;
    float z = (v - p.mean[sc]) * p.rstd[sc];
    if (p.gamma) z = z * p.gamma[ch] + p.beta[ch];
    float y = act_fwd(z, p.act);
    if (p.residual) y = act_fwd(y + p.residual[t], p.post_act);
    out[t] = y;
}

// dz = dy * post'(y) * act'(z); partial sums of dz and dz * xhat per (segment, chunk, channel)
__global__ void __launch_bounds__(256)
segnorm_bwd_stats_kernel(SegApply p, const float* __restrict__ dy, const float* __restrict__ y,
                         double* __restrict__ part) {
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int ch = blockIdx.z * 64 + threadIdx.x % 64;
    const int rg = threadIdx.x / 64;
    const int C = p.a.c;
    const int64_t b = p.a.seg_off[seg], e = p.a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * kRowsChunk;
    double s1 = 0.0, s2 = 0.0;
    if (ch < C && r0 < e) {
        const int64_t sc = (int64_t)seg * C + ch;
        const float mu = p.mean[sc], rs = p.rstd[sc];
        const float g = p.gamma ? p.gamma[ch] : 1.f, bt = p.gamma ? p.beta[ch] : 0.f;
        const int64_t r1 = min(e, r0 + kRowsChunk);
        for (int64_t r = r0 + rg; r < r1; r += 4) {
            const int64_t t = r * C + ch;
            const float v = p.a.row_div ? p.a.x[t] / p.a.row_div[r] : p.a.x[t];
            const float xh = (v - mu) * rs;
            float gr = dy[t];
            if (p.residual) gr *= act_grad(y[t], p.post_act);
            const float dz = gr * act_grad(xh * g + bt, p.act);
            s1 += (double)dz;
            s2 += (double)dz * (double)xh;
        }
    }
    __shared__ double l1[4][64], l2[4][64];
    l1[rg][threadIdx.x % 64] = s1;
    l2[rg][threadIdx.x % 64] = s2;
    __syncthreads();
    if (rg == 0 && ch < C) {
        const int l = threadIdx.x;
        double* q = part + (((int64_t)seg * p.a.n_chunks + chunk) * C + ch) * 2;
        q[0] = ((l1[0][l] + l1[1][l]) + l1[2][l]) + l1[3][l];
        q[1] = ((l2[0][l] + l2[1][l]) + l2[2][l]) + l2[3][l];
    }
}

// Thread per (segment, channel): the chunk sums in order -> sdz, sdzx (per segment); with
// gamma, thread per channel also sums over segments -> dgamma = sum dz xhat, dbeta = sum dz.
__global__ void __launch_bounds__(256)
segnorm_bwd_merge_kernel(SegArgs a, const double* __restrict__ part, float* __restrict__ sums,
                         float* __restrict__ dgamma, float* __restrict__ dbeta) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)a.n_seg * a.c) return;
    const int seg = (int)(t / a.c), ch = (int)(t % a.c);
    double s1 = 0.0, s2 = 0.0;
    for (int k = 0; k < a.n_chunks; ++k) {
        const double* p = part + (((int64_t)seg * a.n_chunks + k) * a.c + ch) * 2;
        s1 += p[0];
        s2 += p[1];
    }
    sums[2 * t] = (float)s1;
    sums[2 * t + 1] = (float)s2;
    if (dgamma && seg == 0) {
        double g1 = 0.0, g2 = 0.0;
        for (int sg = 0; sg < a.n_seg; ++sg)
            for (int k = 0; k < a.n_chunks; ++k) {
                const double* p = part + (((int64_t)sg * a.n_chunks + k) * a.c + ch) * 2;
                g1 += p[0];
                g2 += p[1];
            }
        dbeta[ch] = (float)g1;
        dgamma[ch] = (float)g2;
    }
}

// dx = rstd * gamma * (dz - mean(dz) - xhat * mean(dz xhat)) / row_div; dres = dy * post'(y)
__global__ void __launch_bounds__(256)
segnorm_bwd_apply_kernel(SegApply p, const float* __restrict__ dy, const float* __restrict__ y,
                         const float* __restrict__ sums, float* __restrict__ dx,
                         float* __restrict__ dres) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int C = p.a.c;
    if (t >= p.n * C) return;
    const int64_t r = t / C;
    const int ch = (int)(t - r * C);
    const int seg = find_segment(p.a.seg_off, p.a.n_seg, r);
    const int64_t sc = (int64_t)seg * C + ch;
    const float inv_n = 1.0f / (float)(p.a.seg_off[seg + 1] - p.a.seg_off[seg]);
    const float mu = p.mean[sc], rs = p.rstd[sc];
    const float g = p.gamma ? p.gamma[ch] : 1.f, bt = p.gamma ? p.beta[ch] : 0.f;
    const float rd = p.a.row_div ? p.a.row_div[r] : 1.f;
    const float v = p.a.x[t] / rd;
    const float xh = (v - mu) * rs;
    float gr = dy[t];
    if (p.residual) gr *= act_grad(y[t], p.post_act);
    if (dres) dres[t] = gr;
    const float dz = gr * act_grad(xh * g + bt, p.act);
    const float m1 = sums[2 * sc] * inv_n, m2 = sums[2 * sc + 1] * inv_n;
    dx[t] = rs * g * (dz - m1 - xh * m2) / rd;
}

// ---- LayerNorm backward ------------------------------------------------------------------
// One wave per row (PER = d / 64 columns per lane), rows r = block * 64 + wave + 4 i; the
// wave's lanes keep the column partials of dy * xhat and dy over its rows, merged per block
// in LDS and written as the block's partial row (2 d floats) for fgr_colsum.
constexpr int kLnRows = 64;

template <int PER>
__global__ void __launch_bounds__(256)
layernorm_bwd_kernel(const float* __restrict__ x, int64_t n, int d, const float* __restrict__ g,
                     float eps, const float* __restrict__ dy, float* __restrict__ dx,
                     float* __restrict__ part) {
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    float pg[PER], pb[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) pg[j] = pb[j] = 0.f;
    for (int i = 0; i < kLnRows / 4; ++i) {
        const int64_t r = (int64_t)blockIdx.x * kLnRows + wv + 4 * i;
        if (r >= n) break;
        float v[PER], gy[PER];
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int col = lane + 64 * j;
            v[j] = col < d ? x[r * d + col] : 0.f;
            gy[j] = col < d ? dy[r * d + col] : 0.f;
            s += v[j];
        }
        const float mean = wave_sum(s) / (float)d;
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const float a = (lane + 64 * j) < d ? v[j] - mean : 0.f;
            sq += a * a;
        }
        const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)d + eps);
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int col = lane + 64 * j;
            if (col < d) {
                const float xh = (v[j] - mean) * rstd;
                const float dxh = gy[j] * g[col];
                s1 += dxh;
                s2 += dxh * xh;
                pg[j] += gy[j] * xh;
                pb[j] += gy[j];
                v[j] = xh;
                gy[j] = dxh;
            }
        }
        const float m1 = wave_sum(s1) / (float)d, m2 = wave_sum(s2) / (float)d;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int col = lane + 64 * j;
            if (col < d) dx[r * d + col] = rstd * (gy[j] - m1 - v[j] * m2);
        }
    }
    __shared__ float lg[4][64 * PER], lb[4][64 * PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        lg[wv][lane + 64 * j] = pg[j];
        lb[wv][lane + 64 * j] = pb[j];
    }
    __syncthreads();
    for (int col = threadIdx.x; col < d; col += 256) {
        float* p = part + (int64_t)blockIdx.x * 2 * d;
        p[col] = ((lg[0][col] + lg[1][col]) + lg[2][col]) + lg[3][col];
        p[d + col] = ((lb[0][col] + lb[1][col]) + lb[2][col]) + lb[3][col];
    }
}

// ---- column sums -----------------------------------------------------------------------
constexpr int kColRows = 1024;

__global__ void __launch_bounds__(256)
colsum_part_kernel(const float* __restrict__ x, int64_t n, int c, int64_t ldx, double* __restrict__ part) {
    const int ch = blockIdx.x * 64 + threadIdx.x % 64, rg = threadIdx.x / 64;
    const int64_t r0 = (int64_t)blockIdx.y * kColRows;
    double s = 0.0;
    if (ch < c) {
        const int64_t r1 = min(n, r0 + kColRows);
        for (int64_t r = r0 + rg; r < r1; r += 4) s += (double)x[r * ldx + ch];
    }
    __shared__ double l[4][64];
    l[rg][threadIdx.x % 64] = s;
    __syncthreads();
    if (rg == 0 && ch < c)
        part[(int64_t)blockIdx.y * c + ch] =
            ((l[0][threadIdx.x] + l[1][threadIdx.x]) + l[2][threadIdx.x]) + l[3][threadIdx.x];
}

__global__ void __launch_bounds__(256)
colsum_final_kernel(const double* __restrict__ part, int nparts, int c, float* __restrict__ out) {
    const int ch = blockIdx.x * 256 + threadIdx.x;
    if (ch >= c) return;
    double s = 0.0;
    for (int k = 0; k < nparts; ++k) s += part[(int64_t)k * c + ch];
    out[ch] = (float)s;
}

// ---- attention backward ------------------------------------------------------------------
// Softmax attention per (query segment i -> key segment kv_seg[i], head h), s = scale q.k:
//   P = softmax(S), O = P V;  dV = P^T dO, dP = dO V^T, dS = P (dP - rowsum(dO o O)), dQ =
//   scale dS K, dK = scale dS^T Q.
// Kernel 1: one thread per query row (64-query blocks, K / V tiles of 64 keys in LDS): the
// row's max and sum (pass 1), then dQ (pass 2); writes the row's log-sum-exp and D = dO.O.
// Kernel 2: one thread per key row: over every query segment attending its segment, Q / dO
// tiles in LDS, accumulates dK and dV.
struct AttnBwd {
    const float* q; int64_t ldq;
    const float* k; int64_t ldk;
    const float* v; int64_t ldv;
    const float* o; int64_t ldo;
    const float* dout; int64_t lddo;
    float* dq; int64_t lddq;
    float* dk; int64_t lddk;
    float* dv; int64_t lddv;
    const int64_t* q_off;
    const int64_t* kv_off;
    const int32_t* kv_seg;
    int n_seg, n_kv_seg, nhead;
    int q_blocks, kv_blocks;
    float scale;
    float* lse;      // (Nq, nhead)
    float* dsum;     // (Nq, nhead)
};

template <int DH>
__global__ void __launch_bounds__(64)
attn_bwd_dq_kernel(AttnBwd a) {
    __shared__ float kt[64][DH + 1];
    __shared__ float vt[64][DH + 1];
    const int seg = blockIdx.x / a.q_blocks, qb = blockIdx.x % a.q_blocks, h = blockIdx.y;
    const int lane = threadIdx.x;
    const int64_t qb0 = a.q_off[seg], qe = a.q_off[seg + 1];
    const int64_t r = qb0 + (int64_t)qb * 64 + lane;
    if (qb0 + (int64_t)qb * 64 >= qe) return;                 // whole block past the segment
    const bool ok = r < qe;
    const int ks = a.kv_seg[seg];
    const int64_t kb = a.kv_off[ks], ke = a.kv_off[ks + 1];
    float qv[DH], dov[DH], dqv[DH];
    float dsum = 0.f;
#pragma unroll
    for (int j = 0; j < DH; ++j) {
        qv[j] = ok ? a.q[r * a.ldq + h * DH + j] * a.scale : 0.f;
        dov[j] = ok ? a.dout[r * a.lddo + h * DH + j] : 0.f;
        dsum += ok ? dov[j] * a.o[r * a.ldo + h * DH + j] : 0.f;
        dqv[j] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int64_t t0 = kb; t0 < ke; t0 += 64) {
        const int nt = (int)min((int64_t)64, ke - t0);
        __syncthreads();
        for (int e = lane; e < nt * DH; e += 64) {
            const int kk = e / DH, j = e % DH;
            kt[kk][j] = a.k[(t0 + kk) * a.ldk + h * DH + j];
        }
        __syncthreads();
        for (int kk = 0; kk < nt; ++kk) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < DH; ++j) s = fmaf(qv[j], kt[kk][j], s);
            if (s > m) {
                l = l * expf(m - s) + 1.f;
                m = s;
            } else {
                l += expf(s - m);
            }
        }
    }
    const float inv_l = 1.f / l;
    for (int64_t t0 = kb; t0 < ke; t0 += 64) {
        const int nt = (int)min((int64_t)64, ke - t0);
        __syncthreads();
        for (int e = lane; e < nt * DH; e += 64) {
            const int kk = e / DH, j = e % DH;
            kt[kk][j] = a.k[(t0 + kk) * a.ldk + h * DH + j];
            vt[kk][j] = a.v[(t0 + kk) * a.ldv + h * DH + j];
        }
        __syncthreads();
        for (int kk = 0; kk < nt; ++kk) {
            float s = 0.f, dp = 0.f;
#pragma unroll
            for (int j = 0; j < DH; ++j) {
                s = fmaf(qv[j], kt[kk][j], s);
                dp = fmaf(dov[j], vt[kk][j], dp);
            }
            const float p = expf(s - m) * inv_l;
            const float ds = p * (dp - dsum);
#pragma unroll
            for (int j = 0; j < DH; ++j) dqv[j] = fmaf(ds, kt[kk][j], dqv[j]);
        }
    }
    if (!ok) return;
#pragma unroll
    for (int j = 0; j < DH; ++j) a.dq[r * a.lddq + h * DH + j] = dqv[j] * a.scale;
    a.lse[r * a.nhead + h] = m + logf(l);
    a.dsum[r * a.nhead + h] = dsum;
}

template <int DH>
__global__ void __launch_bounds__(64)
attn_bwd_dkdv_kernel(AttnBwd a) {
    __shared__ float qt[64][DH + 1];
    __shared__ float dot_[64][DH + 1];
    __shared__ float lt[64], dt[64];
    const int ks = blockIdx.x / a.kv_blocks, kbk = blockIdx.x % a.kv_blocks, h = blockIdx.y;
    const int lane = threadIdx.x;
    const int64_t kb0 = a.kv_off[ks], ke = a.kv_off[ks + 1];
    const int64_t r = kb0 + (int64_t)kbk * 64 + lane;
    if (kb0 + (int64_t)kbk * 64 >= ke) return;
    const bool ok = r < ke;
    float kv[DH], vv[DH], dkv[DH], dvv[DH];
#pragma unroll
    for (int j = 0; j < DH; ++j) {
        kv[j] = ok ? a.k[r * a.ldk + h * DH + j] : 0.f;
        vv[j] = ok ? a.v[r * a.ldv + h * DH + j] : 0.f;
        dkv[j] = dvv[j] = 0.f;
    }
    for (int seg = 0; seg < a.n_seg; ++seg) {
        if (a.kv_seg[seg] != ks) continue;
        const int64_t qb = a.q_off[seg], qe = a.q_off[seg + 1];
        for (int64_t t0 = qb; t0 < qe; t0 += 64) {
            const int nt = (int)min((int64_t)64, qe - t0);
            __syncthreads();
            for (int e = lane; e < nt * DH; e += 64) {
                const int qq = e / DH, j = e % DH;
                qt[qq][j] = a.q[(t0 + qq) * a.ldq + h * DH + j] * a.scale;
                dot_[qq][j] = a.dout[(t0 + qq) * a.lddo + h * DH + j];
            }
            if (lane < nt) {
                lt[lane] = a.lse[(t0 + lane) * a.nhead + h];
                dt[lane] = a.dsum[(t0 + lane) * a.nhead + h];
            }
            __syncthreads();
            for (int qq = 0; qq < nt; ++qq) {
                float s = 0.f, dp = 0.f;
#pragma unroll
                for (int j = 0; j < DH; ++j) {
                    s = fmaf(qt[qq][j], kv[j], s);
                    dp = fmaf(dot_[qq][j], vv[j], dp);
                }
                const float p = expf(s - lt[qq]);
                const float ds = p * (dp - dt[qq]);
#pragma unroll
                for (int j = 0; j < DH; ++j) {
                    dvv[j] = fmaf(p, dot_[qq][j], dvv[j]);
                    dkv[j] = fmaf(ds, qt[qq][j], dkv[j]);      // qt holds scale * q
                }
            }
        }
    }
    if (!ok) return;
#pragma unroll
    for (int j = 0; j < DH; ++j) {
        a.dk[r * a.lddk + h * DH + j] = dkv[j];
        a.dv[r * a.lddv + h * DH + j] = dvv[j];
    }
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_kpconv_scatter(const float* q, const float* s, int64_t nq, int64_t ns,
                                  const int64_t* idx, int32_t width, const float* dwf, int32_t cin,
                                  const float* kernel_points, int32_t n_kp, float extent, float* dx,
                                  void* stream) {
    FGR_REQUIRE(nq >= 0 && ns >= 0 && width >= 0 && cin > 0 && n_kp > 0 && n_kp <= kMaxKpT &&
                    extent > 0.f, "fgr_kpconv_scatter: bad arguments");
    if (nq == 0 || width == 0) return FGR_OK;
    FGR_REQUIRE(q && s && idx && dwf && kernel_points && dx, "fgr_kpconv_scatter: null pointer");
    hipLaunchKernelGGL(kpconv_scatter_kernel, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0,
                       as_stream(stream), q, s, nq, ns, idx, width, dwf, cin, kernel_points, n_kp,
                       1.0f / extent, dx);
    FGR_CHECK_LAUNCH("kpconv_scatter_kernel");
    return FGR_OK;
}

extern "C" int fgr_max_pool_bwd(const float* x, int64_t ns, int32_t c, const int64_t* idx, int64_t nq,
                                int32_t width, const float* dy, float* dx, void* stream) {
    FGR_REQUIRE(ns >= 0 && nq >= 0 && c > 0 && width > 0, "fgr_max_pool_bwd: bad arguments");
    if (nq == 0) return FGR_OK;
    FGR_REQUIRE(x && idx && dy && dx, "fgr_max_pool_bwd: null pointer");
    hipLaunchKernelGGL(max_pool_bwd_kernel, dim3((unsigned)ceil_div(nq * c, 256)), dim3(256), 0,
                       as_stream(stream), x, ns, c, idx, nq, width, dy, dx);
    FGR_CHECK_LAUNCH("max_pool_bwd_kernel");
    return FGR_OK;
}

static int seg_chunks(int64_t max_seg_len) { return (int)std::max<int64_t>(1, ceil_div(max_seg_len, kRowsChunk)); }

extern "C" int fgr_segnorm_workspace(int64_t max_seg_len, int32_t c, int32_t n_seg, size_t* bytes) {
    FGR_REQUIRE(bytes && max_seg_len >= 0 && c > 0 && n_seg >= 0, "fgr_segnorm_workspace: bad arguments");
    *bytes = (size_t)n_seg * seg_chunks(max_seg_len) * c * 3 * sizeof(double);
    return FGR_OK;
}

extern "C" int fgr_segnorm_stats(const float* x, int64_t n, int32_t c, const int64_t* seg_off,
                                 int32_t n_seg, int64_t max_seg_len, const float* row_div, float eps,
                                 float* mean, float* rstd, float* var, void* ws, size_t ws_bytes,
                                 void* stream) {
    FGR_REQUIRE(n >= 0 && c > 0 && n_seg > 0 && max_seg_len >= 0, "fgr_segnorm_stats: bad arguments");
    FGR_REQUIRE(x && seg_off && mean && rstd && var && ws, "fgr_segnorm_stats: null pointer");
    size_t need = 0;
    fgr_segnorm_workspace(max_seg_len, c, n_seg, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_segnorm_stats: workspace too small");
    SegArgs a{x, row_div, seg_off, n_seg, c, seg_chunks(max_seg_len)};
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(segnorm_stats_kernel, dim3(a.n_chunks, n_seg, (unsigned)ceil_div(c, 64)), dim3(256),
                       0, st, a, (double*)ws);
    FGR_CHECK_LAUNCH("segnorm_stats_kernel");
    hipLaunchKernelGGL(segnorm_merge_kernel, dim3((unsigned)ceil_div((int64_t)n_seg * c, 256)), dim3(256),
                       0, st, a, (const double*)ws, eps, mean, rstd, var);
    FGR_CHECK_LAUNCH("segnorm_merge_kernel");
    return FGR_OK;
}

extern "C" int fgr_segnorm_apply(const float* x, int64_t n, int32_t c, const int64_t* seg_off,
                                 int32_t n_seg, const float* row_div, const float* mean,
                                 const float* rstd, const float* gamma, const float* beta, int32_t act,
                                 const float* residual, int32_t post_act, float* out, void* stream) {
    FGR_REQUIRE(n >= 0 && c > 0 && n_seg > 0 && (!gamma == !beta), "fgr_segnorm_apply: bad arguments");
    if (n == 0) return FGR_OK;
    FGR_REQUIRE(x && seg_off && mean && rstd && out, "fgr_segnorm_apply: null pointer");
    SegApply p{{x, row_div, seg_off, n_seg, c, 1}, n, mean, rstd, gamma, beta, act, residual, post_act};
    hipLaunchKernelGGL(segnorm_apply_kernel, dim3((unsigned)ceil_div(n * c, 256)), dim3(256), 0,
                       as_stream(stream), p, out);
    FGR_CHECK_LAUNCH("segnorm_apply_kernel");
    return FGR_OK;
}

extern "C" int fgr_segnorm_bwd(const float* x, int64_t n, int32_t c, const int64_t* seg_off,
                               int32_t n_seg, int64_t max_seg_len, const float* row_div,
                               const float* mean, const float* rstd, const float* gamma,
                               const float* beta, int32_t act, int32_t has_residual, int32_t post_act,
                               const float* y, const float* dy, float* dx, float* dres,
                               float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(n >= 0 && c > 0 && n_seg > 0 && (!gamma == !beta) && (!gamma == !dgamma) &&
                    (!dgamma == !dbeta), "fgr_segnorm_bwd: bad arguments");
    FGR_REQUIRE(x && seg_off && mean && rstd && dy && dx && ws && (!has_residual || y),
                "fgr_segnorm_bwd: null pointer");
    // workspace: the chunk partials (2 doubles per entry, inside the stats' 3-double region of
    // fgr_segnorm_workspace bytes) followed by the merged sums (2 floats per (segment, channel))
    size_t part_bytes = 0;
    fgr_segnorm_workspace(max_seg_len, c, n_seg, &part_bytes);
    FGR_REQUIRE(ws_bytes >= part_bytes + (size_t)n_seg * c * 2 * sizeof(float),
                "fgr_segnorm_bwd: workspace too small (fgr_segnorm_workspace + 8 n_seg c bytes)");
    const int nch = seg_chunks(max_seg_len);
    double* part = (double*)ws;
    float* sums = (float*)((char*)ws + part_bytes);
    SegApply p{{x, row_div, seg_off, n_seg, c, nch}, n, mean, rstd, gamma, beta, act,
               has_residual ? y : nullptr, post_act};
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(segnorm_bwd_stats_kernel, dim3(nch, n_seg, (unsigned)ceil_div(c, 64)), dim3(256), 0,
                       st, p, dy, y, part);
    FGR_CHECK_LAUNCH("segnorm_bwd_stats_kernel");
    hipLaunchKernelGGL(segnorm_bwd_merge_kernel, dim3((unsigned)ceil_div((int64_t)n_seg * c, 256)),
                       dim3(256), 0, st, p.a, (const double*)part, sums, dgamma, dbeta);
    FGR_CHECK_LAUNCH("segnorm_bwd_merge_kernel");
    if (n == 0) return FGR_OK;
    hipLaunchKernelGGL(segnorm_bwd_apply_kernel, dim3((unsigned)ceil_div(n * c, 256)), dim3(256), 0, st,
                       p, dy, y, (const float*)sums, dx, has_residual ? dres : nullptr);
    FGR_CHECK_LAUNCH("segnorm_bwd_apply_kernel");
    return FGR_OK;
}

extern "C" int fgr_colsum_workspace(int64_t n, int32_t c, size_t* bytes) {
    FGR_REQUIRE(bytes && n >= 0 && c > 0, "fgr_colsum_workspace: bad arguments");
    *bytes = (size_t)std::max<int64_t>(1, ceil_div(n, kColRows)) * c * sizeof(double);
    return FGR_OK;
}

extern "C" int fgr_colsum(const float* x, int64_t n, int32_t c, int64_t ldx, float* out, void* ws,
                          size_t ws_bytes, void* stream) {
    FGR_REQUIRE(n >= 0 && c > 0 && ldx >= c, "fgr_colsum: bad arguments");
    FGR_REQUIRE(out && ws && (n == 0 || x), "fgr_colsum: null pointer");
    size_t need = 0;
    fgr_colsum_workspace(n, c, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_colsum: workspace too small");
    const int nparts = (int)std::max<int64_t>(1, ceil_div(n, kColRows));
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(colsum_part_kernel, dim3((unsigned)ceil_div(c, 64), nparts), dim3(256), 0, st, x, n,
                       c, ldx, (double*)ws);
    FGR_CHECK_LAUNCH("colsum_part_kernel");
    hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0, st,
                       (const double*)ws, nparts, c, out);
    FGR_CHECK_LAUNCH("colsum_final_kernel");
    return FGR_OK;
}

extern "C" int fgr_layernorm_bwd_workspace(int64_t n, int32_t d, size_t* bytes) {
    FGR_REQUIRE(bytes && n >= 0 && d > 0, "fgr_layernorm_bwd_workspace: bad arguments");
    const int64_t nb = std::max<int64_t>(1, ceil_div(n, kLnRows));
    size_t cs = 0;
    fgr_colsum_workspace(nb, 2 * d, &cs);
    *bytes = (size_t)nb * 2 * d * sizeof(float) + cs;
    return FGR_OK;
}

extern "C" int fgr_layernorm_bwd(const float* x, int64_t n, int32_t d, const float* gamma, float eps,
                                 const float* dy, float* dx, float* dgamma_dbeta, void* ws,
                                 size_t ws_bytes, void* stream) {
    FGR_REQUIRE(n >= 0 && d > 0 && d <= 1024, "fgr_layernorm_bwd: bad arguments (0 < d <= 1024)");
    FGR_REQUIRE(gamma && dgamma_dbeta && ws && (n == 0 || (x && dy && dx)), "fgr_layernorm_bwd: null pointer");
    size_t need = 0;
    fgr_layernorm_bwd_workspace(n, d, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_layernorm_bwd: workspace too small");
    const int64_t nb = std::max<int64_t>(1, ceil_div(n, kLnRows));
    float* part = (float*)ws;
    void* cws = (char*)ws + (size_t)nb * 2 * d * sizeof(float);
    size_t cs = 0;
    fgr_colsum_workspace(nb, 2 * d, &cs);
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        FGR_CHECK_HIP(hipMemsetAsync(part, 0, (size_t)2 * d * sizeof(float), st));
    } else {
        int per = 1;
        while (64 * per < d) per *= 2;
        switch (per) {
#define LNB(P) case P: hipLaunchKernelGGL(layernorm_bwd_kernel<P>, dim3((unsigned)nb), dim3(256), 0, st, x, n, d, gamma, eps, dy, dx, part); break;
            LNB(1) LNB(2) LNB(4) LNB(8) LNB(16)
#undef LNB
            default: FGR_REQUIRE(false, "fgr_layernorm_bwd: unsupported d");
        }
        FGR_CHECK_LAUNCH("layernorm_bwd_kernel");
    }
    return fgr_colsum(part, nb, 2 * d, 2 * d, dgamma_dbeta, cws, cs, stream);
}

extern "C" int fgr_attention_bwd_workspace(int64_t nq, int32_t nhead, size_t* bytes) {
    FGR_REQUIRE(bytes && nq >= 0 && nhead > 0, "fgr_attention_bwd_workspace: bad arguments");
    *bytes = (size_t)std::max<int64_t>(nq, 1) * nhead * 2 * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_attention_bwd(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                                 int64_t ldv, const float* o, int64_t ldo, const float* dout,
                                 int64_t lddo, float* dq, int64_t lddq, float* dk, int64_t lddk,
                                 float* dv, int64_t lddv, const int64_t* q_off, const int64_t* kv_off,
                                 const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg, int64_t nq,
                                 int64_t max_q_len, int64_t max_kv_len, int32_t nhead, int32_t dh,
                                 float scale, void* ws, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(n_seg > 0 && n_kv_seg > 0 && nhead > 0 && nq >= 0 &&
                    (dh == 4 || dh == 8 || dh == 16 || dh == 32 || dh == 64),
                "fgr_attention_bwd: bad arguments (head dim 4 / 8 / 16 / 32 / 64)");
    FGR_REQUIRE(q && k && v && o && dout && dq && dk && dv && q_off && kv_off && kv_seg && ws,
                "fgr_attention_bwd: null pointer");
    size_t need = 0;
    fgr_attention_bwd_workspace(nq, nhead, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_attention_bwd: workspace too small");
    AttnBwd a{q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, dq, lddq, dk, lddk, dv, lddv, q_off, kv_off,
              kv_seg, n_seg, n_kv_seg, nhead, (int)std::max<int64_t>(1, ceil_div(max_q_len, 64)),
              (int)std::max<int64_t>(1, ceil_div(max_kv_len, 64)), scale, (float*)ws,
              (float*)ws + std::max<int64_t>(nq, 1) * nhead};
    hipStream_t st = as_stream(stream);
    dim3 g1((unsigned)(n_seg * a.q_blocks), nhead), g2((unsigned)(n_kv_seg * a.kv_blocks), nhead);
    switch (dh) {
#define ATB(D) case D: \
        hipLaunchKernelGGL(attn_bwd_dq_kernel<D>, g1, dim3(64), 0, st, a); \
        FGR_CHECK_LAUNCH("attn_bwd_dq_kernel"); \
        hipLaunchKernelGGL(attn_bwd_dkdv_kernel<D>, g2, dim3(64), 0, st, a); \
        break;
        ATB(4) ATB(8) ATB(16) ATB(32) ATB(64)
#undef ATB
    }
    FGR_CHECK_LAUNCH("attn_bwd_dkdv_kernel");
    return FGR_OK;
}
