// Training backward of the forward's non-GEMM ops on gfx950 (train.py's
// `loss.backward()`, trainer.py:110-125). The dense products' backward (dX = dY W, dW = dY^T X)
// runs on the f16x3 / bf16 GEMMs with transposed weight images (fgreg/autograd.py); this file
// holds the rest:
//
//   fgr_nbr_inverse         the inverse (CSR) of a neighbour table: for every support row the
//                           (query, slot) entries naming it, in ascending entry order -- built
//                           once per table, shared by every scatter over that table
//   fgr_kpconv_scatter      KPConv gather-weight backward: dx[idx[q,h], c] += sum_k w(q,h,k)
//                           dwf[q,k,c] -- the scatter-add that the reference's
//                           `gather(method=2)` exists for (finegrained_kpconv_blocks.py:66-97)
//   fgr_max_pool_bwd        max_pool (:125-141): the gradient goes to the row's first max entry
//   fgr_corr_attention_bwd  CorrespondenceDecoder.simple_attention (finegrained_regtr.py:328-363)
//                           backward: dq, dk of softmax(q.k scale) xyz
//   fgr_segnorm_stats/_apply/_bwd
//                           per-(segment, channel) normalisation with batch statistics: the
//                           InstanceNorm of BatchNormBlock (:462-518, segment = cloud) and the
//                           Res2Net BatchNorm1d in train() (res2net.py:126-159, one segment, affine)
//   fgr_layernorm_bwd       nn.LayerNorm backward (transformers.py:105-107) + gamma / beta grads
//   fgr_colsum              deterministic column sums (bias gradients)
//   fgr_attention_bwd       MHA core backward (transformers.py:197-226) over packed segments
//
// Every reduction is deterministic: fixed-order partials (fp64 where they are long), merged in
// order, and no floating-point atomics anywhere. The two scatters (KPConv, max-pool) run as
// gathers over the table's inverse: each support row sums its own contributions in ascending
// (query, slot) order, so two backward passes give bit-identical gradients.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <initializer_list>

namespace fgr {
namespace {

constexpr int kMaxKpT = 32;

__device__ __forceinline__ float kp_w(float nx, float ny, float nz, const float* kp, int k,
                                      float inv_extent) {
    float dx = nx - kp[3 * k], dy = ny - kp[3 * k + 1], dz = nz - kp[3 * k + 2];
    float d2 = dx * dx + dy * dy + dz * dz;
    return fmaxf(1.0f - sqrtf(d2) * inv_extent, 0.0f);
}

// ---- inverse neighbour table ----------------------------------------------------------------
// Entry e = q * width + h of an (nq, width) table names support row idx[e] when 0 <= idx[e] < ns
// (the shadow index ns and negatives name none). The inverse lists, per support row s, the
// entries naming s in ascending e: start[s] .. start[s + 1] - 1 index ent[], and pos[e] is the
// CSR slot of entry e (-1 for a non-entry). count (int atomics: an exact count) -> one-block
// exclusive scan -> fill through per-row cursors (arbitrary order) -> per-row rank sort.
__global__ void __launch_bounds__(256)
nbr_count_kernel(const int64_t* __restrict__ idx, int64_t n_ent, int64_t ns, int* __restrict__ cnt) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n_ent) return;
    const int64_t id = idx[e];
    if (id >= 0 && id < ns) atomicAdd(cnt + id, 1);
}

// One 1024-thread block: thread t scans a contiguous run of rows; cnt becomes the fill cursors.
__global__ void __launch_bounds__(1024)
nbr_scan_kernel(int* __restrict__ cnt, int64_t ns, int* __restrict__ start) {
    __shared__ int wtot[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t per = (ns + 1023) / 1024;
    const int64_t b = min(ns, (int64_t)t * per), e = min(ns, b + per);
    int sum = 0;
    for (int64_t i = b; i < e; ++i) sum += cnt[i];
    int inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    int base = inc - sum;
    for (int i = 0; i < w; ++i) base += wtot[i];
    for (int64_t i = b; i < e; ++i) {
        const int c = cnt[i];
        start[i] = base;
        cnt[i] = base;
        base += c;
    }
    if (t == 1023) start[ns] = base;
}

__global__ void __launch_bounds__(256)
nbr_fill_kernel(const int64_t* __restrict__ idx, int64_t n_ent, int64_t ns, int* __restrict__ cursor,
                int* __restrict__ tmp) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n_ent) return;
    const int64_t id = idx[e];
    if (id >= 0 && id < ns) tmp[atomicAdd(cursor + id, 1)] = (int)e;
}

// One wave per support row: entry keys are unique, so each one's rank in the row is the count
// of smaller keys.
__global__ void __launch_bounds__(256)
nbr_sort_kernel(const int* __restrict__ start, int64_t ns, const int* __restrict__ tmp,
                int* __restrict__ ent, int* __restrict__ pos) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= ns) return;
    const int lane = threadIdx.x & 63;
    const int b = start[s], n = start[s + 1] - b;
    for (int j = lane; j < n; j += 64) {
        const int key = tmp[b + j];
        int rank = 0;
        for (int i = 0; i < n; ++i) rank += tmp[b + i] < key ? 1 : 0;
        ent[b + rank] = key;
        pos[key] = b + rank;
    }
}

// Segmented row sums over the inverse: dx[s, c] = sum_{j = start[s]}^{start[s+1]-1} g[j, c], in
// slot (= ascending entry) order; rows nobody names get 0.
__global__ void __launch_bounds__(256)
csr_rowsum_kernel(const int* __restrict__ start, int64_t ns, const float* __restrict__ g, int cin,
                  float* __restrict__ dx) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= ns * cin) return;
    const int64_t s = t / cin;
    const int c = (int)(t - s * cin);
    const int b = start[s], e = start[s + 1];
    float acc = 0.f;
    for (int j = b; j < e; ++j) acc += g[(int64_t)j * cin + c];
    dx[t] = acc;
}

// One wave per query: the valid neighbours of each 64-wide chunk are compacted by ballot and
// their K influences computed once into LDS (the forward gather's recipe, kpconv.hip); then for
// every 64-channel slice the query's dwf rows (K x 64) are held in registers and each valid
// neighbour's contribution sum_k w_hk dwf[q, k, c] is written to its CSR slot of the inverse
// (g[pos[q * width + h], c]); csr_rowsum_kernel then adds each support row's slots in order.
__global__ void __launch_bounds__(256)
kpconv_scatter_rows_kernel(const float* __restrict__ q, const float* __restrict__ s, int64_t nq,
                           int64_t ns, const int64_t* __restrict__ idx, int width,
                           const float* __restrict__ dwf, int cin, const float* __restrict__ kp_g,
                           int n_kp, float inv_extent, const int* __restrict__ pos,
                           float* __restrict__ g) {
    __shared__ float w_lds[4][64][kMaxKpT + 1];
    __shared__ int slot_lds[4][64];
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
            slot_lds[wv][p] = pos[qi * width + h];
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
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < kMaxKpT; ++k)
                    if (k < n_kp) acc = fmaf(w_lds[wv][hh][k], dw[k], acc);
                if (act) g[(int64_t)slot_lds[wv][hh] * cin + c] = acc;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Thread per (query, channel): the slot of the row's first maximum over x[idx[q, h], c] with
// shadow entries reading 0 (the appended zero row, finegrained_kpconv_blocks.py:134-140); -1
// when a shadow entry wins (its gradient goes nowhere).
__global__ void __launch_bounds__(256)
max_pool_argmax_kernel(const float* __restrict__ x, int64_t ns, int c, const int64_t* __restrict__ idx,
                       int64_t nq, int width, int* __restrict__ am) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nq * c) return;
    const int64_t qi = t / c;
    const int ch = (int)(t - qi * c);
    const int64_t* row = idx + qi * width;
    int arg = -1;
    float best = 0.f;
    for (int h = 0; h < width; ++h) {
        const int64_t id = row[h];
        const bool real = id >= 0 && id < ns;
        const float v = real ? x[id * c + ch] : 0.f;
        if (h == 0 || v > best) {
            best = v;
            arg = real ? h : -1;
        }
    }
    am[t] = arg;
}

// Thread per (support row, channel): the gradients of every (query, slot) entry naming the row
// whose channel arg-max is that slot, in ascending entry order.
__global__ void __launch_bounds__(256)
max_pool_bwd_csr_kernel(const int* __restrict__ start, const int* __restrict__ ent, int64_t ns, int c,
                        int width, const int* __restrict__ am, const float* __restrict__ dy,
                        float* __restrict__ dx) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= ns * c) return;
    const int64_t s = t / c;
    const int ch = (int)(t - s * c);
    float acc = 0.f;
    for (int j = start[s]; j < start[s + 1]; ++j) {
        const int e = ent[j];
        const int64_t qi = e / width;
        const int h = e - (int)(qi * width);
        const int64_t qc = qi * c + ch;
        if (am[qc] == h) acc += dy[qc];
    }
    dx[t] = acc;
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
#pragma unroll 8
    for (int k = 0; k < a.n_chunks; ++k) {                     // 8 chunk loads in flight
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
#pragma unroll 8
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
#pragma unroll 8
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

// ---- the same four kernels on 16-B rows (c % 4 == 0, aligned): one float4 of channels per
// thread, four rows in flight per thread in the statistics (the scalar kernels above kept one
// dependent load per row and channel: 22 / 38 us per ModelNet call), 32-bit element indices
// and the segment table in LDS for the elementwise passes. Same partial layout and chunking,
// so the merges are shared.
constexpr int kSegLds = 64;        // segment tables up to this many segments cached in LDS

__device__ __forceinline__ int seg_of_row(const int64_t* so_lds, const int64_t* so, int n_seg, int64_t r) {
    return n_seg <= kSegLds ? find_segment(so_lds, n_seg, r) : find_segment(so, n_seg, r);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__global__ void __launch_bounds__(256)
segnorm_stats4_kernel(SegArgs a, double* __restrict__ part) {
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int qd = threadIdx.x & 15, rg = threadIdx.x >> 4;          // 16 quads x 16 row groups
    const int ch = blockIdx.z * 64 + 4 * qd;
    const int C = a.c;
    const int64_t b = a.seg_off[seg], e = a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * kRowsChunk;
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    int cnt = 0;
    if (ch < C && r0 < e) {
        const float4 pv = ld4(a.x + b * C + ch);
        const float pd = a.row_div ? a.row_div[b] : 1.f;
        const double piv[4] = {(double)(a.row_div ? pv.x / pd : pv.x), (double)(a.row_div ? pv.y / pd : pv.y),
                               (double)(a.row_div ? pv.z / pd : pv.z), (double)(a.row_div ? pv.w / pd : pv.w)};
        const int64_t r1 = min(e, r0 + kRowsChunk);
        for (int64_t r = r0 + rg; r < r1; r += 64) {
            float4 v[4];
            float rd[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t rr = min(r + 16 * u, r1 - 1);
                v[u] = ld4(a.x + rr * C + ch);
                rd[u] = a.row_div ? a.row_div[rr] : 1.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (r + 16 * u >= r1) break;
                const float vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float f = a.row_div ? vv[j] / rd[u] : vv[j];
                    const double d = (double)f - piv[j];
                    s1[j] += d;
                    s2[j] += d * d;
                }
                ++cnt;
            }
        }
    }
    __shared__ double l1[16][64], l2[16][64];
    __shared__ int lc[16][16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        l1[rg][4 * qd + j] = s1[j];
        l2[rg][4 * qd + j] = s2[j];
    }
    lc[rg][qd] = cnt;
    __syncthreads();
    const int l = threadIdx.x;
    if (l < 64 && blockIdx.z * 64 + l < C) {
        double t1 = 0.0, t2 = 0.0;
        int tc = 0;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            t1 += l1[g][l];
            t2 += l2[g][l];
            tc += lc[g][l >> 2];
        }
        double* p = part + (((int64_t)seg * a.n_chunks + chunk) * C + blockIdx.z * 64 + l) * 3;
        p[0] = t1;
        p[1] = t2;
        p[2] = (double)tc;
    }
}

__global__ void __launch_bounds__(256)
segnorm_apply4_kernel(SegApply p, float* __restrict__ out) {
    __shared__ int64_t so[kSegLds + 1];
    if (p.a.n_seg <= kSegLds)
        for (int i = threadIdx.x; i <= p.a.n_seg; i += 256) so[i] = p.a.seg_off[i];
    __syncthreads();
    const int c4 = p.a.c >> 2;
    const int t = blockIdx.x * 256 + threadIdx.x;                  // float4 index (< 2^31)
    if (t >= (int)(p.n * c4)) return;
    const int r = t / c4;
    const int ch = 4 * (t - r * c4);
    const int seg = seg_of_row(so, p.a.seg_off, p.a.n_seg, r);
    const int64_t sc = (int64_t)seg * p.a.c + ch;
    const float4 xv = ld4(p.a.x + 4 * (int64_t)t);
    const float rd = p.a.row_div ? p.a.row_div[r] : 1.f;
    const float4 mu = ld4(p.mean + sc), rs = ld4(p.rstd + sc);
    float4 gm = make_float4(1.f, 1.f, 1.f, 1.f), bt = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.gamma) {
        gm = ld4(p.gamma + ch);
        bt = ld4(p.beta + ch);
    }
    float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.residual) rv = ld4(p.residual + 4 * (int64_t)t);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ms[4] = {mu.x, mu.y, mu.z, mu.w};
    const float ss[4] = {rs.x, rs.y, rs.z, rs.w}, gs[4] = {gm.x, gm.y, gm.z, gm.w};
    const float bs[4] = {bt.x, bt.y, bt.z, bt.w}, res[4] = {rv.x, rv.y, rv.z, rv.w};
    float y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float v = p.a.row_div ? xs[j] / rd : xs[j];
        float z = (v - ms[j]) * ss[j];
        if (p.gamma) z = z * gs[j] + bs[j];
        y[j] = act_fwd(z, p.act);
        if (p.residual) y[j] = act_fwd(y[j] + res[j], p.post_act);
    }
    *reinterpret_cast<float4*>(out + 4 * (int64_t)t) = make_float4(y[0], y[1], y[2], y[3]);
}

__global__ void __launch_bounds__(256)
segnorm_bwd_stats4_kernel(SegApply p, const float* __restrict__ dy, const float* __restrict__ y,
                          double* __restrict__ part) {
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int qd = threadIdx.x & 15, rg = threadIdx.x >> 4;
    const int ch = blockIdx.z * 64 + 4 * qd;
    const int C = p.a.c;
    const int64_t b = p.a.seg_off[seg], e = p.a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * kRowsChunk;
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if (ch < C && r0 < e) {
        const int64_t sc = (int64_t)seg * C + ch;
        const float4 mu4 = ld4(p.mean + sc), rs4 = ld4(p.rstd + sc);
        float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.gamma) {
            g4 = ld4(p.gamma + ch);
            b4 = ld4(p.beta + ch);
        }
        const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, rs[4] = {rs4.x, rs4.y, rs4.z, rs4.w};
        const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
        const int64_t r1 = min(e, r0 + kRowsChunk);
        for (int64_t r = r0 + rg; r < r1; r += 64) {
            float4 xv[4], dv[4], yv[4];
            float rd[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t rr = min(r + 16 * u, r1 - 1);
                const int64_t o = rr * C + ch;
                xv[u] = ld4(p.a.x + o);
                dv[u] = ld4(dy + o);
                yv[u] = p.residual ? ld4(y + o) : make_float4(0.f, 0.f, 0.f, 0.f);
                rd[u] = p.a.row_div ? p.a.row_div[rr] : 1.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (r + 16 * u >= r1) break;
                const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
                const float ds[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w};
                const float ys[4] = {yv[u].x, yv[u].y, yv[u].z, yv[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = p.a.row_div ? xs[j] / rd[u] : xs[j];
                    const float xh = (v - mu[j]) * rs[j];
                    float gr = ds[j];
                    if (p.residual) gr *= act_grad(ys[j], p.post_act);
                    const float dz = gr * act_grad(xh * gg[j] + bb[j], p.act);
                    s1[j] += (double)dz;
                    s2[j] += (double)dz * (double)xh;
                }
            }
        }
    }
    __shared__ double l1[16][64], l2[16][64];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        l1[rg][4 * qd + j] = s1[j];
        l2[rg][4 * qd + j] = s2[j];
    }
    __syncthreads();
    const int l = threadIdx.x;
    if (l < 64 && blockIdx.z * 64 + l < C) {
        double t1 = 0.0, t2 = 0.0;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            t1 += l1[g][l];
            t2 += l2[g][l];
        }
        double* q = part + (((int64_t)seg * p.a.n_chunks + chunk) * C + blockIdx.z * 64 + l) * 2;
        q[0] = t1;
        q[1] = t2;
    }
}

__global__ void __launch_bounds__(256)
segnorm_bwd_apply4_kernel(SegApply p, const float* __restrict__ dy, const float* __restrict__ y,
                          const float* __restrict__ sums, float* __restrict__ dx,
                          float* __restrict__ dres) {
    __shared__ int64_t so[kSegLds + 1];
    if (p.a.n_seg <= kSegLds)
        for (int i = threadIdx.x; i <= p.a.n_seg; i += 256) so[i] = p.a.seg_off[i];
    __syncthreads();
    const int C = p.a.c, c4 = C >> 2;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= (int)(p.n * c4)) return;
    const int r = t / c4;
    const int ch = 4 * (t - r * c4);
    const int seg = seg_of_row(so, p.a.seg_off, p.a.n_seg, r);
    const int64_t sc = (int64_t)seg * C + ch;
    const int64_t o = 4 * (int64_t)t;
    const float inv_n = 1.0f / (float)(p.a.seg_off[seg + 1] - p.a.seg_off[seg]);
    const float4 mu4 = ld4(p.mean + sc), rs4 = ld4(p.rstd + sc);
    float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.gamma) {
        g4 = ld4(p.gamma + ch);
        b4 = ld4(p.beta + ch);
    }
    const float rd = p.a.row_div ? p.a.row_div[r] : 1.f;
    const float4 xv = ld4(p.a.x + o), dv = ld4(dy + o);
    const float4 yv = p.residual ? ld4(y + o) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 sa = ld4(sums + 2 * sc), sb = ld4(sums + 2 * sc + 4);   // (s1, s2) per channel
    const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, rs[4] = {rs4.x, rs4.y, rs4.z, rs4.w};
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ds[4] = {dv.x, dv.y, dv.z, dv.w};
    const float ys[4] = {yv.x, yv.y, yv.z, yv.w};
    const float m1s[4] = {sa.x, sa.z, sb.x, sb.z}, m2s[4] = {sa.y, sa.w, sb.y, sb.w};
    float gx[4], gres[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float v = xs[j] / rd;
        const float xh = (v - mu[j]) * rs[j];
        float gr = ds[j];
        if (p.residual) gr *= act_grad(ys[j], p.post_act);
        gres[j] = gr;
        const float dz = gr * act_grad(xh * gg[j] + bb[j], p.act);
        const float m1 = m1s[j] * inv_n, m2 = m2s[j] * inv_n;
        gx[j] = rs[j] * gg[j] * (dz - m1 - xh * m2) / rd;
    }
    if (dres) *reinterpret_cast<float4*>(dres + o) = make_float4(gres[0], gres[1], gres[2], gres[3]);
    *reinterpret_cast<float4*>(dx + o) = make_float4(gx[0], gx[1], gx[2], gx[3]);
}

// ---- the merges folded into the apply passes (segments of at most kSegFuseChunks chunks, e.g.
// ModelNet's per-cloud InstanceNorms): one block per (chunk, segment, 64 channels) as the
// statistics pass, whose first 64 threads merge the 64 channels' chunk partials exactly as the
// merge kernels do (same order, same roundings: bit-identical results) into LDS, then the block
// applies them to its chunk's rows. The chunk-0 block writes mean / rstd / var (forward) or
// dgamma / dbeta (backward, segment 0). One launch per norm and direction instead of two.
constexpr int kSegFuseChunks = 16;          // up to here the merge order of the merge kernels
constexpr int kSegFuseChunksMax = 64;       // beyond: the separate merge kernels

__global__ void __launch_bounds__(256)
segnorm_merge_apply4_kernel(SegApply p, const double* __restrict__ part, float eps, float* __restrict__ mean,
                            float* __restrict__ rstd, float* __restrict__ var, float* __restrict__ out) {
    __shared__ float smu[64], srs[64];
    __shared__ double sred[3][3][64];
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int C = p.a.c;
    const int64_t b = p.a.seg_off[seg], e = p.a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * kRowsChunk;
    if (r0 >= e && chunk != 0) return;                         // block-uniform
    const int tid = threadIdx.x;
    // more than kSegFuseChunks chunks (the BatchNorms over every row): the four waves sum the
    // chunks congruent to their index mod 4, combined in wave order
    const bool split4 = p.a.n_chunks > kSegFuseChunks;
    if (split4 && tid >= 64 && blockIdx.z * 64 + (tid & 63) < C) {
        const int ch = blockIdx.z * 64 + (tid & 63), w = tid >> 6;
        double s1 = 0.0, s2 = 0.0, n = 0.0;
#pragma unroll 4
        for (int k = w; k < p.a.n_chunks; k += 4) {
            const double* q = part + (((int64_t)seg * p.a.n_chunks + k) * C + ch) * 3;
            s1 += q[0];
            s2 += q[1];
            n += q[2];
        }
        sred[w - 1][0][tid & 63] = s1;
        sred[w - 1][1][tid & 63] = s2;
        sred[w - 1][2][tid & 63] = n;
    }
    if (split4) __syncthreads();
    if (tid < 64 && blockIdx.z * 64 + tid < C) {
        const int ch = blockIdx.z * 64 + tid;
        const int64_t t = (int64_t)seg * C + ch;
        float mu = 0.f, rs = 0.f, vr = 0.f;
        if (e > b) {
            double s1 = 0.0, s2 = 0.0, n = 0.0;
#pragma unroll 8
            for (int k = 0; k < p.a.n_chunks; k += split4 ? 4 : 1) {
                const double* q = part + (((int64_t)seg * p.a.n_chunks + k) * C + ch) * 3;
                s1 += q[0];
                s2 += q[1];
                n += q[2];
            }
            if (split4)
                for (int w = 0; w < 3; ++w) {
                    s1 += sred[w][0][tid];
                    s2 += sred[w][1][tid];
                    n += sred[w][2][tid];
                }
            const double piv = (double)(p.a.row_div ? p.a.x[b * C + ch] / p.a.row_div[b] : p.a.x[b * C + ch]);
            const double m1 = s1 / n;
            const double vv = fmax(s2 / n - m1 * m1, 0.0);
            mu = (float)(piv + m1);
            vr = (float)vv;
            rs = (float)(1.0 / sqrt(vv + (double)eps));
        }
        smu[tid] = mu;
        srs[tid] = rs;
        if (chunk == 0) {
            mean[t] = mu;
            rstd[t] = rs;
            var[t] = vr;
        }
    }
    __syncthreads();
    if (r0 >= e) return;
    const int qd = tid & 15, rg = tid >> 4;
    const int ch = blockIdx.z * 64 + 4 * qd;
    if (ch >= C) return;
    const float ms[4] = {smu[4 * qd], smu[4 * qd + 1], smu[4 * qd + 2], smu[4 * qd + 3]};
    const float ss[4] = {srs[4 * qd], srs[4 * qd + 1], srs[4 * qd + 2], srs[4 * qd + 3]};
    float4 gm = make_float4(1.f, 1.f, 1.f, 1.f), bt = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.gamma) {
        gm = ld4(p.gamma + ch);
        bt = ld4(p.beta + ch);
    }
    const float gs[4] = {gm.x, gm.y, gm.z, gm.w}, bs[4] = {bt.x, bt.y, bt.z, bt.w};
    const int64_t r1 = min(e, r0 + kRowsChunk);
    for (int64_t r = r0 + rg; r < r1; r += 64) {
        float4 xv[4], rv[4];
        float rd[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t rr = min(r + 16 * u, r1 - 1);
            xv[u] = ld4(p.a.x + rr * C + ch);
            rd[u] = p.a.row_div ? p.a.row_div[rr] : 1.f;
            rv[u] = p.residual ? ld4(p.residual + rr * C + ch) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (r + 16 * u >= r1) break;
            const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
            const float res[4] = {rv[u].x, rv[u].y, rv[u].z, rv[u].w};
            float y[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float v = p.a.row_div ? xs[j] / rd[u] : xs[j];
                float z = (v - ms[j]) * ss[j];
                if (p.gamma) z = z * gs[j] + bs[j];
                y[j] = act_fwd(z, p.act);
                if (p.residual) y[j] = act_fwd(y[j] + res[j], p.post_act);
            }
            *reinterpret_cast<float4*>(out + (r + 16 * u) * C + ch) = make_float4(y[0], y[1], y[2], y[3]);
        }
    }
}

__global__ void __launch_bounds__(256)
segnorm_bwd_merge_apply4_kernel(SegApply p, const float* __restrict__ dy, const float* __restrict__ y,
                                const double* __restrict__ part, float* __restrict__ dgamma,
                                float* __restrict__ dbeta, float* __restrict__ dx, float* __restrict__ dres) {
    __shared__ float sm1[64], sm2[64];
    __shared__ double sred[3][2][64];
    const int seg = blockIdx.y, chunk = blockIdx.x;
    const int C = p.a.c;
    const int64_t b = p.a.seg_off[seg], e = p.a.seg_off[seg + 1];
    const int64_t r0 = b + (int64_t)chunk * kRowsChunk;
    const bool gblock = dgamma && seg == 0 && chunk == 0;
    if (r0 >= e && !gblock) return;                            // block-uniform
    const int tid = threadIdx.x;
    const bool split4 = p.a.n_chunks > kSegFuseChunks;         // as the forward
    if (split4 && tid >= 64 && blockIdx.z * 64 + (tid & 63) < C) {
        const int ch = blockIdx.z * 64 + (tid & 63), w = tid >> 6;
        double s1 = 0.0, s2 = 0.0;
#pragma unroll 4
        for (int k = w; k < p.a.n_chunks; k += 4) {
            const double* q = part + (((int64_t)seg * p.a.n_chunks + k) * C + ch) * 2;
            s1 += q[0];
            s2 += q[1];
        }
        sred[w - 1][0][tid & 63] = s1;
        sred[w - 1][1][tid & 63] = s2;
    }
    if (split4) __syncthreads();
    if (tid < 64 && blockIdx.z * 64 + tid < C) {
        const int ch = blockIdx.z * 64 + tid;
        double s1 = 0.0, s2 = 0.0;
#pragma unroll 8
        for (int k = 0; k < p.a.n_chunks; k += split4 ? 4 : 1) {
            const double* q = part + (((int64_t)seg * p.a.n_chunks + k) * C + ch) * 2;
            s1 += q[0];
            s2 += q[1];
        }
        if (split4)
            for (int w = 0; w < 3; ++w) {
                s1 += sred[w][0][tid];
                s2 += sred[w][1][tid];
            }
        sm1[tid] = (float)s1;
        sm2[tid] = (float)s2;
        if (gblock) {
            double g1 = 0.0, g2 = 0.0;
            for (int sg = 0; sg < p.a.n_seg; ++sg)
#pragma unroll 8
                for (int k = 0; k < p.a.n_chunks; ++k) {
                    const double* q = part + (((int64_t)sg * p.a.n_chunks + k) * C + ch) * 2;
                    g1 += q[0];
                    g2 += q[1];
                }
            dbeta[ch] = (float)g1;
            dgamma[ch] = (float)g2;
        }
    }
    __syncthreads();
    if (r0 >= e) return;
    const int qd = tid & 15, rg = tid >> 4;
    const int ch = blockIdx.z * 64 + 4 * qd;
    if (ch >= C) return;
    const int64_t sc = (int64_t)seg * C + ch;
    const float inv_n = 1.0f / (float)(e - b);
    const float4 mu4 = ld4(p.mean + sc), rs4 = ld4(p.rstd + sc);
    float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.gamma) {
        g4 = ld4(p.gamma + ch);
        b4 = ld4(p.beta + ch);
    }
    const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, rs[4] = {rs4.x, rs4.y, rs4.z, rs4.w};
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
    const float m1s[4] = {sm1[4 * qd], sm1[4 * qd + 1], sm1[4 * qd + 2], sm1[4 * qd + 3]};
    const float m2s[4] = {sm2[4 * qd], sm2[4 * qd + 1], sm2[4 * qd + 2], sm2[4 * qd + 3]};
    const int64_t r1 = min(e, r0 + kRowsChunk);
    for (int64_t r = r0 + rg; r < r1; r += 64) {
        float4 xv[4], dv[4], yv[4];
        float rdv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t rr = min(r + 16 * u, r1 - 1);
            const int64_t o = rr * C + ch;
            xv[u] = ld4(p.a.x + o);
            dv[u] = ld4(dy + o);
            yv[u] = p.residual ? ld4(y + o) : make_float4(0.f, 0.f, 0.f, 0.f);
            rdv[u] = p.a.row_div ? p.a.row_div[rr] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (r + 16 * u >= r1) break;
            const int64_t o = (r + 16 * u) * C + ch;
            const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w}, ds[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w};
            const float ys[4] = {yv[u].x, yv[u].y, yv[u].z, yv[u].w};
            const float rd = rdv[u];
            float gx[4], gres[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float v = xs[j] / rd;
                const float xh = (v - mu[j]) * rs[j];
                float gr = ds[j];
                if (p.residual) gr *= act_grad(ys[j], p.post_act);
                gres[j] = gr;
                const float dz = gr * act_grad(xh * gg[j] + bb[j], p.act);
                const float m1 = m1s[j] * inv_n, m2 = m2s[j] * inv_n;
                gx[j] = rs[j] * gg[j] * (dz - m1 - xh * m2) / rd;
            }
            if (dres) *reinterpret_cast<float4*>(dres + o) = make_float4(gres[0], gres[1], gres[2], gres[3]);
            *reinterpret_cast<float4*>(dx + o) = make_float4(gx[0], gx[1], gx[2], gx[3]);
        }
    }
}

// ---- LayerNorm backward ------------------------------------------------------------------
// One wave per row (PER = d / 64 columns per lane), rows r = block * 64 + wave + 4 i; the
// wave's lanes keep the column partials of dy * xhat and dy over its rows, merged per block
// in LDS and written as the block's partial row (2 d floats) for fgr_colsum.
constexpr int kLnRowsWave = 4;                 // rows per wave, loaded together
constexpr int kLnRows = 4 * kLnRowsWave;       // rows per block (16: ~600 blocks at 9.5k rows)

template <int PER>
__global__ void __launch_bounds__(256)
layernorm_bwd_kernel(const float* __restrict__ x, int64_t n, int d, const float* __restrict__ g,
                     float eps, const float* __restrict__ dy, float* __restrict__ dx,
                     float* __restrict__ part) {
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    float pg[PER], pb[PER], gm[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        pg[j] = pb[j] = 0.f;
        const int col = lane + 64 * j;
        gm[j] = col < d ? g[col] : 0.f;
    }
    // every load of the wave's rows first (one memory round trip), then the rows in turn
    float v[kLnRowsWave][PER], gy[kLnRowsWave][PER];
    const int64_t rb = (int64_t)blockIdx.x * kLnRows + wv * kLnRowsWave;
#pragma unroll
    for (int i = 0; i < kLnRowsWave; ++i) {
        const int64_t r = min(rb + i, n - 1);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int col = min(lane + 64 * j, d - 1);
            v[i][j] = x[r * d + col];
            gy[i][j] = dy[r * d + col];
        }
    }
#pragma unroll
    for (int i = 0; i < kLnRowsWave; ++i) {
        const int64_t r = rb + i;
        if (r >= n) break;                         // wave-uniform
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < PER; ++j) s += (lane + 64 * j) < d ? v[i][j] : 0.f;
        const float mean = wave_sum(s) / (float)d;
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const float a = (lane + 64 * j) < d ? v[i][j] - mean : 0.f;
            sq += a * a;
        }
        const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)d + eps);
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int col = lane + 64 * j;
            if (col < d) {
                const float xh = (v[i][j] - mean) * rstd;
                const float dxh = gy[i][j] * gm[j];
                s1 += dxh;
                s2 += dxh * xh;
                pg[j] += gy[i][j] * xh;
                pb[j] += gy[i][j];
                v[i][j] = xh;
                gy[i][j] = dxh;
            }
        }
        const float m1 = wave_sum(s1) / (float)d, m2 = wave_sum(s2) / (float)d;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int col = lane + 64 * j;
            if (col < d) dx[r * d + col] = rstd * (gy[i][j] - m1 - v[i][j] * m2);
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
constexpr int kColRows = 256;     // rows per partial: >= 4 blocks per CU on the tall inputs

__global__ void __launch_bounds__(256)
colsum_part_kernel(const float* __restrict__ x, int64_t n, int c, int64_t ldx, double* __restrict__ part) {
    const int ch = blockIdx.x * 64 + threadIdx.x % 64, rg = threadIdx.x / 64;
    const int64_t r0 = (int64_t)blockIdx.y * kColRows;
    double s = 0.0;
    if (ch < c) {
        const int64_t r1 = min(n, r0 + kColRows);
        double s1 = 0.0, s2 = 0.0, s3 = 0.0;       // four chains: the loads stay in flight
        int64_t r = r0 + rg;
        for (; r + 12 < r1; r += 16) {
            s += (double)x[r * ldx + ch];
            s1 += (double)x[(r + 4) * ldx + ch];
            s2 += (double)x[(r + 8) * ldx + ch];
            s3 += (double)x[(r + 12) * ldx + ch];
        }
        for (; r < r1; r += 4) s += (double)x[r * ldx + ch];
        s = (s + s1) + (s2 + s3);
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
    // attention-weight dropout (MFMA kernels, DROP): entries with attn_drop_hash < drop_thresh
    // are dropped, kept ones scaled by inv_keep (the forward's mask: fgr_attention_f16x3_drop)
    uint32_t drop_seed, drop_thresh;
    float inv_keep;
    // training: the forward's log2-sum-exp per (row, head) (fgr_attention_f16x3_train); the
    // MFMA dQ kernel then skips its max / sum pass
    const float* lse_in;
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

// ---- attention backward on the fp32 matrix cores (head dim 16 / 32 / 64; round 5) -----------
// The same two-kernel split as above, as tiled v_mfma_f32_16x16x4_f32 products (exact fp32
// products, fp32 accumulation: the precision of the scalar kernels, ~6-10x their speed on the
// forward's shapes). A wave owns 16 rows of its side (kernel 1: queries; kernel 2: keys), a
// 256-thread block 64; the other side streams through LDS in tiles of 64 rows.
// Lane maps of the 16x16x4 product (lane l, g = l >> 4, c = l & 15): A[i = c][k = g],
// B[k = g][j = c], D[i = 4g + r][j = c]. The head-dim contraction pairs lane g with dims
// g * KS + s at k-step s (KS = DH / 4), so a lane holds KS CONSECUTIVE dims of its row (vector
// loads); the key / query contraction (dV, dK, dQ) pairs lane g with row 16n + 4g + r at k-step
// (n, r) -- exactly the rows whose scores the lane holds after the score product, so P and dS
// feed the next product from registers. Scores run in the log2 domain (q pre-scaled by
// scale * log2 e, P = exp2(s - lse2)); the workspace keeps lse2 and D = dO . O per (row, head).
__device__ __forceinline__ float xg_sum_tr(float v) {     // sum over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float xg_max_tr(float v) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr float kLog2e = 1.4426950408889634f;

// KS consecutive floats of a row (16-B aligned when KS % 4 == 0)
template <int KS>
__device__ __forceinline__ void load_ks(const float* p, float (&v)[KS], bool ok, float mul) {
    if constexpr (KS % 4 == 0) {
#pragma unroll
        for (int s = 0; s < KS; s += 4) {
            const float4 x = ok ? *reinterpret_cast<const float4*>(p + s) : make_float4(0.f, 0.f, 0.f, 0.f);
            v[s] = x.x * mul; v[s + 1] = x.y * mul; v[s + 2] = x.z * mul; v[s + 3] = x.w * mul;
        }
    } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) v[s] = ok ? p[s] * mul : 0.f;
    }
}

// stage 64 rows x DH of `src` (row stride ld, head offset applied) into LDS rows of pitch LD,
// rows >= n zero, each row scaled by mul
template <int DH, int LD>
__device__ __forceinline__ void stage_rows(float* dst, const float* src, int64_t ld, int n, float mul) {
    constexpr int R4 = DH / 4;
    for (int e = threadIdx.x; e < 64 * R4; e += 256) {
        const int row = e / R4, d4 = (e % R4) * 4;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < n) x = *reinterpret_cast<const float4*>(src + row * ld + d4);
        float* o = dst + row * LD + d4;
        o[0] = x.x * mul; o[1] = x.y * mul; o[2] = x.z * mul; o[3] = x.w * mul;
    }
}

// DROP: with M the forward's scaled mask (0 or 1 / (1 - p)), O = (P o M) V, so dV = (P o M)^T dO,
// dP = M o (dO V^T) and dS = P o (dP - D) with D = rowsum(dO o O) unchanged.
template <int DH, bool DROP = false>
__global__ void __launch_bounds__(256)
attn_bwd_dq_mfma_kernel(AttnBwd a) {
    constexpr int KS = DH / 4, DT = DH / 16, LD = DH + 4;
    __shared__ float kt[64 * LD];
    __shared__ float vt[64 * LD];
    const int seg = blockIdx.x / a.q_blocks, qb = blockIdx.x % a.q_blocks, h = blockIdx.y;
    const int64_t qb0 = a.q_off[seg], qe = a.q_off[seg + 1];
    if (qb0 + (int64_t)qb * 64 >= qe) return;                 // block-uniform
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
    const int64_t r = qb0 + (int64_t)qb * 64 + wv * 16 + c;  // this lane's query row
    const bool ok = r < qe;
    const int ks = a.kv_seg[seg];
    const int64_t kb = a.kv_off[ks], ke = a.kv_off[ks + 1];
    float qv[KS], dov[KS], ov[KS];
    load_ks<KS>(a.q + r * a.ldq + h * DH + g * KS, qv, ok, a.scale * kLog2e);
    load_ks<KS>(a.dout + r * a.lddo + h * DH + g * KS, dov, ok, 1.f);
    load_ks<KS>(a.o + r * a.ldo + h * DH + g * KS, ov, ok, 1.f);
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) dsum = fmaf(dov[s], ov[s], dsum);
    dsum = xg_sum_tr(dsum);
    // S^T tile n of the staged keys: lane (g, c) -> keys 16n + 4g + r of query c
    auto scores = [&](const float* tile, const float (&rv)[KS], int n) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
        const float* kr = tile + (16 * n + c) * LD + g * KS;
#pragma unroll
        for (int s = 0; s < KS; ++s)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kr[s], rv[s], acc, 0, 0, 0);
        return acc;
    };
    // pass 1: the row's max and sum (per lane over its keys, then over the 4 lanes of the row)
    // -- or the forward's log-sum-exp
    float m = -INFINITY, l = 0.f;
    for (int64_t t0 = a.lse_in ? ke : kb; t0 < ke; t0 += 64) {
        const int nt = (int)min((int64_t)64, ke - t0);
        __syncthreads();
        stage_rows<DH, LD>(kt, a.k + t0 * a.ldk + h * DH, a.ldk, nt, 1.f);
        __syncthreads();
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const f32x4_t s4 = scores(kt, qv, n);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                if (16 * n + 4 * g + rr >= nt) continue;
                const float sv = s4[rr];
                if (sv > m) { l = l * __builtin_amdgcn_exp2f(m - sv) + 1.f; m = sv; }
                else l += __builtin_amdgcn_exp2f(sv - m);
            }
        }
    }
    const float M = xg_max_tr(m);
    const float lse2 = a.lse_in ? (ok ? a.lse_in[r * a.nhead + h] : 0.f)
                                : M + __builtin_amdgcn_logf(xg_sum_tr(m == -INFINITY ? 0.f : l * __builtin_amdgcn_exp2f(m - M)));
    // pass 2: P, dP, dS and dQ^T += K^T dS^T
    f32x4_t dq[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) dq[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int64_t t0 = kb; t0 < ke; t0 += 64) {
        const int nt = (int)min((int64_t)64, ke - t0);
        __syncthreads();
        stage_rows<DH, LD>(kt, a.k + t0 * a.ldk + h * DH, a.ldk, nt, 1.f);
        stage_rows<DH, LD>(vt, a.v + t0 * a.ldv + h * DH, a.ldv, nt, 1.f);
        __syncthreads();
        float ds[4][4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const f32x4_t s4 = scores(kt, qv, n);
            const f32x4_t p4 = scores(vt, dov, n);                // dP^T = V dO^T
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const bool in = 16 * n + 4 * g + rr < nt;
                const float p = in ? __builtin_amdgcn_exp2f(s4[rr] - lse2) : 0.f;
                float dp = p4[rr];
                if constexpr (DROP)
                    dp = attn_drop_hash(a.drop_seed, h, r, t0 + 16 * n + 4 * g + rr) < a.drop_thresh
                             ? 0.f : dp * a.inv_keep;
                ds[n][rr] = p * (dp - dsum);
            }
        }
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    dq[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        kt[(16 * n + 4 * g + rr) * LD + 16 * t + c], ds[n][rr], dq[t], 0, 0, 0);
    }
    // dQ = scale * sum dS K; lane (g, c) holds dims 16t + 4g .. + 3 of query c
    const int64_t rq = qb0 + (int64_t)qb * 64 + wv * 16 + c;
    if (rq < qe) {
#pragma unroll
        for (int t = 0; t < DT; ++t)
            *reinterpret_cast<float4*>(a.dq + rq * a.lddq + h * DH + 16 * t + 4 * g) =
                make_float4(dq[t][0] * a.scale, dq[t][1] * a.scale, dq[t][2] * a.scale, dq[t][3] * a.scale);
        if (g == 0) {
            a.lse[rq * a.nhead + h] = lse2;
            a.dsum[rq * a.nhead + h] = dsum;
        }
    }
}

template <int DH, bool DROP = false>
__global__ void __launch_bounds__(256)
attn_bwd_dkdv_mfma_kernel(AttnBwd a) {
    constexpr int KS = DH / 4, DT = DH / 16, LD = DH + 4;
    __shared__ float qt[64 * LD];
    __shared__ float dt[64 * LD];
    __shared__ float lt[64], st[64];
    const int ks = blockIdx.x / a.kv_blocks, kbk = blockIdx.x % a.kv_blocks, h = blockIdx.y;
    const int64_t kb0 = a.kv_off[ks], ke = a.kv_off[ks + 1];
    if (kb0 + (int64_t)kbk * 64 >= ke) return;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
    const int64_t rk = kb0 + (int64_t)kbk * 64 + wv * 16 + c;   // this lane's key row
    const bool ok = rk < ke;
    float kv[KS], vv[KS];
    load_ks<KS>(a.k + rk * a.ldk + h * DH + g * KS, kv, ok, 1.f);
    load_ks<KS>(a.v + rk * a.ldv + h * DH + g * KS, vv, ok, 1.f);
    f32x4_t dk[DT], dv[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) dk[t] = dv[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int seg = 0; seg < a.n_seg; ++seg) {
        if (a.kv_seg[seg] != ks) continue;
        const int64_t qb = a.q_off[seg], qe = a.q_off[seg + 1];
        for (int64_t t0 = qb; t0 < qe; t0 += 64) {
            const int nt = (int)min((int64_t)64, qe - t0);
            __syncthreads();
            stage_rows<DH, LD>(qt, a.q + t0 * a.ldq + h * DH, a.ldq, nt, a.scale * kLog2e);
            stage_rows<DH, LD>(dt, a.dout + t0 * a.lddo + h * DH, a.lddo, nt, 1.f);
            if (tid < 64) {
                lt[tid] = tid < nt ? a.lse[(t0 + tid) * a.nhead + h] : INFINITY;   // P = 0 past the end
                st[tid] = tid < nt ? a.dsum[(t0 + tid) * a.nhead + h] : 0.f;
            }
            __syncthreads();
            float p[4][4], ds[4][4];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                // S[query 16n + 4g + r][key c] = Q K^T, dP = dO V^T
                f32x4_t s4 = {0.f, 0.f, 0.f, 0.f}, d4 = s4;
                const float* qr = qt + (16 * n + c) * LD + g * KS;
                const float* dr = dt + (16 * n + c) * LD + g * KS;
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    s4 = __builtin_amdgcn_mfma_f32_16x16x4f32(qr[s], kv[s], s4, 0, 0, 0);
                    d4 = __builtin_amdgcn_mfma_f32_16x16x4f32(dr[s], vv[s], d4, 0, 0, 0);
                }
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int qi = 16 * n + 4 * g + rr;
                    const float pv = __builtin_amdgcn_exp2f(s4[rr] - lt[qi]);
                    if constexpr (DROP) {
                        const float mk = attn_drop_hash(a.drop_seed, h, t0 + qi, rk) < a.drop_thresh
                                             ? 0.f : a.inv_keep;
                        p[n][rr] = pv * mk;                    // dV uses the dropped weights
                        ds[n][rr] = pv * (d4[rr] * mk - st[qi]);
                    } else {
                        p[n][rr] = pv;
                        ds[n][rr] = pv * (d4[rr] - st[qi]);
                    }
                }
            }
            // dV^T += dO^T P, dK^T += Q^T dS (k-step (n, r): query 16n + 4g + r)
#pragma unroll
            for (int t = 0; t < DT; ++t)
#pragma unroll
                for (int n = 0; n < 4; ++n)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int qi = 16 * n + 4 * g + rr;
                        dv[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(dt[qi * LD + 16 * t + c], p[n][rr], dv[t], 0, 0, 0);
                        dk[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(qt[qi * LD + 16 * t + c], ds[n][rr], dk[t], 0, 0, 0);
                    }
        }
    }
    if (!ok) return;
    // the staged q carried scale * log2 e: dK = scale * sum dS q = (sum dS qt) / log2 e
    constexpr float il2 = 1.0f / kLog2e;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
        *reinterpret_cast<float4*>(a.dk + rk * a.lddk + h * DH + 16 * t + 4 * g) =
            make_float4(dk[t][0] * il2, dk[t][1] * il2, dk[t][2] * il2, dk[t][3] * il2);
        *reinterpret_cast<float4*>(a.dv + rk * a.lddv + h * DH + 16 * t + 4 * g) =
            make_float4(dv[t][0], dv[t][1], dv[t][2], dv[t][3]);
    }
}

// ---- CorrespondenceDecoder.simple_attention backward ----------------------------------------
// corr[i] = sum_j P_ij v_j, P = softmax_j(s_ij), s_ij = scale q_i.k_j, v_j = the partner cloud's
// xyz (3 columns, no gradient). With D_i = dO_i . corr_i and dS_ij = P_ij (dO_i . v_j - D_i):
//   dq_i = scale sum_j dS_ij k_j,   dk_j = scale sum_i dS_ij q_i.
// The forward kernel's layout (attention.hip corr_attention_kernel): 32 rows x 8 lanes per
// block, each lane a D/8 slice of the dot products reduced over its 8 lanes with DPP, the other
// side's rows staged 32 at a time through LDS; fp32, no atomics (kernel 2 owns its key rows).
constexpr int kCbQ = 32;

__device__ __forceinline__ float sum8(float s) {
    s += dpp<0xB1>(s);
    s += dpp<0x4E>(s);
    s += dpp<0x141>(s);
    return s;
}

struct CorrBwd {
    const float* q; int64_t ld_q;
    const float* k; int64_t ld_k;
    const float* xyz;
    const float* dout;
    float* dq; int64_t ld_dq;
    float* dk; int64_t ld_dk;
    const int64_t* q_off;
    const int64_t* kv_off;
    const int32_t* kv_seg;
    const int64_t* v_off;
    int n_seg;
    float scale;
    float* lse;
    float* dsum;
};

template <int D>
__global__ void __launch_bounds__(256)
corr_attn_bwd_dq_kernel(CorrBwd a) {
    constexpr int DL = D / 8;
    __shared__ float kt[kCbQ][D + 4];
    __shared__ float vt[kCbQ][3];
    const int seg = blockIdx.y;
    const int64_t qb = a.q_off[seg], qe = a.q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)blockIdx.x * kCbQ;
    if (q0 >= qe) return;                                  // block-uniform
    const int ks = a.kv_seg[seg];
    const int64_t kb = a.kv_off[ks], ke = a.kv_off[ks + 1];
    const int64_t vb = a.v_off[ks];
    const int tid = threadIdx.x, qi = tid >> 3, sl = tid & 7;
    const int64_t row = q0 + qi;
    const bool active = row < qe;
    float qv[DL], dqv[DL];
#pragma unroll
    for (int e = 0; e < DL; ++e) {
        qv[e] = active ? a.q[row * a.ld_q + sl * DL + e] * a.scale : 0.f;
        dqv[e] = 0.f;
    }
    const float d0 = active ? a.dout[row * 3] : 0.f, d1 = active ? a.dout[row * 3 + 1] : 0.f,
                d2 = active ? a.dout[row * 3 + 2] : 0.f;
    float m = -INFINITY, l = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int pass = 0; pass < 2; ++pass) {
        float inv_l = 0.f, dsum = 0.f;
        if (pass == 1) {
            inv_l = 1.0f / l;
            dsum = d0 * (a0 * inv_l) + d1 * (a1 * inv_l) + d2 * (a2 * inv_l);   // dO . corr
        }
        for (int64_t j0 = kb; j0 < ke; j0 += kCbQ) {
            const int nk = (int)min((int64_t)kCbQ, ke - j0);
            __syncthreads();
            for (int e = tid; e < kCbQ * D; e += 256) {
                const int r = e / D, cc = e - r * D;
                kt[r][cc] = r < nk ? a.k[(j0 + r) * a.ld_k + cc] : 0.f;
            }
            if (tid < kCbQ * 3) {
                const int r = tid / 3, cc = tid - r * 3;
                vt[r][cc] = r < nk ? a.xyz[(vb + (j0 - kb) + r) * 3 + cc] : 0.f;
            }
            __syncthreads();
            for (int r = 0; r < nk; ++r) {
                float s = 0.f;
#pragma unroll
                for (int e = 0; e < DL; ++e) s = fmaf(qv[e], kt[r][sl * DL + e], s);
                s = sum8(s);
                if (pass == 0) {                           // the forward's online softmax
                    if (s > m) {
                        const float f = __expf(m - s);
                        l *= f; a0 *= f; a1 *= f; a2 *= f;
                        m = s;
                    }
                    const float p = __expf(s - m);
                    l += p;
                    a0 = fmaf(p, vt[r][0], a0);
                    a1 = fmaf(p, vt[r][1], a1);
                    a2 = fmaf(p, vt[r][2], a2);
                } else {
                    const float p = __expf(s - m) * inv_l;
                    const float dp = d0 * vt[r][0] + d1 * vt[r][1] + d2 * vt[r][2];
                    const float ds = p * (dp - dsum);
#pragma unroll
                    for (int e = 0; e < DL; ++e) dqv[e] = fmaf(ds, kt[r][sl * DL + e], dqv[e]);
                }
            }
        }
        if (pass == 1 && active) {
#pragma unroll
            for (int e = 0; e < DL; ++e) a.dq[row * a.ld_dq + sl * DL + e] = dqv[e] * a.scale;
            if (sl == 0) {
                a.lse[row] = m + logf(l);
                a.dsum[row] = dsum;
            }
        }
    }
}

template <int D>
__global__ void __launch_bounds__(256)
corr_attn_bwd_dk_kernel(CorrBwd a) {
    constexpr int DL = D / 8;
    __shared__ float qt[kCbQ][D + 4];
    __shared__ float dt[kCbQ][5];                          // dO (3), lse, D of each staged query
    const int ks = blockIdx.y;
    const int64_t kb = a.kv_off[ks], ke = a.kv_off[ks + 1];
    const int64_t k0 = kb + (int64_t)blockIdx.x * kCbQ;
    if (k0 >= ke) return;                                  // block-uniform
    const int tid = threadIdx.x, ki = tid >> 3, sl = tid & 7;
    const int64_t row = k0 + ki;
    const bool active = row < ke;
    float kv[DL], dkv[DL];
#pragma unroll
    for (int e = 0; e < DL; ++e) {
        kv[e] = active ? a.k[row * a.ld_k + sl * DL + e] : 0.f;
        dkv[e] = 0.f;
    }
    for (int seg = 0; seg < a.n_seg; ++seg) {
        if (a.kv_seg[seg] != ks) continue;
        const int64_t vb = a.v_off[ks] + (row - kb);
        const float v0 = active ? a.xyz[vb * 3] : 0.f, v1 = active ? a.xyz[vb * 3 + 1] : 0.f,
                    v2 = active ? a.xyz[vb * 3 + 2] : 0.f;
        const int64_t qb = a.q_off[seg], qe = a.q_off[seg + 1];
        for (int64_t i0 = qb; i0 < qe; i0 += kCbQ) {
            const int nq = (int)min((int64_t)kCbQ, qe - i0);
            __syncthreads();
            for (int e = tid; e < kCbQ * D; e += 256) {
                const int r = e / D, cc = e - r * D;
                qt[r][cc] = r < nq ? a.q[(i0 + r) * a.ld_q + cc] * a.scale : 0.f;
            }
            if (tid < kCbQ) {
                const bool ok = tid < nq;
                const int64_t r = i0 + tid;
                dt[tid][0] = ok ? a.dout[r * 3] : 0.f;
                dt[tid][1] = ok ? a.dout[r * 3 + 1] : 0.f;
                dt[tid][2] = ok ? a.dout[r * 3 + 2] : 0.f;
                dt[tid][3] = ok ? a.lse[r] : 0.f;
                dt[tid][4] = ok ? a.dsum[r] : 0.f;
            }
            __syncthreads();
            for (int r = 0; r < nq; ++r) {
                float s = 0.f;
#pragma unroll
                for (int e = 0; e < DL; ++e) s = fmaf(qt[r][sl * DL + e], kv[e], s);
                s = sum8(s);
                const float p = __expf(s - dt[r][3]);
                const float dp = dt[r][0] * v0 + dt[r][1] * v1 + dt[r][2] * v2;
                const float ds = p * (dp - dt[r][4]);
#pragma unroll
                for (int e = 0; e < DL; ++e) dkv[e] = fmaf(ds, qt[r][sl * DL + e], dkv[e]);   // qt = scale q
            }
        }
    }
    if (!active) return;
#pragma unroll
    for (int e = 0; e < DL; ++e) a.dk[row * a.ld_dk + sl * DL + e] = dkv[e];
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_nbr_inverse_workspace(int64_t nq, int32_t width, int64_t ns, size_t* bytes) {
    FGR_REQUIRE(bytes && nq >= 0 && width >= 0 && ns >= 0 && nq * (int64_t)width < (1ll << 31),
                "fgr_nbr_inverse_workspace: bad arguments");
    *bytes = (size_t)(ns + 1) * sizeof(int) + (size_t)nq * width * sizeof(int);
    return FGR_OK;
}

extern "C" int fgr_nbr_inverse(const int64_t* idx, int64_t nq, int32_t width, int64_t ns, int32_t* start,
                               int32_t* pos, int32_t* ent, void* ws, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(nq >= 0 && width >= 0 && ns >= 0 && nq * (int64_t)width < (1ll << 31),
                "fgr_nbr_inverse: bad arguments");
    FGR_REQUIRE(start && pos && ent && ws && (nq * width == 0 || idx), "fgr_nbr_inverse: null pointer");
    size_t need = 0;
    fgr_nbr_inverse_workspace(nq, width, ns, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_nbr_inverse: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    const int64_t n_ent = nq * (int64_t)width;
    int* cnt = (int*)ws;
    int* tmp = cnt + (ns + 1);
    FGR_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)(ns + 1) * sizeof(int), st));
    if (n_ent > 0)
        FGR_CHECK_HIP(hipMemsetAsync(pos, 0xFF, (size_t)n_ent * sizeof(int), st));
    const unsigned eb = (unsigned)std::max<int64_t>(1, ceil_div(n_ent, 256));
    if (n_ent > 0) {
        hipLaunchKernelGGL(nbr_count_kernel, dim3(eb), dim3(256), 0, st, idx, n_ent, ns, cnt);
        FGR_CHECK_LAUNCH("nbr_count_kernel");
    }
    hipLaunchKernelGGL(nbr_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, ns, start);
    FGR_CHECK_LAUNCH("nbr_scan_kernel");
    if (n_ent == 0 || ns == 0) return FGR_OK;
    hipLaunchKernelGGL(nbr_fill_kernel, dim3(eb), dim3(256), 0, st, idx, n_ent, ns, cnt, tmp);
    FGR_CHECK_LAUNCH("nbr_fill_kernel");
    hipLaunchKernelGGL(nbr_sort_kernel, dim3((unsigned)ceil_div(ns, 4)), dim3(256), 0, st, start, ns,
                       (const int*)tmp, ent, pos);
    FGR_CHECK_LAUNCH("nbr_sort_kernel");
    return FGR_OK;
}

extern "C" int fgr_kpconv_scatter_workspace(int64_t nq, int32_t width, int32_t cin, size_t* bytes) {
    FGR_REQUIRE(bytes && nq >= 0 && width >= 0 && cin > 0, "fgr_kpconv_scatter_workspace: bad arguments");
    *bytes = std::max<size_t>(1, (size_t)nq * width * cin * sizeof(float));
    return FGR_OK;
}

extern "C" int fgr_kpconv_scatter(const float* q, const float* s, int64_t nq, int64_t ns,
                                  const int64_t* idx, int32_t width, const float* dwf, int32_t cin,
                                  const float* kernel_points, int32_t n_kp, float extent,
                                  const int32_t* start, const int32_t* pos, float* dx, void* ws,
                                  size_t ws_bytes, void* stream) {
    FGR_REQUIRE(nq >= 0 && ns >= 0 && width >= 0 && cin > 0 && n_kp > 0 && n_kp <= kMaxKpT &&
                    extent > 0.f, "fgr_kpconv_scatter: bad arguments");
    if (ns == 0) return FGR_OK;
    FGR_REQUIRE(start && dx && ws, "fgr_kpconv_scatter: null pointer");
    size_t need = 0;
    fgr_kpconv_scatter_workspace(nq, width, cin, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_kpconv_scatter: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    float* g = (float*)ws;
    if (nq > 0 && width > 0) {
        FGR_REQUIRE(q && s && idx && dwf && kernel_points && pos, "fgr_kpconv_scatter: null pointer");
        hipLaunchKernelGGL(kpconv_scatter_rows_kernel, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, st,
                           q, s, nq, ns, idx, width, dwf, cin, kernel_points, n_kp, 1.0f / extent,
                           (const int*)pos, g);
        FGR_CHECK_LAUNCH("kpconv_scatter_rows_kernel");
    }
    hipLaunchKernelGGL(csr_rowsum_kernel, dim3((unsigned)ceil_div(ns * cin, 256)), dim3(256), 0, st,
                       (const int*)start, ns, (const float*)g, cin, dx);
    FGR_CHECK_LAUNCH("csr_rowsum_kernel");
    return FGR_OK;
}

extern "C" int fgr_max_pool_bwd_workspace(int64_t nq, int32_t c, size_t* bytes) {
    FGR_REQUIRE(bytes && nq >= 0 && c > 0, "fgr_max_pool_bwd_workspace: bad arguments");
    *bytes = std::max<size_t>(1, (size_t)nq * c * sizeof(int));
    return FGR_OK;
}

extern "C" int fgr_max_pool_bwd(const float* x, int64_t ns, int32_t c, const int64_t* idx, int64_t nq,
                                int32_t width, const float* dy, const int32_t* start,
                                const int32_t* ent, float* dx, void* ws, size_t ws_bytes,
                                void* stream) {
    FGR_REQUIRE(ns >= 0 && nq >= 0 && c > 0 && width > 0, "fgr_max_pool_bwd: bad arguments");
    if (ns == 0) return FGR_OK;
    FGR_REQUIRE(start && ent && dx && ws && (nq == 0 || (x && idx && dy)), "fgr_max_pool_bwd: null pointer");
    size_t need = 0;
    fgr_max_pool_bwd_workspace(nq, c, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_max_pool_bwd: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    int* am = (int*)ws;
    if (nq > 0) {
        hipLaunchKernelGGL(max_pool_argmax_kernel, dim3((unsigned)ceil_div(nq * c, 256)), dim3(256), 0, st,
                           x, ns, c, idx, nq, width, am);
        FGR_CHECK_LAUNCH("max_pool_argmax_kernel");
    }
    hipLaunchKernelGGL(max_pool_bwd_csr_kernel, dim3((unsigned)ceil_div(ns * c, 256)), dim3(256), 0, st,
                       (const int*)start, (const int*)ent, ns, c, width, (const int*)am, dy, dx);
    FGR_CHECK_LAUNCH("max_pool_bwd_csr_kernel");
    return FGR_OK;
}

extern "C" int fgr_corr_attention_bwd_workspace(int64_t n_rows, size_t* bytes) {
    FGR_REQUIRE(bytes && n_rows >= 0, "fgr_corr_attention_bwd_workspace: bad arguments");
    *bytes = (size_t)std::max<int64_t>(n_rows, 1) * 2 * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_corr_attention_bwd(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                      const float* xyz, const float* dout, float* dq, int64_t ld_dq,
                                      float* dk, int64_t ld_dk, const int64_t* q_off,
                                      const int64_t* kv_off, const int32_t* kv_seg,
                                      const int64_t* v_off, int32_t n_seg, int32_t n_kv_seg,
                                      int64_t n_rows, int32_t max_q_len, int32_t max_kv_len, int32_t d,
                                      float scale, void* ws, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(n_seg > 0 && n_kv_seg > 0 && n_rows >= 0 && max_q_len >= 0 && max_kv_len >= 0 &&
                    ld_q >= d && ld_k >= d && ld_dq >= d && ld_dk >= d,
                "fgr_corr_attention_bwd: bad arguments");
    FGR_REQUIRE(d == 32 || d == 64 || d == 128 || d == 256 || d == 512,
                "fgr_corr_attention_bwd: d %d unsupported (32, 64, 128, 256, 512)", d);
    FGR_REQUIRE(q && k && xyz && dout && dq && dk && q_off && kv_off && kv_seg && v_off && ws,
                "fgr_corr_attention_bwd: null pointer");
    size_t need = 0;
    fgr_corr_attention_bwd_workspace(n_rows, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_corr_attention_bwd: workspace %zu < %zu bytes", ws_bytes, need);
    const int64_t nr = std::max<int64_t>(n_rows, 1);
    CorrBwd a{q, ld_q, k, ld_k, xyz, dout, dq, ld_dq, dk, ld_dk, q_off, kv_off, kv_seg, v_off, n_seg,
              scale, (float*)ws, (float*)ws + nr};
    hipStream_t st = as_stream(stream);
    const dim3 g1((unsigned)std::max<int64_t>(1, ceil_div(max_q_len, kCbQ)), (unsigned)n_seg);
    const dim3 g2((unsigned)std::max<int64_t>(1, ceil_div(max_kv_len, kCbQ)), (unsigned)n_kv_seg);
    switch (d) {
#define CAB(DD) case DD: \
        hipLaunchKernelGGL(corr_attn_bwd_dq_kernel<DD>, g1, dim3(256), 0, st, a); \
        FGR_CHECK_LAUNCH("corr_attn_bwd_dq_kernel"); \
        hipLaunchKernelGGL(corr_attn_bwd_dk_kernel<DD>, g2, dim3(256), 0, st, a); \
        break;
        CAB(32) CAB(64) CAB(128) CAB(256) CAB(512)
#undef CAB
    }
    FGR_CHECK_LAUNCH("corr_attn_bwd_dk_kernel");
    return FGR_OK;
}

// the float4 segment-norm kernels: c % 4 == 0, every given pointer 16-B aligned (NULL
// allowed), float4 indices below 2^31
static bool seg_vec_ok(int64_t n, int c, std::initializer_list<const void*> ptrs) {
    if (c % 4 != 0 || n * c / 4 >= (int64_t)1 << 31) return false;
    for (const void* q : ptrs)
        if (reinterpret_cast<uintptr_t>(q) & 15) return false;
    return true;
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
    if (seg_vec_ok(n, c, {x}))
        hipLaunchKernelGGL(segnorm_stats4_kernel, dim3(a.n_chunks, n_seg, (unsigned)ceil_div(c, 64)),
                           dim3(256), 0, st, a, (double*)ws);
    else
        hipLaunchKernelGGL(segnorm_stats_kernel, dim3(a.n_chunks, n_seg, (unsigned)ceil_div(c, 64)),
                           dim3(256), 0, st, a, (double*)ws);
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
    if (seg_vec_ok(n, c, {x, out, residual, mean, rstd, gamma, beta}))
        hipLaunchKernelGGL(segnorm_apply4_kernel, dim3((unsigned)ceil_div(n * c / 4, 256)), dim3(256), 0,
                           as_stream(stream), p, out);
    else
        hipLaunchKernelGGL(segnorm_apply_kernel, dim3((unsigned)ceil_div(n * c, 256)), dim3(256), 0,
                           as_stream(stream), p, out);
    FGR_CHECK_LAUNCH("segnorm_apply_kernel");
    return FGR_OK;
}

extern "C" int fgr_segnorm_fwd(const float* x, int64_t n, int32_t c, const int64_t* seg_off,
                               int32_t n_seg, int64_t max_seg_len, const float* row_div, float eps,
                               float* mean, float* rstd, float* var, const float* gamma,
                               const float* beta, int32_t act, const float* residual,
                               int32_t post_act, float* out, void* ws, size_t ws_bytes,
                               void* stream) {
    static const bool fuse = [] { const char* e = getenv("FGR_SEG_FUSED"); return !(e && e[0] == '0'); }();
    if (fuse && n > 0 && c > 0 && n_seg > 0 && max_seg_len > 0 && seg_chunks(max_seg_len) <= kSegFuseChunksMax &&
        x && seg_off && mean && rstd && var && out && ws &&
        seg_vec_ok(n, c, {x, out, residual, mean, rstd, gamma, beta}) && (!gamma == !beta)) {
        size_t need = 0;
        fgr_segnorm_workspace(max_seg_len, c, n_seg, &need);
        FGR_REQUIRE(ws_bytes >= need, "fgr_segnorm_fwd: workspace too small");
        SegApply p{{x, row_div, seg_off, n_seg, c, seg_chunks(max_seg_len)}, n, mean, rstd, gamma, beta, act,
                   residual, post_act};
        hipStream_t st = as_stream(stream);
        const dim3 grid(p.a.n_chunks, n_seg, (unsigned)ceil_div(c, 64));
        hipLaunchKernelGGL(segnorm_stats4_kernel, grid, dim3(256), 0, st, p.a, (double*)ws);
        FGR_CHECK_LAUNCH("segnorm_stats4_kernel");
        hipLaunchKernelGGL(segnorm_merge_apply4_kernel, grid, dim3(256), 0, st, p, (const double*)ws, eps,
                           mean, rstd, var, out);
        FGR_CHECK_LAUNCH("segnorm_merge_apply4_kernel");
        return FGR_OK;
    }
    const int rc = fgr_segnorm_stats(x, n, c, seg_off, n_seg, max_seg_len, row_div, eps, mean, rstd,
                                     var, ws, ws_bytes, stream);
    if (rc != FGR_OK) return rc;
    return fgr_segnorm_apply(x, n, c, seg_off, n_seg, row_div, mean, rstd, gamma, beta, act, residual,
                             post_act, out, stream);
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
    const bool vec = seg_vec_ok(n, c, {x, dy, has_residual ? y : nullptr, dx, has_residual ? dres : nullptr,
                                       mean, rstd, gamma, beta, sums});
    static const bool fuse = [] { const char* e = getenv("FGR_SEG_FUSED"); return !(e && e[0] == '0'); }();
    if (fuse && vec && n > 0 && nch <= kSegFuseChunksMax) {
        const dim3 grid(nch, n_seg, (unsigned)ceil_div(c, 64));
        hipLaunchKernelGGL(segnorm_bwd_stats4_kernel, grid, dim3(256), 0, st, p, dy, y, part);
        FGR_CHECK_LAUNCH("segnorm_bwd_stats4_kernel");
        hipLaunchKernelGGL(segnorm_bwd_merge_apply4_kernel, grid, dim3(256), 0, st, p, dy, y,
                           (const double*)part, dgamma, dbeta, dx, has_residual ? dres : nullptr);
        FGR_CHECK_LAUNCH("segnorm_bwd_merge_apply4_kernel");
        return FGR_OK;
    }
    if (vec)
        hipLaunchKernelGGL(segnorm_bwd_stats4_kernel, dim3(nch, n_seg, (unsigned)ceil_div(c, 64)), dim3(256),
                           0, st, p, dy, y, part);
    else
        hipLaunchKernelGGL(segnorm_bwd_stats_kernel, dim3(nch, n_seg, (unsigned)ceil_div(c, 64)), dim3(256),
                           0, st, p, dy, y, part);
    FGR_CHECK_LAUNCH("segnorm_bwd_stats_kernel");
    hipLaunchKernelGGL(segnorm_bwd_merge_kernel, dim3((unsigned)ceil_div((int64_t)n_seg * c, 256)),
                       dim3(256), 0, st, p.a, (const double*)part, sums, dgamma, dbeta);
    FGR_CHECK_LAUNCH("segnorm_bwd_merge_kernel");
    if (n == 0) return FGR_OK;
    if (vec)
        hipLaunchKernelGGL(segnorm_bwd_apply4_kernel, dim3((unsigned)ceil_div(n * c / 4, 256)), dim3(256), 0,
                           st, p, dy, y, (const float*)sums, dx, has_residual ? dres : nullptr);
    else
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

static int attention_bwd_impl(const float* q, int64_t ldq, const float* k, int64_t ldk,
                              const float* v, int64_t ldv, const float* o, int64_t ldo,
                              const float* dout, int64_t lddo, float* dq, int64_t lddq, float* dk,
                              int64_t lddk, float* dv, int64_t lddv, const int64_t* q_off,
                              const int64_t* kv_off, const int32_t* kv_seg, int32_t n_seg,
                              int32_t n_kv_seg, int64_t nq, int64_t max_q_len, int64_t max_kv_len,
                              int32_t nhead, int32_t dh, float scale, void* ws, size_t ws_bytes,
                              uint32_t drop_seed, float drop_p, void* stream,
                              const float* lse_in = nullptr, int64_t n_kv_rows = -1) {
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
              (float*)ws + std::max<int64_t>(nq, 1) * nhead, drop_seed,
              (uint32_t)std::min(4294967295.0, (double)drop_p * 4294967296.0),
              drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.f, lse_in};
    const bool drop = drop_p > 0.f;
    hipStream_t st = as_stream(stream);
    dim3 g1((unsigned)(n_seg * a.q_blocks), nhead), g2((unsigned)(n_kv_seg * a.kv_blocks), nhead);
    // head dim 16 / 32 / 64 with 16-B aligned rows: the fp32-MFMA kernels (FGR_ATTN_BWD=scalar:
    // the scalar ones, for A/B)
    const bool al = ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
                      reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o) |
                      reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dq) |
                      reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) & 15) == 0 &&
                    (ldq | ldk | ldv | ldo | lddo | lddq | lddk | lddv) % 4 == 0;
    static const bool scalar_only = [] { const char* e = getenv("FGR_ATTN_BWD"); return e && e[0] == 's'; }();
    const bool mfma = al && !scalar_only && (dh == 16 || dh == 32 || dh == 64);
    FGR_REQUIRE(!drop || (al && (dh == 16 || dh == 32 || dh == 64)),
                "fgr_attention_bwd_drop: dropout needs head dim 16 / 32 / 64 and 16-B aligned rows");
    // training with the forward's lse (head dim 32 / 64): the f16x3 kernels (attention16.hip
    // attn_bwd_f16x3), their K / V / Q / dO images after lse / D in ws
    // (fgr_attention_bwd_train_workspace). FGR_ATTN_BWD16=0: the fp32-MFMA kernels, =q: only dQ
    // on the f16 matrix cores (A/B)
    static const int bwd16 = [] {
        const char* e = getenv("FGR_ATTN_BWD16");
        return e && e[0] == '0' ? 0 : e && e[0] == 'q' ? 1 : 2;
    }();
    const size_t lse_bytes = (need + 255) & ~(size_t)255;
    const int64_t n_rows = std::max(nq, n_kv_rows);
    if (bwd16 && lse_in && n_kv_rows >= 0 && al && (dh == 32 || dh == 64) &&
        ws_bytes >= lse_bytes + attn_bwd_f16x3_bytes(n_rows, std::max(n_seg, n_kv_seg), nhead, dh)) {
        FGR_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0, "fgr_attention_bwd_train: ws alignment");
        const bool dkdv16 = bwd16 == 2;
        const int rc = attn_bwd_f16x3(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, dq, lddq, dk, lddk, dv,
                                      lddv, q_off, kv_off, kv_seg, n_seg, n_kv_seg, n_rows, max_q_len,
                                      max_kv_len, nhead, dh, scale, lse_in, a.lse, a.dsum, dkdv16,
                                      static_cast<char*>(ws) + lse_bytes, a.drop_seed,
                                      a.drop_thresh, a.inv_keep, st);
        if (rc != FGR_OK || dkdv16) return rc;
        switch (dh) {
#define AT16(D) case D: \
            if (drop) hipLaunchKernelGGL((attn_bwd_dkdv_mfma_kernel<D, true>), g2, dim3(256), 0, st, a); \
            else hipLaunchKernelGGL((attn_bwd_dkdv_mfma_kernel<D, false>), g2, dim3(256), 0, st, a); \
            break;
            AT16(32) AT16(64)
#undef AT16
        }
        FGR_CHECK_LAUNCH("attn_bwd_dkdv_mfma_kernel");
        return FGR_OK;
    }
    if (drop) {
        switch (dh) {
#define ATD(D) case D: \
            hipLaunchKernelGGL((attn_bwd_dq_mfma_kernel<D, true>), g1, dim3(256), 0, st, a); \
            FGR_CHECK_LAUNCH("attn_bwd_dq_mfma_kernel"); \
            hipLaunchKernelGGL((attn_bwd_dkdv_mfma_kernel<D, true>), g2, dim3(256), 0, st, a); \
            break;
            ATD(16) ATD(32) ATD(64)
#undef ATD
        }
        FGR_CHECK_LAUNCH("attn_bwd_dkdv_mfma_kernel");
        return FGR_OK;
    }
    if (mfma) {
        switch (dh) {
#define ATM(D) case D: \
            hipLaunchKernelGGL(attn_bwd_dq_mfma_kernel<D>, g1, dim3(256), 0, st, a); \
            FGR_CHECK_LAUNCH("attn_bwd_dq_mfma_kernel"); \
            hipLaunchKernelGGL(attn_bwd_dkdv_mfma_kernel<D>, g2, dim3(256), 0, st, a); \
            break;
            ATM(16) ATM(32) ATM(64)
#undef ATM
        }
        FGR_CHECK_LAUNCH("attn_bwd_dkdv_mfma_kernel");
        return FGR_OK;
    }
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

extern "C" int fgr_attention_bwd(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                                 int64_t ldv, const float* o, int64_t ldo, const float* dout,
                                 int64_t lddo, float* dq, int64_t lddq, float* dk, int64_t lddk,
                                 float* dv, int64_t lddv, const int64_t* q_off, const int64_t* kv_off,
                                 const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg, int64_t nq,
                                 int64_t max_q_len, int64_t max_kv_len, int32_t nhead, int32_t dh,
                                 float scale, void* ws, size_t ws_bytes, void* stream) {
    return attention_bwd_impl(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, dq, lddq, dk, lddk, dv,
                              lddv, q_off, kv_off, kv_seg, n_seg, n_kv_seg, nq, max_q_len,
                              max_kv_len, nhead, dh, scale, ws, ws_bytes, 0u, 0.f, stream);
}

extern "C" int fgr_attention_bwd_train(const float* q, int64_t ldq, const float* k, int64_t ldk,
                                       const float* v, int64_t ldv, const float* o, int64_t ldo,
                                       const float* dout, int64_t lddo, float* dq, int64_t lddq,
                                       float* dk, int64_t lddk, float* dv, int64_t lddv,
                                       const int64_t* q_off, const int64_t* kv_off,
                                       const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg,
                                       int64_t nq, int64_t max_q_len, int64_t max_kv_len,
                                       int32_t nhead, int32_t dh, float scale, void* ws,
                                       size_t ws_bytes, uint32_t seed, float p, const float* lse,
                                       int64_t n_kv_rows, void* stream) {
    FGR_REQUIRE(p >= 0.f && p < 1.f, "fgr_attention_bwd_train: dropout p %f not in [0, 1)", p);
    FGR_REQUIRE(lse, "fgr_attention_bwd_train: null lse");
    return attention_bwd_impl(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, dq, lddq, dk, lddk, dv,
                              lddv, q_off, kv_off, kv_seg, n_seg, n_kv_seg, nq, max_q_len,
                              max_kv_len, nhead, dh, scale, ws, ws_bytes, seed, p, stream, lse,
                              n_kv_rows);
}

// fgr_attention_bwd_train's workspace: lse / D per (query row, head), then (head dim 32 / 64)
// the f16x3 kernels' K / V / Q / dO tile images (nq query rows in n_seg segments, n_kv_rows key
// rows in n_kv_seg segments, one packed row space)
extern "C" int fgr_attention_bwd_train_workspace(int64_t nq, int32_t n_seg, int64_t n_kv_rows,
                                                 int32_t n_kv_seg, int32_t nhead, int32_t dh,
                                                 size_t* bytes) {
    FGR_REQUIRE(bytes && nq >= 0 && n_seg > 0 && n_kv_rows >= 0 && n_kv_seg > 0 && nhead > 0,
                "fgr_attention_bwd_train_workspace: bad arguments");
    size_t need = 0;
    fgr_attention_bwd_workspace(nq, nhead, &need);
    *bytes = need;
    if (dh == 32 || dh == 64)
        *bytes = ((need + 255) & ~(size_t)255) +
                 attn_bwd_f16x3_bytes(std::max(nq, n_kv_rows), std::max(n_seg, n_kv_seg), nhead, dh);
    return FGR_OK;
}

extern "C" int fgr_attention_bwd_drop(const float* q, int64_t ldq, const float* k, int64_t ldk,
                                      const float* v, int64_t ldv, const float* o, int64_t ldo,
                                      const float* dout, int64_t lddo, float* dq, int64_t lddq,
                                      float* dk, int64_t lddk, float* dv, int64_t lddv,
                                      const int64_t* q_off, const int64_t* kv_off,
                                      const int32_t* kv_seg, int32_t n_seg, int32_t n_kv_seg,
                                      int64_t nq, int64_t max_q_len, int64_t max_kv_len,
                                      int32_t nhead, int32_t dh, float scale, void* ws,
                                      size_t ws_bytes, uint32_t seed, float p, void* stream) {
    FGR_REQUIRE(p >= 0.f && p < 1.f, "fgr_attention_bwd_drop: dropout p %f not in [0, 1)", p);
    return attention_bwd_impl(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, dq, lddq, dk, lddk, dv,
                              lddv, q_off, kv_off, kv_seg, n_seg, n_kv_seg, nq, max_q_len,
                              max_kv_len, nhead, dh, scale, ws, ws_bytes, seed, p, stream);
}
