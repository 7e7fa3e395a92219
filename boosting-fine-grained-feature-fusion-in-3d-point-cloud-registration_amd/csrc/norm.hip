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

constexpr int kInWaves = 8;  // waves per block, each sweeps rows with stride kInWaves

// Block = (segment, 64-channel slab). Two-pass mean / biased variance over the segment's
// rows, then the normalised write (nn.InstanceNorm1d, affine=False, eps inside the sqrt).
__global__ void __launch_bounds__(64 * kInWaves)
instnorm_kernel(const float* __restrict__ x, int c, const int64_t* __restrict__ seg_off,
                const float* __restrict__ row_div, float eps, int act,
                const float* __restrict__ residual, int post_act, float* __restrict__ out) {
    __shared__ float red[kInWaves][64];
    const int seg = blockIdx.y;
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int ch = blockIdx.x * 64 + lane;
    const bool cok = ch < c;
    const int64_t b = seg_off[seg], e = seg_off[seg + 1];
    const float n = (float)(e - b);
    if (e <= b) return;

    float s = 0.f;
    for (int64_t r = b + wv; r < e; r += kInWaves) {
        if (cok) {
            float v = x[r * c + ch];
            if (row_div) v = v / row_div[r];
            s += v;
        }
    }
    red[wv][lane] = s;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < kInWaves; ++w) tot += red[w][lane];
    const float mean = tot / n;
    __syncthreads();

    float sq = 0.f;
    for (int64_t r = b + wv; r < e; r += kInWaves) {
        if (cok) {
            float v = x[r * c + ch];
            if (row_div) v = v / row_div[r];
            const float d = v - mean;
            sq += d * d;
        }
    }
    red[wv][lane] = sq;
    __syncthreads();
    float tsq = 0.f;
#pragma unroll
    for (int w = 0; w < kInWaves; ++w) tsq += red[w][lane];
    const float rstd = 1.0f / sqrtf(tsq / n + eps);

    if (!cok) return;
    for (int64_t r = b + wv; r < e; r += kInWaves) {
        float v = x[r * c + ch];
        if (row_div) v = v / row_div[r];
        float y = act_fn((v - mean) * rstd, act);
        if (residual) y = act_fn(y + residual[r * c + ch], post_act);
        out[r * c + ch] = y;
    }
}

// One wave per row; d <= 64 * 16.
template <int PER>
__global__ void __launch_bounds__(256)
layernorm_kernel(const float* __restrict__ x, int64_t n, int d, const float* __restrict__ g,
                 const float* __restrict__ bta, float eps, const float* __restrict__ add,
                 float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const int lane = threadIdx.x % 64;
    if (r >= n) return;
    const float* xr = x + r * d;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int col = lane + 64 * j;
        v[j] = col < d ? xr[col] : 0.f;
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
__global__ void sine_pe_kernel(const float* __restrict__ xyz, int64_t n, int d, int npf,
                               float temperature, float scale, float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * d) return;
    const int64_t r = t / d;
    const int col = (int)(t - r * d);
    float y = 0.f;
    if (col < 3 * npf) {
        const int dim = col / npf, i = col - dim * npf;
        // torch: stack([sin(pd[..., 0::2]), cos(pd[..., 1::2])], -1).reshape -> pairs (sin, cos)
        const int pair = i >> 1, is_cos = i & 1;
        const int src_i = 2 * pair + is_cos;   // sin uses even feature 2p, cos odd 2p+1
        const float dim_t = powf(temperature, (float)(2 * (src_i / 2)) / (float)npf);
        const float pd = (xyz[r * 3 + dim] * scale) / dim_t;
        y = is_cos ? cosf(pd) : sinf(pd);
    }
    out[t] = y;
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_instnorm(const float* x, int64_t n, int32_t c, const int64_t* seg_off,
                            int32_t n_seg, const float* row_div, float eps, int32_t act,
                            const float* residual, int32_t post_act, float* out, void* stream) {
    FGR_REQUIRE(n >= 0 && c > 0 && n_seg > 0 && seg_off && eps >= 0.f,
                "fgr_instnorm: bad arguments");
    FGR_REQUIRE(n == 0 || (x && out), "fgr_instnorm: null pointer");
    if (n == 0) return FGR_OK;
    dim3 grid((unsigned)ceil_div(c, 64), (unsigned)n_seg);
    hipLaunchKernelGGL(instnorm_kernel, grid, dim3(64 * kInWaves), 0, as_stream(stream), x, c,
                       seg_off, row_div, eps, act, residual, post_act, out);
    FGR_CHECK_LAUNCH("instnorm_kernel");
    return FGR_OK;
}

extern "C" int fgr_layernorm(const float* x, int64_t n, int32_t d, const float* gamma,
                             const float* beta, float eps, const float* add, float* out,
                             void* stream) {
    FGR_REQUIRE(n >= 0 && d > 0 && d <= 1024 && gamma && beta, "fgr_layernorm: bad arguments");
    FGR_REQUIRE(n == 0 || (x && out), "fgr_layernorm: null pointer");
    if (n == 0) return FGR_OK;
    dim3 grid((unsigned)ceil_div(n, 4));
    hipStream_t st = as_stream(stream);
    if (d <= 64)
        hipLaunchKernelGGL(layernorm_kernel<1>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, out);
    else if (d <= 256)
        hipLaunchKernelGGL(layernorm_kernel<4>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, out);
    else if (d <= 512)
        hipLaunchKernelGGL(layernorm_kernel<8>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, out);
    else
        hipLaunchKernelGGL(layernorm_kernel<16>, grid, dim3(256), 0, st, x, n, d, gamma, beta, eps, add, out);
    FGR_CHECK_LAUNCH("layernorm_kernel");
    return FGR_OK;
}

extern "C" int fgr_sine_pos_embed(const float* xyz, int64_t n, int32_t d_model, float temperature,
                                  float scale, float* out, void* stream) {
    FGR_REQUIRE(n >= 0 && d_model >= 6, "fgr_sine_pos_embed: bad arguments");
    FGR_REQUIRE(n == 0 || (xyz && out), "fgr_sine_pos_embed: null pointer");
    if (n == 0) return FGR_OK;
    const int npf = d_model / 3 / 2 * 2;
    const int64_t tot = n * d_model;
    hipLaunchKernelGGL(sine_pe_kernel, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0,
                       as_stream(stream), xyz, n, d_model, npf, temperature, scale, out);
    FGR_CHECK_LAUNCH("sine_pe_kernel");
    return FGR_OK;
}
