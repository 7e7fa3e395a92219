// GPU-resident ModelNet "crop" test pipeline, the geometry half of
// data_loaders/modelnet_transforms.py as data_loaders/modelnet.py:111-117 chains it:
//   RandomCrop            :176-246   fgr_crop_pairs_mask      (one block per cloud)
//   RandomTransformSE3    :300-355   fgr_crop_pairs_assemble  (one block per pair; also
//   Resampler / RandomJitter / ShufflePoints  :92-173, :374-397   the index bookkeeping and
//   the correspondence list of modelnet.py:160-185)
// The random draws stay on the host in NumPy's stream (fgreg/transforms_gpu.py): they need
// only the seed and the cropped counts, never the points. Every arithmetic step repeats
// NumPy's own evaluation order so the outputs equal fgreg.transforms.modelnet_crop_test
// (pinned to the reference's transform objects) bit for bit:
//   np.mean over axis 0 of float32 rows = one float32 running sum in row order, / n;
//   np.percentile 'linear' = _lerp(s_k, s_k+1, gamma) with the branch at gamma >= 0.5;
//   np.einsum('ij,bj->bi') in float32 = ((0 + r0 x) + r1 y) + r2 z, no fused multiply-add;
//   float32 cloud += float64 noise = the float64 sum rounded to float32.
// The crop projection d = (p - mean) . u is float64 here and in NumPy (OpenBLAS dgemv may
// round its last bit differently; only the order of d matters, and ties are equal values
// in both).
#include "common.h"

#pragma clang fp contract(off)

namespace fgr {
namespace {

constexpr int kCropThreads = 1024;
constexpr int kCropMaxN = 4096;   // points per raw cloud (LDS: 12 B + 2 x 8 B per point)

// Exclusive block scan of one int flag per thread (1024 threads); returns the prefix and
// sets *total. Deterministic (fixed wave order).
__device__ __forceinline__ int block_scan(int flag, int* sh, int* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t bal = __ballot(flag);
    const int pre = __popcll(bal & ((lane ? (~0ull >> (64 - lane)) : 0ull)));
    if (lane == 0) sh[wv] = __popcll(bal);
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < kCropThreads / 64; ++w) {
        const int c = sh[w];
        base += w < wv ? c : 0;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return base + pre;
}

// One block per (pair, cloud): cloud 0 = source, 1 = reference, both cropped from the
// pair's raw cloud (SplitSourceRef copies it) with their own direction.
__global__ void __launch_bounds__(kCropThreads)
crop_mask_kernel(const float* __restrict__ raw, int ld, const int64_t* __restrict__ off,
                 const double* __restrict__ dirs, const int32_t* __restrict__ crop_k,
                 const double* __restrict__ gamma, uint8_t* __restrict__ mask,
                 int32_t* __restrict__ keep, int32_t* __restrict__ count) {
    __shared__ float px[kCropMaxN], py[kCropMaxN], pz[kCropMaxN];
    __shared__ double dd[kCropMaxN], ss[kCropMaxN];
    __shared__ double sk[2];
    __shared__ float mean[3];
    __shared__ int sh[kCropThreads / 64];
    const int b = blockIdx.x >> 1, c = blockIdx.x & 1, tid = threadIdx.x;
    const int64_t o = off[b];
    const int n = (int)(off[b + 1] - o);
    uint8_t* mk = mask + (int64_t)c * off[gridDim.x >> 1] + o;
    int32_t* kp = keep + (int64_t)c * off[gridDim.x >> 1] + o;
    if (n > kCropMaxN || n < 1) {           // the host checks; never index past the tiles
        if (tid == 0) count[blockIdx.x] = -1;
        return;
    }
    for (int i = tid; i < n; i += kCropThreads) {
        const float* p = raw + (o + i) * ld;
        px[i] = p[0];
        py[i] = p[1];
        pz[i] = p[2];
    }
    __syncthreads();
    if (tid < 3) {                          // np.mean(points[:, :3], axis=0), float32
        const float* col = tid == 0 ? px : (tid == 1 ? py : pz);
        float s = 0.f;
        int i = 0;
        for (; i + 32 <= n; i += 32) {      // 32 loads in flight, then the ordered adds
            float v[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) v[u] = col[i + u];
#pragma unroll
            for (int u = 0; u < 32; ++u) s = s + v[u];
        }
        for (; i < n; ++i) s = s + col[i];
        mean[tid] = s / (float)n;
    }
    __syncthreads();
    const double u0 = dirs[blockIdx.x * 3], u1 = dirs[blockIdx.x * 3 + 1],
                 u2 = dirs[blockIdx.x * 3 + 2];
    for (int i = tid; i < n; i += kCropThreads) {
        const double x = (double)(px[i] - mean[0]), y = (double)(py[i] - mean[1]),
                     z = (double)(pz[i] - mean[2]);
        dd[i] = x * u0 + y * u1 + z * u2;
    }
    __syncthreads();
    const int k = crop_k[b];
    double t = 0.0;                         // p_keep == 0.5: d > 0 (modelnet_transforms.py)
    if (k >= 0) {
        // order statistics s_k, s_k+1 of d: bitonic sort of a copy, padded with +inf to a
        // power of two (<= 12 * 13 / 2 = 78 compare-exchange stages of <= 2 pairs per thread)
        int P = 1;
        while (P < n) P <<= 1;
        for (int i = tid; i < P; i += kCropThreads) ss[i] = i < n ? dd[i] : __builtin_inf();
        __syncthreads();
        for (int size = 2; size <= P; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int h = tid; h < (P >> 1); h += kCropThreads) {
                    const int i = 2 * h - (h & (stride - 1));      // low index of the pair
                    const int j = i + stride;
                    const bool up = (i & size) == 0;
                    const double a = ss[i], c2 = ss[j];
                    if ((a > c2) == up) {
                        ss[i] = c2;
                        ss[j] = a;
                    }
                }
                __syncthreads();
            }
        }
        if (tid == 0) {
            sk[0] = ss[k];
            sk[1] = ss[k + 1 < n ? k + 1 : n - 1];
        }
        __syncthreads();
        const double g = gamma[b], a = sk[0], bb = sk[1], diff = bb - a;
        t = g >= 0.5 ? bb - diff * (1.0 - g) : a + diff * g;
    }
    int base = 0;
    for (int i0 = 0; i0 < n; i0 += kCropThreads) {
        const int i = i0 + tid;
        const int f = i < n && dd[i] > t;
        int tot;
        const int pos = block_scan(f, sh, &tot);
        if (i < n) mk[i] = (uint8_t)f;
        if (f) kp[base + pos] = i;
        base += tot;
    }
    if (tid == 0) count[blockIdx.x] = base;
}

// One block per pair. For cloud c and output row i < m: the raw point
// keep[c][sel[c][i]] (the host composed Resampler's choice with ShufflePoints' permutation),
// moved by the source's (R | t) when c == 0, plus the shuffled jitter noise; its overlap flag
// is the OTHER cloud's crop mask at the same raw index; inverse maps raw index -> output
// row give the correspondences, listed in raw-index order as the reference's remaps keep them.
__global__ void __launch_bounds__(kCropThreads)
crop_assemble_kernel(const float* __restrict__ raw, int ld, const int64_t* __restrict__ off,
                     const uint8_t* __restrict__ mask, const int32_t* __restrict__ keep,
                     const int32_t* __restrict__ sel, const double* __restrict__ noise,
                     const float* __restrict__ rt, int m, float* __restrict__ xyz,
                     uint8_t* __restrict__ ov, int64_t* __restrict__ corr,
                     int32_t* __restrict__ ncorr) {
    __shared__ int inv[2][kCropMaxN];
    __shared__ int sh[kCropThreads / 64];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int64_t o = off[b], ntot = off[gridDim.x];
    const int n = (int)(off[b + 1] - o);
    if (n > kCropMaxN || n < 1) {
        if (tid == 0) ncorr[b] = -1;
        return;
    }
    for (int i = tid; i < n; i += kCropThreads) inv[0][i] = inv[1][i] = -1;
    __syncthreads();
    const float* R = rt + b * 12;
    for (int c = 0; c < 2; ++c) {
        const int32_t* sl = sel + ((int64_t)b * 2 + c) * m;
        const double* nz = noise + ((int64_t)b * 2 + c) * m * 3;
        float* out = xyz + ((int64_t)b * 2 + c) * m * 3;
        for (int i = tid; i < m; i += kCropThreads) {
            const int si = sl[i];                   // host-drawn: 0 <= si < count[c]
            int r = keep[c * ntot + o + ((unsigned)si < (unsigned)n ? si : 0)];
            r = (unsigned)r < (unsigned)n ? r : 0;
            const float* p = raw + (o + r) * ld;
            float v[3] = {p[0], p[1], p[2]};
            if (c == 0) {
                float w[3];
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    float acc = 0.f;
                    acc = acc + R[e * 4 + 0] * v[0];
                    acc = acc + R[e * 4 + 1] * v[1];
                    acc = acc + R[e * 4 + 2] * v[2];
                    w[e] = acc + R[e * 4 + 3];
                }
                v[0] = w[0], v[1] = w[1], v[2] = w[2];
            }
#pragma unroll
            for (int e = 0; e < 3; ++e) out[i * 3 + e] = (float)((double)v[e] + nz[i * 3 + e]);
            ov[((int64_t)b * 2 + c) * m + i] = mask[(1 - c) * ntot + o + r];
            inv[c][r] = i;
        }
    }
    __syncthreads();
    int base = 0;
    for (int j0 = 0; j0 < n; j0 += kCropThreads) {
        const int j = j0 + tid;
        const int s = j < n ? inv[0][j] : -1, q = j < n ? inv[1][j] : -1;
        const int f = s >= 0 && q >= 0;
        int tot;
        const int pos = block_scan(f, sh, &tot);
        if (f) {
            corr[o + base + pos] = s;
            corr[ntot + o + base + pos] = q;
        }
        base += tot;
    }
    if (tid == 0) ncorr[b] = base;
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_crop_pairs_mask(const float* raw, int32_t ld, const int64_t* offsets,
                                   int32_t n_pairs, const double* dirs, const int32_t* crop_k,
                                   const double* gamma, uint8_t* mask, int32_t* keep,
                                   int32_t* count, void* stream) {
    FGR_REQUIRE(n_pairs > 0 && ld >= 3, "fgr_crop_pairs_mask: bad arguments");
    FGR_REQUIRE(raw && offsets && dirs && crop_k && gamma && mask && keep && count,
                "fgr_crop_pairs_mask: null pointer");
    TimedCall tc(as_stream(stream));
    hipLaunchKernelGGL(crop_mask_kernel, dim3((unsigned)n_pairs * 2), dim3(kCropThreads), 0,
                       as_stream(stream), raw, ld, offsets, dirs, crop_k, gamma, mask, keep,
                       count);
    FGR_CHECK_LAUNCH("crop_mask_kernel");
    return FGR_OK;
}

extern "C" int fgr_crop_pairs_assemble(const float* raw, int32_t ld, const int64_t* offsets,
                                       int32_t n_pairs, const uint8_t* mask, const int32_t* keep,
                                       const int32_t* sel, const double* noise, const float* rt,
                                       int32_t m, float* xyz, uint8_t* overlap, int64_t* corr,
                                       int32_t* n_corr, void* stream) {
    FGR_REQUIRE(n_pairs > 0 && ld >= 3 && m > 0, "fgr_crop_pairs_assemble: bad arguments");
    FGR_REQUIRE(raw && offsets && mask && keep && sel && noise && rt && xyz && overlap && corr &&
                    n_corr,
                "fgr_crop_pairs_assemble: null pointer");
    TimedCall tc(as_stream(stream));
    hipLaunchKernelGGL(crop_assemble_kernel, dim3((unsigned)n_pairs), dim3(kCropThreads), 0,
                       as_stream(stream), raw, ld, offsets, mask, keep, sel, noise, rt, m, xyz,
                       overlap, corr, n_corr);
    FGR_CHECK_LAUNCH("crop_assemble_kernel");
    return FGR_OK;
}

extern "C" int fgr_crop_max_points(int32_t* n_max) {
    FGR_REQUIRE(n_max, "fgr_crop_max_points: null pointer");
    *n_max = kCropMaxN;
    return FGR_OK;
}
