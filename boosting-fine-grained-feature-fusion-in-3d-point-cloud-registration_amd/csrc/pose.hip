// Weighted Procrustes (Kabsch) with a 3x3 Jacobi SVD, one block per problem.
//
// Restates fast_compute_rigid_transform (utils/se3_torch.py:226-273):
//   w <- w if w > threshold else 0                         (:240-242)
//   wn = w / max(sum w, 1e-6); ca = sum a wn; cb = sum b wn (:248-251)
//   H  = (a - ca)^T ((b - cb) wn)                          (:252-254)
//   U S V^T = svd(H); R = V U^T, or V diag(1,1,-1) U^T if det(V U^T) <= 0  (:264-269)
//   t  = -R ca + cb                                        (:272)
// Reductions and the SVD run in fp64 (one-sided Jacobi), results rounded to fp32.
// A zero covariance (all weights under the threshold) gives U = V = I -> R = I,
// which is what torch.svd returns for the zero matrix.
#include "common.h"

namespace fgr {
namespace {

constexpr int kPoseThreads = 256;

struct Sums {
    double w, a[3], b[3];
};

__device__ void block_reduce(double* vals, int n, double* sh) {
    // vals: per-thread partials (n <= 16); sh: [kPoseThreads/64][16]
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (int i = 0; i < n; ++i) {
        double v = vals[i];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) sh[wv * 16 + i] = v;
    }
    __syncthreads();
    for (int i = 0; i < n; ++i) {
        double t = 0.0;
        for (int w = 0; w < kPoseThreads / 64; ++w) t += sh[w * 16 + i];
        vals[i] = t;
    }
    __syncthreads();
}

__device__ void svd3_rotation(const double H[3][3], double R[3][3]) {
    // one-sided Jacobi: A = H V with orthogonal columns -> A = U S
    double A[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[i][j] = H[i][j];
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 2; ++p) {
            for (int qq = p + 1; qq < 3; ++qq) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < 3; ++i) {
                    al += A[i][p] * A[i][p];
                    be += A[i][qq] * A[i][qq];
                    ga += A[i][p] * A[i][qq];
                }
                if (fabs(ga) <= 1e-300 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
                off = fmax(off, fabs(ga) / sqrt(al * be));
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
                for (int i = 0; i < 3; ++i) {
                    const double x = A[i][p], y = A[i][qq];
                    A[i][p] = cs * x - sn * y;
                    A[i][qq] = sn * x + cs * y;
                    const double vx = V[i][p], vy = V[i][qq];
                    V[i][p] = cs * vx - sn * vy;
                    V[i][qq] = sn * vx + cs * vy;
                }
            }
        }
        if (off < 1e-15) break;
    }
    double sig[3], U[3][3];
    for (int j = 0; j < 3; ++j) sig[j] = sqrt(A[0][j] * A[0][j] + A[1][j] * A[1][j] + A[2][j] * A[2][j]);
    // sort singular values descending (permute columns of A and V)
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2 - i; ++j)
            if (sig[j] < sig[j + 1]) {
                double ts = sig[j]; sig[j] = sig[j + 1]; sig[j + 1] = ts;
                for (int r = 0; r < 3; ++r) {
                    double ta = A[r][j]; A[r][j] = A[r][j + 1]; A[r][j + 1] = ta;
                    double tv = V[r][j]; V[r][j] = V[r][j + 1]; V[r][j + 1] = tv;
                }
            }
    const double tiny = 1e-30 + 1e-13 * sig[0];
    int rank = 0;
    for (int j = 0; j < 3; ++j) {
        if (sig[j] > tiny) {
            for (int r = 0; r < 3; ++r) U[r][j] = A[r][j] / sig[j];
            ++rank;
        }
    }
    if (rank == 0) {
        for (int r = 0; r < 3; ++r)
            for (int j = 0; j < 3; ++j) U[r][j] = (r == j) ? 1.0 : 0.0;
    } else {
        if (rank == 1) {
            // any unit vector orthogonal to u0
            double e[3] = {0, 0, 0};
            int m = fabs(U[0][0]) < fabs(U[1][0]) ? (fabs(U[0][0]) < fabs(U[2][0]) ? 0 : 2)
                                                  : (fabs(U[1][0]) < fabs(U[2][0]) ? 1 : 2);
            e[m] = 1.0;
            double d = e[0] * U[0][0] + e[1] * U[1][0] + e[2] * U[2][0];
            double u1[3] = {e[0] - d * U[0][0], e[1] - d * U[1][0], e[2] - d * U[2][0]};
            double nn = sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
            for (int r = 0; r < 3; ++r) U[r][1] = u1[r] / nn;
        }
        if (rank <= 2) {
            U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
            U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
            U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
        }
    }
    // R = V U^T ; reflection fix flips V[:, 2]
    double Rp[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            Rp[i][j] = V[i][0] * U[j][0] + V[i][1] * U[j][1] + V[i][2] * U[j][2];
    const double det = Rp[0][0] * (Rp[1][1] * Rp[2][2] - Rp[1][2] * Rp[2][1]) -
                       Rp[0][1] * (Rp[1][0] * Rp[2][2] - Rp[1][2] * Rp[2][0]) +
                       Rp[0][2] * (Rp[1][0] * Rp[2][1] - Rp[1][1] * Rp[2][0]);
    const double f = det > 0 ? 1.0 : -1.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            R[i][j] = V[i][0] * U[j][0] + V[i][1] * U[j][1] + f * V[i][2] * U[j][2];
}

// Generic accessor-driven solver: point i of problem p -> (a, b, w).
template <class Get>
__device__ void solve(int64_t n, float threshold, Get get, float* out) {
    __shared__ double sh[(kPoseThreads / 64) * 16];
    double s[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = threadIdx.x; i < n; i += kPoseThreads) {
        float a[3], b[3], w;
        get(i, a, b, w);
        if (threshold >= 0.f && !(w > threshold)) w = 0.f;
        s[0] += w;
        for (int d = 0; d < 3; ++d) { s[1 + d] += (double)w * a[d]; s[4 + d] += (double)w * b[d]; }
    }
    block_reduce(s, 7, sh);
    const double W = fmax(s[0], 1e-6);
    double ca[3], cb[3];
    for (int d = 0; d < 3; ++d) { ca[d] = s[1 + d] / W; cb[d] = s[4 + d] / W; }
    double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = threadIdx.x; i < n; i += kPoseThreads) {
        float a[3], b[3], w;
        get(i, a, b, w);
        if (threshold >= 0.f && !(w > threshold)) w = 0.f;
        const double wn = (double)w / W;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) h[3 * r + c] += (a[r] - ca[r]) * ((b[c] - cb[c]) * wn);
    }
    block_reduce(h, 9, sh);
    if (threadIdx.x == 0) {
        double H[3][3], R[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) H[r][c] = h[3 * r + c];
        svd3_rotation(H, R);
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) out[4 * r + c] = (float)R[r][c];
            out[4 * r + 3] = (float)(-(R[r][0] * ca[0] + R[r][1] * ca[1] + R[r][2] * ca[2]) + cb[r]);
        }
    }
}

__global__ void __launch_bounds__(kPoseThreads)
procrustes_kernel(const float* __restrict__ a, const float* __restrict__ b,
                  const float* __restrict__ w, int64_t n_pts, float threshold,
                  float* __restrict__ out) {
    const int64_t p = blockIdx.x;
    const float* ap = a + p * n_pts * 3;
    const float* bp = b + p * n_pts * 3;
    const float* wp = w + p * n_pts;
    solve(n_pts, threshold,
          [&](int64_t i, float* av, float* bv, float& wv) {
              for (int d = 0; d < 3; ++d) { av[d] = ap[3 * i + d]; bv[d] = bp[3 * i + d]; }
              wv = wp[i];
          },
          out + p * 12);
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// grid = (n_pairs, n_layers)
__global__ void __launch_bounds__(kPoseThreads)
pair_pose_kernel(const float* __restrict__ xyz, const float* __restrict__ corr,
                 const float* __restrict__ logits, int64_t n_tot,
                 const int64_t* __restrict__ seg_off, int n_pairs, float threshold,
                 float* __restrict__ out) {
    const int pr = blockIdx.x, l = blockIdx.y;
    const int64_t sb = seg_off[pr], se = seg_off[pr + 1];
    const int64_t tb = seg_off[n_pairs + pr], te = seg_off[n_pairs + pr + 1];
    const int64_t ns = se - sb, nt = te - tb;
    const float* cl = corr + (int64_t)l * n_tot * 3;
    const float* lg = logits + (int64_t)l * n_tot;
    solve(ns + nt, threshold,
          [&](int64_t i, float* av, float* bv, float& wv) {
              if (i < ns) {            // [src_xyz | src_corr]
                  const int64_t r = sb + i;
                  for (int d = 0; d < 3; ++d) { av[d] = xyz[3 * r + d]; bv[d] = cl[3 * r + d]; }
                  wv = sigmoidf(lg[r]);
              } else {                 // [tgt_corr | tgt_xyz]
                  const int64_t r = tb + (i - ns);
                  for (int d = 0; d < 3; ++d) { av[d] = cl[3 * r + d]; bv[d] = xyz[3 * r + d]; }
                  wv = sigmoidf(lg[r]);
              }
          },
          out + ((int64_t)l * n_pairs + pr) * 12);
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_procrustes(const float* a, const float* b, const float* w, int64_t n_batch,
                              int64_t n_pts, float threshold, float* out, void* stream) {
    FGR_REQUIRE(n_batch >= 0 && n_pts >= 0, "fgr_procrustes: bad arguments");
    FGR_REQUIRE(n_batch == 0 || (a && b && w && out), "fgr_procrustes: null pointer");
    if (n_batch == 0) return FGR_OK;
    hipLaunchKernelGGL(procrustes_kernel, dim3((unsigned)n_batch), dim3(kPoseThreads), 0,
                       as_stream(stream), a, b, w, n_pts, threshold, out);
    FGR_CHECK_LAUNCH("procrustes_kernel");
    return FGR_OK;
}

extern "C" int fgr_pair_pose(const float* xyz, const float* corr, const float* logits,
                             int64_t n_tot, const int64_t* seg_off, int32_t n_pairs,
                             int32_t n_layers, float threshold, float* out, void* stream) {
    FGR_REQUIRE(n_pairs > 0 && n_layers > 0 && n_tot >= 0 && seg_off && xyz && corr && logits &&
                    out,
                "fgr_pair_pose: bad arguments");
    TimedCall timed_(as_stream(stream));
    hipLaunchKernelGGL(pair_pose_kernel, dim3((unsigned)n_pairs, (unsigned)n_layers),
                       dim3(kPoseThreads), 0, as_stream(stream), xyz, corr, logits, n_tot,
                       seg_off, n_pairs, threshold, out);
    FGR_CHECK_LAUNCH("pair_pose_kernel");
    return FGR_OK;
}
