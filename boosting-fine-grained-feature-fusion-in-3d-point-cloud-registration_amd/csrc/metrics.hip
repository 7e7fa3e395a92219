// The ModelNet evaluation metrics of the reference's test step (benchmark/benchmark_modelnet.py:
// 33-82 compute_metrics, called by models/generic_reg_model.py:138-147 on the last layer's pose)
// for a batch of pairs, on the GPU:
//
//   * DCP Euler errors: r_mse / r_mae of the 'xyz' (extrinsic) Euler angles in degrees of the
//     ground-truth and predicted rotations (scipy Rotation.from_matrix(R).as_euler('xyz')),
//     t_mse / t_mae of the translations;
//   * isotropic errors: err_r_deg = acos(clamp((tr(R_gt^T R_pred) - 1) / 2)) in degrees,
//     err_t = |t of se3_cat(se3_inv(gt), pred)| (fp32, as the reference);
//   * the modified Chamfer distance: mean over the src points of min_raw |pred(src) - raw|^2
//     plus mean over the ref points of min_raw |ref - (pred o gt^-1)(raw)|^2 (points_raw = the
//     clean reference cloud before cropping).
//
// Two launches: mn_chamfer_kernel (one thread per query point and direction, the candidate cloud
// staged through LDS 2048 points at a time -- an N x M row-min, bound by LDS reads) writes every
// query's squared distance; mn_pair_kernel (one block per pair) reduces them in a fixed order and
// forms the pose metrics in fp64. scipy's from_matrix orthogonalises its input (the polar factor
// U V^T of the SVD, scipy 1.15) before as_euler: restated as Newton's polar iteration
// X <- (X + X^-T) / 2 in fp64 (quadratic convergence from a nearly orthogonal fp32 matrix),
// then the extrinsic-xyz angles of the orthogonal matrix, alpha = atan2(M21, M22),
// beta = -asin(M20), gamma = atan2(M10, M00) (equal to scipy's quaternion algorithm to ~1e-12
// degrees away from gimbal lock, |beta| = 90 degrees, where the two pick different splits of
// alpha / gamma).
#include "common.h"

namespace fgr {
namespace {

constexpr int kMnChunk = 2048;          // candidate points per LDS stage (24 KB)

// x -> R x + t with R, t of a (3, 4) pose (fp32, no contraction: as the reference's einsum +
// add, each component a three-term sum)
__device__ __forceinline__ void apply_pose(const float* P, float x, float y, float z, float& ox,
                                           float& oy, float& oz) {
    ox = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(P[0], x), __fmul_rn(P[1], y)), __fmul_rn(P[2], z)), P[3]);
    oy = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(P[4], x), __fmul_rn(P[5], y)), __fmul_rn(P[6], z)), P[7]);
    oz = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(P[8], x), __fmul_rn(P[9], y)), __fmul_rn(P[10], z)), P[11]);
}

// C = se3_cat(A, se3_inv(B)) = (R_A R_B^T, t_A - R_A R_B^T t_B), fp32
__device__ void cat_inv(const float* A, const float* B, float* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[4 * i + j] = __fadd_rn(__fadd_rn(__fmul_rn(A[4 * i + 0], B[4 * j + 0]),
                                               __fmul_rn(A[4 * i + 1], B[4 * j + 1])),
                                     __fmul_rn(A[4 * i + 2], B[4 * j + 2]));
    for (int i = 0; i < 3; ++i)
        C[4 * i + 3] = __fsub_rn(A[4 * i + 3],
                                 __fadd_rn(__fadd_rn(__fmul_rn(C[4 * i + 0], B[3]), __fmul_rn(C[4 * i + 1], B[7])),
                                           __fmul_rn(C[4 * i + 2], B[11])));
}

// grid (ceil(n_pts / 256), 2, n_pairs): direction 0 = src queries pred(src) against raw, 1 = ref
// queries against (pred o gt^-1)(raw)
__global__ void __launch_bounds__(256)
mn_chamfer_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                  const float* __restrict__ src, const float* __restrict__ ref,
                  const float* __restrict__ raw, int n_pts, int n_raw, float* __restrict__ dmin) {
    __shared__ float cx[kMnChunk], cy[kMnChunk], cz[kMnChunk];
    __shared__ float T[12];
    const int b = blockIdx.z, dir = blockIdx.y, tid = threadIdx.x;
    const int i = blockIdx.x * 256 + tid;
    const float* Pp = pred + 12 * b;
    if (tid == 0) {
        if (dir == 1) cat_inv(Pp, gt + 12 * b, T);
        else
            for (int e = 0; e < 12; ++e) T[e] = Pp[e];
    }
    __syncthreads();
    float qx = 0.f, qy = 0.f, qz = 0.f;
    const int ii = min(i, n_pts - 1);
    if (dir == 0) {
        const float* s = src + ((int64_t)b * n_pts + ii) * 3;
        apply_pose(T, s[0], s[1], s[2], qx, qy, qz);
    } else {
        const float* s = ref + ((int64_t)b * n_pts + ii) * 3;
        qx = s[0]; qy = s[1]; qz = s[2];
    }
    float best = INFINITY;
    const float* rb = raw + (int64_t)b * n_raw * 3;
    for (int c0 = 0; c0 < n_raw; c0 += kMnChunk) {
        const int nc = min(kMnChunk, n_raw - c0);
        __syncthreads();
        for (int j = tid; j < nc; j += 256) {
            const float* r = rb + (int64_t)(c0 + j) * 3;
            float x = r[0], y = r[1], z = r[2];
            if (dir == 1) apply_pose(T, r[0], r[1], r[2], x, y, z);
            cx[j] = x; cy[j] = y; cz[j] = z;
        }
        __syncthreads();
        for (int j = 0; j < nc; ++j) {
            const float dx = __fsub_rn(qx, cx[j]), dy = __fsub_rn(qy, cy[j]), dz = __fsub_rn(qz, cz[j]);
            const float d = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
            best = fminf(best, d);
        }
    }
    if (i < n_pts) dmin[((int64_t)b * 2 + dir) * n_pts + i] = best;
}

// orthogonal polar factor of a 3 x 3 matrix (fp64 Newton iteration X <- (X + X^-T) / 2)
__device__ void polar3(double (&X)[3][3]) {
    for (int it = 0; it < 40; ++it) {
        const double c00 = X[1][1] * X[2][2] - X[1][2] * X[2][1];
        const double c01 = X[1][2] * X[2][0] - X[1][0] * X[2][2];
        const double c02 = X[1][0] * X[2][1] - X[1][1] * X[2][0];
        const double c10 = X[0][2] * X[2][1] - X[0][1] * X[2][2];
        const double c11 = X[0][0] * X[2][2] - X[0][2] * X[2][0];
        const double c12 = X[0][1] * X[2][0] - X[0][0] * X[2][1];
        const double c20 = X[0][1] * X[1][2] - X[0][2] * X[1][1];
        const double c21 = X[0][2] * X[1][0] - X[0][0] * X[1][2];
        const double c22 = X[0][0] * X[1][1] - X[0][1] * X[1][0];
        const double det = X[0][0] * c00 + X[0][1] * c01 + X[0][2] * c02;
        if (det == 0.0) return;
        // X^-T = cofactor matrix / det
        const double C[3][3] = {{c00, c01, c02}, {c10, c11, c12}, {c20, c21, c22}};
        double delta = 0.0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                const double nv = 0.5 * (X[i][j] + C[i][j] / det);
                delta = fmax(delta, fabs(nv - X[i][j]));
                X[i][j] = nv;
            }
        if (delta < 1e-16) return;
    }
}

__device__ void euler_xyz_deg(const float* P, double (&e)[3]) {
    double X[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) X[i][j] = (double)P[4 * i + j];
    polar3(X);
    const double r2d = 180.0 / 3.14159265358979323846;
    e[0] = atan2(X[2][1], X[2][2]) * r2d;
    e[1] = -asin(fmin(fmax(X[2][0], -1.0), 1.0)) * r2d;
    e[2] = atan2(X[1][0], X[0][0]) * r2d;
}

// one block per pair: out[b] = {r_mse, r_mae, t_mse, t_mae, err_r_deg, err_t, chamfer_dist}
__global__ void __launch_bounds__(256)
mn_pair_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
               const float* __restrict__ dmin, int n_pts, double* __restrict__ out) {
    __shared__ float red[2][256];
    const int b = blockIdx.x, tid = threadIdx.x;
    for (int dir = 0; dir < 2; ++dir) {
        const float* d = dmin + ((int64_t)b * 2 + dir) * n_pts;
        float s = 0.f;
        for (int i = tid; i < n_pts; i += 256) s += d[i];
        red[dir][tid] = s;
    }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) {
            red[0][tid] += red[0][tid + w];
            red[1][tid] += red[1][tid + w];
        }
        __syncthreads();
    }
    if (tid != 0) return;
    const float* Pp = pred + 12 * b;
    const float* Pg = gt + 12 * b;
    double eg[3], ep[3];
    euler_xyz_deg(Pg, eg);
    euler_xyz_deg(Pp, ep);
    double r_mse = 0.0, r_mae = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double dd = eg[k] - ep[k];
        r_mse += dd * dd;
        r_mae += fabs(dd);
    }
    float t_mse = 0.f, t_mae = 0.f;
    for (int k = 0; k < 3; ++k) {
        const float dt = __fsub_rn(Pg[4 * k + 3], Pp[4 * k + 3]);
        t_mse = __fadd_rn(t_mse, __fmul_rn(dt, dt));
        t_mae = __fadd_rn(t_mae, fabsf(dt));
    }
    // se3_cat(se3_inv(gt), pred) in fp32 as the reference (se3_torch.py:32-48): irot = Rg^T,
    // itrans = -irot tg, rot = irot Rp, trans = irot tp + itrans (near a zero error the
    // isotropic angle is acos of a value within fp32 rounding of 1: the reference's own fp32
    // value, not an fp64 one, is the metric)
    float rt[3], it[3], tr3[3];
    for (int i = 0; i < 3; ++i) {
        rt[i] = __fadd_rn(__fadd_rn(__fmul_rn(Pg[0 + i], Pp[0 + i]), __fmul_rn(Pg[4 + i], Pp[4 + i])),
                          __fmul_rn(Pg[8 + i], Pp[8 + i]));                       // rot[i][i]
        it[i] = -__fadd_rn(__fadd_rn(__fmul_rn(Pg[0 + i], Pg[3]), __fmul_rn(Pg[4 + i], Pg[7])),
                           __fmul_rn(Pg[8 + i], Pg[11]));
        tr3[i] = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(Pg[0 + i], Pp[3]), __fmul_rn(Pg[4 + i], Pp[7])),
                                     __fmul_rn(Pg[8 + i], Pp[11])), it[i]);
    }
    const float trace = __fadd_rn(__fadd_rn(rt[0], rt[1]), rt[2]);
    const float cth = fminf(fmaxf(__fmul_rn(0.5f, __fsub_rn(trace, 1.0f)), -1.0f), 1.0f);
    double* o = out + 7 * b;
    o[0] = r_mse / 3.0;
    o[1] = r_mae / 3.0;
    o[2] = (double)t_mse / 3.0;
    o[3] = (double)t_mae / 3.0;
    o[4] = (double)(acosf(cth) * 180.0f / 3.14159265358979323846f);
    o[5] = (double)sqrtf(__fadd_rn(__fadd_rn(__fmul_rn(tr3[0], tr3[0]), __fmul_rn(tr3[1], tr3[1])),
                                   __fmul_rn(tr3[2], tr3[2])));
    o[6] = (double)red[0][0] / n_pts + (double)red[1][0] / n_pts;
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_modelnet_metrics_workspace(int32_t n_pairs, int32_t n_pts, size_t* bytes) {
    FGR_REQUIRE(bytes && n_pairs >= 0 && n_pts >= 0, "fgr_modelnet_metrics_workspace: bad arguments");
    *bytes = (size_t)n_pairs * 2 * n_pts * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_modelnet_metrics(const float* pred, const float* gt, const float* src,
                                    const float* ref, const float* raw, int32_t n_pairs,
                                    int32_t n_pts, int32_t n_raw, void* ws, size_t ws_bytes,
                                    double* out, void* stream) {
    FGR_REQUIRE(pred && gt && src && ref && raw && out && ws && n_pairs > 0 && n_pts > 0 &&
                    n_raw > 0,
                "fgr_modelnet_metrics: bad arguments");
    size_t need = 0;
    fgr_modelnet_metrics_workspace(n_pairs, n_pts, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_modelnet_metrics: workspace %zu < %zu bytes", ws_bytes, need);
    FGR_REQUIRE(n_pairs <= 65535, "fgr_modelnet_metrics: at most 65535 pairs per call");
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    float* dmin = static_cast<float*>(ws);
    hipLaunchKernelGGL(mn_chamfer_kernel, dim3((unsigned)ceil_div(n_pts, 256), 2u, (unsigned)n_pairs),
                       dim3(256), 0, st, pred, gt, src, ref, raw, n_pts, n_raw, dmin);
    FGR_CHECK_LAUNCH("mn_chamfer_kernel");
    hipLaunchKernelGGL(mn_pair_kernel, dim3((unsigned)n_pairs), dim3(256), 0, st, pred, gt,
                       (const float*)dmin, n_pts, out);
    FGR_CHECK_LAUNCH("mn_pair_kernel");
    return FGR_OK;
}
