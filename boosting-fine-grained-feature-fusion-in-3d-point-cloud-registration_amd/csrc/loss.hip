// Test-step tail of the reference on gfx950: what
// GenericRegModel.test_step runs after the forward (generic_reg_model.py:128-132).
//   compute_overlaps      finegrained_kpconv.py:545-571    fgr_overlap_pool
//   overlap loss          finegrained_regtr.py:264-267     fgr_bce_logits_mean
//   se3_transform_list    utils/se3_torch.py:70-90         fgr_transform_points
//   InfoNCELossFull       losses/feature_loss.py:268-314   (GEMMs) + fgr_infonce_rows/_reduce
//   CircleLossFull        losses/feature_loss.py:160-243   fgr_circle_loss (feature_loss_type
//                         circle, finegrained_regtr.py:86-88: Euclidean feature distances)
//   CorrCriterion (mae)   losses/corr_loss.py:18-38         fgr_corr_loss
//   se3_compare           utils/se3_torch.py:117-129        fgr_se3_compare
// All reductions are deterministic (fixed lane / wave / block order).
#include "common.h"

namespace fgr {
namespace {

constexpr int kRed = 1024;    // threads of the single-block reductions

// Block-wide sums of N values, deterministic: DPP wave sums, then wave 0's lanes in order.
template <int N>
__device__ __forceinline__ void block_sum(float (&v)[N]) {
    __shared__ float sh[N][kRed / 64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = wave_sum_dpp(v[i]);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) sh[i][wv] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        float t = 0.f;
        for (int w = 0; w < nw; ++w) t += sh[i][w];
        v[i] = t;
    }
    __syncthreads();
}

// compute_overlaps, one pyramid step (finegrained_kpconv.py:560-569): mean of the previous
// level's overlap over the pool entries with idx < n_prev, clamped to [0, 1]. A row with no
// valid entry gives 0 / 0 = NaN, and torch.clamp passes NaN through: so do we.
__global__ void overlap_pool_kernel(const float* __restrict__ prev, int64_t n_prev,
                                    const int64_t* __restrict__ idx, int64_t nq, int width,
                                    float* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const int64_t* row = idx + q * width;
    float s = 0.f, cnt = 0.f;
    for (int h = 0; h < width; ++h) {
        const int64_t id = row[h];
        if (id < n_prev && id >= -n_prev) {           // torch indexing wraps negative ids
            s += prev[id < 0 ? id + n_prev : id];
            cnt += 1.f;
        }
    }
    const float v = s / cnt;
    out[q] = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
}

// nn.BCEWithLogitsLoss (mean): (1 - y) x - log_sigmoid(x), log_sigmoid(x) =
// min(x, 0) - log1p(exp(-|x|)) (ATen's form). One block.
__global__ void __launch_bounds__(kRed)
bce_logits_mean_kernel(const float* __restrict__ x, int64_t sx, const float* __restrict__ y,
                       int64_t n, float* __restrict__ out) {
    float v[1] = {0.f};
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float xi = x[i * sx], yi = y[i];
        const float ls = fminf(xi, 0.f) - log1pf(expf(-fabsf(xi)));
        v[0] += (1.f - yi) * xi - ls;
    }
    block_sum<1>(v);
    if (threadIdx.x == 0) out[0] = v[0] / (float)n;
}

__device__ __forceinline__ void load_pose(const float* __restrict__ pose, bool inverse,
                                          float (&R)[3][3], float (&t)[3]) {
    float P[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) P[i][j] = pose[4 * i + j];
    if (!inverse) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) R[i][j] = P[i][j];
            t[i] = P[i][3];
        }
    } else {                                          // se3_inv: R^T, -(R^T t)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) R[i][j] = P[j][i];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i)
            t[i] = -fmaf(R[i][2], P[2][3], fmaf(R[i][1], P[1][3], R[i][0] * P[0][3]));
    }
}

__device__ __forceinline__ void apply_pose(const float (&R)[3][3], const float (&t)[3], float x,
                                           float y, float z, float (&o)[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = fmaf(R[i][2], z, fmaf(R[i][1], y, R[i][0] * x)) + t[i];
}

// se3_transform_list over packed segments: rows of segment s get pose[s] (or its inverse).
__global__ void transform_points_kernel(const float* __restrict__ xyz, int64_t n,
                                        const int64_t* __restrict__ seg_off, int n_seg,
                                        const float* __restrict__ pose, int inverse,
                                        float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int s = find_segment(seg_off, n_seg, r);
    float R[3][3], t[3], o[3];
    load_pose(pose + 12 * s, inverse != 0, R, t);
    apply_pose(R, t, xyz[3 * r], xyz[3 * r + 1], xyz[3 * r + 2], o);
    out[3 * r] = o[0];
    out[3 * r + 1] = o[1];
    out[3 * r + 2] = o[2];
}

// torch.cdist's matrix-multiply form (used for > 25 rows): sqrt(max(x.x2 - 2 x.y + y.y, 1e-30))
// with the 5-term dot [-2x, |x|^2, 1] . [y, 1, |y|^2] accumulated in that order.
__device__ __forceinline__ float cdist_mm(float ax, float ay, float az, float a2,
                                          const float* __restrict__ p) {
    const float px = p[0], py = p[1], pz = p[2];
    const float p2 = (px * px + py * py) + pz * pz;
    float t = (-2.f * ax) * px;
    t = fmaf(-2.f * ay, py, t);
    t = fmaf(-2.f * az, pz, t);
    t = t + a2;
    t = t + p2;
    return sqrtf(fmaxf(t, 1e-30f));
}

// InfoNCE per anchor row i of pair b (feature_loss.py:280-294), one wave per row, given the
// match logits row (already A W_sym P^T): the positive is the nearest point of the pair's
// positive cloud (lowest index on ties), mask = its distance < r_p, every other point
// closer than r_n is ignored (-inf), loss_i = logsumexp(row) - logit(positive).
__global__ void __launch_bounds__(256)
infonce_rows_kernel(const float* __restrict__ logits, int64_t ld, const float* __restrict__ axyz,
                    const float* __restrict__ pxyz, const int64_t* __restrict__ a_off,
                    const int64_t* __restrict__ p_off, int n_pairs, int64_t n_anchor, float r_p,
                    float r_n, float* __restrict__ row_loss, float* __restrict__ row_mask) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n_anchor) return;                            // wave-uniform
    const int b = find_segment(a_off, n_pairs, i);
    const int p0 = (int)p_off[b], p1 = (int)p_off[b + 1];
    if (p1 <= p0) {
        if (lane == 0) { row_loss[i] = __builtin_nanf(""); row_mask[i] = 0.f; }
        return;
    }
    const float ax = axyz[3 * i], ay = axyz[3 * i + 1], az = axyz[3 * i + 2];
    const float a2 = (ax * ax + ay * ay) + az * az;
    float best = INFINITY;
    int bj = p1;
    for (int j = p0 + lane; j < p1; j += 64) {
        const float d = cdist_mm(ax, ay, az, a2, pxyz + 3 * (int64_t)j);
        if (d < best) { best = d; bj = j; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oj = __shfl_xor(bj, o, 64);
        if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
    }
    if (bj >= p1) bj = p0;                                // all distances NaN: keep in range
    const float* lrow = logits + i * ld;
    float m = -INFINITY, s = 0.f;
    for (int j = p0 + lane; j < p1; j += 64) {
        const float d = cdist_mm(ax, ay, az, a2, pxyz + 3 * (int64_t)j);
        if (d < r_n && j != bj) continue;                 // ignored: exp(-inf) = 0
        const float l = lrow[j];
        if (l > m) { s = s * expf(m - l) + 1.f; m = l; }
        else s += expf(l - m);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
        const float M = fmaxf(m, om);
        const float a = m == -INFINITY ? 0.f : s * expf(m - M);
        const float c = om == -INFINITY ? 0.f : os * expf(om - M);
        s = a + c;
        m = M;
    }
    if (lane == 0) {
        row_loss[i] = -lrow[bj] + (m + logf(s));
        row_mask[i] = best < r_p ? 1.f : 0.f;
    }
}

// Backward of infonce_rows_kernel + the reduce (training: loss.backward() through
// InfoNCELossFull, feature_loss.py:268-314): for anchor row i of pair b with weight
// w_i = row_mask_i / (K_b n_pairs) (K_b = the pair's kept rows) and upstream gradient g,
//   dlogits[i][j] = g w_i (softmax_ij - [j == positive])  over the pair's non-ignored columns,
// 0 on ignored columns and on every column of the other pairs (the logits span all pairs).
// The positive, the ignore mask and the log-sum-exp are recomputed exactly as the forward.
__global__ void __launch_bounds__(256)
infonce_rows_bwd_kernel(const float* __restrict__ logits, int64_t ld, const float* __restrict__ axyz,
                        const float* __restrict__ pxyz, const int64_t* __restrict__ a_off,
                        const int64_t* __restrict__ p_off, int n_pairs, int64_t n_anchor,
                        int64_t n_cols, float r_n, const float* __restrict__ w,
                        const float* __restrict__ g, float* __restrict__ dl, int64_t ldd) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n_anchor) return;                            // wave-uniform
    const int b = find_segment(a_off, n_pairs, i);
    const int p0 = (int)p_off[b], p1 = (int)p_off[b + 1];
    float* drow = dl + i * ldd;
    const float wi = w[i] * g[0];
    // columns outside the pair's block, and every column of an unkept row: 0
    for (int64_t j = lane; j < n_cols; j += 64)
        if (j < p0 || j >= p1 || wi == 0.f) drow[j] = 0.f;
    if (p1 <= p0 || wi == 0.f) return;
    const float ax = axyz[3 * i], ay = axyz[3 * i + 1], az = axyz[3 * i + 2];
    const float a2 = (ax * ax + ay * ay) + az * az;
    float best = INFINITY;
    int bj = p1;
    for (int j = p0 + lane; j < p1; j += 64) {
        const float d = cdist_mm(ax, ay, az, a2, pxyz + 3 * (int64_t)j);
        if (d < best) { best = d; bj = j; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oj = __shfl_xor(bj, o, 64);
        if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
    }
    if (bj >= p1) bj = p0;
    const float* lrow = logits + i * ld;
    float m = -INFINITY, s = 0.f;
    for (int j = p0 + lane; j < p1; j += 64) {
        const float d = cdist_mm(ax, ay, az, a2, pxyz + 3 * (int64_t)j);
        if (d < r_n && j != bj) continue;
        const float l = lrow[j];
        if (l > m) { s = s * expf(m - l) + 1.f; m = l; }
        else s += expf(l - m);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
        const float M = fmaxf(m, om);
        const float a = m == -INFINITY ? 0.f : s * expf(m - M);
        const float c = om == -INFINITY ? 0.f : os * expf(om - M);
        s = a + c;
        m = M;
    }
    const float lse = m + logf(s);
    for (int j = p0 + lane; j < p1; j += 64) {
        const float d = cdist_mm(ax, ay, az, a2, pxyz + 3 * (int64_t)j);
        float v = 0.f;
        if (!(d < r_n && j != bj)) v = wi * (expf(lrow[j] - lse) - (j == bj ? 1.f : 0.f));
        drow[j] = v;
    }
}

// sum(loss[mask]) / sum(mask) per pair, then the mean over pairs (feature_loss.py:295, 314).
__global__ void __launch_bounds__(kRed)
infonce_reduce_kernel(const float* __restrict__ row_loss, const float* __restrict__ row_mask,
                      const int64_t* __restrict__ a_off, int n_pairs, float* __restrict__ out) {
    float total = 0.f;
    for (int b = 0; b < n_pairs; ++b) {
        float v[2] = {0.f, 0.f};
        for (int64_t i = a_off[b] + threadIdx.x; i < a_off[b + 1]; i += blockDim.x) {
            const bool mk = row_mask[i] != 0.f;
            v[0] += mk ? row_loss[i] : 0.f;
            v[1] += mk ? 1.f : 0.f;
        }
        block_sum<2>(v);
        total += v[0] / v[1];
    }
    if (threadIdx.x == 0) out[0] = total / (float)n_pairs;
}

// ---- CircleLossFull (feature_loss.py:160-243, Euclidean feature distances) ----------------
// Per pair b: fd[i][j] = sqrt(sum_k (a_ik - p_jk)^2 + 1e-12) (cdist 'euclidean', :34-36),
// cd[i][j] = torch.cdist of the points (its matrix-multiply form, cdist_mm); positives
// cd < r_p, negatives cd > r_n. The reference masks by shifting fd by -/+1e5 and multiplying
// by a clamped weight that is 0 on the masked entries, so a non-positive (non-negative) entry
// contributes exp(0) = 1 to the positive (negative) log-sum-exp:
//   tp = pos ? 10 (fd - 0.1) max(fd - 0.1, 0) : 0,  tn = neg ? 10 (1.4 - fd) max(1.4 - fd, 0) : 0
//   line loss = softplus(lse(tp) + lse(tn)) / 10 over each row (and each column),
// averaged over the rows (columns) that hold a positive and a negative; pair loss = (row mean
// + column mean) / 2, the call's loss the mean over pairs. Three launches: fd tiles, one wave
// per row / column, one reduction block; every sum in a fixed order.
constexpr float kCircleScale = 10.f, kCirclePos = 0.1f, kCircleNeg = 1.4f;
constexpr int kCdTile = 16, kCdChunk = 64;

// fd of pair b in 16 x 16 tiles, features staged through LDS 64 at a time (rows padded by one
// float: the 16 positive rows of a k step sit in distinct banks); packed per pair at fd_off[b]
__global__ void __launch_bounds__(256)
circle_fd_kernel(const float* __restrict__ af, const float* __restrict__ pf, int d,
                 const int64_t* __restrict__ a_off, const int64_t* __restrict__ p_off,
                 const int64_t* __restrict__ fd_off, float* __restrict__ fd) {
    __shared__ float as[kCdTile][kCdChunk + 1], ps[kCdTile][kCdChunk + 1];
    const int b = blockIdx.z;
    const int64_t a0 = a_off[b], p0 = p_off[b];
    const int na = (int)(a_off[b + 1] - a0), np = (int)(p_off[b + 1] - p0);
    const int i0 = blockIdx.y * kCdTile, j0 = blockIdx.x * kCdTile;
    if (i0 >= na || j0 >= np) return;                      // block-uniform
    const int t = threadIdx.x, ti = t / kCdTile, tj = t % kCdTile;
    float acc = 0.f;
    for (int k0 = 0; k0 < d; k0 += kCdChunk) {
#pragma unroll
        for (int u = 0; u < kCdTile * kCdChunk / 256; ++u) {
            const int e = t + 256 * u, r = e / kCdChunk, k = e % kCdChunk;
            const bool kin = k0 + k < d;
            as[r][k] = (kin && i0 + r < na) ? af[(a0 + i0 + r) * d + k0 + k] : 0.f;
            ps[r][k] = (kin && j0 + r < np) ? pf[(p0 + j0 + r) * d + k0 + k] : 0.f;
        }
        __syncthreads();
#pragma unroll 16
        for (int k = 0; k < kCdChunk; ++k) {
            const float df = as[ti][k] - ps[tj][k];
            acc = fmaf(df, df, acc);
        }
        __syncthreads();
    }
    if (i0 + ti < na && j0 + tj < np)
        fd[fd_off[b] + (int64_t)(i0 + ti) * np + j0 + tj] = sqrtf(acc + 1e-12f);
}

__device__ __forceinline__ void lse_push(float& m, float& s, float x) {
    if (x > m) { s = s * expf(m - x) + 1.f; m = x; }
    else s += expf(x - m);
}
__device__ __forceinline__ void lse_wave(float& m, float& s) {      // fixed butterfly order
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
        const float M = fmaxf(m, om);
        const float x = m == -INFINITY ? 0.f : s * expf(m - M);
        const float y = om == -INFINITY ? 0.f : os * expf(om - M);
        s = x + y;
        m = M;
    }
}
__device__ __forceinline__ float softplus_t(float x) {               // F.softplus, threshold 20
    return x > 20.f ? x : log1pf(expf(x));
}

// one wave per line: waves [0, n_anchor) are the anchor rows, then one per positive column
__global__ void __launch_bounds__(256)
circle_lines_kernel(const float* __restrict__ fd, const float* __restrict__ axyz,
                    const float* __restrict__ pxyz, const int64_t* __restrict__ a_off,
                    const int64_t* __restrict__ p_off, const int64_t* __restrict__ fd_off,
                    int n_pairs, int64_t n_anchor, int64_t n_pos, float r_p, float r_n,
                    float* __restrict__ line_loss, float* __restrict__ line_sel) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= n_anchor + n_pos) return;                     // wave-uniform
    const bool row = w < n_anchor;
    const int64_t r = row ? w : w - n_anchor;
    const int b = find_segment(row ? a_off : p_off, n_pairs, r);
    const int64_t a0 = a_off[b], p0 = p_off[b];
    const int na = (int)(a_off[b + 1] - a0), np = (int)(p_off[b + 1] - p0);
    const int me = (int)(r - (row ? a0 : p0));              // this line's index in the pair
    const int n_other = row ? np : na;
    const float* base = fd + fd_off[b];
    float mp = -INFINITY, sp = 0.f, mn = -INFINITY, sn = 0.f;
    bool anyp = false, anyn = false;
    for (int o = lane; o < n_other; o += 64) {
        const int i = row ? me : o, j = row ? o : me;
        const float* av = axyz + 3 * (a0 + i);
        const float ax = av[0], ay = av[1], az = av[2];
        const float cd = cdist_mm(ax, ay, az, (ax * ax + ay * ay) + az * az, pxyz + 3 * (p0 + j));
        const float f = base[(int64_t)i * np + j];
        const bool pos = cd < r_p, neg = cd > r_n;
        anyp |= pos;
        anyn |= neg;
        lse_push(mp, sp, pos ? kCircleScale * (f - kCirclePos) * fmaxf(f - kCirclePos, 0.f) : 0.f);
        lse_push(mn, sn, neg ? kCircleScale * (kCircleNeg - f) * fmaxf(kCircleNeg - f, 0.f) : 0.f);
    }
    lse_wave(mp, sp);
    lse_wave(mn, sn);
    const bool sel = __any(anyp) && __any(anyn);
    if (lane == 0) {
        line_loss[w] = n_other > 0 ? softplus_t((mp + logf(sp)) + (mn + logf(sn))) / kCircleScale
                                   : __builtin_nanf("");
        line_sel[w] = sel ? 1.f : 0.f;
    }
}

// per pair: (mean of the selected rows + mean of the selected columns) / 2 (0 / 0 = NaN for a
// pair without one, as torch's mean of an empty selection), then the mean over the pairs
__global__ void __launch_bounds__(kRed)
circle_reduce_kernel(const float* __restrict__ line_loss, const float* __restrict__ line_sel,
                     const int64_t* __restrict__ a_off, const int64_t* __restrict__ p_off,
                     int n_pairs, float* __restrict__ out) {
    const int64_t n_anchor = a_off[n_pairs];
    float total = 0.f;
    for (int b = 0; b < n_pairs; ++b) {
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        for (int64_t i = a_off[b] + threadIdx.x; i < a_off[b + 1]; i += blockDim.x) {
            const bool sl = line_sel[i] != 0.f;
            v[0] += sl ? line_loss[i] : 0.f;
            v[1] += sl ? 1.f : 0.f;
        }
        for (int64_t j = p_off[b] + threadIdx.x; j < p_off[b + 1]; j += blockDim.x) {
            const bool sl = line_sel[n_anchor + j] != 0.f;
            v[2] += sl ? line_loss[n_anchor + j] : 0.f;
            v[3] += sl ? 1.f : 0.f;
        }
        block_sum<4>(v);
        total += (v[0] / v[1] + v[2] / v[3]) / 2.f;
    }
    if (threadIdx.x == 0) out[0] = total / (float)n_pairs;
}

// CorrCriterion('mae') for both directions of finegrained_regtr.py:283-296: rows of cloud
// c < B are compared with pose[c] applied to the coarse point, rows of tgt cloud c with
// se3_inv(pose[c - B]); err = |dx| + |dy| + |dz|; each direction is an overlap-weighted mean
// over ALL its rows (the reference concatenates the pairs), the two are added.
__global__ void __launch_bounds__(kRed)
corr_loss_kernel(const float* __restrict__ xyz, const float* __restrict__ corr,
                 const float* __restrict__ w, const int64_t* __restrict__ seg_off, int n_pairs,
                 const float* __restrict__ pose, float* __restrict__ out) {
    const int64_t n = seg_off[2 * n_pairs];
    float v[4] = {0.f, 0.f, 0.f, 0.f};                    // num_s, den_s, num_t, den_t
    for (int64_t r = threadIdx.x; r < n; r += blockDim.x) {
        const int c = find_segment(seg_off, 2 * n_pairs, r);
        const bool tgt = c >= n_pairs;
        float R[3][3], t[3], g[3];
        load_pose(pose + 12 * (tgt ? c - n_pairs : c), tgt, R, t);
        apply_pose(R, t, xyz[3 * r], xyz[3 * r + 1], xyz[3 * r + 2], g);
        const float err = (fabsf(corr[3 * r] - g[0]) + fabsf(corr[3 * r + 1] - g[1])) +
                          fabsf(corr[3 * r + 2] - g[2]);
        const float wr = w[r];
        v[tgt ? 2 : 0] += wr * err;
        v[tgt ? 3 : 1] += wr;
    }
    block_sum<4>(v);
    if (threadIdx.x == 0)
        out[0] = v[0] / fmaxf(v[1], 1e-6f) + v[2] / fmaxf(v[3], 1e-6f);
}

// se3_compare(pred[l, b], gt[b]): combined = pred . inv(gt); rotation error in degrees from
// its trace, translation error = |combined translation|.
__global__ void se3_compare_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                   int n_layers, int n_pairs, float* __restrict__ rot_deg,
                                   float* __restrict__ trans) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_layers * n_pairs) return;
    const int b = u % n_pairs;
    float Rg[3][3], tg[3], Rp[3][3], tp[3];
    load_pose(gt + 12 * b, true, Rg, tg);                 // inv(gt)
    load_pose(pred + 12 * u, false, Rp, tp);
    float C[3][3], ct[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
            C[i][j] = fmaf(Rp[i][2], Rg[2][j], fmaf(Rp[i][1], Rg[1][j], Rp[i][0] * Rg[0][j]));
        ct[i] = fmaf(Rp[i][2], tg[2], fmaf(Rp[i][1], tg[1], Rp[i][0] * tg[0])) + tp[i];
    }
    const float trace = (C[0][0] + C[1][1]) + C[2][2];
    const float cosv = fminf(fmaxf(0.5f * (trace - 1.f), -1.f), 1.f);
    rot_deg[u] = (acosf(cosv) * 180.f) / 3.14159265358979323846f;
    trans[u] = sqrtf((ct[0] * ct[0] + ct[1] * ct[1]) + ct[2] * ct[2]);
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_overlap_pool(const float* prev, int64_t n_prev, const int64_t* idx, int64_t nq,
                                int32_t width, float* out, void* stream) {
    FGR_REQUIRE(n_prev >= 0 && nq >= 0 && width > 0, "fgr_overlap_pool: bad arguments");
    FGR_REQUIRE(nq == 0 || (prev && idx && out), "fgr_overlap_pool: null pointer");
    if (nq == 0) return FGR_OK;
    hipLaunchKernelGGL(overlap_pool_kernel, dim3((unsigned)ceil_div(nq, 256)), dim3(256), 0,
                       as_stream(stream), prev, n_prev, idx, nq, width, out);
    FGR_CHECK_LAUNCH("overlap_pool_kernel");
    return FGR_OK;
}

extern "C" int fgr_bce_logits_mean(const float* x, int64_t stride_x, const float* y, int64_t n,
                                   float* out, void* stream) {
    FGR_REQUIRE(x && y && out && n > 0 && stride_x >= 1, "fgr_bce_logits_mean: bad arguments");
    hipLaunchKernelGGL(bce_logits_mean_kernel, dim3(1), dim3(kRed), 0, as_stream(stream), x,
                       stride_x, y, n, out);
    FGR_CHECK_LAUNCH("bce_logits_mean_kernel");
    return FGR_OK;
}

extern "C" int fgr_transform_points(const float* xyz, int64_t n, const int64_t* seg_off,
                                    int32_t n_seg, const float* pose, int32_t inverse, float* out,
                                    void* stream) {
    FGR_REQUIRE(n >= 0 && n_seg > 0, "fgr_transform_points: bad arguments");
    FGR_REQUIRE(n == 0 || (xyz && seg_off && pose && out), "fgr_transform_points: null pointer");
    if (n == 0) return FGR_OK;
    hipLaunchKernelGGL(transform_points_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                       as_stream(stream), xyz, n, seg_off, n_seg, pose, inverse, out);
    FGR_CHECK_LAUNCH("transform_points_kernel");
    return FGR_OK;
}

extern "C" int fgr_infonce_rows(const float* logits, int64_t ld, const float* axyz,
                                const float* pxyz, const int64_t* a_off, const int64_t* p_off,
                                int32_t n_pairs, int64_t n_anchor, float r_p, float r_n,
                                float* row_loss, float* row_mask, void* stream) {
    FGR_REQUIRE(n_pairs > 0 && n_anchor >= 0 && ld >= 0, "fgr_infonce_rows: bad arguments");
    FGR_REQUIRE(n_anchor == 0 || (logits && axyz && pxyz && a_off && p_off && row_loss &&
                                  row_mask),
                "fgr_infonce_rows: null pointer");
    if (n_anchor == 0) return FGR_OK;
    hipLaunchKernelGGL(infonce_rows_kernel, dim3((unsigned)ceil_div(n_anchor, 4)), dim3(256), 0,
                       as_stream(stream), logits, ld, axyz, pxyz, a_off, p_off, n_pairs, n_anchor,
                       r_p, r_n, row_loss, row_mask);
    FGR_CHECK_LAUNCH("infonce_rows_kernel");
    return FGR_OK;
}

extern "C" int fgr_infonce_rows_bwd(const float* logits, int64_t ld, const float* axyz,
                                    const float* pxyz, const int64_t* a_off, const int64_t* p_off,
                                    int32_t n_pairs, int64_t n_anchor, int64_t n_cols, float r_n,
                                    const float* row_weight, const float* grad, float* dlogits,
                                    int64_t ld_d, void* stream) {
    FGR_REQUIRE(n_pairs > 0 && n_anchor >= 0 && n_cols >= 0 && ld >= n_cols && ld_d >= n_cols,
                "fgr_infonce_rows_bwd: bad arguments");
    FGR_REQUIRE(n_anchor == 0 || (logits && axyz && pxyz && a_off && p_off && row_weight && grad &&
                                  dlogits),
                "fgr_infonce_rows_bwd: null pointer");
    if (n_anchor == 0) return FGR_OK;
    hipLaunchKernelGGL(infonce_rows_bwd_kernel, dim3((unsigned)ceil_div(n_anchor, 4)), dim3(256), 0,
                       as_stream(stream), logits, ld, axyz, pxyz, a_off, p_off, n_pairs, n_anchor,
                       n_cols, r_n, row_weight, grad, dlogits, ld_d);
    FGR_CHECK_LAUNCH("infonce_rows_bwd_kernel");
    return FGR_OK;
}

extern "C" int fgr_infonce_reduce(const float* row_loss, const float* row_mask,
                                  const int64_t* a_off, int32_t n_pairs, float* out, void* stream) {
    FGR_REQUIRE(row_loss && row_mask && a_off && out && n_pairs > 0,
                "fgr_infonce_reduce: bad arguments");
    hipLaunchKernelGGL(infonce_reduce_kernel, dim3(1), dim3(kRed), 0, as_stream(stream), row_loss,
                       row_mask, a_off, n_pairs, out);
    FGR_CHECK_LAUNCH("infonce_reduce_kernel");
    return FGR_OK;
}

extern "C" int fgr_circle_loss_workspace(int64_t fd_elems, int64_t n_anchor, int64_t n_pos,
                                         size_t* bytes) {
    FGR_REQUIRE(bytes && fd_elems >= 0 && n_anchor >= 0 && n_pos >= 0,
                "fgr_circle_loss_workspace: bad arguments");
    *bytes = (size_t)(fd_elems + 2 * (n_anchor + n_pos)) * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_circle_loss(const float* anchor_feat, const float* pos_feat, int32_t d,
                               const float* axyz, const float* pxyz, const int64_t* a_off,
                               const int64_t* p_off, const int64_t* fd_off, int32_t n_pairs,
                               int64_t n_anchor, int64_t n_pos, int32_t max_anchor,
                               int32_t max_pos, int64_t fd_elems, float r_p, float r_n,
                               void* ws, size_t ws_bytes, float* out, void* stream) {
    FGR_REQUIRE(n_pairs > 0 && d > 0 && n_anchor >= 0 && n_pos >= 0 && max_anchor >= 0 &&
                    max_pos >= 0 && fd_elems >= 0,
                "fgr_circle_loss: bad arguments");
    FGR_REQUIRE(anchor_feat && pos_feat && axyz && pxyz && a_off && p_off && fd_off && ws && out,
                "fgr_circle_loss: null pointer");
    size_t need = 0;
    fgr_circle_loss_workspace(fd_elems, n_anchor, n_pos, &need);
    FGR_REQUIRE(ws_bytes >= need, "fgr_circle_loss: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    float* fd = static_cast<float*>(ws);
    float* line_loss = fd + fd_elems;
    float* line_sel = line_loss + (n_anchor + n_pos);
    if (max_anchor > 0 && max_pos > 0) {
        hipLaunchKernelGGL(circle_fd_kernel,
                           dim3((unsigned)ceil_div(max_pos, kCdTile),
                                (unsigned)ceil_div(max_anchor, kCdTile), (unsigned)n_pairs),
                           dim3(256), 0, st, anchor_feat, pos_feat, d, a_off, p_off, fd_off, fd);
        FGR_CHECK_LAUNCH("circle_fd_kernel");
    }
    if (n_anchor + n_pos > 0) {
        hipLaunchKernelGGL(circle_lines_kernel, dim3((unsigned)ceil_div(n_anchor + n_pos, 4)),
                           dim3(256), 0, st, (const float*)fd, axyz, pxyz, a_off, p_off, fd_off,
                           n_pairs, n_anchor, n_pos, r_p, r_n, line_loss, line_sel);
        FGR_CHECK_LAUNCH("circle_lines_kernel");
    }
    hipLaunchKernelGGL(circle_reduce_kernel, dim3(1), dim3(kRed), 0, st, (const float*)line_loss,
                       (const float*)line_sel, a_off, p_off, n_pairs, out);
    FGR_CHECK_LAUNCH("circle_reduce_kernel");
    return FGR_OK;
}

// the Euclidean feature distances alone (feature_loss.py:11-36 cdist 'euclidean': direct
// differences, sqrt(sum + 1e-12)), packed per pair at fd_off[b]: the forward of the training
// CircleLoss (fgreg.loss, its backward on the GEMMs)
extern "C" int fgr_pair_cdist(const float* anchor_feat, const float* pos_feat, int32_t d,
                              const int64_t* a_off, const int64_t* p_off, const int64_t* fd_off,
                              int32_t n_pairs, int32_t max_anchor, int32_t max_pos, float* fd,
                              void* stream) {
    FGR_REQUIRE(n_pairs > 0 && d > 0 && max_anchor >= 0 && max_pos >= 0,
                "fgr_pair_cdist: bad arguments");
    FGR_REQUIRE(anchor_feat && pos_feat && a_off && p_off && fd_off && fd,
                "fgr_pair_cdist: null pointer");
    if (max_anchor > 0 && max_pos > 0) {
        hipLaunchKernelGGL(circle_fd_kernel,
                           dim3((unsigned)ceil_div(max_pos, kCdTile),
                                (unsigned)ceil_div(max_anchor, kCdTile), (unsigned)n_pairs),
                           dim3(256), 0, as_stream(stream), anchor_feat, pos_feat, d, a_off, p_off,
                           fd_off, fd);
        FGR_CHECK_LAUNCH("circle_fd_kernel");
    }
    return FGR_OK;
}

extern "C" int fgr_corr_loss(const float* xyz, const float* corr, const float* w,
                             const int64_t* seg_off, int32_t n_pairs, const float* pose,
                             float* out, void* stream) {
    FGR_REQUIRE(xyz && corr && w && seg_off && pose && out && n_pairs > 0,
                "fgr_corr_loss: bad arguments");
    hipLaunchKernelGGL(corr_loss_kernel, dim3(1), dim3(kRed), 0, as_stream(stream), xyz, corr, w,
                       seg_off, n_pairs, pose, out);
    FGR_CHECK_LAUNCH("corr_loss_kernel");
    return FGR_OK;
}

extern "C" int fgr_se3_compare(const float* pred, const float* gt, int32_t n_layers,
                               int32_t n_pairs, float* rot_deg, float* trans, void* stream) {
    FGR_REQUIRE(pred && gt && rot_deg && trans && n_layers > 0 && n_pairs > 0,
                "fgr_se3_compare: bad arguments");
    const int n = n_layers * n_pairs;
    hipLaunchKernelGGL(se3_compare_kernel, dim3((unsigned)ceil_div(n, 64)), dim3(64), 0,
                       as_stream(stream), pred, gt, n_layers, n_pairs, rot_deg, trans);
    FGR_CHECK_LAUNCH("se3_compare_kernel");
    return FGR_OK;
}
