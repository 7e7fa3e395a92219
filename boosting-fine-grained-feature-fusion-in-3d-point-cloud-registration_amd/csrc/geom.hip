// KPConv pyramid geometry on gfx950: brute-force radius neighbour search (grid subsampling
// and the voxel-binned radius search live in grid.hip).
//
// Built with -ffp-contract=off: every float expression below rounds exactly as
// written, which is what makes voxel keys, barycentres and the d2 < r2 test
// bit-identical to the reference's C++ (grid_subsampling.cpp, neighbors.cpp +
// nanoflann.hpp) and to oracle/geom_oracle.c.
#include "common.h"

namespace fgr {
namespace {

// ------------------------------------------------------------------------------------
// Radius search
// ------------------------------------------------------------------------------------
constexpr int kRadBlock = 256;
constexpr int kRadTile = 1024;

// d2 exactly as nanoflann's L2_Simple_Adaptor::evalMetric (result = 0 + dx^2 ...).
__device__ __forceinline__ float dist2(float qx, float qy, float qz, float sx, float sy, float sz) {
    float dx = qx - sx, dy = qy - sy, dz = qz - sz;
    float d2 = dx * dx;
    d2 = d2 + dy * dy;
    d2 = d2 + dz * dz;
    return d2;
}

// mode INDEX (ball_query) and uncapped count; one thread per query, supports of the
// query's cloud staged through LDS tiles shared by the block.
template <bool kCountOnly>
__global__ void __launch_bounds__(kRadBlock)
radius_index_kernel(const float* __restrict__ q, const int64_t* __restrict__ q_off,
                    const float* __restrict__ s, const int64_t* __restrict__ s_off, float r2,
                    int width, int64_t ns_total, int64_t* __restrict__ out,
                    int* __restrict__ counts, int* __restrict__ max_count) {
    __shared__ float tile[3 * kRadTile];
    const int c = blockIdx.y;
    const int64_t qb = q_off[c], qe = q_off[c + 1];
    const int64_t sb = s_off[c], se = s_off[c + 1];
    const int64_t qi = qb + (int64_t)blockIdx.x * kRadBlock + threadIdx.x;
    if (qb + (int64_t)blockIdx.x * kRadBlock >= qe) return;  // block-uniform
    const bool active = qi < qe;
    float qx = 0.f, qy = 0.f, qz = 0.f;
    if (active) { qx = q[3 * qi]; qy = q[3 * qi + 1]; qz = q[3 * qi + 2]; }
    int cnt = 0;
    int64_t* row = active && !kCountOnly ? out + qi * width : nullptr;
    for (int64_t t0 = sb; t0 < se; t0 += kRadTile) {
        const int nt = (int)min((int64_t)kRadTile, se - t0);
        __syncthreads();
        for (int j = threadIdx.x; j < 3 * nt; j += kRadBlock) tile[j] = s[3 * t0 + j];
        __syncthreads();
        if (active && (kCountOnly || cnt < width)) {
            for (int j = 0; j < nt; ++j) {
                float d2 = dist2(qx, qy, qz, tile[3 * j], tile[3 * j + 1], tile[3 * j + 2]);
                if (d2 < r2) {
                    if (!kCountOnly) {
                        row[cnt] = t0 + j;
                        if (++cnt == width) break;
                    } else {
                        ++cnt;
                    }
                }
            }
        }
        if (!kCountOnly && __syncthreads_and(!active || cnt >= width)) break;
    }
    if (!active) return;
    if (kCountOnly) {
        counts[qi] = cnt;
        atomicMax(max_count, cnt);
    } else {
        for (int k = cnt; k < width; ++k) row[k] = ns_total;
    }
}

// mode INDEX, one wave per query: the wave sweeps the cloud's supports 64 at a time in
// index order (coalesced 768-B loads), keeps hits with a ballot and writes them at their
// prefix-count positions, and stops as soon as `width` hits are stored.
constexpr int kWaveQueries = 4;

__global__ void __launch_bounds__(64 * kWaveQueries)
radius_index_wave_kernel(const float* __restrict__ q, const int64_t* __restrict__ q_off,
                         const float* __restrict__ s, const int64_t* __restrict__ s_off, float r2,
                         int width, int64_t ns_total, int64_t* __restrict__ out) {
    const int c = blockIdx.y;
    const int lane = threadIdx.x % 64;
    const int64_t qb = q_off[c], qe = q_off[c + 1];
    const int64_t qi = qb + (int64_t)blockIdx.x * kWaveQueries + threadIdx.x / 64;
    if (qi >= qe) return;                                   // wave-uniform
    const int64_t sb = s_off[c], se = s_off[c + 1];
    const float qx = q[3 * qi], qy = q[3 * qi + 1], qz = q[3 * qi + 2];
    int64_t* row = out + qi * width;
    int cnt = 0;
    for (int64_t j0 = sb; j0 < se && cnt < width; j0 += 64) {
        const int64_t j = j0 + lane;
        bool hit = false;
        if (j < se) hit = dist2(qx, qy, qz, s[3 * j], s[3 * j + 1], s[3 * j + 2]) < r2;
        const unsigned long long m = __ballot(hit);
        const int pos = cnt + __popcll(m & ((1ull << lane) - 1ull));
        if (hit && pos < width) row[pos] = j;
        cnt += __popcll(m);
    }
    for (int k = (cnt < width ? cnt : width) + lane; k < width; k += 64) row[k] = ns_total;
}

// mode DIST (nanoflann sorted + [:, :K]): per-thread sorted (d2, idx) list in LDS.
constexpr int kDistBlock = 64;
constexpr int kDistTile = 512;
constexpr int kDistMaxWidth = 64;

__global__ void __launch_bounds__(kDistBlock)
radius_dist_kernel(const float* __restrict__ q, const int64_t* __restrict__ q_off,
                   const float* __restrict__ s, const int64_t* __restrict__ s_off, float r2,
                   int width, int64_t ns_total, int64_t* __restrict__ out) {
    __shared__ float tile[3 * kDistTile];
    __shared__ float ld2[kDistMaxWidth][kDistBlock];
    __shared__ int lidx[kDistMaxWidth][kDistBlock];
    const int c = blockIdx.y;
    const int64_t qb = q_off[c], qe = q_off[c + 1];
    const int64_t sb = s_off[c], se = s_off[c + 1];
    const int64_t qi = qb + (int64_t)blockIdx.x * kDistBlock + threadIdx.x;
    if (qb + (int64_t)blockIdx.x * kDistBlock >= qe) return;
    const bool active = qi < qe;
    const int t = threadIdx.x;
    float qx = 0.f, qy = 0.f, qz = 0.f;
    if (active) { qx = q[3 * qi]; qy = q[3 * qi + 1]; qz = q[3 * qi + 2]; }
    int cnt = 0;
    for (int64_t t0 = sb; t0 < se; t0 += kDistTile) {
        const int nt = (int)min((int64_t)kDistTile, se - t0);
        __syncthreads();
        for (int j = t; j < 3 * nt; j += kDistBlock) tile[j] = s[3 * t0 + j];
        __syncthreads();
        if (!active) continue;
        for (int j = 0; j < nt; ++j) {
            float d2 = dist2(qx, qy, qz, tile[3 * j], tile[3 * j + 1], tile[3 * j + 2]);
            if (!(d2 < r2)) continue;
            int pos;
            if (cnt < width) {
                pos = cnt++;
            } else if (d2 < ld2[width - 1][t]) {
                pos = width - 1;
            } else {
                continue;
            }
            // supports arrive in index order, so an equal d2 already stored has a smaller
            // index and stays in front: the list is sorted by (d2, index)
            while (pos > 0 && ld2[pos - 1][t] > d2) {
                ld2[pos][t] = ld2[pos - 1][t];
                lidx[pos][t] = lidx[pos - 1][t];
                --pos;
            }
            ld2[pos][t] = d2;
            lidx[pos][t] = (int)(t0 - sb + j);
        }
    }
    if (!active) return;
    int64_t* row = out + qi * width;
    for (int k = 0; k < width; ++k) row[k] = k < cnt ? sb + lidx[k][t] : ns_total;
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_radius_count(const float* q, const int64_t* q_off, const float* s,
                                const int64_t* s_off, int32_t n_clouds, int64_t nq,
                                int32_t max_q_len, float radius, int32_t* counts,
                                int32_t* max_count, void* stream) {
    FGR_REQUIRE(q_off && s_off && counts && max_count && n_clouds > 0 && max_q_len >= 0 &&
                    radius > 0.f,
                "fgr_radius_count: bad arguments");
    hipStream_t st = as_stream(stream);
    FGR_CHECK_HIP(hipMemsetAsync(max_count, 0, sizeof(int32_t), st));
    if (nq == 0 || max_q_len == 0) return FGR_OK;
    dim3 grid((unsigned)ceil_div(max_q_len, kRadBlock), (unsigned)n_clouds);
    hipLaunchKernelGGL(radius_index_kernel<true>, grid, dim3(kRadBlock), 0, st, q, q_off, s,
                       s_off, radius * radius, 0, (int64_t)0, (int64_t*)nullptr, counts,
                       max_count);
    FGR_CHECK_LAUNCH("radius_count_kernel");
    return FGR_OK;
}

extern "C" int fgr_radius_search(const float* q, const int64_t* q_off, const float* s,
                                 const int64_t* s_off, int32_t n_clouds, int64_t nq, int64_t ns,
                                 int32_t max_q_len, float radius, int32_t mode, int32_t width,
                                 int64_t* out, void* stream) {
    FGR_REQUIRE(q_off && s_off && n_clouds > 0 && max_q_len >= 0 && radius > 0.f && width >= 0 &&
                    (out || nq == 0 || width == 0),
                "fgr_radius_search: bad arguments");
    FGR_REQUIRE(mode == FGR_NB_INDEX || (mode == FGR_NB_DIST && width <= kDistMaxWidth),
                "fgr_radius_search: mode %d / width %d unsupported", mode, width);
    if (nq == 0 || width == 0 || max_q_len == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const float r2 = radius * radius;
    if (mode == FGR_NB_INDEX) {
        dim3 grid((unsigned)ceil_div(max_q_len, kWaveQueries), (unsigned)n_clouds);
        hipLaunchKernelGGL(radius_index_wave_kernel, grid, dim3(64 * kWaveQueries), 0, st, q, q_off,
                           s, s_off, r2, width, ns, out);
    } else {
        dim3 grid((unsigned)ceil_div(max_q_len, kDistBlock), (unsigned)n_clouds);
        hipLaunchKernelGGL(radius_dist_kernel, grid, dim3(kDistBlock), 0, st, q, q_off, s, s_off,
                           r2, width, ns, out);
    }
    FGR_CHECK_LAUNCH("radius_search_kernel");
    return FGR_OK;
}
