// KPConv pyramid geometry on gfx950: grid subsampling and radius neighbour search.
//
// Built with -ffp-contract=off: every float expression below rounds exactly as
// written, which is what makes voxel keys, barycentres and the d2 < r2 test
// bit-identical to the reference's C++ (grid_subsampling.cpp, neighbors.cpp +
// nanoflann.hpp) and to oracle/geom_oracle.c.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace fgr {
namespace {

// ------------------------------------------------------------------------------------
// Grid subsampling
// ------------------------------------------------------------------------------------
struct CloudGrid {
    float org[3];
    float pad;
    unsigned long long nx, ny;
};

// One block per cloud: bounding box -> origin and grid dims (grid_subsampling.cpp:25-31).
__global__ void __launch_bounds__(256) grid_bbox_kernel(const float* __restrict__ pts,
                                                        const int64_t* __restrict__ off,
                                                        float dl, CloudGrid* __restrict__ grids) {
    const int c = blockIdx.x;
    const int64_t b = off[c], e = off[c + 1];
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            float v = pts[3 * i + d];
            mn[d] = fminf(mn[d], v);
            mx[d] = fmaxf(mx[d], v);
        }
    }
    __shared__ float red[2][3][4];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        for (int o = 32; o > 0; o >>= 1) {
            mn[d] = fminf(mn[d], __shfl_xor(mn[d], o, kWave));
            mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o, kWave));
        }
    }
    const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
    if (l == 0) {
        for (int d = 0; d < 3; ++d) { red[0][d][w] = mn[d]; red[1][d][w] = mx[d]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        CloudGrid g;
        float inv = 1.0f / dl;
        float fmn[3], fmx[3];
        for (int d = 0; d < 3; ++d) {
            fmn[d] = fminf(fminf(red[0][d][0], red[0][d][1]), fminf(red[0][d][2], red[0][d][3]));
            fmx[d] = fmaxf(fmaxf(red[1][d][0], red[1][d][1]), fmaxf(red[1][d][2], red[1][d][3]));
            g.org[d] = floorf(fmn[d] * inv) * dl;
        }
        g.pad = 0.f;
        g.nx = (unsigned long long)(long long)floorf((fmx[0] - g.org[0]) / dl) + 1ull;
        g.ny = (unsigned long long)(long long)floorf((fmx[1] - g.org[1]) / dl) + 1ull;
        grids[c] = g;
    }
}

// Voxel key per point (grid_subsampling.cpp:53-56); value = point index.
__global__ void grid_key_kernel(const float* __restrict__ pts, const int64_t* __restrict__ off,
                                int n_clouds, int64_t n, float dl,
                                const CloudGrid* __restrict__ grids,
                                unsigned long long* __restrict__ keys, int* __restrict__ vals) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = find_segment(off, n_clouds, i);
    const CloudGrid g = grids[c];
    unsigned long long ix = (unsigned long long)(long long)floorf((pts[3 * i] - g.org[0]) / dl);
    unsigned long long iy = (unsigned long long)(long long)floorf((pts[3 * i + 1] - g.org[1]) / dl);
    unsigned long long iz = (unsigned long long)(long long)floorf((pts[3 * i + 2] - g.org[2]) / dl);
    keys[i] = ix + g.nx * iy + g.nx * g.ny * iz;
    vals[i] = (int)i;
}

// Voxel-head flags over the (cloud, key)-sorted keys.
__global__ void grid_head_kernel(const unsigned long long* __restrict__ skeys,
                                 const int64_t* __restrict__ off, int n_clouds, int64_t n,
                                 int* __restrict__ flags) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = find_segment(off, n_clouds, i);
    flags[i] = (i == off[c] || skeys[i] != skeys[i - 1]) ? 1 : 0;
}

// Per-cloud voxel counts + total (from the inclusive scan of head flags); voxel starts.
__global__ void grid_count_kernel(const int* __restrict__ scan, const int* __restrict__ flags,
                                  const int64_t* __restrict__ off, int n_clouds, int64_t n,
                                  int64_t* __restrict__ counts, int* __restrict__ vstart) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && flags[i]) vstart[scan[i] - 1] = (int)i;
    if (i < n_clouds) {
        int64_t b = off[i], e = off[i + 1];
        int64_t before = b > 0 ? scan[b - 1] : 0;
        int64_t upto = e > 0 ? scan[e - 1] : 0;
        counts[i] = e > b ? upto - before : 0;
    }
    if (i == 0) {
        int total = n > 0 ? scan[n - 1] : 0;
        counts[n_clouds] = total;
        vstart[total] = (int)n;
    }
}

// Barycentre per voxel: members summed in input order (grid_subsampling.cpp:70, 87).
__global__ void grid_fill_kernel(const float* __restrict__ pts, const int* __restrict__ svals,
                                 const unsigned long long* __restrict__ skeys,
                                 const int* __restrict__ vstart, int64_t n_out,
                                 float* __restrict__ out, int64_t* __restrict__ out_keys) {
    int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n_out) return;
    const int b = vstart[v], e = vstart[v + 1];
    float sx = 0.f, sy = 0.f, sz = 0.f;
    for (int j = b; j < e; ++j) {
        const int p = svals[j];
        sx += pts[3 * p];
        sy += pts[3 * p + 1];
        sz += pts[3 * p + 2];
    }
    const float s = (float)(1.0 / (double)(e - b));
    out[3 * v] = sx * s;
    out[3 * v + 1] = sy * s;
    out[3 * v + 2] = sz * s;
    if (out_keys) out_keys[v] = (int64_t)skeys[b];
}

struct GridWs {
    CloudGrid* grids;
    unsigned long long *keys, *skeys;
    int *vals, *svals, *flags, *scan, *vstart;
    void* temp;
    size_t temp_bytes;
    size_t total;
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

int carve(void* ws, int64_t n, int32_t n_clouds, size_t temp_bytes, GridWs* g) {
    char* p = static_cast<char*>(ws);
    size_t o = 0;
    auto take = [&](size_t bytes) { void* r = p ? p + o : nullptr; o += align_up(bytes); return r; };
    g->grids = (CloudGrid*)take(sizeof(CloudGrid) * n_clouds);
    g->keys = (unsigned long long*)take(8 * n);
    g->skeys = (unsigned long long*)take(8 * n);
    g->vals = (int*)take(4 * n);
    g->svals = (int*)take(4 * n);
    g->flags = (int*)take(4 * n);
    g->scan = (int*)take(4 * n);
    g->vstart = (int*)take(4 * (n + 1));
    g->temp = take(temp_bytes);
    g->temp_bytes = temp_bytes;
    g->total = o;
    return 0;
}

size_t cub_temp_bytes(int64_t n, int32_t n_clouds) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceSegmentedRadixSort::SortPairs(
        nullptr, a, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
        (const int*)nullptr, (int*)nullptr, (int)n, n_clouds, (const int64_t*)nullptr,
        (const int64_t*)nullptr + 1);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (const int*)nullptr, (int*)nullptr, (int)n);
    return a > b ? a : b;
}

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

namespace fgr {

// The radix-sort path of grid subsampling (hipCUB segmented sort of the voxel keys), used by
// the entry points in grid.hip when the caller selects it (max_cells < 0): it handles any key
// space, the dense counting-sort path only those that fit its histogram.
size_t grid_radix_ws_bytes(int64_t n_points, int32_t n_clouds) {
    GridWs g;
    carve(nullptr, n_points, n_clouds, cub_temp_bytes(n_points, n_clouds), &g);
    return g.total;
}

int grid_radix_count(const float* points, const int64_t* off, int32_t n_clouds, int64_t n_points,
                     float dl, void* ws, size_t ws_bytes, int64_t* counts, hipStream_t st) {
    GridWs g;
    size_t tb = cub_temp_bytes(n_points, n_clouds);
    carve(ws, n_points, n_clouds, tb, &g);
    if (g.total > ws_bytes) {
        set_error("fgr_grid_subsample_count: workspace %zu < %zu bytes", ws_bytes, g.total);
        return FGR_E_WORKSPACE;
    }
    hipLaunchKernelGGL(grid_bbox_kernel, dim3(n_clouds), dim3(256), 0, st, points, off, dl,
                       g.grids);
    FGR_CHECK_LAUNCH("grid_bbox_kernel");
    if (n_points > 0) {
        const int64_t nb = ceil_div(n_points, 256);
        hipLaunchKernelGGL(grid_key_kernel, dim3(nb), dim3(256), 0, st, points, off, n_clouds,
                           n_points, dl, g.grids, g.keys, g.vals);
        FGR_CHECK_LAUNCH("grid_key_kernel");
        size_t tmp = g.temp_bytes;
        FGR_CHECK_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(
            g.temp, tmp, g.keys, g.skeys, g.vals, g.svals, (int)n_points, n_clouds, off, off + 1,
            0, 64, st));
        hipLaunchKernelGGL(grid_head_kernel, dim3(nb), dim3(256), 0, st, g.skeys, off, n_clouds,
                           n_points, g.flags);
        FGR_CHECK_LAUNCH("grid_head_kernel");
        tmp = g.temp_bytes;
        FGR_CHECK_HIP(hipcub::DeviceScan::InclusiveSum(g.temp, tmp, g.flags, g.scan,
                                                       (int)n_points, st));
    }
    const int64_t nthreads = n_points > n_clouds ? n_points : n_clouds;
    hipLaunchKernelGGL(grid_count_kernel, dim3(ceil_div(nthreads, 256)), dim3(256), 0, st, g.scan,
                       g.flags, off, n_clouds, n_points, counts, g.vstart);
    FGR_CHECK_LAUNCH("grid_count_kernel");
    return FGR_OK;
}

int grid_radix_fill(int64_t n_points, int32_t n_clouds, int64_t n_out, void* ws, size_t ws_bytes,
                    const float* points, float* out_points, int64_t* out_keys, hipStream_t st) {
    GridWs g;
    carve(ws, n_points, n_clouds, cub_temp_bytes(n_points, n_clouds), &g);
    if (g.total > ws_bytes) {
        set_error("fgr_grid_subsample_fill: workspace %zu < %zu bytes", ws_bytes, g.total);
        return FGR_E_WORKSPACE;
    }
    if (n_out == 0) return FGR_OK;
    hipLaunchKernelGGL(grid_fill_kernel, dim3(ceil_div(n_out, 256)), dim3(256), 0, st, points,
                       g.svals, g.skeys, g.vstart, n_out, out_points, out_keys);
    FGR_CHECK_LAUNCH("grid_fill_kernel");
    return FGR_OK;
}

}  // namespace fgr

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
