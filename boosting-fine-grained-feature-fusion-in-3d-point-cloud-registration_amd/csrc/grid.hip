// Counting-sort geometry on gfx950: dense voxel-key grid subsampling and cell-binned radius
// search, without a comparison / radix sort on the hot path.
//
// Both replace a sort of per-point keys by a counting sort over a DENSE key space:
//   1. every point adds itself to its cell's counter (atomicAdd returns its slot),
//   2. a device-wide exclusive scan of the counters gives each cell's start (and, for the
//      voxel grid, each non-empty cell's ordinal = the voxel index in ascending key order),
//   3. each point is scattered to start[cell] + slot.
// The order of points inside a cell is arbitrary (atomic arrival order); every consumer
// below restores the order the semantics need (ascending point index) itself.
//
// * Grid subsampling (grid_subsampling.cpp:5-106 semantics, voxel key ix + nx iy + nx ny iz
//   from the cloud's floor(min/dl) origin): the dense key space of cloud c is
//   nx * ny * nz; clouds are laid end to end in one histogram of `max_cells` counters sized
//   by the caller. Voxels come out in ascending key order per cloud (= histogram order) and
//   each barycentre sums its members in ascending point index, i.e. the reference's input
//   order -- bit-identical to oracle/geom_oracle.c. A key space larger than the histogram
//   is reported back (counts[n_clouds] = -cells needed), never truncated; the host redoes the
//   count with that capacity, up to 2^28 cells (fgreg.ops.grid_subsample raises past it).
// * Radius search: supports binned into cubic cells of edge >= 1.0625 r (grown by 1.25x
//   steps until the cloud's grid fits 4 n_c + 1024 cells, so the workspace size depends on
//   the point count only); a query scans the 27 cells around its own. Every support within r
//   lies in those cells: the 1/16 margin covers the fp32 rounding of the cell coordinates
//   for grids up to 2^16 cells per axis. Hits are ranked by (index) for ball_query
//   semantics or (d2, index) for nanoflann semantics and the first `width` are written in
//   that order -- the same rows as the brute-force scan.
// Built with -ffp-contract=off (see geom.hip): keys, barycentres and d2 round as written.
#include "common.h"

namespace fgr {

namespace {

typedef unsigned long long u64;

// ------------------------------------------------------------------------------------------
// device-wide exclusive scan of int32 counters (3 launches), optionally dual: the second
// component counts the non-zero counters (the voxel ordinal)
// ------------------------------------------------------------------------------------------
constexpr int kSB = 256, kSI = 16, kST = kSB * kSI;

__device__ __forceinline__ int2 add2(int2 a, int2 b) { return make_int2(a.x + b.x, a.y + b.y); }

__device__ __forceinline__ int2 wave_incl_scan2(int2 v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int tx = __shfl_up(v.x, o, 64), ty = __shfl_up(v.y, o, 64);
        if (lane >= o) { v.x += tx; v.y += ty; }
    }
    return v;
}

// 256-thread block exclusive scan of int2; *tot = the block total (all threads)
__device__ __forceinline__ int2 block_excl_scan2(int2 v, int2* tot) {
    __shared__ int2 wsum[kSB / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int2 inc = wave_incl_scan2(v, lane);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int2 pre = make_int2(0, 0), all = make_int2(0, 0);
#pragma unroll
    for (int i = 0; i < kSB / 64; ++i) {
        if (i < w) pre = add2(pre, wsum[i]);
        all = add2(all, wsum[i]);
    }
    __syncthreads();
    *tot = all;
    return make_int2(pre.x + inc.x - v.x, pre.y + inc.y - v.y);
}

// n = *n_dev (device-side element count) when n_dev, else n_static; element n itself reads as
// 0, so the exclusive scan's entry n is the total.
__device__ __forceinline__ int64_t scan_n(const int64_t* n_dev, int64_t n_static) {
    return n_dev ? *n_dev : n_static;
}

template <bool DUAL>
__global__ void __launch_bounds__(kSB) scan_tile_kernel(const int* __restrict__ in,
                                                        const int64_t* __restrict__ n_dev,
                                                        int64_t n_static, int2* __restrict__ tiles) {
    const int64_t n = scan_n(n_dev, n_static);
    const int64_t base = (int64_t)blockIdx.x * kST;
    int2 s = make_int2(0, 0);
    if (base <= n) {
#pragma unroll 4
        for (int k = 0; k < kSI; ++k) {
            const int64_t i = base + k * kSB + threadIdx.x;
            const int v = i < n ? in[i] : 0;
            s.x += v;
            if (DUAL) s.y += v > 0 ? 1 : 0;
        }
    }
    int2 tot;
    block_excl_scan2(s, &tot);
    if (threadIdx.x == 0) tiles[blockIdx.x] = tot;
}

// one block: tile totals -> exclusive tile offsets, in place
__global__ void __launch_bounds__(kSB) scan_offsets_kernel(int2* __restrict__ tiles, int ntiles) {
    int2 carry = make_int2(0, 0);
    for (int b0 = 0; b0 < ntiles; b0 += kSB) {
        const int i = b0 + threadIdx.x;
        const int2 v = i < ntiles ? tiles[i] : make_int2(0, 0);
        int2 tot;
        const int2 ex = block_excl_scan2(v, &tot);
        if (i < ntiles) tiles[i] = add2(ex, carry);
        carry = add2(carry, tot);
    }
}

// io[i] <- exclusive prefix (in place) for i in [0, n]; ord[i] <- exclusive count of non-zero.
// RAW: `tiles` holds the raw tile totals (at most kSB tiles) and each block sums those before
// its own (one load per thread and a block reduction) -- the scan without its one-block
// offsets launch; else `tiles` holds the exclusive tile offsets (scan_offsets_kernel)
template <bool DUAL, bool RAW = false>
__global__ void __launch_bounds__(kSB) scan_final_kernel(int* __restrict__ io, int* __restrict__ ord,
                                                         const int64_t* __restrict__ n_dev,
                                                         int64_t n_static,
                                                         const int2* __restrict__ tiles) {
    const int64_t n = scan_n(n_dev, n_static);
    const int64_t base = (int64_t)blockIdx.x * kST;
    if (base > n) return;                                   // block-uniform
    int2 carry;
    if constexpr (RAW) {
        const int2 v = (int)threadIdx.x < (int)blockIdx.x ? tiles[threadIdx.x] : make_int2(0, 0);
        block_excl_scan2(v, &carry);                        // carry = the sum over earlier tiles
    } else {
        carry = tiles[blockIdx.x];
    }
    for (int k = 0; k < kSI; ++k) {
        const int64_t i = base + k * kSB + threadIdx.x;
        const int v = i < n ? io[i] : 0;
        int2 tot;
        const int2 ex = block_excl_scan2(make_int2(v, DUAL ? (v > 0 ? 1 : 0) : 0), &tot);
        if (i <= n) {
            io[i] = carry.x + ex.x;
            if (DUAL) ord[i] = carry.y + ex.y;
        }
        carry = add2(carry, tot);
    }
}

int scan_tiles(int64_t n_max) { return (int)ceil_div(n_max + 1, kST); }

template <bool DUAL>
int launch_scan(int* io, int* ord, const int64_t* n_dev, int64_t n_max, int2* tiles,
                hipStream_t st) {
    const int nt = scan_tiles(n_max);
    hipLaunchKernelGGL(scan_tile_kernel<DUAL>, dim3(nt), dim3(kSB), 0, st, io, n_dev, n_max, tiles);
    FGR_CHECK_LAUNCH("scan_tile_kernel");
    static const bool two = [] { const char* e = getenv("FGR_SCAN2"); return !(e && e[0] == '0'); }();
    if (two && nt <= kSB) {                                 // <= 1M counters: two launches
        hipLaunchKernelGGL((scan_final_kernel<DUAL, true>), dim3(nt), dim3(kSB), 0, st, io, ord, n_dev,
                           n_max, tiles);
        FGR_CHECK_LAUNCH("scan_final_kernel");
        return FGR_OK;
    }
    hipLaunchKernelGGL(scan_offsets_kernel, dim3(1), dim3(kSB), 0, st, tiles, nt);
    FGR_CHECK_LAUNCH("scan_offsets_kernel");
    hipLaunchKernelGGL(scan_final_kernel<DUAL>, dim3(nt), dim3(kSB), 0, st, io, ord, n_dev, n_max,
                       tiles);
    FGR_CHECK_LAUNCH("scan_final_kernel");
    return FGR_OK;
}

// per-cloud min / max of xyz (256 threads, one block per cloud); valid in thread 0
// bounding box of pts[b, e) over the whole block (<= 1024 threads); every thread keeps 4
// points' loads in flight per round (the loop is latency-bound: one block per cloud)
__device__ __forceinline__ void block_bbox(const float* __restrict__ pts, int64_t b, int64_t e,
                                           float mn[3], float mx[3]) {
    mn[0] = mn[1] = mn[2] = INFINITY;
    mx[0] = mx[1] = mx[2] = -INFINITY;
    const int64_t bs = blockDim.x;
    for (int64_t i0 = b + threadIdx.x; i0 < e; i0 += 4 * bs) {
        float v[4][3];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + u * bs;
            const int64_t ic = i < e ? i : i0;              // i0 < e: always a valid point
#pragma unroll
            for (int d = 0; d < 3; ++d) v[u][d] = pts[3 * ic + d];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                mn[d] = fminf(mn[d], v[u][d]);
                mx[d] = fmaxf(mx[d], v[u][d]);
            }
    }
    __shared__ float red[2][3][16];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        for (int o = 32; o > 0; o >>= 1) {
            mn[d] = fminf(mn[d], __shfl_xor(mn[d], o, kWave));
            mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o, kWave));
        }
    }
    const int w = threadIdx.x / kWave, l = threadIdx.x % kWave, nw = (int)(bs / kWave);
    if (l == 0)
        for (int d = 0; d < 3; ++d) { red[0][d][w] = mn[d]; red[1][d][w] = mx[d]; }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int d = 0; d < 3; ++d) {
            mn[d] = red[0][d][0];
            mx[d] = red[1][d][0];
            for (int k = 1; k < nw; ++k) {
                mn[d] = fminf(mn[d], red[0][d][k]);
                mx[d] = fmaxf(mx[d], red[1][d][k]);
            }
        }
}

// ------------------------------------------------------------------------------------------
// grid subsampling, dense voxel keys
// ------------------------------------------------------------------------------------------
struct DGrid {
    float org[3];
    int pad;
    u64 nx, ny;
    long long base, cells;          // first counter of the cloud, its key-space size
};

constexpr long long kHuge = 1ll << 62;

// blocks >= n_clouds zero the histogram (4096 counters each) -- one launch instead of a
// bbox launch plus a memset
__global__ void __launch_bounds__(1024) dgrid_bbox_kernel(const float* __restrict__ pts,
                                                         const int64_t* __restrict__ off, float dl,
                                                         DGrid* __restrict__ grids, int n_clouds,
                                                         int* __restrict__ zero, int64_t n_zero) {
    const int c = blockIdx.x;
    if (c >= n_clouds) {                                   // block-uniform
        const int64_t z0 = (int64_t)(c - n_clouds) * 4096;
        for (int64_t i = z0 + threadIdx.x; i < min(z0 + 4096, n_zero); i += 1024) zero[i] = 0;
        return;
    }
    const int64_t b = off[c], e = off[c + 1];
    float mn[3], mx[3];
    block_bbox(pts, b, e, mn, mx);
    if (threadIdx.x != 0) return;
    DGrid g;
    g.pad = 0;
    g.base = 0;
    if (e <= b) {
        g.org[0] = g.org[1] = g.org[2] = 0.f;
        g.nx = g.ny = 1;
        g.cells = 0;
    } else {
        // origin and dims exactly as grid_subsampling.cpp:25-31
        const float inv = 1.0f / dl;
        long long dims[3];
        for (int d = 0; d < 3; ++d) {
            g.org[d] = floorf(mn[d] * inv) * dl;
            dims[d] = (long long)floorf((mx[d] - g.org[d]) / dl) + 1;
        }
        g.nx = (u64)dims[0];
        g.ny = (u64)dims[1];
        const bool big = dims[0] > (1 << 20) || dims[1] > (1 << 20) || dims[2] > (1 << 20);
        g.cells = big ? kHuge : dims[0] * dims[1] * dims[2];
    }
    grids[c] = g;
}

// ctl[0] = cells to scan (0 when the key space does not fit), ctl[1] = cells needed
__global__ void dgrid_base_kernel(DGrid* __restrict__ grids, int n_clouds, long long cap,
                                  int64_t* __restrict__ ctl) {
    if (threadIdx.x != 0) return;
    long long b = 0;
    for (int c = 0; c < n_clouds; ++c) {
        grids[c].base = b;
        b = (b >= kHuge - grids[c].cells) ? kHuge : b + grids[c].cells;
    }
    ctl[0] = b <= cap ? b : 0;
    ctl[1] = b;
}

__global__ void dgrid_key_kernel(const float* __restrict__ pts, const int64_t* __restrict__ off,
                                 int n_clouds, int64_t n, float dl, const DGrid* __restrict__ grids,
                                 const int64_t* __restrict__ ctl, int* __restrict__ hist,
                                 int* __restrict__ cellof, int* __restrict__ slot,
                                 u64* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || ctl[0] == 0) return;
    const int c = find_segment(off, n_clouds, i);
    const DGrid g = grids[c];
    // key exactly as grid_subsampling.cpp:53-56 (geom.hip grid_key_kernel)
    const u64 ix = (u64)(long long)floorf((pts[3 * i] - g.org[0]) / dl);
    const u64 iy = (u64)(long long)floorf((pts[3 * i + 1] - g.org[1]) / dl);
    const u64 iz = (u64)(long long)floorf((pts[3 * i + 2] - g.org[2]) / dl);
    const u64 key = ix + g.nx * iy + g.nx * g.ny * iz;
    const long long cell = g.base + (long long)key;
    cellof[i] = (int)cell;
    slot[i] = atomicAdd(&hist[cell], 1);
    keys[i] = key;
}

__global__ void dgrid_scatter_kernel(int64_t n, const int64_t* __restrict__ ctl,
                                     const int* __restrict__ cellof, const int* __restrict__ slot,
                                     const u64* __restrict__ keys, const int* __restrict__ start,
                                     const int* __restrict__ ord, int* __restrict__ svals,
                                     int* __restrict__ vstart, u64* __restrict__ vkey) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || ctl[0] == 0) return;
    const int cell = cellof[i], sl = slot[i];
    svals[start[cell] + sl] = (int)i;
    if (sl == 0) {
        const int v = ord[cell];
        vstart[v] = start[cell];
        vkey[v] = keys[i];
    }
}

__global__ void dgrid_count_kernel(const DGrid* __restrict__ grids, int n_clouds, int64_t n,
                                   const int64_t* __restrict__ ctl, const int* __restrict__ ord,
                                   int64_t* __restrict__ counts, int* __restrict__ vstart) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c > n_clouds) return;
    const int64_t cells = ctl[0];
    if (cells == 0) {                                   // no points, or the key space overflowed
        counts[c] = (c < n_clouds || ctl[1] == 0) ? 0 : -ctl[1];
        return;
    }
    if (c < n_clouds) {
        const DGrid g = grids[c];
        counts[c] = (int64_t)ord[g.base + g.cells] - ord[g.base];
    } else {
        const int m = ord[cells];
        counts[n_clouds] = m;
        vstart[m] = (int)n;
    }
}

// Barycentre per voxel; members are summed in ascending point index (the reference's input
// order, grid_subsampling.cpp:70, 87) -- the counting sort leaves them in arrival order.
__global__ void dgrid_fill_kernel(const float* __restrict__ pts, const int* __restrict__ svals,
                                  const int* __restrict__ vstart, const u64* __restrict__ vkey,
                                  int64_t n_out, float* __restrict__ out,
                                  int64_t* __restrict__ out_keys) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n_out) return;
    const int b = vstart[v], e = vstart[v + 1], cnt = e - b;
    float sx = 0.f, sy = 0.f, sz = 0.f;
    if (cnt <= 16) {
        int m[16];
        for (int j = 0; j < cnt; ++j) {                 // insertion sort by point index
            int x = svals[b + j], k = j;
            while (k > 0 && m[k - 1] > x) { m[k] = m[k - 1]; --k; }
            m[k] = x;
        }
        for (int j = 0; j < cnt; ++j) {
            const int p = m[j];
            sx += pts[3 * p];
            sy += pts[3 * p + 1];
            sz += pts[3 * p + 2];
        }
    } else {                                            // long voxels: repeated min-selection
        int prev = -1;
        for (int t = 0; t < cnt; ++t) {
            int nxt = 0x7fffffff;
            for (int j = b; j < e; ++j) {
                const int x = svals[j];
                if (x > prev && x < nxt) nxt = x;
            }
            sx += pts[3 * nxt];
            sy += pts[3 * nxt + 1];
            sz += pts[3 * nxt + 2];
            prev = nxt;
        }
    }
    const float s = (float)(1.0 / (double)cnt);
    out[3 * v] = sx * s;
    out[3 * v + 1] = sy * s;
    out[3 * v + 2] = sz * s;
    if (out_keys) out_keys[v] = (int64_t)vkey[v];
}

struct DGridWs {
    DGrid* grids;
    int64_t* ctl;
    int *hist, *ord;
    int2* tiles;
    int *cellof, *slot, *svals, *vstart;
    u64 *keys, *vkey;
    size_t total;
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

void carve_dense(void* ws, int64_t n, int32_t nc, int64_t cap, DGridWs* g) {
    char* p = static_cast<char*>(ws);
    size_t o = 0;
    auto take = [&](size_t bytes) { void* r = p ? p + o : nullptr; o += align_up(bytes); return r; };
    g->grids = (DGrid*)take(sizeof(DGrid) * nc);
    g->ctl = (int64_t*)take(4 * sizeof(int64_t));
    g->hist = (int*)take(4 * (cap + 1));
    g->ord = (int*)take(4 * (cap + 1));
    g->tiles = (int2*)take(sizeof(int2) * scan_tiles(cap));
    g->cellof = (int*)take(4 * n);
    g->slot = (int*)take(4 * n);
    g->svals = (int*)take(4 * n);
    g->vstart = (int*)take(4 * (n + 1));
    g->keys = (u64*)take(8 * n);
    g->vkey = (u64*)take(8 * n);
    g->total = o;
}

int64_t dense_cap(int64_t n, int64_t max_cells) {
    return max_cells > 0 ? max_cells : 8 * n + (1 << 20);
}

// ------------------------------------------------------------------------------------------
// radius search over cells
// ------------------------------------------------------------------------------------------
struct RGrid {
    float org[3];
    float cell;
    int nx, ny, nz;
    float radius;                   // the radius the grid was built for (queries use <= it)
    long long base;                 // first cell counter of the cloud (= 4 s_off[c] + 1024 c)
};

__host__ __device__ inline long long rgrid_cap(int64_t n_c) { return 4 * n_c + 1024; }

// blocks >= n_clouds zero the cell starts (4096 each), as dgrid_bbox_kernel
__global__ void __launch_bounds__(1024) rgrid_bbox_kernel(const float* __restrict__ s,
                                                         const int64_t* __restrict__ s_off,
                                                         float radius, RGrid* __restrict__ grids,
                                                         int n_clouds, int* __restrict__ zero,
                                                         int64_t n_zero) {
    const int c = blockIdx.x;
    if (c >= n_clouds) {                                   // block-uniform
        const int64_t z0 = (int64_t)(c - n_clouds) * 4096;
        for (int64_t i = z0 + threadIdx.x; i < min(z0 + 4096, n_zero); i += 1024) zero[i] = 0;
        return;
    }
    const int64_t b = s_off[c], e = s_off[c + 1];
    float mn[3], mx[3];
    block_bbox(s, b, e, mn, mx);
    if (threadIdx.x != 0) return;
    RGrid g;
    g.radius = radius;
    g.base = 4 * b + 1024ll * c;
    if (e <= b) {
        g.org[0] = g.org[1] = g.org[2] = 0.f;
        g.cell = radius;
        g.nx = g.ny = g.nz = 1;
    } else {
        const long long cap = rgrid_cap(e - b);
        float cell = radius * 1.0625f;
        long long d[3];
        for (int it = 0; it < 200; ++it) {
            for (int k = 0; k < 3; ++k) d[k] = (long long)floorf((mx[k] - mn[k]) / cell) + 1;
            if (d[0] * d[1] * d[2] <= cap && d[0] <= 65536 && d[1] <= 65536 && d[2] <= 65536) break;
            cell *= 1.25f;
        }
        for (int k = 0; k < 3; ++k) g.org[k] = mn[k];
        g.cell = cell;
        g.nx = (int)d[0];
        g.ny = (int)d[1];
        g.nz = (int)d[2];
    }
    grids[c] = g;
}

__device__ __forceinline__ int cell_coord(float x, float org, float cell) {
    return (int)floorf((x - org) / cell);
}

__global__ void rgrid_key_kernel(const float* __restrict__ s, const int64_t* __restrict__ s_off,
                                 int n_clouds, int64_t ns, const RGrid* __restrict__ grids,
                                 int* __restrict__ hist, int* __restrict__ cellof,
                                 int* __restrict__ slot) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns) return;
    const int c = find_segment(s_off, n_clouds, i);
    const RGrid g = grids[c];
    const int x = min(max(cell_coord(s[3 * i], g.org[0], g.cell), 0), g.nx - 1);
    const int y = min(max(cell_coord(s[3 * i + 1], g.org[1], g.cell), 0), g.ny - 1);
    const int z = min(max(cell_coord(s[3 * i + 2], g.org[2], g.cell), 0), g.nz - 1);
    const int cell = (int)(g.base + ((long long)z * g.ny + y) * g.nx + x);
    cellof[i] = cell;
    slot[i] = atomicAdd(&hist[cell], 1);
}

__global__ void rgrid_scatter_kernel(int64_t ns, const int* __restrict__ cellof,
                                     const int* __restrict__ slot, const int* __restrict__ start,
                                     int* __restrict__ members) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns) return;
    members[start[cellof[i]] + slot[i]] = (int)i;
}

// d2 exactly as nanoflann's L2_Simple_Adaptor::evalMetric (and geom.hip's dist2)
__device__ __forceinline__ float dist2g(float qx, float qy, float qz, float sx, float sy, float sz) {
    float dx = qx - sx, dy = qy - sy, dz = qz - sz;
    float d2 = dx * dx;
    d2 = d2 + dy * dy;
    d2 = d2 + dz * dz;
    return d2;
}

constexpr int kRQ = 4;        // queries (waves) per block
constexpr int kRCap = 256;    // hits ranked in LDS per query (more: threshold bisection)

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One wave per query: the 27 cells around the query's cell are flattened into one candidate
// range (lane k < 27 holds cell k's start / length and their exclusive prefix), candidates are
// tested 64 at a time, hits compacted by ballot into an LDS list of rank keys, then ranked:
// key = local support index (MODE 0, ball_query: first `width` in index order) or
// (d2 bits << 32 | index) (MODE 1, nanoflann: `width` nearest, ties by index).
template <int MODE, bool COUNT>
__global__ void __launch_bounds__(64 * kRQ)
rgrid_query_kernel(const float* __restrict__ q, const int64_t* __restrict__ q_off,
                   const float* __restrict__ s, const int64_t* __restrict__ s_off,
                   const RGrid* __restrict__ grids, const int* __restrict__ start,
                   const int* __restrict__ members, float r2, int width, int64_t ns_total,
                   int64_t* __restrict__ out, int* __restrict__ counts,
                   int* __restrict__ max_count) {
    __shared__ u64 lst[kRQ][kRCap];
    const int c = blockIdx.y;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t qb = q_off[c], qe = q_off[c + 1];
    const int64_t qi = qb + (int64_t)blockIdx.x * kRQ + w;
    if (qi >= qe) return;                                   // wave-uniform; no block barrier
    const int64_t sb = s_off[c];
    const RGrid g = grids[c];
    const float qx = q[3 * qi], qy = q[3 * qi + 1], qz = q[3 * qi + 2];
    const int cx = cell_coord(qx, g.org[0], g.cell);
    const int cy = cell_coord(qy, g.org[1], g.cell);
    const int cz = cell_coord(qz, g.org[2], g.cell);
    int st = 0, len = 0;
    if (lane < 27) {
        const int x = cx + lane % 3 - 1, y = cy + (lane / 3) % 3 - 1, z = cz + lane / 9 - 1;
        if (x >= 0 && x < g.nx && y >= 0 && y < g.ny && z >= 0 && z < g.nz) {
            const long long cell = g.base + ((long long)z * g.ny + y) * g.nx + x;
            st = start[cell];
            len = start[cell + 1] - st;
        }
    }
    int inc = len;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    const int exc = inc - len;
    const int T = __shfl(inc, 26, 64);
    const u64 lt_mask = (1ull << lane) - 1ull;

    // candidate j (0 <= j < T) -> (hit, key); every lane runs the shuffles
    auto probe = [&](int j, u64& key) -> bool {
        int pos = 0;
#pragma unroll
        for (int step = 16; step >= 1; step >>= 1) {
            const int cand = pos + step;
            const int e = __shfl(exc, cand & 31, 64);
            if (cand < 27 && e <= j) pos = cand;
        }
        const int stk = __shfl(st, pos, 64), exk = __shfl(exc, pos, 64);
        if (j >= T) return false;
        const int m = members[stk + (j - exk)];
        const float d2 = dist2g(qx, qy, qz, s[3 * m], s[3 * m + 1], s[3 * m + 2]);
        const unsigned loc = (unsigned)(m - sb);
        key = MODE == 0 ? (u64)loc : (((u64)__float_as_uint(d2) << 32) | (u64)loc);
        return d2 < r2;
    };

    int n = 0;
    for (int j0 = 0; j0 < T; j0 += 64) {
        u64 key = 0;
        const bool hit = probe(j0 + lane, key);
        const u64 bal = __ballot(hit);
        if (!COUNT) {
            const int p = n + __popcll(bal & lt_mask);
            if (hit && p < kRCap) lst[w][p] = key;
        }
        n += __popcll(bal);
    }
    if (COUNT) {
        if (lane == 0) {
            counts[qi] = n;
            atomicMax(max_count, n);
        }
        return;
    }
    int64_t* row = out + qi * width;
    int kept = n;
    if (n > kRCap) {
        // rare: find the smallest key t with #{hits with key <= t} >= width by bisection over
        // the key space (each probe re-tests the candidates), then keep the keys <= t
        u64 lo = 0, hi = MODE == 0 ? 0xffffffffull : ~0ull;
        while (lo < hi) {
            const u64 mid = lo + (hi - lo) / 2;
            int cnt = 0;
            for (int j0 = 0; j0 < T; j0 += 64) {
                u64 key = 0;
                const bool hit = probe(j0 + lane, key);
                cnt += __popcll(__ballot(hit && key <= mid));
            }
            if (cnt >= width) hi = mid; else lo = mid + 1;
        }
        kept = 0;
        for (int j0 = 0; j0 < T; j0 += 64) {
            u64 key = 0;
            const bool hit = probe(j0 + lane, key) && key <= lo;
            const u64 bal = __ballot(hit);
            const int p = kept + __popcll(bal & lt_mask);
            if (hit && p < kRCap) lst[w][p] = key;
            kept += __popcll(bal);
        }
        kept = min(kept, kRCap);
    }
    wave_sync_lds();
    for (int e = lane; e < kept; e += 64) {
        const u64 ke = lst[w][e];
        int rank = 0;
        for (int f = 0; f < kept; ++f) rank += lst[w][f] < ke ? 1 : 0;
        if (rank < width) row[rank] = sb + (int64_t)(ke & 0xffffffffull);
    }
    for (int k = min(n, width) + lane; k < width; k += 64) row[k] = ns_total;
}

struct RGridWs {
    RGrid* grids;
    int* start;
    int2* tiles;
    int *cellof, *slot, *members;
    size_t total;
};

void carve_rgrid(void* ws, int64_t ns, int32_t nc, RGridWs* g) {
    char* p = static_cast<char*>(ws);
    size_t o = 0;
    auto take = [&](size_t bytes) { void* r = p ? p + o : nullptr; o += align_up(bytes); return r; };
    const int64_t cap = 4 * ns + 1024ll * nc;
    g->grids = (RGrid*)take(sizeof(RGrid) * nc);
    g->start = (int*)take(4 * (cap + 1));
    g->tiles = (int2*)take(sizeof(int2) * scan_tiles(cap));
    g->cellof = (int*)take(4 * ns);
    g->slot = (int*)take(4 * ns);
    g->members = (int*)take(4 * ns);
    g->total = o;
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_grid_subsample_workspace(int64_t n_points, int32_t n_clouds, int64_t max_cells,
                                            size_t* bytes) {
    FGR_REQUIRE(bytes && n_points >= 0 && n_clouds > 0 && n_points < (1ll << 31) &&
                    max_cells < (1ll << 31) - 1,
                "fgr_grid_subsample_workspace: bad arguments");
    FGR_REQUIRE(max_cells >= 0, "fgr_grid_subsample_workspace: max_cells < 0 (the radix-sort path "
                "was removed: the dense counting sort takes key spaces up to 2^28 cells)");
    DGridWs g;
    carve_dense(nullptr, n_points, n_clouds, dense_cap(n_points, max_cells), &g);
    *bytes = g.total;
    return FGR_OK;
}

extern "C" int fgr_grid_subsample_count(const float* points, const int64_t* off, int32_t n_clouds,
                                        int64_t n_points, float dl, int64_t max_cells, void* ws,
                                        size_t ws_bytes, int64_t* counts, void* stream) {
    FGR_REQUIRE(off && counts && ws && n_clouds > 0 && n_points >= 0 && dl > 0.f &&
                    (points || n_points == 0) && n_points < (1ll << 31) &&
                    max_cells < (1ll << 31) - 1,
                "fgr_grid_subsample_count: bad arguments");
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    FGR_REQUIRE(max_cells >= 0, "fgr_grid_subsample_count: max_cells < 0 (no radix-sort path)");
    const int64_t cap = dense_cap(n_points, max_cells);
    DGridWs g;
    carve_dense(ws, n_points, n_clouds, cap, &g);
    if (g.total > ws_bytes) {
        set_error("fgr_grid_subsample_count: workspace %zu < %zu bytes", ws_bytes, g.total);
        return FGR_E_WORKSPACE;
    }
    hipLaunchKernelGGL(dgrid_bbox_kernel, dim3((unsigned)(n_clouds + ceil_div(cap + 1, 4096))),
                       dim3(1024), 0, st, points, off, dl, g.grids, n_clouds, g.hist,
                       (int64_t)(cap + 1));
    FGR_CHECK_LAUNCH("dgrid_bbox_kernel");
    hipLaunchKernelGGL(dgrid_base_kernel, dim3(1), dim3(64), 0, st, g.grids, n_clouds,
                       (long long)cap, g.ctl);
    FGR_CHECK_LAUNCH("dgrid_base_kernel");
    const unsigned nb = (unsigned)ceil_div(n_points > 0 ? n_points : 1, 256);
    hipLaunchKernelGGL(dgrid_key_kernel, dim3(nb), dim3(256), 0, st, points, off, n_clouds,
                       n_points, dl, g.grids, g.ctl, g.hist, g.cellof, g.slot, g.keys);
    FGR_CHECK_LAUNCH("dgrid_key_kernel");
    int rc = launch_scan<true>(g.hist, g.ord, g.ctl, cap, g.tiles, st);
    if (rc != FGR_OK) return rc;
    hipLaunchKernelGGL(dgrid_scatter_kernel, dim3(nb), dim3(256), 0, st, n_points, g.ctl, g.cellof,
                       g.slot, g.keys, g.hist, g.ord, g.svals, g.vstart, g.vkey);
    FGR_CHECK_LAUNCH("dgrid_scatter_kernel");
    hipLaunchKernelGGL(dgrid_count_kernel, dim3((unsigned)ceil_div(n_clouds + 1, 64)), dim3(64), 0,
                       st, g.grids, n_clouds, n_points, g.ctl, g.ord, counts, g.vstart);
    FGR_CHECK_LAUNCH("dgrid_count_kernel");
    return FGR_OK;
}

extern "C" int fgr_grid_subsample_fill(int64_t n_points, int32_t n_clouds, int64_t max_cells,
                                       int64_t n_out, void* ws, size_t ws_bytes,
                                       const float* points, float* out_points, int64_t* out_keys,
                                       void* stream) {
    FGR_REQUIRE(ws && n_clouds > 0 && n_out >= 0 && n_out <= n_points &&
                    (out_points || n_out == 0) && max_cells < (1ll << 31) - 1,
                "fgr_grid_subsample_fill: bad arguments");
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    FGR_REQUIRE(max_cells >= 0, "fgr_grid_subsample_fill: max_cells < 0 (no radix-sort path)");
    DGridWs g;
    carve_dense(ws, n_points, n_clouds, dense_cap(n_points, max_cells), &g);
    if (g.total > ws_bytes) {
        set_error("fgr_grid_subsample_fill: workspace %zu < %zu bytes", ws_bytes, g.total);
        return FGR_E_WORKSPACE;
    }
    if (n_out == 0) return FGR_OK;
    hipLaunchKernelGGL(dgrid_fill_kernel, dim3((unsigned)ceil_div(n_out, 256)), dim3(256), 0, st,
                       points, g.svals, g.vstart, g.vkey, n_out, out_points, out_keys);
    FGR_CHECK_LAUNCH("dgrid_fill_kernel");
    return FGR_OK;
}

extern "C" int fgr_radius_grid_workspace(int64_t ns, int32_t n_clouds, size_t* bytes) {
    FGR_REQUIRE(bytes && ns >= 0 && n_clouds > 0 && 4 * ns + 1024ll * n_clouds < (1ll << 31) - 1,
                "fgr_radius_grid_workspace: bad arguments");
    RGridWs g;
    carve_rgrid(nullptr, ns, n_clouds, &g);
    *bytes = g.total;
    return FGR_OK;
}

extern "C" int fgr_radius_grid_build(const float* s, const int64_t* s_off, int32_t n_clouds,
                                     int64_t ns, float radius, void* grid, size_t grid_bytes,
                                     void* stream) {
    FGR_REQUIRE(s_off && grid && n_clouds > 0 && ns >= 0 && (s || ns == 0) && radius > 0.f &&
                    4 * ns + 1024ll * n_clouds < (1ll << 31) - 1,
                "fgr_radius_grid_build: bad arguments");
    RGridWs g;
    carve_rgrid(grid, ns, n_clouds, &g);
    if (g.total > grid_bytes) {
        set_error("fgr_radius_grid_build: workspace %zu < %zu bytes", grid_bytes, g.total);
        return FGR_E_WORKSPACE;
    }
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const int64_t cap = 4 * ns + 1024ll * n_clouds;
    hipLaunchKernelGGL(rgrid_bbox_kernel, dim3((unsigned)(n_clouds + ceil_div(cap + 1, 4096))),
                       dim3(1024), 0, st, s, s_off, radius, g.grids, n_clouds, g.start,
                       (int64_t)(cap + 1));
    FGR_CHECK_LAUNCH("rgrid_bbox_kernel");
    if (ns > 0) {
        hipLaunchKernelGGL(rgrid_key_kernel, dim3((unsigned)ceil_div(ns, 256)), dim3(256), 0, st, s,
                           s_off, n_clouds, ns, g.grids, g.start, g.cellof, g.slot);
        FGR_CHECK_LAUNCH("rgrid_key_kernel");
    }
    int rc = launch_scan<false>(g.start, nullptr, nullptr, cap, g.tiles, st);
    if (rc != FGR_OK) return rc;
    if (ns > 0) {
        hipLaunchKernelGGL(rgrid_scatter_kernel, dim3((unsigned)ceil_div(ns, 256)), dim3(256), 0,
                           st, ns, g.cellof, g.slot, g.start, g.members);
        FGR_CHECK_LAUNCH("rgrid_scatter_kernel");
    }
    return FGR_OK;
}

extern "C" int fgr_radius_search_grid(const float* q, const int64_t* q_off, int32_t n_clouds,
                                      int64_t nq, int32_t max_q_len, const float* s,
                                      const int64_t* s_off, int64_t ns, const void* grid,
                                      size_t grid_bytes, float radius, int32_t mode, int32_t width,
                                      int64_t* out, int32_t* counts, int32_t* max_count,
                                      void* stream) {
    FGR_REQUIRE(q_off && s_off && grid && n_clouds > 0 && max_q_len >= 0 && radius > 0.f &&
                    width >= 0 && width <= kRCap && (mode == FGR_NB_INDEX || mode == FGR_NB_DIST),
                "fgr_radius_search_grid: bad arguments (mode %d width %d)", mode, width);
    const bool count_only = counts != nullptr;
    FGR_REQUIRE(count_only ? (max_count != nullptr) : (out || nq == 0 || width == 0),
                "fgr_radius_search_grid: need out (search) or counts + max_count (count)");
    RGridWs g;
    carve_rgrid(const_cast<void*>(grid), ns, n_clouds, &g);
    FGR_REQUIRE(g.total <= grid_bytes, "fgr_radius_search_grid: grid workspace %zu < %zu bytes",
                grid_bytes, g.total);
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    if (count_only) FGR_CHECK_HIP(hipMemsetAsync(max_count, 0, sizeof(int32_t), st));
    if (nq == 0 || max_q_len == 0 || (!count_only && width == 0)) return FGR_OK;
    const float r2 = radius * radius;
    dim3 grd((unsigned)ceil_div(max_q_len, kRQ), (unsigned)n_clouds);
    // a query radius above the build radius would need cells past the 27 scanned: refused on
    // the device side by clamping nothing -- the host checks it (fgreg.ops.RadiusGrid)
    if (count_only)
        hipLaunchKernelGGL((rgrid_query_kernel<0, true>), grd, dim3(64 * kRQ), 0, st, q, q_off, s,
                           s_off, g.grids, g.start, g.members, r2, 0, ns, (int64_t*)nullptr,
                           counts, max_count);
    else if (mode == FGR_NB_INDEX)
        hipLaunchKernelGGL((rgrid_query_kernel<0, false>), grd, dim3(64 * kRQ), 0, st, q, q_off, s,
                           s_off, g.grids, g.start, g.members, r2, width, ns, out,
                           (int*)nullptr, (int*)nullptr);
    else
        hipLaunchKernelGGL((rgrid_query_kernel<1, false>), grd, dim3(64 * kRQ), 0, st, q, q_off, s,
                           s_off, g.grids, g.start, g.members, r2, width, ns, out,
                           (int*)nullptr, (int*)nullptr);
    FGR_CHECK_LAUNCH("rgrid_query_kernel");
    return FGR_OK;
}
