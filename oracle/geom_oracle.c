/* oracle/geom_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded CPU restatement of the KPConv preprocessing
 * geometry (grid subsampling + radius neighbour search). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path never does. It is pinned against the reference's own C++
 * (oracle/_ref/libkpconv_ref.so) through tests/golden/geom_*.npz.
 *
 * Build: gcc -O2 -ffp-contract=off (see oracle/Makefile): no FMA contraction, so
 * every float expression rounds exactly as written, like the reference's x86 build.
 *
 * grid_subsample  restates grid_subsampling.cpp:5-106 (per cloud, :109-211):
 *   origin = floor(min * (1/dl)) * dl                         (:27)
 *   nx = floor((max.x - origin.x)/dl) + 1, ny likewise        (:30-31)
 *   i* = floor((p - origin)/dl);  key = ix + nx*iy + nx*ny*iz (:53-56)
 *   centroid = (sequential float sum of member points) * float(1.0/count) (:87)
 * The reference emits voxels in std::unordered_map iteration order, which is
 * unspecified; this restatement (and the HIP kernel) emit them in ascending key
 * order per cloud. Comparisons against the reference are therefore made as
 * sets keyed by voxel.
 *
 * radius_search restates the two neighbour semantics the reference uses:
 *   mode 0 (INDEX): PyTorch3D ball_query as called by batch_neighbors_kpconv_gpu
 *     (finegrained_kpconv.py:266-293): the first K supports of the same cloud in
 *     index order with d2 < r2, padded to width K with the shadow index Ns_total.
 *   mode 1 (DIST):  nanoflann radiusSearch(sorted=true) as called by
 *     batch_nanoflann_neighbors (neighbors.cpp:211-332) + the python truncation
 *     [:, :K] (finegrained_kpconv.py:260-261): supports sorted by distance, the
 *     K nearest kept, padded with Ns_total; width = min(max_count, K). Exact
 *     distance ties are broken by support index (nanoflann's order among equal
 *     distances is its kd-tree visit order, which is unspecified).
 *   d2 = ((qx-sx)^2 + (qy-sy)^2) + (qz-sz)^2 in float (nanoflann.hpp:433-440,
 *   L2_Simple_Adaptor::evalMetric), r2 = r*r in float (neighbors.cpp:226),
 *   strict d2 < r2 (nanoflann.hpp:249-250).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t key; int idx; } kv_t;

static int cmp_kv(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a;
    const kv_t* y = (const kv_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx - y->idx;
}

/* Pass 1: counts voxels per cloud. Returns the total. */
long long oracle_grid_count(const float* pts, const long long* lens, int ncloud, float dl,
                            long long* out_lens) {
    long long total = 0, off = 0;
    for (int c = 0; c < ncloud; ++c) {
        long long n = lens[c];
        if (n == 0) { out_lens[c] = 0; continue; }
        const float* p = pts + 3 * off;
        float mn[3] = {p[0], p[1], p[2]}, mx[3] = {p[0], p[1], p[2]};
        for (long long i = 0; i < n; ++i)
            for (int d = 0; d < 3; ++d) {
                float v = p[3 * i + d];
                if (v < mn[d]) mn[d] = v;
                if (v > mx[d]) mx[d] = v;
            }
        float inv = 1.0f / dl, org[3];
        for (int d = 0; d < 3; ++d) org[d] = floorf(mn[d] * inv) * dl;
        uint64_t nx = (uint64_t)(int64_t)floorf((mx[0] - org[0]) / dl) + 1;
        uint64_t ny = (uint64_t)(int64_t)floorf((mx[1] - org[1]) / dl) + 1;
        kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)n);
        for (long long i = 0; i < n; ++i) {
            uint64_t ix = (uint64_t)(int64_t)floorf((p[3 * i] - org[0]) / dl);
            uint64_t iy = (uint64_t)(int64_t)floorf((p[3 * i + 1] - org[1]) / dl);
            uint64_t iz = (uint64_t)(int64_t)floorf((p[3 * i + 2] - org[2]) / dl);
            kv[i].key = ix + nx * iy + nx * ny * iz;
            kv[i].idx = (int)i;
        }
        qsort(kv, (size_t)n, sizeof(kv_t), cmp_kv);
        long long m = 0;
        for (long long i = 0; i < n; ++i)
            if (i == 0 || kv[i].key != kv[i - 1].key) ++m;
        free(kv);
        out_lens[c] = m;
        total += m;
        off += n;
    }
    return total;
}

/* Pass 2: writes the barycentres (ascending voxel key per cloud) and, optionally,
 * the voxel keys. */
void oracle_grid_fill(const float* pts, const long long* lens, int ncloud, float dl,
                      float* out_pts, long long* out_keys) {
    long long off = 0, o = 0;
    for (int c = 0; c < ncloud; ++c) {
        long long n = lens[c];
        if (n == 0) continue;
        const float* p = pts + 3 * off;
        float mn[3] = {p[0], p[1], p[2]}, mx[3] = {p[0], p[1], p[2]};
        for (long long i = 0; i < n; ++i)
            for (int d = 0; d < 3; ++d) {
                float v = p[3 * i + d];
                if (v < mn[d]) mn[d] = v;
                if (v > mx[d]) mx[d] = v;
            }
        float inv = 1.0f / dl, org[3];
        for (int d = 0; d < 3; ++d) org[d] = floorf(mn[d] * inv) * dl;
        uint64_t nx = (uint64_t)(int64_t)floorf((mx[0] - org[0]) / dl) + 1;
        uint64_t ny = (uint64_t)(int64_t)floorf((mx[1] - org[1]) / dl) + 1;
        kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)n);
        for (long long i = 0; i < n; ++i) {
            uint64_t ix = (uint64_t)(int64_t)floorf((p[3 * i] - org[0]) / dl);
            uint64_t iy = (uint64_t)(int64_t)floorf((p[3 * i + 1] - org[1]) / dl);
            uint64_t iz = (uint64_t)(int64_t)floorf((p[3 * i + 2] - org[2]) / dl);
            kv[i].key = ix + nx * iy + nx * ny * iz;
            kv[i].idx = (int)i;
        }
        qsort(kv, (size_t)n, sizeof(kv_t), cmp_kv);
        long long i = 0;
        while (i < n) {
            long long j = i;
            float sx = 0.f, sy = 0.f, sz = 0.f;
            while (j < n && kv[j].key == kv[i].key) {
                const float* q = p + 3 * kv[j].idx;   /* members in input order */
                sx += q[0]; sy += q[1]; sz += q[2];
                ++j;
            }
            float s = (float)(1.0 / (double)(j - i));
            out_pts[3 * o] = sx * s;
            out_pts[3 * o + 1] = sy * s;
            out_pts[3 * o + 2] = sz * s;
            if (out_keys) out_keys[o] = (long long)kv[i].key;
            ++o;
            i = j;
        }
        free(kv);
        off += n;
    }
}

typedef struct { float d2; int idx; } cand_t;

static int cmp_cand(const void* a, const void* b) {
    const cand_t* x = (const cand_t*)a;
    const cand_t* y = (const cand_t*)b;
    if (x->d2 != y->d2) return x->d2 < y->d2 ? -1 : 1;
    return x->idx - y->idx;
}

/* Uncapped counts: out_counts[q] = #{s in cloud(q): d2 < r2}. Returns max count. */
long long oracle_radius_count(const float* q, const long long* qlens, const float* s,
                              const long long* slens, int ncloud, float radius,
                              long long* out_counts) {
    float r2 = radius * radius;
    long long qo = 0, so = 0, mx = 0;
    for (int c = 0; c < ncloud; ++c) {
        for (long long i = 0; i < qlens[c]; ++i) {
            const float* a = q + 3 * (qo + i);
            long long cnt = 0;
            for (long long j = 0; j < slens[c]; ++j) {
                const float* b = s + 3 * (so + j);
                float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
                float d2 = dx * dx;
                d2 = d2 + dy * dy;
                d2 = d2 + dz * dz;
                if (d2 < r2) ++cnt;
            }
            out_counts[qo + i] = cnt;
            if (cnt > mx) mx = cnt;
        }
        qo += qlens[c];
        so += slens[c];
    }
    return mx;
}

/* Fills out[Nq_total * width] (int64). mode 0 = INDEX, 1 = DIST. */
void oracle_radius_fill(const float* q, const long long* qlens, const float* s,
                        const long long* slens, int ncloud, float radius, int mode,
                        int width, long long* out) {
    float r2 = radius * radius;
    long long qo = 0, so = 0, ns_total = 0;
    for (int c = 0; c < ncloud; ++c) ns_total += slens[c];
    long long maxs = 0;
    for (int c = 0; c < ncloud; ++c) if (slens[c] > maxs) maxs = slens[c];
    cand_t* cand = (cand_t*)malloc(sizeof(cand_t) * (size_t)(maxs > 0 ? maxs : 1));
    for (int c = 0; c < ncloud; ++c) {
        for (long long i = 0; i < qlens[c]; ++i) {
            const float* a = q + 3 * (qo + i);
            int cnt = 0;
            for (long long j = 0; j < slens[c]; ++j) {
                const float* b = s + 3 * (so + j);
                float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
                float d2 = dx * dx;
                d2 = d2 + dy * dy;
                d2 = d2 + dz * dz;
                if (d2 < r2) { cand[cnt].d2 = d2; cand[cnt].idx = (int)j; ++cnt; }
            }
            if (mode == 1) qsort(cand, (size_t)cnt, sizeof(cand_t), cmp_cand);
            long long* row = out + (qo + i) * (long long)width;
            for (int k = 0; k < width; ++k)
                row[k] = k < cnt ? so + cand[k].idx : ns_total;
        }
        qo += qlens[c];
        so += slens[c];
    }
    free(cand);
}
