// oracle/ref_shim.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
//
// A tiny extern "C" adaptor written for this repo that calls the reference's
// own KPConv preprocessing algorithms, compiled unmodified from their sources
// under /root/reference (see oracle/Makefile):
//   batch_nanoflann_neighbors  models/backbone_kpconv/cpp_wrappers/cpp_neighbors/neighbors/neighbors.cpp:211-332
//   batch_grid_subsampling     models/backbone_kpconv/cpp_wrappers/cpp_subsampling/grid_subsampling/grid_subsampling.cpp:109-211
// It replaces the reference's CPython/NumPy-1 wrapper (cpp_*/wrapper.cpp), which
// is not used: arguments arrive as plain pointers from ctypes instead.
#include <cstring>
#include <vector>
#include "neighbors/neighbors.h"
#include "grid_subsampling/grid_subsampling.h"

static std::vector<int> g_last_nb;          // result of the last neighbour query
static std::vector<PointXYZ> g_last_pts;    // result of the last subsampling
static std::vector<int> g_last_lens;

extern "C" {

// Runs the reference radius search (nanoflann, sorted by distance, padded with
// Ns_total). Returns max_count (row width); fetch rows with ref_neighbors_fetch.
int ref_neighbors_run(const float* q, int nq, const float* s, int ns,
                      const int* qb, const int* sb, int nb, float radius) {
    std::vector<PointXYZ> queries((const PointXYZ*)q, (const PointXYZ*)q + nq);
    std::vector<PointXYZ> supports((const PointXYZ*)s, (const PointXYZ*)s + ns);
    std::vector<int> q_batches(qb, qb + nb), s_batches(sb, sb + nb);
    g_last_nb.clear();
    batch_nanoflann_neighbors(queries, supports, q_batches, s_batches, g_last_nb, radius);
    return nq > 0 ? (int)(g_last_nb.size() / nq) : 0;
}

void ref_neighbors_fetch(int* out) {
    std::memcpy(out, g_last_nb.data(), g_last_nb.size() * sizeof(int));
}

// Runs the reference barycentre grid subsampling. Returns total output points.
int ref_subsample_run(const float* p, int n, const int* lens, int nb, float dl) {
    std::vector<PointXYZ> pts((const PointXYZ*)p, (const PointXYZ*)p + n);
    std::vector<float> of, sf;
    std::vector<int> oc, sc;
    std::vector<int> ob(lens, lens + nb);
    g_last_pts.clear();
    g_last_lens.clear();
    batch_grid_subsampling(pts, g_last_pts, of, sf, oc, sc, ob, g_last_lens, dl, 0);
    return (int)g_last_pts.size();
}

void ref_subsample_fetch(float* out_pts, int* out_lens) {
    std::memcpy(out_pts, g_last_pts.data(), g_last_pts.size() * sizeof(PointXYZ));
    std::memcpy(out_lens, g_last_lens.data(), g_last_lens.size() * sizeof(int));
}

}  // extern "C"
