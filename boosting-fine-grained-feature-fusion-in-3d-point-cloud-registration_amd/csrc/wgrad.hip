// Weight-gradient GEMM of the training backward (loss.backward() of
// trainer.py:110-125 through every nn.Linear / KPConv weight, dW = dY^T X):
//   dw[i][j] = sum_r dy[r][i] * x[r][j]          (i < m, j < n, r < rows)
// read straight from the two row-major activations: no transposed copy of dY and no split
// operand image of X (the generic GEMM path needs both: three extra launches and two extra
// passes over the activations per Linear).
//
// One 256-thread workgroup per (128 x 128 output tile, chunk of rows), one pass over the
// chunk: every 32-row k-step is scaled per column by a running power of two (the largest
// |value| seen so far in [2^14, 2^15); when a k-step raises a column's maximum the exponent
// drops and the accumulated products are rescaled by the exact power of two -- the dynamic
// row scaling of the g5 GEMM, here on the contraction's columns), split into two fp16 terms
// (h = f16(s x), m = f16(s x - h)) straight into LDS in MFMA fragment order (per column, 32 k
// contiguous, 80-B pitch: conflict-free ds_read_b128), and the three products mh + hm + hh
// accumulate in fp32 on mfma_f32_16x16x32_f16. The four row groups of a column quad sit in one
// wave, so a k-step's column maxima are two lane shuffles. The four waves each own a 64 x 64
// quarter (4 x 4 fragments); one set of LDS images (40 KB: three workgroups per CU hide each
// other's barriers), the next k-step's global loads in flight during the matrix-core work.
// With more than one chunk the tiles are fp32 partials that wgrad_reduce_kernel sums in
// chunk order: deterministic, no atomics. With a bias gradient the tile column j0 = 0 also
// sums its dy columns in fp64 (db = sum_r dy[r][i]), partials per chunk summed in the same
// reduce launch: the separate column-sum pass goes away. (Round 5: a pre-pass of per-chunk
// column maxima read every chunk twice: 1141 -> 938 us over the 13 training shapes,
// profiles/r05_wgrad_shapes.txt.)
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kWgT = 128;                  // output tile edge
constexpr int kWgK = 32;                   // rows per k-step
constexpr int kWgPitch = 40;               // halves per image column: 32 k + 8 pad (80 B)
constexpr int kWgImg = kWgT * kWgPitch;    // halves per (operand, term) image

struct WgradArgs {
    const float* dy;
    int64_t ldy;
    const float* x;
    int64_t ldx;
    int64_t rows;
    int m, n;
    int64_t kc;        // rows per chunk (multiple of kWgK)
    int tiles_n;       // ceil(n / 128)
    float* out;        // one chunk: the result, row stride ldo
    int64_t ldo;
    float* part;       // several chunks: partial tiles [chunk][m][n]
    float* db;         // optional: db[i] = sum_r dy[r][i] (the bias gradient)
    double* part_db;   // several chunks: its partials [chunk][m]
};

__device__ __forceinline__ int wg_scale_exp(float mx) {
    return mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
}

// one register set of k-step rows (the next k-step's loads in flight during the matrix-core
// work; 166 VGPRs = 3 workgroups per CU -- a second set spilled or cost the occupancy)
__global__ void __launch_bounds__(256, 3) wgrad_f16x3_kernel(WgradArgs p) {
    __shared__ _Float16 img[2][2][kWgImg];         // [operand][term]: 40 KB (3 workgroups / CU)
    __shared__ int edel[2][kWgT];                  // per operand column: this k-step's exponent change
    __shared__ int eend[2][kWgT];                  // per operand column: the final exponent
    __shared__ int chg[2];                         // any exponent change at k-step parity
    __shared__ double bred[4][kWgT];               // bias partial sums per row group
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, g = lane >> 4, c = lane & 15;
    const int ti = blockIdx.x / p.tiles_n, tj = blockIdx.x % p.tiles_n;
    const int i0 = ti * kWgT, j0 = tj * kWgT;
    const int64_t rb = (int64_t)blockIdx.y * p.kc;
    const int64_t re = min(p.rows, rb + p.kc);
    // thread -> (operand, column quad, row group of 8): waves 0-1 read dy, 2-3 x; in a wave
    // lanes 16 kg + c4l, so the 4 row groups of a column quad sit in one wave (the column
    // maxima of a k-step are two lane shuffles, no LDS round)
    const int op = tid >> 7, kg = lane >> 4, c4 = ((tid >> 6) & 1) * 16 + (lane & 15);
    const int64_t ld = op ? p.ldx : p.ldy;
    const int lim = op ? p.n : p.m;
    const int col0 = (op ? j0 : i0) + 4 * c4;      // first of this thread's 4 columns
    const bool cok = col0 < lim;                   // lim % 4 == 0: all four or none
    const float* base = (op ? p.x : p.dy) + (cok ? col0 : 0);
    const bool bias_sums = p.db && op == 0 && tj == 0;
    if (bias_sums) {
#pragma unroll
        for (int q = 0; q < 4; ++q) bred[kg][4 * c4 + q] = 0.0;
    }
    // running column exponents: the scale 2^e keeps the largest |value| seen so far in
    // [2^14, 2^15); when a k-step raises a column's maximum the exponent drops and the
    // accumulated products are rescaled by the (exact) power of two -- one pass over the data
    int ecur[4] = {127, 127, 127, 127};
    if (tid < 2) chg[tid] = 0;

    const int nk = (int)((re - rb + kWgK - 1) / kWgK);
    float va[8][4];
    auto load = [&](float (&v)[8][4], int ks) {
        const int64_t r0 = rb + (int64_t)ks * kWgK + 8 * kg;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int64_t rr = r0 + e;
            const float4 t = *reinterpret_cast<const float4*>(base + min(rr, re - 1) * ld);
            const bool ok = rr < re && cok;
            v[e][0] = ok ? t.x : 0.f;
            v[e][1] = ok ? t.y : 0.f;
            v[e][2] = ok ? t.z : 0.f;
            v[e][3] = ok ? t.w : 0.f;
        }
    };
    // exponents of this k-step, then the split images (and the bias sums)
    auto store = [&](const float (&v)[8][4], int par) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float m = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e][q]));
            m = fmaxf(m, __shfl_xor(m, 16, 64));
            m = fmaxf(m, __shfl_xor(m, 32, 64));
            const int en = m > 0.f ? min(ecur[q], wg_scale_exp(m)) : ecur[q];
            if (kg == 0) edel[op][4 * c4 + q] = en - ecur[q];
            if (en != ecur[q]) chg[par] = 1;
            ecur[q] = en;
            const float sc = __builtin_ldexpf(1.f, en);
            f16x8 th, tm;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float xs = v[e][q] * sc;
                const _Float16 hh = (_Float16)xs;
                th[e] = hh;
                tm[e] = (_Float16)(xs - (float)hh);
            }
            const int o = (4 * c4 + q) * kWgPitch + 8 * kg;
            *reinterpret_cast<u32x4*>(&img[op][0][o]) = __builtin_bit_cast(u32x4, th);
            *reinterpret_cast<u32x4*>(&img[op][1][o]) = __builtin_bit_cast(u32x4, tm);
        }
        if (bias_sums) {                           // fp64 running sums in this thread's LDS slots
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float t = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) t += v[e][q];
                bred[kg][4 * c4 + q] += (double)t;
            }
        }
    };

    const int wi = wv & 1, wj = wv >> 1;
    f32x4 acc[4][4];
#pragma unroll
    for (int fi = 0; fi < 4; ++fi)
#pragma unroll
        for (int fj = 0; fj < 4; ++fj) acc[fi][fj] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mfma_step = [&](int par) {
        if (chg[par]) {                            // block-uniform: rescale to the new exponents
            float fb[4];
#pragma unroll
            for (int fj = 0; fj < 4; ++fj) fb[fj] = __builtin_ldexpf(1.f, edel[1][64 * wj + 16 * fj + c]);
#pragma unroll
            for (int fi = 0; fi < 4; ++fi)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float fa = __builtin_ldexpf(1.f, edel[0][64 * wi + 16 * fi + 4 * g + r]);
#pragma unroll
                    for (int fj = 0; fj < 4; ++fj) acc[fi][fj][r] *= fa * fb[fj];
                }
        }
        f16x8 bh[4], bm[4];
#pragma unroll
        for (int fj = 0; fj < 4; ++fj) {
            const int o = (64 * wj + 16 * fj + c) * kWgPitch + 8 * g;
            bh[fj] = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4*>(&img[1][0][o]));
            bm[fj] = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4*>(&img[1][1][o]));
        }
#pragma unroll
        for (int fi = 0; fi < 4; ++fi) {
            const int o = (64 * wi + 16 * fi + c) * kWgPitch + 8 * g;
            const f16x8 ah = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4*>(&img[0][0][o]));
            const f16x8 am = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4*>(&img[0][1][o]));
#pragma unroll
            for (int fj = 0; fj < 4; ++fj) {
                acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(am, bh[fj], acc[fi][fj], 0, 0, 0);
                acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bm[fj], acc[fi][fj], 0, 0, 0);
                acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[fj], acc[fi][fj], 0, 0, 0);
            }
        }
    };
    load(va, 0);
    for (int ks = 0; ks < nk; ++ks) {
        const int par = ks & 1;
        // every wave is done with the last images, edel and chg[par ^ 1] (ks = 0: chg zeroed)
        __syncthreads();
        if (tid == 0) chg[par ^ 1] = 0;
        store(va, par);
        if (ks + 1 < nk) load(va, ks + 1);
        __syncthreads();
        mfma_step(par);
    }
    if (kg == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) eend[op][4 * c4 + q] = ecur[q];
    }
    if (p.db && tj == 0) {                         // (block-uniform) fold the 4 row groups
        __syncthreads();
        if (tid < kWgT && i0 + tid < p.m) {
            const double t = ((bred[0][tid] + bred[1][tid]) + bred[2][tid]) + bred[3][tid];
            if (p.part_db)
                p.part_db[(int64_t)blockIdx.y * p.m + i0 + tid] = t;
            else
                p.db[i0 + tid] = (float)t;
        }
    }
    __syncthreads();
    // epilogue: lane (g, c) holds D[64 wi + 16 fi + 4 g + r][64 wj + 16 fj + c]; both
    // inverse scales are powers of two (exact)
    float* dst;
    int64_t ldd;
    if (p.part) {
        dst = p.part + (int64_t)blockIdx.y * p.m * p.n;
        ldd = p.n;
    } else {
        dst = p.out;
        ldd = p.ldo;
    }
    float jb[4];
#pragma unroll
    for (int fj = 0; fj < 4; ++fj) jb[fj] = __builtin_ldexpf(1.f, -eend[1][64 * wj + 16 * fj + c]);
#pragma unroll
    for (int fi = 0; fi < 4; ++fi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int il = 64 * wi + 16 * fi + 4 * g + r;
            const int i = i0 + il;
            const float ia = __builtin_ldexpf(1.f, -eend[0][il]);
#pragma unroll
            for (int fj = 0; fj < 4; ++fj) {
                const int j = j0 + 64 * wj + 16 * fj + c;
                if (i < p.m && j < p.n) dst[(int64_t)i * ldd + j] = acc[fi][fj][r] * ia * jb[fj];
            }
        }
}

// out[i][j] = the sum over chunks of part[chunk][i][j]: a block takes 32 float4 outputs, its
// 8 thread rows the chunks congruent to their row mod 8 (consecutive threads read consecutive
// float4s of one chunk), the 8 partial sums combined in row order -- a fixed order, so the
// result is deterministic. Blocks past the tile items sum the bias partials (fp64) the same way.
constexpr int kRdQ = 32, kRdL = 8;
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ part, int chunks,
                                                           int m, int n, float* __restrict__ out,
                                                           int64_t ldo, const double* __restrict__ part_db,
                                                           float* __restrict__ db) {
    const int tq = threadIdx.x % kRdQ, tl = threadIdx.x / kRdQ;
    const int64_t mn4 = (int64_t)m * n / 4;
    const int64_t tile_blocks = (mn4 + kRdQ - 1) / kRdQ;
    if ((int64_t)blockIdx.x >= tile_blocks) {      // the bias gradient
        __shared__ double sd[kRdL][kRdQ];
        const int64_t i = ((int64_t)blockIdx.x - tile_blocks) * kRdQ + tq;
        double t = 0.0;
        if (db && i < m)
            for (int ch = tl; ch < chunks; ch += kRdL) t += part_db[(int64_t)ch * m + i];
        sd[tl][tq] = t;
        __syncthreads();
        if (tl == 0 && db && i < m) {
            double u = 0.0;
#pragma unroll
            for (int l = 0; l < kRdL; ++l) u += sd[l][tq];
            db[i] = (float)u;
        }
        return;
    }
    const int64_t q = (int64_t)blockIdx.x * kRdQ + tq;
    const int64_t qc = q < mn4 ? q : mn4 - 1;
    const float4* p4 = reinterpret_cast<const float4*>(part);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int ch = tl;
    for (; ch + 3 * kRdL < chunks; ch += 4 * kRdL) {
        float4 t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = p4[(int64_t)(ch + u * kRdL) * mn4 + qc];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            s.x += t[u].x; s.y += t[u].y; s.z += t[u].z; s.w += t[u].w;
        }
    }
    for (; ch < chunks; ch += kRdL) {
        const float4 t = p4[(int64_t)ch * mn4 + qc];
        s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    __shared__ float4 sf[kRdL][kRdQ];
    sf[tl][tq] = s;
    __syncthreads();
    if (tl == 0 && q < mn4) {
        float4 u = sf[0][tq];
#pragma unroll
        for (int l = 1; l < kRdL; ++l) {
            const float4 t = sf[l][tq];
            u.x += t.x; u.y += t.y; u.z += t.z; u.w += t.w;
        }
        const int64_t e = 4 * q;
        const int64_t i = e / n, j = e - i * n;
        *reinterpret_cast<float4*>(out + i * ldo + j) = u;
    }
}

// chunks of rows per output tile: about two workgroups per CU (512) over the tiles, at least
// 32 rows each, and no more partial bytes than the two operands' bytes
struct WgradPlan {
    int64_t kc;
    int chunks;
    int tiles;
    int tiles_n;
};

WgradPlan wgrad_plan(int64_t rows, int m, int n) {
    static const int64_t target = [] {           // FGR_WGRAD_WGS: workgroup target (A/B)
        const char* e = getenv("FGR_WGRAD_WGS");
        return (int64_t)(e ? std::max(1, atoi(e)) : 512);
    }();
    WgradPlan pl;
    pl.tiles_n = (int)ceil_div(n, kWgT);
    pl.tiles = (int)ceil_div(m, kWgT) * pl.tiles_n;
    static const double part_ratio = [] {       // FGR_WGRAD_PART: partial / operand bytes cap
        const char* e = getenv("FGR_WGRAD_PART");
        return e ? std::max(0.01, atof(e)) : 1.0;
    }();
    int64_t ch = ceil_div(target, pl.tiles);
    ch = std::min(ch, std::max<int64_t>(1, (int64_t)(part_ratio * (double)(rows * (m + n)) /
                                                     ((double)m * n))));
    ch = std::max<int64_t>(1, std::min(ch, ceil_div(rows, kWgK)));
    pl.kc = std::max<int64_t>(kWgK, ceil_div(ceil_div(rows, ch), kWgK) * kWgK);
    pl.chunks = (int)std::max<int64_t>(1, ceil_div(rows, pl.kc));
    return pl;
}

}  // namespace
}  // namespace fgr

using namespace fgr;

static size_t wgrad_ws_bytes(const WgradPlan& pl, int m, int n, bool bias) {
    if (pl.chunks <= 1) return 0;
    return (size_t)pl.chunks * m * n * sizeof(float) + (bias ? (size_t)pl.chunks * m * sizeof(double) : 0);
}

extern "C" int fgr_gemm_wgrad_workspace(int64_t rows, int32_t m, int32_t n, int32_t with_bias,
                                        size_t* bytes) {
    FGR_REQUIRE(bytes && rows >= 0 && m > 0 && n > 0, "fgr_gemm_wgrad_workspace: bad arguments");
    *bytes = 0;
    if (rows == 0) return FGR_OK;
    *bytes = wgrad_ws_bytes(wgrad_plan(rows, m, n), m, n, with_bias != 0);
    return FGR_OK;
}

extern "C" int fgr_gemm_f16x3_wgrad(const float* dy, int64_t ld_dy, const float* x, int64_t ld_x,
                                    int64_t rows, int32_t m, int32_t n, float* dw, int64_t ld_dw,
                                    float* db, void* ws, size_t ws_bytes, void* stream) {
    FGR_REQUIRE(rows >= 0 && m > 0 && n > 0 && m % 4 == 0 && n % 4 == 0,
                "fgr_gemm_f16x3_wgrad: m, n must be positive multiples of 4 (got %d, %d)", m, n);
    FGR_REQUIRE(ld_dy >= m && ld_x >= n && ld_dw >= n && ld_dy % 4 == 0 && ld_x % 4 == 0 &&
                    ld_dw % 4 == 0,
                "fgr_gemm_f16x3_wgrad: row strides must cover the rows and be multiples of 4");
    FGR_REQUIRE(dw && (rows == 0 || (dy && x)), "fgr_gemm_f16x3_wgrad: null pointer");
    FGR_REQUIRE(((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) |
                  reinterpret_cast<uintptr_t>(dw)) & 15) == 0,
                "fgr_gemm_f16x3_wgrad: dy / x / dw must be 16-B aligned");
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    if (rows == 0) {
        FGR_CHECK_HIP(hipMemset2DAsync(dw, (size_t)ld_dw * sizeof(float), 0, (size_t)n * sizeof(float),
                                       (size_t)m, st));
        if (db) FGR_CHECK_HIP(hipMemsetAsync(db, 0, (size_t)m * sizeof(float), st));
        return FGR_OK;
    }
    const WgradPlan pl = wgrad_plan(rows, m, n);
    const size_t need = wgrad_ws_bytes(pl, m, n, db != nullptr);
    FGR_REQUIRE(ws_bytes >= need && (need == 0 || (ws && (reinterpret_cast<uintptr_t>(ws) & 15) == 0)),
                "fgr_gemm_f16x3_wgrad: workspace of %zu bytes (16-B aligned) needed", need);
    float* part = pl.chunks > 1 ? static_cast<float*>(ws) : nullptr;
    double* part_db = part && db ? reinterpret_cast<double*>(part + (size_t)pl.chunks * m * n) : nullptr;
    WgradArgs a{dy, ld_dy, x, ld_x, rows, m, n, pl.kc, pl.tiles_n, dw, ld_dw, part, db, part_db};
    hipLaunchKernelGGL(wgrad_f16x3_kernel, dim3((unsigned)pl.tiles, (unsigned)pl.chunks), dim3(256), 0, st, a);
    FGR_CHECK_LAUNCH("wgrad_f16x3_kernel");
    if (pl.chunks > 1) {
        const int64_t blocks = ceil_div((int64_t)m * n / 4, kRdQ) + (db ? ceil_div(m, kRdQ) : 0);
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(kRdQ * kRdL), 0, st,
                           static_cast<const float*>(ws), pl.chunks, m, n, dw, ld_dw,
                           static_cast<const double*>(part_db), db);
        FGR_CHECK_LAUNCH("wgrad_reduce_kernel");
    }
    return FGR_OK;
}
