// Fused Res2Net hierarchy (the "fine-grained feature fusion" of my_Bottle2neck,
// res2net.py:126-148) on the split matrix cores.
//
// Given h = ReLU(BN1(conv1(x))) split into `scale` chunks of width w, computes in one
// launch, for i < nums (= scale - 1):
//   sp_i = ReLU(BN_i(conv_i(sp_{i-1} + h_i)))      (sp_{-1} = 0)
// with BN folded into (W_i, b_i) on the host, and writes the concatenation input of
// conv3 + downsample: cat = [sp_0 .. sp_{nums-1} | h_{nums..scale-1} | x].
// The reference runs this as 7 dependent (Linear, BN, ReLU) triples plus adds and a
// cat (21+ launches over HBM); here sp never leaves the chip between steps.
// Two fp32-accurate variants: fgr_res2net_chain6 (three exact bf16 terms, six products;
// w = 112, 224 -- dispatched at w = 224, where it measured faster) and fgr_res2net_chain_h3
// (scaled split fp16, three products; w % 4 == 0 up to 224).
#include "common.h"

namespace fgr {
namespace {

// dst[r0 + row][0..cols) = src[r0 + row][0..cols) for row < rows (rows past n skipped): the
// concatenation tail of the chain kernels. 16-B accesses when every row start is 16-B aligned,
// kCpU of them in flight per thread: every load unconditional (element index and row clamped
// to valid ones, the store masked) -- round 5: guarded loads had put the staging array in
// scratch with a vmcnt(0) wait after each load, one memory round trip per float4
constexpr int kCpU = 8;
__device__ __forceinline__ void copy_rows(float* __restrict__ dst, int64_t ldd,
                                          const float* __restrict__ src, int64_t lds, int64_t r0,
                                          int rows, int64_t n, int cols, int tid, int nth) {
    const bool v4 = ((cols | (int)(ldd & 3) | (int)(lds & 3)) & 3) == 0 &&
                    ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
    if (v4) {
        const int c4 = cols / 4;
        const int nr = (int)min<int64_t>(rows, n - r0);   // rows of this block below n
        if (nr <= 0 || c4 == 0) return;
        const int tot = nr * c4;
        for (int e0 = tid; e0 < tot; e0 += kCpU * nth) {
            float4 v[kCpU];
#pragma unroll
            for (int u = 0; u < kCpU; ++u) {
                const int e = min(e0 + u * nth, tot - 1);
                const int row = e / c4, cc = (e - row * c4) * 4;
                v[u] = *reinterpret_cast<const float4*>(src + (r0 + row) * lds + cc);
            }
#pragma unroll
            for (int u = 0; u < kCpU; ++u) {
                const int e = e0 + u * nth;
                if (e < tot) {
                    const int row = e / c4, cc = (e - row * c4) * 4;
                    *reinterpret_cast<float4*>(dst + (r0 + row) * ldd + cc) = v[u];
                }
            }
        }
        return;
    }
    for (int e = tid; e < rows * cols; e += nth) {
        const int row = e / cols, cc = e - row * cols;
        if (r0 + row < n) dst[(r0 + row) * ldd + cc] = src[(r0 + row) * lds + cc];
    }
}


using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kRows = 32;

// ------------------------------------------------------------------------------------
// bf16x6 variant (fp32-accurate): the hierarchy on the bf16 matrix cores, every fp32 value
// split exactly into three bf16 terms h + m + l (residual <= 2^-27 |x|), the six products
// hh + hm + mh + hl + lh + mm accumulated in fp32. Per step the A operand
// a = sp_{i-1} + h_i is formed in fp32, split and stored as fragment-ordered LDS images
//   img[t][ks][g][row] (16-B units: row, k = 32 ks + 8 g .. + 7),
// read with conflict-free ds_read_b128; sp_i stays in an fp32 LDS tile between steps.
// W_i comes pre-split from the host in fragment order [i][jt][ks][t][g][c][8] (1 KB per
// wave-load), streamed two k-steps ahead. K is padded to a multiple of 32 (w = 112 -> 128)
// with zero weights and zero A columns. 2 barriers per step (build | MFMA + epilogue).
// ------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

// R rows per block (16, 32 or 48: R / 16 row fragments per wave; 48 puts ModelNet's 9544
// rows in 199 blocks -- one round of one 14-wave block per CU -- instead of 256 + 43, 16
// spreads 3DMatch's ~2k rows over twice the CUs)
template <int KT, int R = kRows>   // KT = w / 16 column tiles (= waves); KS = ceil(w / 32) k-steps
__global__ void __launch_bounds__(64 * KT)
res2net_chain6_kernel(const float* __restrict__ h, int64_t n, int scale, int nums,
                      const u32x4* __restrict__ wf, const float* __restrict__ bias,
                      const float* __restrict__ x, int cin, float* __restrict__ cat, int64_t ld) {
    constexpr int W = 16 * KT, KS = (W + 31) / 32, NU = R * KS * 4;   // A units per term
    // sp rows padded to W + 4 floats: at a stride of W (a multiple of 32 floats here) the
    // build's reads -- consecutive lanes on consecutive rows -- hit 2-4 of the 64 LDS banks
    // (16-32-way conflicts); at W + 4 the 16-B reads of a wave spread over all of them
    constexpr int SPW = W + 4;
    __shared__ u32x4 img[3 * NU];
    __shared__ float sp[R * SPW];
    const int tid = threadIdx.x, nth = 64 * KT;
    const int wv = tid / 64, lane = tid % 64, g = lane >> 4, c = lane & 15;
    const int64_t r0 = (int64_t)blockIdx.x * R;
    const int64_t hw = (int64_t)scale * W;
    const int col = wv * 16 + c;

    for (int i = 0; i < nums; ++i) {
        const u32x4* wb = wf + (((int64_t)i * KT + wv) * KS) * 192 + lane;
        u32x4 bq[3][3];                                // ring: k-steps ks, ks+1, ks+2
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (q < KS) {
#pragma unroll
                for (int t = 0; t < 3; ++t) bq[q][t] = wb[(q * 3 + t) * 64];
            }
        const float bc = bias[i * W + col];
        // build the split A images: unit u -> (row = u % 32, kg = u / 32), 8 k each
        for (int u = tid; u < NU; u += nth) {
            const int row = u % R, kg = u / R;       // kg = 4 ks + g'
            const int k0 = 8 * kg;
            float a[8];
            const int64_t gr = r0 + row;
#pragma unroll
            for (int e = 0; e < 8; e += 4) {
                float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (gr < n && k0 + e < W)
                    hv = *reinterpret_cast<const float4*>(h + gr * hw + (int64_t)i * W + k0 + e);
                a[e] = hv.x; a[e + 1] = hv.y; a[e + 2] = hv.z; a[e + 3] = hv.w;
            }
            if (i > 0 && k0 < W) {                      // k0 + 8 <= W: W % 16 == 0
                const float4 s0 = *reinterpret_cast<const float4*>(sp + row * SPW + k0);
                const float4 s1 = *reinterpret_cast<const float4*>(sp + row * SPW + k0 + 4);
                a[0] += s0.x; a[1] += s0.y; a[2] += s0.z; a[3] += s0.w;
                a[4] += s1.x; a[5] += s1.y; a[6] += s1.z; a[7] += s1.w;
            }
            bf16x8 th, tm, tl;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                __bf16 hh, mm, ll;
                split3(a[e], hh, mm, ll);
                th[e] = hh; tm[e] = mm; tl[e] = ll;
            }
            img[0 * NU + kg * R + row] = __builtin_bit_cast(u32x4, th);
            img[1 * NU + kg * R + row] = __builtin_bit_cast(u32x4, tm);
            img[2 * NU + kg * R + row] = __builtin_bit_cast(u32x4, tl);
        }
        __syncthreads();
        constexpr int RF = R / 16;
        f32x4 acc[RF];
#pragma unroll
        for (int f = 0; f < RF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ks + 2 < KS) {
#pragma unroll
                for (int t = 0; t < 3; ++t) bq[(ks + 2) % 3][t] = wb[((ks + 2) * 3 + t) * 64];
            }
            const bf16x8 bh = __builtin_bit_cast(bf16x8, bq[ks % 3][0]);
            const bf16x8 bm = __builtin_bit_cast(bf16x8, bq[ks % 3][1]);
            const bf16x8 bl = __builtin_bit_cast(bf16x8, bq[ks % 3][2]);
            const int base = (ks * 4 + g) * R;
            bf16x8 ah[RF], am[RF], al[RF];
#pragma unroll
            for (int f = 0; f < RF; ++f) {
                ah[f] = __builtin_bit_cast(bf16x8, img[0 * NU + base + 16 * f + c]);
                am[f] = __builtin_bit_cast(bf16x8, img[1 * NU + base + 16 * f + c]);
                al[f] = __builtin_bit_cast(bf16x8, img[2 * NU + base + 16 * f + c]);
            }
            // the six products of three-term bf16 splits, smallest first
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[f], bm, acc[f], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[f], bh, acc[f], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f], bl, acc[f], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[f], bh, acc[f], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f], bm, acc[f], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f], bh, acc[f], 0, 0, 0);
        }
        // epilogue: sp_i -> cat and the fp32 LDS tile (read by the next step's build,
        // which starts after the barrier below)
#pragma unroll
        for (int rg = 0; rg < RF; ++rg) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = rg * 16 + 4 * g + r;
                const float y = fmaxf(acc[rg][r] + bc, 0.f);
                if (r0 + row < n) cat[(r0 + row) * ld + (int64_t)i * W + col] = y;
                sp[row * SPW + col] = y;
            }
        }
        __syncthreads();
    }
    copy_rows(cat + (int64_t)nums * W, ld, h + (int64_t)nums * W, hw, r0, R, n,
              (scale - nums) * W, tid, nth);
    if (x) copy_rows(cat + hw, ld, x, cin, r0, R, n, cin, tid, nth);
}

// ------------------------------------------------------------------------------------
// f16x3 variant (scaled two-term fp16 splits, see gemm16.hip): the same hierarchy at half
// the matrix-core work of bf16x6. Swapped products (C^T = W a^T: W_i fragments as the A
// operand, activation rows as the B operand) so each lane owns ONE activation row and
// four output columns. Each step forms a = sp_{i-1} + h_i for the block's 32 rows, takes
// the row max (LDS atomics: the whole row is on chip, so the scale is exact per row, no
// online rescaling), scales the row by 2^e (max in [2^14, 2^15)) and splits it into fp16
// (h, m) images img[t][ks][g][row]; W_i rows come pre-scaled per output column with their
// inverse scales wsc[i][col] (fgreg.ops.res2net_fragments_h3).
// ------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// R rows per block (32, or 48 at w = 224 when that saves a round of blocks, as in chain6).
// Each step issues the whole step's W_i fragments (KS x 2 per lane) before the build, so the
// matrix-core loop never waits on L2; rmax is double-buffered (reset in the previous step's
// epilogue): 3 barriers per step.
template <int KT, int R = kRows>
__global__ void __launch_bounds__(64 * KT)
res2net_chain_h3_kernel(const float* __restrict__ h, int64_t n, int w, int scale, int nums,
                        const u32x4* __restrict__ wf, const float* __restrict__ wsc,
                        const float* __restrict__ bias, const float* __restrict__ x, int cin,
                        float* __restrict__ cat, int64_t ld) {
    // W = the width padded to whole 16-column tiles (one wave each); w <= W the real width
    // (w % 4 == 0): columns past w carry zero weights and are never stored
    constexpr int W = 16 * KT, KS = (W + 31) / 32, NU = R * KS * 4;       // A units per term
    constexpr int IT = (NU + 64 * KT - 1) / (64 * KT);                    // build units / thread
    constexpr int RF = R / 16;                                            // row fragments
    constexpr int SPW = W + 4;                 // padded sp rows (bank spread, as in chain6)
    __shared__ u32x4 img[2 * NU];
    __shared__ float sp[R * SPW];
    __shared__ int rmax[2][R];
    const int tid = threadIdx.x, nth = 64 * KT;
    const int wv = tid / 64, lane = tid % 64, g = lane >> 4, c = lane & 15;
    const int64_t r0 = (int64_t)blockIdx.x * R;
    const int64_t hw = (int64_t)scale * w;
    const int col0 = wv * 16 + 4 * g;                  // this lane's 4 output columns
    const bool col_ok = col0 < w;
    if (tid < R) rmax[0][tid] = 0;
    __syncthreads();

    for (int i = 0; i < nums; ++i) {
        int* rm = rmax[i & 1];
        const u32x4* wb = wf + (((int64_t)i * KT + wv) * KS) * 128 + lane;
        u32x4 bq[KS][2];
#pragma unroll
        for (int q = 0; q < KS; ++q)
#pragma unroll
            for (int t = 0; t < 2; ++t) bq[q][t] = wb[(q * 2 + t) * 64];
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 wsv = col_ok ? *reinterpret_cast<const float4*>(wsc + i * w + col0) : z4;
        const float4 bc = col_ok ? *reinterpret_cast<const float4*>(bias + i * w + col0) : z4;
        // a = sp_{i-1} + h_i: unit u -> (row = u % R, kg = u / R), 8 k each
        float a[IT][8];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int u = tid + nth * it;
            const int row = u % R, kg = u / R, k0 = 8 * kg;
            const int64_t gr = r0 + row;
#pragma unroll
            for (int e = 0; e < 8; e += 4) {
                float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (u < NU && gr < n && k0 + e < w)
                    hv = *reinterpret_cast<const float4*>(h + gr * hw + (int64_t)i * w + k0 + e);
                a[it][e] = hv.x; a[it][e + 1] = hv.y; a[it][e + 2] = hv.z; a[it][e + 3] = hv.w;
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int u = tid + nth * it;
            const int row = u % R, kg = u / R, k0 = 8 * kg;
            float cm = 0.f;
            if (i > 0 && u < NU && k0 < W) {            // k0 < W => k0 + 8 <= W (W % 16 == 0)
                // sp columns in [w, W) hold 0 (zero weights and bias there); units at k0 >= W
                // are the k32 steps' padding past W (no sp columns)
                const float4 s0 = *reinterpret_cast<const float4*>(sp + row * SPW + k0);
                const float4 s1 = *reinterpret_cast<const float4*>(sp + row * SPW + k0 + 4);
                a[it][0] += s0.x; a[it][1] += s0.y; a[it][2] += s0.z; a[it][3] += s0.w;
                a[it][4] += s1.x; a[it][5] += s1.y; a[it][6] += s1.z; a[it][7] += s1.w;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) cm = fmaxf(cm, fabsf(a[it][e]));
            if (u < NU && cm > 0.f) atomicMax(&rm[row], __float_as_int(cm));
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int u = tid + nth * it;
            if (u >= NU) break;
            const int row = u % R, kg = u / R;
            const float mx = __int_as_float(rm[row]);
            const float s = __builtin_ldexpf(1.f, mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0);
            f16x8 th, tm;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float xs = a[it][e] * s;
                const _Float16 hh = (_Float16)xs;
                th[e] = hh;
                tm[e] = (_Float16)(xs - (float)hh);
            }
            img[0 * NU + kg * R + row] = __builtin_bit_cast(u32x4, th);
            img[1 * NU + kg * R + row] = __builtin_bit_cast(u32x4, tm);
        }
        __syncthreads();
        f32x4 acc[RF];
#pragma unroll
        for (int f = 0; f < RF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const f16x8 wh = __builtin_bit_cast(f16x8, bq[ks][0]);
            const f16x8 wl = __builtin_bit_cast(f16x8, bq[ks][1]);
            const int base = (ks * 4 + g) * R;
            f16x8 ah[RF], am[RF];
#pragma unroll
            for (int f = 0; f < RF; ++f) {
                ah[f] = __builtin_bit_cast(f16x8, img[0 * NU + base + 16 * f + c]);
                am[f] = __builtin_bit_cast(f16x8, img[1 * NU + base + 16 * f + c]);
            }
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah[f], acc[f], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, am[f], acc[f], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < RF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah[f], acc[f], 0, 0, 0);
        }
        // epilogue: lane (g, c) holds sp_i[row rg * 16 + c][cols col0 .. col0 + 3]
#pragma unroll
        for (int rg = 0; rg < RF; ++rg) {
            const int row = rg * 16 + c;
            const float mx = __int_as_float(rm[row]);
            const float rs = __builtin_ldexpf(1.f, mx > 0.f ? -min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0);
            const f32x4 av = acc[rg];
            float4 y;
            y.x = fmaxf(av[0] * rs * wsv.x + bc.x, 0.f);
            y.y = fmaxf(av[1] * rs * wsv.y + bc.y, 0.f);
            y.z = fmaxf(av[2] * rs * wsv.z + bc.z, 0.f);
            y.w = fmaxf(av[3] * rs * wsv.w + bc.w, 0.f);
            if (r0 + row < n && col_ok)
                *reinterpret_cast<float4*>(cat + (r0 + row) * ld + (int64_t)i * w + col0) = y;
            *reinterpret_cast<float4*>(sp + row * SPW + col0) = y;
        }
        if (tid < R) rmax[(i + 1) & 1][tid] = 0;       // next step's row maxima
        __syncthreads();
    }
    copy_rows(cat + (int64_t)nums * w, ld, h + (int64_t)nums * w, hw, r0, R, n,
              (scale - nums) * w, tid, nth);
    if (x) copy_rows(cat + hw, ld, x, cin, r0, R, n, cin, tid, nth);
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_res2net_chain_h3(const float* h, int64_t n, int32_t w, int32_t scale,
                                    const void* w_img, const float* w_scale, const float* bias,
                                    const float* x, int32_t cin, float* cat, int64_t ld_cat,
                                    void* stream) {
    FGR_REQUIRE(n >= 0 && scale >= 2 && w > 0 && w <= 224 && w % 4 == 0 && cin >= 0,
                "fgr_res2net_chain_h3: unsupported width %d / scale %d (w %% 4 == 0, <= 224)", w,
                scale);
    FGR_REQUIRE(ld_cat >= (int64_t)scale * w + (x ? cin : 0) && ld_cat % 4 == 0,
                "fgr_res2net_chain_h3: ld_cat too small or not a multiple of 4");
    FGR_REQUIRE(n == 0 || (h && w_img && w_scale && bias && cat), "fgr_res2net_chain_h3: null pointer");
    FGR_REQUIRE(((reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(cat) |
                  reinterpret_cast<uintptr_t>(w_scale) | reinterpret_cast<uintptr_t>(bias)) & 15) == 0 &&
                    (scale * w) % 4 == 0,
                "fgr_res2net_chain_h3: h / cat / w_scale / bias must be 16-B aligned");
    if (n == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const int kt = (w + 15) / 16;
    // w > 112 (one 14-wave block per CU): 48-row blocks when that saves a round of blocks
    // (rounds x rows per block over 256 CUs, as fgr_res2net_chain6); FGR_R2N_ROWS=32 forces 32
    const char* rr = getenv("FGR_R2N_ROWS");
    const bool r48 = kt == 14 && !(rr && rr[0] == '3') &&
                     ceil_div(ceil_div(n, 48), 256) * 48 < ceil_div(ceil_div(n, 32), 256) * 32;
#define FGR_H3_CASE(KT)                                                                         \
    case KT:                                                                                    \
        hipLaunchKernelGGL(res2net_chain_h3_kernel<KT>, dim3((unsigned)ceil_div(n, kRows)),     \
                           dim3(64 * KT), 0, st, h, n, w, scale, scale - 1, (const u32x4*)w_img, \
                           w_scale, bias, x, cin, cat, ld_cat);                                 \
        break;
    if (r48) {
        hipLaunchKernelGGL((res2net_chain_h3_kernel<14, 48>), dim3((unsigned)ceil_div(n, 48)),
                           dim3(64 * 14), 0, st, h, n, w, scale, scale - 1, (const u32x4*)w_img,
                           w_scale, bias, x, cin, cat, ld_cat);
        FGR_CHECK_LAUNCH("res2net_chain_h3_kernel");
        return FGR_OK;
    }
    switch (kt) {
        FGR_H3_CASE(2)
        FGR_H3_CASE(4)
        FGR_H3_CASE(7)
        FGR_H3_CASE(14)
        default:
            set_error("fgr_res2net_chain_h3: width %d has no kernel instance (28, 56, 112, 224)", w);
            return FGR_E_ARG;
    }
#undef FGR_H3_CASE
    FGR_CHECK_LAUNCH("res2net_chain_h3_kernel");
    return FGR_OK;
}

extern "C" int fgr_res2net_chain6(const float* h, int64_t n, int32_t w, int32_t scale,
                                  const void* w_img, const float* bias, const float* x,
                                  int32_t cin, float* cat, int64_t ld_cat, void* stream) {
    FGR_REQUIRE(n >= 0 && scale >= 2 && (w == 112 || w == 224) && cin >= 0,
                "fgr_res2net_chain6: unsupported width %d / scale %d (needs 112 or 224)", w, scale);
    FGR_REQUIRE(ld_cat >= (int64_t)scale * w + (x ? cin : 0), "fgr_res2net_chain6: ld_cat too small");
    FGR_REQUIRE(n == 0 || (h && w_img && bias && cat), "fgr_res2net_chain6: null pointer");
    FGR_REQUIRE(((reinterpret_cast<uintptr_t>(h) & 15) == 0) && (scale * w) % 4 == 0,
                "fgr_res2net_chain6: h must be 16-B aligned");
    if (n == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    // w = 224 (one 14-wave block per CU): 48-row blocks when that saves a round of blocks
    // over 32-row ones (rounds x rows per block; 256 CUs); FGR_R2N_ROWS=32 forces 32 (A/B)
    const char* rr = getenv("FGR_R2N_ROWS");
    int rows = 32;
    if (w == 224 && !(rr && rr[0] == '3')) {       // min over R of rounds(R) x R, larger R on ties
        int64_t best = ceil_div(ceil_div(n, 32), 256) * 32;
        for (int r : {48, 16}) {
            const int64_t cost = ceil_div(ceil_div(n, r), 256) * r;
            if (cost < best) { best = cost; rows = r; }
        }
    }
    const int64_t b32 = ceil_div(n, 32);
    if (w == 112)
        hipLaunchKernelGGL(res2net_chain6_kernel<7>, dim3((unsigned)b32), dim3(64 * 7), 0, st, h, n,
                           scale, scale - 1, (const u32x4*)w_img, bias, x, cin, cat, ld_cat);
    else if (rows == 48)
        hipLaunchKernelGGL((res2net_chain6_kernel<14, 48>), dim3((unsigned)ceil_div(n, 48)), dim3(64 * 14),
                           0, st, h, n, scale, scale - 1, (const u32x4*)w_img, bias, x, cin, cat, ld_cat);
    else if (rows == 16)
        hipLaunchKernelGGL((res2net_chain6_kernel<14, 16>), dim3((unsigned)ceil_div(n, 16)), dim3(64 * 14),
                           0, st, h, n, scale, scale - 1, (const u32x4*)w_img, bias, x, cin, cat, ld_cat);
    else
        hipLaunchKernelGGL(res2net_chain6_kernel<14>, dim3((unsigned)b32), dim3(64 * 14), 0, st, h, n,
                           scale, scale - 1, (const u32x4*)w_img, bias, x, cin, cat, ld_cat);
    FGR_CHECK_LAUNCH("res2net_chain6_kernel");
    return FGR_OK;
}
