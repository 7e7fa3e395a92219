// The pre-norm transformer's position-wise feed-forward sub-layer in ONE launch
// (transformers.py:231-238, forward_pre):
//
//   y = x + linear2(ReLU(linear1(LayerNorm3(x))))        x (M, d), d = 256, hidden F
//
// fp32-accurate f16x3 products (three fp16 MFMA term products per product, as gemm_rs.hip).
//
// Why one launch. The two-launch form writes the (M, F) hidden activations (F = 4d) to HBM and
// reads them back, and pays two prologues / fill-drain tails (ModelNet: 9544 x 1024 fp32 = 39 MB
// each way, 2 x ~31 us per layer). Here a block owns 64 rows (4 waves x 16 rows) end to end:
//
//   * prologue: each wave loads its 16 rows whole, forms LayerNorm3 in registers (as the LN
//     prologue of gemm_rs.hip) and splits them into the two fp16 terms with one power-of-two
//     scale per row (max in [2^14, 2^15)): the A operand of linear1, resident for the launch;
//   * per chunk of 32 hidden units: linear1's two 16-column panels (W1 fragments from LDS) give
//     the lane's 8 hidden values of its row, bias + ReLU in registers, split once into fp16
//     terms -- and those registers ARE linear2's B fragment (no LDS, no shuffle): with the swapped
//     orientation (W fragments = MFMA A operand, activations = B operand) lane (g, c) holds
//     hidden 16 p + 4 g + r (p = 0, 1, r = 0..3) of row c after linear1, and linear2's B lane map
//     wants k = 8 g + e of row c; so linear2's contraction runs over the hidden units in the
//     order k = 8 g + e <-> 16 (e / 4) + 4 g + e % 4, and linear2's weight image is built in that
//     order (ffn_w2_split_kernel). 16 output panels of linear2 accumulate over all chunks in
//     registers (64 accumulators per lane);
//   * the weights stream global -> LDS by LDS-DMA through a ring of 8 x 16 KB units (a W1
//     panel, or half of a chunk's W2 slice): while a wave multiplies unit u (fragments in
//     registers), unit u + 1's fragments are read from LDS and units u + 2 .. u + 8 are in
//     flight; one barrier per unit;
//   * epilogue: y = acc * wsc2 / S + b2 + x (x re-read from L2), one 16-B store per lane and
//     output panel. The hidden activations never reach memory.
//
// Precision of the hidden split: linear2's B operand needs ONE scale per row before the row's
// hidden values exist. It comes from a bound: |h_j| <= ||a|| ||W1_j|| + |b1_j| <= ||a|| M1 + Mb
// (Cauchy-Schwarz; a = the LayerNorm'd row, M1 = max_j ||W1_j||_2, Mb = max |b1|, `bound` =
// {M1, Mb} from the host), so h S <= 2^15 with S = 2^e, bound S in [2^14, 2^15): no fp16
// overflow. Values below the bound keep an ABSOLUTE split error <= 2^-25 / S <= 2^-39 bound
// (fp16 subnormal spacing), far under the fp32 rounding of the products they feed.
//
// Weight images: W1 (F, d) is the plain fgr_split_weights_h3 image ([panel][kstep][term][g][16]
// x 16 B, then the F per-row inverse scales); W2 (d, F) the chunk-major image of
// fgr_split_weights_ffn2 below ([chunk F/32][panel d/16][term][g][16] x 16 B in the permuted k
// order, then the d per-row inverse scales).
#include <algorithm>
#include <cstdlib>

#include "common.h"

#ifdef FGR_FFN_STAMP
// Diagnostic build only (tools/ffn_stamp.py): per (block, wave) cycle sums of the loop's phases
// (s_memtime): [0] prologue, [1] waits for the DMA, [2] barriers, [3] DMA + read issue, [4] MFMA
// sections (incl. the hidden epilogue), [5] read waits, [6] epilogue, [7] total
__device__ unsigned long long g_ffn_stamp[4096][4][8];
#define FFN_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define FFN_T(v)
#endif

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kFfnD = 256;                  // d_model
constexpr int kFfnKS = kFfnD / 32;          // k32 steps of linear1 (8)
constexpr int kFfnNP = kFfnD / 16;          // output panels of linear2 (16)
constexpr int kFfnMaxF = 2048;              // hidden units (LDS for their scales / bias)
constexpr int kUnit = 1024;                 // 16-B units per ring unit (16 KB)
constexpr int kRing = 8;                    // ring units (128 KB of LDS)
static_assert(kFfnKS * 128 == kUnit, "a W1 panel is one ring unit");
static_assert(kFfnNP / 2 * 128 == kUnit, "half of a chunk's W2 slice is one ring unit");

struct FfnArgs {
    const float* x; int64_t ldx;
    const float* ln_g; const float* ln_b; float eps;
    const u32x4* w1; const float* wsc1; const float* b1;
    const u32x4* w2; const float* wsc2; const float* b2;
    const float* bound;                     // {max_j ||W1_j||_2, max_j |b1_j|}
    float* out; int64_t ldo;
    int M, F;
};

// s_waitcnt vmcnt(N) lgkmcnt(0) (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0_f() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}
// vmcnt(4 n) lgkmcnt(0) for a wave-uniform n in [0, kRing - 2]
__device__ __forceinline__ void wait_units(int n) {
    static_assert(kRing - 2 <= 6, "extend the switch");
    switch (n) {
        case 0: wait_vm_lgkm0_f<0>(); break;
        case 1: wait_vm_lgkm0_f<4>(); break;
        case 2: wait_vm_lgkm0_f<8>(); break;
        case 3: wait_vm_lgkm0_f<12>(); break;
        case 4: wait_vm_lgkm0_f<16>(); break;
        case 5: wait_vm_lgkm0_f<20>(); break;
        default: wait_vm_lgkm0_f<24>(); break;
    }
}

__device__ __forceinline__ float xg_sum_f(float v) {      // sum over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float xg_max_f(float v) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

typedef __attribute__((address_space(3))) u32x4 lds_u4;

// The ring: one LDS object per slot, addressed with a compile-time slot index (the chunk loop
// is unrolled over a whole ring turn).
__shared__ u32x4 g_ffn_ring0[kUnit], g_ffn_ring1[kUnit], g_ffn_ring2[kUnit], g_ffn_ring3[kUnit],
                 g_ffn_ring4[kUnit], g_ffn_ring5[kUnit], g_ffn_ring6[kUnit], g_ffn_ring7[kUnit];
static_assert(kRing == 8, "one object per slot below");

__device__ __forceinline__ u32x4* ring_slot(int s) {
    switch (s & 7) {
        case 0: return g_ffn_ring0; case 1: return g_ffn_ring1;
        case 2: return g_ffn_ring2; case 3: return g_ffn_ring3;
        case 4: return g_ffn_ring4; case 5: return g_ffn_ring5;
        case 6: return g_ffn_ring6; default: return g_ffn_ring7;
    }
}

// The 8 fragment pairs (term 0 / 1) of one ring unit at rows (g, c): [j][term][g][16] x 16 B
// (j = the k32 step of a W1 panel, or the output panel of a W2 half slice). The reads are
// issued by one asm statement and waited for by another (read_wait: the fragments are its
// in-out operands, so nothing uses them before the wait), with the current unit's MFMAs in
// between. Compiler-visible reads of the ring made its wait insertion drain every LDS-DMA in
// flight (vmcnt(0)) once per ring turn (its LDS-DMA tracking does not survive the loop's back
// edge); the kernel waits for the DMA itself (wait_units + barrier).
__device__ __forceinline__ void read_issue(const u32x4* slot, int lane_u, u32x4 (&r)[16]) {
    const uint32_t a = (uint32_t)(uintptr_t)((const lds_u4*)slot + lane_u);
    asm volatile(
        "ds_read_b128 %0, %16 offset:0\n\t"
        "ds_read_b128 %1, %16 offset:1024\n\t"
        "ds_read_b128 %2, %16 offset:2048\n\t"
        "ds_read_b128 %3, %16 offset:3072\n\t"
        "ds_read_b128 %4, %16 offset:4096\n\t"
        "ds_read_b128 %5, %16 offset:5120\n\t"
        "ds_read_b128 %6, %16 offset:6144\n\t"
        "ds_read_b128 %7, %16 offset:7168\n\t"
        "ds_read_b128 %8, %16 offset:8192\n\t"
        "ds_read_b128 %9, %16 offset:9216\n\t"
        "ds_read_b128 %10, %16 offset:10240\n\t"
        "ds_read_b128 %11, %16 offset:11264\n\t"
        "ds_read_b128 %12, %16 offset:12288\n\t"
        "ds_read_b128 %13, %16 offset:13312\n\t"
        "ds_read_b128 %14, %16 offset:14336\n\t"
        "ds_read_b128 %15, %16 offset:15360"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
          "=&v"(r[6]), "=&v"(r[7]), "=&v"(r[8]), "=&v"(r[9]), "=&v"(r[10]), "=&v"(r[11]),
          "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]), "=&v"(r[15])
        : "v"(a)
        : "memory");
}
__device__ __forceinline__ void read_wait(u32x4 (&r)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                   "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]),
                   "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])
                 :
                 : "memory");
}
// fragment j, term t of a unit read into r
__device__ __forceinline__ f16x8 frag(const u32x4 (&r)[16], int j, int t) {
    return __builtin_bit_cast(f16x8, r[2 * j + t]);
}

__global__ void __launch_bounds__(256, 1) ffn_f16x3_kernel(FfnArgs p) {
    __shared__ float4 cw1[kFfnMaxF / 4], cb1[kFfnMaxF / 4];     // linear1 column scales / bias
    __shared__ float4 cw2[kFfnD / 4], cb2[kFfnD / 4];           // linear2
    __shared__ float4 lng[kFfnD / 4], lnb[kFfnD / 4];           // LayerNorm3 gamma / beta

#ifdef FGR_FFN_STAMP
    unsigned long long acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    FFN_T(t_begin);
    const int nbm = (p.M + 63) / 64;
    int t = blockIdx.x;
    {   // XCD-aware order: each XCD a contiguous range of row blocks
        const int q = nbm / 8, r = nbm % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const int mw = t * 64 + wv * 16;                   // this wave's first row
    const int64_t row = min(mw + c, p.M - 1);          // lane's row (loads clamp, stores guard)
    const int nch = p.F / 32;
    const int nu = 4 * nch;                            // ring units: [W1 2c, W1 2c+1, W2 lo, W2 hi]

    // 1. the wave's rows: lane (g, c) holds row c, k = 32 s + 8 g + e
    float xr[kFfnKS][8];
    {
        const float* ar = p.x + row * p.ldx;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s) {
            const float4 a0 = *reinterpret_cast<const float4*>(ar + 32 * s + 8 * g);
            const float4 a1 = *reinterpret_cast<const float4*>(ar + 32 * s + 8 * g + 4);
            xr[s][0] = a0.x; xr[s][1] = a0.y; xr[s][2] = a0.z; xr[s][3] = a0.w;
            xr[s][4] = a1.x; xr[s][5] = a1.y; xr[s][6] = a1.z; xr[s][7] = a1.w;
        }
    }
    // 2. per-column parameters (16-B loads from clamped indices, no branches around them: a
    //    guarded load puts a vmcnt(0) in its branch; staged in LDS after the wait below)
    const int nf4 = p.F / 4;
    static_assert(kFfnMaxF / 4 == 2 * 256, "two float4 per thread");
    const int j0 = min(tid, nf4 - 1), j1 = min(tid + 256, nf4 - 1);
    const float4 pw1a = reinterpret_cast<const float4*>(p.wsc1)[j0];
    const float4 pb1a = reinterpret_cast<const float4*>(p.b1)[j0];
    const float4 pw1b = reinterpret_cast<const float4*>(p.wsc1)[j1];
    const float4 pb1b = reinterpret_cast<const float4*>(p.b1)[j1];
    const int t4 = tid & (kFfnD / 4 - 1);
    const float4 pw2 = reinterpret_cast<const float4*>(p.wsc2)[t4];
    const float4 pb2 = reinterpret_cast<const float4*>(p.b2)[t4];
    const float4 pg = reinterpret_cast<const float4*>(p.ln_g)[t4];
    const float4 pbe = reinterpret_cast<const float4*>(p.ln_b)[t4];
    const float bM1 = p.bound[0], bMb = p.bound[1];

    // 3. the first kRing ring units by LDS-DMA: wave wv moves 1-KB pieces wv, wv + 4, wv + 8, wv + 12
    auto unit_src = [&](int u) -> const u32x4* {
        const int ch = u >> 2, j = u & 3;
        return j < 2 ? p.w1 + (int64_t)(2 * ch + j) * kUnit
                     : p.w2 + (int64_t)ch * (2 * kUnit) + (j - 2) * kUnit;
    };
    auto dma = [&](int u, int slot) {                   // slot = u % kRing, compile-time
        const u32x4* src = unit_src(u) + wv * 64 + lane;
        __attribute__((address_space(3))) char* dst =
            (__attribute__((address_space(3))) char*)(lds_u4*)ring_slot(slot) + wv * 1024;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(src + j * 256),
                                             (__attribute__((address_space(3))) void*)(dst + j * 4096),
                                             16, 0, 0);
    };
#pragma unroll
    for (int u = 0; u < kRing; ++u) dma(u, u);         // nu >= 8 (f >= 64: supported())
    // the row and parameter loads are older than the DMA pieces: vmcnt(4 kRing) leaves the
    // pieces in flight
    wait_vm_lgkm0_f<4 * kRing>();
    if (tid < nf4) { cw1[tid] = pw1a; cb1[tid] = pb1a; }
    if (tid + 256 < nf4) { cw1[tid + 256] = pw1b; cb1[tid + 256] = pb1b; }
    if (tid < kFfnD / 4) { cw2[tid] = pw2; cb2[tid] = pb2; lng[tid] = pg; lnb[tid] = pbe; }
    wait_vm_lgkm0_f<4 * kRing - 4>();     // the LDS writes (lgkmcnt 0) and unit 0's pieces
    __builtin_amdgcn_s_barrier();
    const int lane_u = g * 16 + c;
    u32x4 wa[16], wb[16];                 // fragment double buffer: units of even / odd index
    read_issue(ring_slot(0), lane_u, wa); // waited for after the LayerNorm below

    // 4. LayerNorm3 of the rows (two passes over registers, as gemm_rs.hip), ||a||, split
    f16x8 af[kFfnKS][2];
    float rsS, inv_s;                                   // rs_a * S, 1 / S
    {
        float sm = 0.f;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s)
            sm += ((xr[s][0] + xr[s][1]) + (xr[s][2] + xr[s][3])) +
                  ((xr[s][4] + xr[s][5]) + (xr[s][6] + xr[s][7]));
        const float mean = xg_sum_f(sm) / (float)kFfnD;
        float sq = 0.f;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float d = xr[s][e] - mean;
                sq += d * d;
            }
        const float rstd = 1.0f / sqrtf(xg_sum_f(sq) / (float)kFfnD + p.eps);
        float mx = 0.f, nn = 0.f;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s) {
            const int k = 32 * s + 8 * g;
            const float4 g0 = lng[k / 4], g1 = lng[k / 4 + 1];
            const float4 b0 = lnb[k / 4], b1 = lnb[k / 4 + 1];
            const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
            const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float a = (xr[s][e] - mean) * rstd * gg[e] + bb[e];
                xr[s][e] = a;
                nn = fmaf(a, a, nn);
            }
            mx = fmaxf(mx, max3_abs(xr[s][0], xr[s][1], xr[s][2]));
            mx = fmaxf(mx, max3_abs(xr[s][3], xr[s][4], xr[s][5]));
            mx = fmaxf(mx, max3_abs(xr[s][6], xr[s][7], 0.f));
        }
        mx = xg_max_f(mx);
        nn = xg_sum_f(nn);
        const int ea = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
        const float sca = __builtin_ldexpf(1.f, ea);
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s) {
            u32x4 h, l;
            split8_f16(xr[s], sca, h, l);
            af[s][0] = __builtin_bit_cast(f16x8, h);
            af[s][1] = __builtin_bit_cast(f16x8, l);
        }
        // the hidden values' scale S from the bound ||a|| M1 + Mb (bound S in [2^14, 2^15))
        const float bnd = sqrtf(nn) * bM1 + bMb;
        const int eh = bnd > 0.f ? max(min(15 - __builtin_amdgcn_frexp_expf(bnd), 127), -126) : 0;
        rsS = __builtin_ldexpf(1.f, eh - ea);
        inv_s = __builtin_ldexpf(1.f, -eh);
    }
    const float sS = inv_s > 0.f ? 1.f / inv_s : 1.f;   // S (exact: a power of two)

    // 5. the chunk loop: unit u of chunk ch = u / 4: j 0, 1 linear1 panels 2 ch + j; j 2, 3
    //    linear2 output panels 8 (j - 2) .. + 7 over the chunk's 32 hidden units
    f32x4 accy[kFfnNP];
#pragma unroll
    for (int q = 0; q < kFfnNP; ++q) accy[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 acc1[2];
    f16x8 hb[2];
    read_wait(wa);
    FFN_T(t_loop);
#ifdef FGR_FFN_STAMP
    acc_[0] = t_loop - t_begin;
#endif
    for (int ch2 = 0; ch2 < nch; ch2 += 2) {            // one ring turn (8 units) per iteration
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const int j = jj & 3, ch = ch2 + (jj >> 2);
            const int u = 4 * ch2 + jj;                   // slot jj
            u32x4 (&cur)[16] = (jj & 1) ? wb : wa;
            u32x4 (&nxt)[16] = (jj & 1) ? wa : wb;
            const bool more = u + 1 < nu;                 // block-uniform
            FFN_T(t0);
            if (more) {
                // unit u + 1 landed (units issued after it: min(6, nu - 2 - u)); every wave has
                // read unit u (its fragments are in registers), whose slot the DMA of unit u + 8
                // refills
                wait_units(min(kRing - 2, nu - 2 - u));
                FFN_T(t1);
                __builtin_amdgcn_s_barrier();
                FFN_T(t2);
                if (u + kRing < nu) dma(u + kRing, jj);
                read_issue(ring_slot(jj + 1), lane_u, nxt);
#ifdef FGR_FFN_STAMP
                acc_[1] += t1 - t0;
                acc_[2] += t2 - t1;
                acc_[3] += __builtin_amdgcn_s_memtime() - t2;
#endif
            }
            __builtin_amdgcn_sched_barrier(0);
            FFN_T(t3);
            if (j < 2) {
                f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < kFfnKS; ++s) {
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(frag(cur, s, 1), af[s][0], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(frag(cur, s, 0), af[s][1], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(frag(cur, s, 0), af[s][0], a, 0, 0, 0);
                }
                acc1[j] = a;
                if (j == 1) {
                    // bias + ReLU, scaled by S, split: linear2's B fragment of row c
                    float hv[8];
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp) {
                        const int n = 32 * ch + 16 * pp + 4 * g;
                        const float4 w4 = cw1[n / 4], b4 = cb1[n / 4];
                        hv[4 * pp + 0] = fmaxf(fmaf(acc1[pp][0], rsS * w4.x, sS * b4.x), 0.f);
                        hv[4 * pp + 1] = fmaxf(fmaf(acc1[pp][1], rsS * w4.y, sS * b4.y), 0.f);
                        hv[4 * pp + 2] = fmaxf(fmaf(acc1[pp][2], rsS * w4.z, sS * b4.z), 0.f);
                        hv[4 * pp + 3] = fmaxf(fmaf(acc1[pp][3], rsS * w4.w, sS * b4.w), 0.f);
                    }
                    u32x4 h, l;
                    split8_f16(hv, 1.f, h, l);
                    hb[0] = __builtin_bit_cast(f16x8, h);
                    hb[1] = __builtin_bit_cast(f16x8, l);
                }
            } else {
#pragma unroll
                for (int qq = 0; qq < 8; ++qq) {
                    const int q = 8 * (j - 2) + qq;
                    accy[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(frag(cur, qq, 1), hb[0], accy[q], 0, 0, 0);
                    accy[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(frag(cur, qq, 0), hb[1], accy[q], 0, 0, 0);
                    accy[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(frag(cur, qq, 0), hb[0], accy[q], 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            FFN_T(t4);
            if (more) read_wait(nxt);
#ifdef FGR_FFN_STAMP
            acc_[4] += t4 - t3;
            acc_[5] += __builtin_amdgcn_s_memtime() - t4;
#endif
        }
    }
    FFN_T(t_epi);

    // 6. y = acc * wsc2 / S + b2 + x: lane (g, c) holds row c, columns 16 q + 4 g .. + 3
    const bool ok = mw + c < p.M;
    const float* xrow = p.x + row * p.ldx;
    float4 res[kFfnNP];
#pragma unroll
    for (int q = 0; q < kFfnNP; ++q) res[q] = *reinterpret_cast<const float4*>(xrow + 16 * q + 4 * g);
    float* orow = p.out + row * p.ldo;
#pragma unroll
    for (int q = 0; q < kFfnNP; ++q) {
        const int n = 16 * q + 4 * g;
        const float4 w4 = cw2[n / 4], b4 = cb2[n / 4];
        const float4 y = make_float4(fmaf(accy[q][0], w4.x * inv_s, b4.x) + res[q].x,
                                     fmaf(accy[q][1], w4.y * inv_s, b4.y) + res[q].y,
                                     fmaf(accy[q][2], w4.z * inv_s, b4.z) + res[q].z,
                                     fmaf(accy[q][3], w4.w * inv_s, b4.w) + res[q].w);
        if (ok) *reinterpret_cast<float4*>(orow + n) = y;
    }
#ifdef FGR_FFN_STAMP
    __builtin_amdgcn_s_waitcnt(0);
    FFN_T(t_end);
    acc_[6] = t_end - t_epi;
    acc_[7] = t_end - t_begin;
    if (lane < 8 && blockIdx.x < 4096) g_ffn_stamp[blockIdx.x][wv][lane] = acc_[lane];
#endif
}

// ---------------------------------------------------------------------------------------------
// Version 2 (default): the same sub-layer with the waves splitting the WEIGHTS instead of the rows.
//
// The ring version above streams every weight unit to all 4 waves of a block through LDS (each
// wave multiplies it against its own 16 rows): per 16 KB unit the CU pays 16 LDS-DMA pieces, 64
// KB of LDS fragment reads and a barrier for 96 MFMAs, and its in-kernel clock stamps put the
// DMA / read issue (446 cycles per unit) and the DMA wait (209) beside 384 cycles of MFMA.
// Here the block's 64 LayerNorm'd rows are split ONCE into an LDS image (4 row tiles x 8 k32
// steps x 2 terms, 64 KB), and each wave owns weights, read straight from global memory (L2)
// into registers, each byte by one wave only:
//   * linear1: wave w computes hidden chunk 4 st + w (32 units) of step st for all 64 rows (its
//     W1 fragments x the row image from LDS), bias + ReLU + scale + split as in version 1, and
//     writes the 64 rows x 32 hidden fragments to an LDS hand-off buffer (8 KB per wave);
//   * one barrier per step (128 hidden units), then linear2: wave w owns output panels
//     4 w .. 4 w + 3 (64 columns) and contracts them over the step's 128 hidden units (the four
//     waves' fragments from LDS, its W2 fragments from global), accumulating 4 row tiles x 4
//     panels in registers; no cross-wave reduction at the end.
// Per step and wave: 64 x 16-B weight loads per lane (its 32 KB of W1 and 32 KB of W2), 96 LDS
// fragment reads, 384 MFMAs; 8 barriers per launch at F = 1024. The weight loads run 3 groups
// (12 loads) ahead of their MFMAs through a 4-group register ring.
constexpr int kV2Groups = 16;          // load groups per step: 8 linear1 k32 steps, 8 linear2 halves
constexpr int kCusFfn = 256;           // MI355X compute units (one block per CU)
#ifndef FGR_FFN_RING
#define FGR_FFN_RING 4
#endif
constexpr int kV2Ring = FGR_FFN_RING;  // register ring of groups (kV2Ring - 1 in flight)
static_assert(kV2Groups % kV2Ring == 0, "ring slot = group index mod kV2Ring at compile time");

// s_waitcnt vmcnt(n) (lgkmcnt / expcnt untouched) for n = 4 k <= 28
__device__ __forceinline__ void wait_vm_only(int n) {
    // vmcnt field bits 3:0 and 15:14, expcnt 6:4 = 7, lgkmcnt 11:8 = 15 (no wait)
#define FGR_VMW(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | (7 << 4) | (15 << 8))
    switch (n) {
        case 0: FGR_VMW(0); break;   case 4: FGR_VMW(4); break;
        case 8: FGR_VMW(8); break;   case 12: FGR_VMW(12); break;
        case 16: FGR_VMW(16); break; case 20: FGR_VMW(20); break;
        case 24: FGR_VMW(24); break; default: FGR_VMW(28); break;
    }
#undef FGR_VMW
}

// RT row tiles per block (16 RT rows): 4, or 3 where 48-row blocks still fit the CUs in one
// round (ModelNet's 9544 rows: 199 blocks instead of 150 -- every block 25 % shorter)
template <int RT>
__global__ void __launch_bounds__(256, 1) ffn_nsplit_kernel(FfnArgs p) {
    static_assert(RT >= 1 && RT <= 4, "row tiles");
    __shared__ u32x4 act[RT * kFfnKS * 2 * 64];           // [row tile][k32 step][term][lane]
    __shared__ u32x4 hbuf[2][4][RT][2][64];               // [step & 1][src wave][row tile][term][lane]
    __shared__ float4 cw1[kFfnMaxF / 4], cb1[kFfnMaxF / 4];
    __shared__ float4 cw2[kFfnD / 4], cb2[kFfnD / 4];
    __shared__ float4 lng[kFfnD / 4], lnb[kFfnD / 4];
    __shared__ float2 rowpar[64];                         // per row: (rs_a S, S)

    constexpr int BR = 16 * RT;                           // rows per block
    const int nbm = (p.M + BR - 1) / BR;
    int t = blockIdx.x;
    {   // XCD-aware order: each XCD a contiguous range of row blocks
        const int q = nbm / 8, r = nbm % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c = lane & 15;
    const int r0 = t * BR;                                // the block's first row
    const int nst = p.F / 128;                            // steps of 128 hidden units

    // 1. parameters (issued first: their LDS stores wait for them alone), this wave's row tile
    //    (rows r0 + 16 wv + c); parameters -> LDS
    const int nf4 = p.F / 4;
    const int j0 = min(tid, nf4 - 1), j1 = min(tid + 256, nf4 - 1);
    const float4 pw1a = reinterpret_cast<const float4*>(p.wsc1)[j0];
    const float4 pb1a = reinterpret_cast<const float4*>(p.b1)[j0];
    const float4 pw1b = reinterpret_cast<const float4*>(p.wsc1)[j1];
    const float4 pb1b = reinterpret_cast<const float4*>(p.b1)[j1];
    const int t4 = tid & (kFfnD / 4 - 1);
    const float4 pw2 = reinterpret_cast<const float4*>(p.wsc2)[t4];
    const float4 pb2 = reinterpret_cast<const float4*>(p.b2)[t4];
    const float4 pg = reinterpret_cast<const float4*>(p.ln_g)[t4];
    const float4 pbe = reinterpret_cast<const float4*>(p.ln_b)[t4];
    __builtin_amdgcn_sched_barrier(0);                    // keep them ahead of the row loads
    float xr[kFfnKS][8];
    {
        const int64_t row = min(r0 + 16 * min(wv, RT - 1) + c, p.M - 1);   // RT < 4: wave 3 idles
        const float* ar = p.x + row * p.ldx;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s) {
            const float4 a0 = *reinterpret_cast<const float4*>(ar + 32 * s + 8 * g);
            const float4 a1 = *reinterpret_cast<const float4*>(ar + 32 * s + 8 * g + 4);
            xr[s][0] = a0.x; xr[s][1] = a0.y; xr[s][2] = a0.z; xr[s][3] = a0.w;
            xr[s][4] = a1.x; xr[s][5] = a1.y; xr[s][6] = a1.z; xr[s][7] = a1.w;
        }
    }
    {
        if (tid < nf4) { cw1[tid] = pw1a; cb1[tid] = pb1a; }
        if (tid + 256 < nf4) { cw1[tid + 256] = pw1b; cb1[tid + 256] = pb1b; }
        if (tid < kFfnD / 4) { cw2[tid] = pw2; cb2[tid] = pb2; lng[tid] = pg; lnb[tid] = pbe; }
    }
    const float bM1 = p.bound[0], bMb = p.bound[1];
    __syncthreads();

    // 2. LayerNorm3, ||a||, the row split into the LDS row image, the per-row scales
    {
        float sm = 0.f;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s)
            sm += ((xr[s][0] + xr[s][1]) + (xr[s][2] + xr[s][3])) +
                  ((xr[s][4] + xr[s][5]) + (xr[s][6] + xr[s][7]));
        const float mean = xg_sum_f(sm) / (float)kFfnD;
        float sq = 0.f;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float d = xr[s][e] - mean;
                sq += d * d;
            }
        const float rstd = 1.0f / sqrtf(xg_sum_f(sq) / (float)kFfnD + p.eps);
        float mx = 0.f, nn = 0.f;
#pragma unroll
        for (int s = 0; s < kFfnKS; ++s) {
            const int k = 32 * s + 8 * g;
            const float4 g0 = lng[k / 4], g1 = lng[k / 4 + 1];
            const float4 b0 = lnb[k / 4], b1 = lnb[k / 4 + 1];
            const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
            const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float a = (xr[s][e] - mean) * rstd * gg[e] + bb[e];
                xr[s][e] = a;
                nn = fmaf(a, a, nn);
            }
            mx = fmaxf(mx, max3_abs(xr[s][0], xr[s][1], xr[s][2]));
            mx = fmaxf(mx, max3_abs(xr[s][3], xr[s][4], xr[s][5]));
            mx = fmaxf(mx, max3_abs(xr[s][6], xr[s][7], 0.f));
        }
        mx = xg_max_f(mx);
        nn = xg_sum_f(nn);
        const int ea = mx > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(mx), 127) : 0;
        const float sca = __builtin_ldexpf(1.f, ea);
        if (wv < RT) {
#pragma unroll
            for (int s = 0; s < kFfnKS; ++s) {
                u32x4 h, l;
                split8_f16(xr[s], sca, h, l);
                act[((wv * kFfnKS + s) * 2 + 0) * 64 + lane] = h;
                act[((wv * kFfnKS + s) * 2 + 1) * 64 + lane] = l;
            }
        }
        const float bnd = sqrtf(nn) * bM1 + bMb;
        const int eh = bnd > 0.f ? max(min(15 - __builtin_amdgcn_frexp_expf(bnd), 127), -126) : 0;
        if (g == 0 && wv < RT)
            rowpar[16 * wv + c] = make_float2(__builtin_ldexpf(1.f, eh - ea), __builtin_ldexpf(1.f, eh));
    }
    __syncthreads();

    // 3. the steps. Load group j of a step: j < 8 = linear1 k32 step j of this wave's chunk (W1
    //    panels 2 ch, 2 ch + 1 x 2 terms); j >= 8 = linear2 source wave (j - 8) / 2, output panel
    //    pair (j - 8) % 2 of this wave's four (x 2 terms)
    auto issue = [&](int st, int j, u32x4 (&slot)[4]) {
        if (j < 8) {
            const int ch = 4 * st + wv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int pp = e >> 1, tt = e & 1;
                slot[e] = p.w1[(int64_t)(2 * ch + pp) * kUnit + (j * 2 + tt) * 64 + lane];
            }
        } else {
            const int ch = 4 * st + ((j - 8) >> 1), q0 = 4 * wv + 2 * ((j - 8) & 1);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int qq = e >> 1, tt = e & 1;
                slot[e] = p.w2[((int64_t)(ch * kFfnNP + q0 + qq) * 2 + tt) * 64 + lane];
            }
        }
    };
    u32x4 ring[kV2Ring][4];
    f32x4 accy[RT][4];                                    // [row tile][output panel of the wave]
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int q = 0; q < 4; ++q) accy[rt][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < kV2Ring - 1; ++j) issue(0, j, ring[j]);
    // LDS fragments of a group, double-buffered: the 4 row tiles' (hi, lo) row-image fragments
    // of a k32 step (linear1), or the 4 row tiles' (hi, lo) hidden fragments of a source wave
    // (linear2); the next group's are read while this group's MFMAs run
    u32x4 fa[2][2 * RT];
    auto read_act = [&](int s, u32x4 (&f)[2 * RT]) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            f[2 * rt + 0] = act[((rt * kFfnKS + s) * 2 + 0) * 64 + lane];
            f[2 * rt + 1] = act[((rt * kFfnKS + s) * 2 + 1) * 64 + lane];
        }
    };
    auto read_h = [&](int buf, int sw, u32x4 (&f)[2 * RT]) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            f[2 * rt + 0] = hbuf[buf][sw][rt][0][lane];
            f[2 * rt + 1] = hbuf[buf][sw][rt][1][lane];
        }
    };

    for (int st = 0; st < nst; ++st) {
        const int ch = 4 * st + wv;
        // the last step's look-ahead re-reads its own groups (no branch in the body; drained
        // after the loop)
        const int stn = min(st + 1, nst - 1);
        f32x4 acc1[RT][2];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc1[rt][0] = acc1[rt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        read_act(0, fa[0]);
#pragma unroll
        for (int j = 0; j < kV2Groups; ++j) {
            const int jn = j + kV2Ring - 1;               // group j + 3 (this step or the next)
            issue(jn < kV2Groups ? st : stn, jn % kV2Groups, ring[jn % kV2Ring]);
            wait_vm_only(4 * (kV2Ring - 1));              // group j landed
            u32x4 (&wf)[4] = ring[j % kV2Ring];
            if (j < 8) {
                u32x4 (&cur)[2 * RT] = fa[j & 1];
                if (j < 7) read_act(j + 1, fa[(j + 1) & 1]);
                __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);      // this group's + 3 loads
                if (j < 7) __builtin_amdgcn_sched_group_barrier(0x100, 2 * RT, 0);   // next reads
                // linear1 k32 step j: W1 (panel pp, term) x the row tiles' fragments
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    const f16x8 ah = __builtin_bit_cast(f16x8, cur[2 * rt + 0]);
                    const f16x8 al = __builtin_bit_cast(f16x8, cur[2 * rt + 1]);
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp) {
                        const f16x8 wh = __builtin_bit_cast(f16x8, wf[2 * pp]);
                        const f16x8 wl = __builtin_bit_cast(f16x8, wf[2 * pp + 1]);
                        acc1[rt][pp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, acc1[rt][pp], 0, 0, 0);
                        acc1[rt][pp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, al, acc1[rt][pp], 0, 0, 0);
                        acc1[rt][pp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, acc1[rt][pp], 0, 0, 0);
                    }
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 6 * RT, 0);
                __builtin_amdgcn_sched_barrier(0);                      // nothing crosses groups
                if (j == 7) {
                    // bias + ReLU + S, split: the chunk's linear2 B fragments -> the hand-off buffer
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) {
                        const float2 rp = rowpar[16 * rt + c];
                        float hv[8];
#pragma unroll
                        for (int pp = 0; pp < 2; ++pp) {
                            const int n = 32 * ch + 16 * pp + 4 * g;
                            const float4 w4 = cw1[n / 4], b4 = cb1[n / 4];
                            hv[4 * pp + 0] = fmaxf(fmaf(acc1[rt][pp][0], rp.x * w4.x, rp.y * b4.x), 0.f);
                            hv[4 * pp + 1] = fmaxf(fmaf(acc1[rt][pp][1], rp.x * w4.y, rp.y * b4.y), 0.f);
                            hv[4 * pp + 2] = fmaxf(fmaf(acc1[rt][pp][2], rp.x * w4.z, rp.y * b4.z), 0.f);
                            hv[4 * pp + 3] = fmaxf(fmaf(acc1[rt][pp][3], rp.x * w4.w, rp.y * b4.w), 0.f);
                        }
                        u32x4 h, l;
                        split8_f16(hv, 1.f, h, l);
                        hbuf[st & 1][wv][rt][0][lane] = h;
                        hbuf[st & 1][wv][rt][1][lane] = l;
                    }
                    // every wave's chunk in LDS (and every wave done with the buffer's previous
                    // use, step st - 2, which ended before its barrier of step st - 1)
                    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
                    __builtin_amdgcn_s_barrier();
                    read_h(st & 1, 0, fa[0]);
                }
            } else {
                // linear2: source wave sw's chunk (k32 step of 32 hidden), output panels 2 qh, +1
                const int sw = (j - 8) >> 1, qh = (j - 8) & 1;
                u32x4 (&cur)[2 * RT] = fa[sw & 1];
                const bool pre = qh == 0 && sw < 3;
                if (pre) read_h(st & 1, sw + 1, fa[(sw + 1) & 1]);
                __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);
                if (pre) __builtin_amdgcn_sched_group_barrier(0x100, 2 * RT, 0);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    const f16x8 hh = __builtin_bit_cast(f16x8, cur[2 * rt + 0]);
                    const f16x8 hl = __builtin_bit_cast(f16x8, cur[2 * rt + 1]);
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq) {
                        const f16x8 wh = __builtin_bit_cast(f16x8, wf[2 * qq]);
                        const f16x8 wl = __builtin_bit_cast(f16x8, wf[2 * qq + 1]);
                        f32x4& a = accy[rt][2 * qh + qq];
                        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, hh, a, 0, 0, 0);
                        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, hl, a, 0, 0, 0);
                        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, hh, a, 0, 0, 0);
                    }
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 6 * RT, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    wait_vm_only(0);                                      // the last step's redundant look-ahead

    // 4. y = acc * wsc2 / S + b2 + x for the wave's 4 output panels of the block's rows
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int rr = r0 + 16 * rt + c;
        const int64_t row = min(rr, p.M - 1);
        const float inv_s = 1.f / rowpar[16 * rt + c].y;       // exact: a power of two
        const float* xrow = p.x + row * p.ldx;
        float4 res[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) res[q] = *reinterpret_cast<const float4*>(xrow + 16 * (4 * wv + q) + 4 * g);
        float* orow = p.out + row * p.ldo;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int n = 16 * (4 * wv + q) + 4 * g;
            const float4 w4 = cw2[n / 4], b4 = cb2[n / 4];
            const float4 y = make_float4(fmaf(accy[rt][q][0], w4.x * inv_s, b4.x) + res[q].x,
                                         fmaf(accy[rt][q][1], w4.y * inv_s, b4.y) + res[q].y,
                                         fmaf(accy[rt][q][2], w4.z * inv_s, b4.z) + res[q].z,
                                         fmaf(accy[rt][q][3], w4.w * inv_s, b4.w) + res[q].w);
            if (rr < p.M) *reinterpret_cast<float4*>(orow + n) = y;
        }
    }
}

// W2 (d, F) -> the chunk-major, k-permuted f16x3 image: block = output panel q (16 rows);
// unit (chunk cc, panel q, term t, g, i) holds W2s[16 q + i][32 cc + 16 (e / 4) + 4 g + e % 4],
// e = 0..7, W2s = the row scaled by 2^e_row (max in [2^14, 2^15)); then wsc2[n] = 2^-e_row
__global__ void __launch_bounds__(256)
ffn_w2_split_kernel(const float* __restrict__ w, int n, int f, int64_t sn, int64_t sk,
                    float* __restrict__ wsc, u32x4* __restrict__ img) {
    const int tid = threadIdx.x, q = blockIdx.x, r0 = q * 16;
    const int ri = tid >> 4, kl = tid & 15;
    float mx = 0.f;
    if (r0 + ri < n)
        for (int j = kl; j < f; j += 16) mx = fmaxf(mx, fabsf(w[(int64_t)(r0 + ri) * sn + (int64_t)j * sk]));
    __shared__ float red[16][17];
    __shared__ float scale_inv[16];
    red[ri][kl] = mx;
    __syncthreads();
    if (tid < 16) {
        float m = 0.f;
#pragma unroll
        for (int z = 0; z < 16; ++z) m = fmaxf(m, red[tid][z]);
        const int e = m > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(m), 127) : 0;
        const bool ok = r0 + tid < n;
        scale_inv[tid] = ok ? __builtin_ldexpf(1.f, e) : 0.f;
        wsc[r0 + tid] = ok ? __builtin_ldexpf(1.f, -e) : 0.f;
    }
    __syncthreads();
    const int np = (n + 15) / 16, units = (f / 32) * 128;
    for (int u = tid; u < units; u += 256) {
        const int i = u & 15, gg = (u >> 4) & 3, t = (u >> 6) & 1, cc = u >> 7;
        const int rr = r0 + i;
        const float sc = scale_inv[i];
        f16x8 out;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int col = 32 * cc + 16 * (e >> 2) + 4 * gg + (e & 3);
            const float v = rr < n ? w[(int64_t)rr * sn + (int64_t)col * sk] * sc : 0.f;
            const _Float16 h = (_Float16)v;
            out[e] = t == 0 ? h : (_Float16)(v - (float)h);
        }
        img[((int64_t)cc * np + q) * 128 + (u & 127)] = __builtin_bit_cast(u32x4, out);
    }
}

size_t ffn_image_bytes(int n, int f) { return (size_t)(f / 32) * ((n + 15) / 16) * 128 * 16; }

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_split_weights_ffn2_bytes(int32_t n, int32_t k, size_t* bytes) {
    FGR_REQUIRE(bytes && n > 0 && k > 0 && k % 32 == 0,
                "fgr_split_weights_ffn2_bytes: bad arguments (n %d, k %d: k %% 32 == 0)", n, k);
    *bytes = ffn_image_bytes(n, k) + (size_t)((n + 15) / 16) * 16 * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_split_weights_ffn2(const float* w, int32_t n, int32_t k, int64_t stride_n,
                                      int64_t stride_k, void* img, void* stream) {
    FGR_REQUIRE(w && img && n > 0 && k > 0 && k % 32 == 0,
                "fgr_split_weights_ffn2: bad arguments (n %d, k %d)", n, k);
    FGR_REQUIRE((reinterpret_cast<uintptr_t>(img) & 15) == 0,
                "fgr_split_weights_ffn2: image not 16-B aligned");
    float* wsc = reinterpret_cast<float*>(static_cast<char*>(img) + ffn_image_bytes(n, k));
    hipLaunchKernelGGL(ffn_w2_split_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                       as_stream(stream), w, n, k, stride_n, stride_k, wsc, (u32x4*)img);
    FGR_CHECK_LAUNCH("ffn_w2_split_kernel");
    return FGR_OK;
}

extern "C" int fgr_ffn_f16x3_supported(int32_t m, int32_t d, int32_t f) {
    return (m > 0 && d == kFfnD && f >= 64 && f % 64 == 0 && f <= kFfnMaxF) ? 1 : 0;
}

extern "C" int fgr_ffn_f16x3(const float* x, int64_t ldx, const float* gamma, const float* beta,
                             float eps, const void* w1_img, const float* b1, const void* w2_img,
                             const float* b2, const float* bound, float* out, int64_t ldo,
                             int32_t m, int32_t d, int32_t f, void* stream) {
    FGR_REQUIRE(x && gamma && beta && w1_img && b1 && w2_img && b2 && bound && out && m >= 0 &&
                    ldx >= d && ldo >= d && eps >= 0.f,
                "fgr_ffn_f16x3: bad arguments");
    FGR_REQUIRE(m == 0 || fgr_ffn_f16x3_supported(m, d, f),
                "fgr_ffn_f16x3: d %d, hidden %d not supported (fgr_ffn_f16x3_supported)", d, f);
    const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gamma) |
                         reinterpret_cast<uintptr_t>(beta) | reinterpret_cast<uintptr_t>(w1_img) |
                         reinterpret_cast<uintptr_t>(b1) | reinterpret_cast<uintptr_t>(w2_img) |
                         reinterpret_cast<uintptr_t>(b2) | reinterpret_cast<uintptr_t>(out);
    FGR_REQUIRE((al & 15) == 0 && ldx % 4 == 0 && ldo % 4 == 0,
                "fgr_ffn_f16x3: operands must be 16-B aligned with row strides %% 4 == 0");
    FGR_REQUIRE(out + (size_t)m * ldo <= x || x + (size_t)m * ldx <= out || out == x,
                "fgr_ffn_f16x3: out overlaps x partially");
    if (m == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    // W1 image: fgr_split_weights_h3 of (f, d): f / 16 panels of ksteps_h3(d) = 8 k32 steps
    const char* i1 = static_cast<const char*>(w1_img);
    const char* i2 = static_cast<const char*>(w2_img);
    FfnArgs a{x, ldx, gamma, beta, eps,
              (const u32x4*)i1, (const float*)(i1 + (size_t)(f / 16) * kFfnKS * 128 * 16), b1,
              (const u32x4*)i2, (const float*)(i2 + ffn_image_bytes(d, f)), b2,
              bound, out, ldo, m, f};
    // FGR_FFN_V=1: the LDS-ring version (A/B); default the weight-split version 2 (f % 128 == 0)
    static const int ver = [] { const char* e = getenv("FGR_FFN_V"); return (e && e[0] == '1') ? 1 : 2; }();
    // row tiles per block (version 2): 3 when 48-row blocks fit one round of the CUs and
    // 64-row ones do not fill them, else 4 (FGR_FFN_RT overrides: A/B)
    static const int rt_env = [] { const char* e = getenv("FGR_FFN_RT"); return e ? atoi(e) : 0; }();
    const int rt = (rt_env >= 1 && rt_env <= 4) ? rt_env
                   : ((m + 47) / 48 <= kCusFfn && (m + 63) / 64 < kCusFfn) ? 3 : 4;
    if (ver == 2 && f % 128 == 0) {
        const unsigned nb = (unsigned)((m + 16 * rt - 1) / (16 * rt));
        switch (rt) {
            case 1: hipLaunchKernelGGL(ffn_nsplit_kernel<1>, dim3(nb), dim3(256), 0, st, a); break;
            case 2: hipLaunchKernelGGL(ffn_nsplit_kernel<2>, dim3(nb), dim3(256), 0, st, a); break;
            case 3: hipLaunchKernelGGL(ffn_nsplit_kernel<3>, dim3(nb), dim3(256), 0, st, a); break;
            default: hipLaunchKernelGGL(ffn_nsplit_kernel<4>, dim3(nb), dim3(256), 0, st, a); break;
        }
    } else
        hipLaunchKernelGGL(ffn_f16x3_kernel, dim3((unsigned)((m + 63) / 64)), dim3(256), 0, st, a);
    FGR_CHECK_LAUNCH("ffn_f16x3_kernel");
    return FGR_OK;
}

#ifdef FGR_FFN_STAMP
extern "C" int fgr_debug_ffn_stamps(void* dst, int32_t nblocks) {
    if (nblocks > 4096) nblocks = 4096;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ffn_stamp), (size_t)nblocks * 4 * 8 * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
