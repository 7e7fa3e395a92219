// Fused Res2Net hierarchy (the "fine-grained feature fusion" of my_Bottle2neck,
// res2net.py:126-148) on fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Given h = ReLU(BN1(conv1(x))) split into `scale` chunks of width w, computes in one
// launch, for i < nums (= scale - 1):
//   sp_i = ReLU(BN_i(conv_i(sp_{i-1} + h_i)))      (sp_{-1} = 0)
// with BN folded into (W_i, b_i) on the host, and writes the concatenation input of
// conv3 + downsample: cat = [sp_0 .. sp_{nums-1} | h_{nums..scale-1} | x].
// The reference runs this as 7 dependent (Linear, BN, ReLU) triples plus adds and a
// cat (21+ launches over HBM); here sp never leaves the chip between steps.
//
// Block = 32 rows (two 16-row MFMA groups) x w/16 waves; wave v owns output column
// tile v for both row groups, so every B fragment feeds 2 MFMAs and the chip holds
// ~2.5 waves per SIMD at the ModelNet sizes. The A operand (sp + h) lives in an LDS
// image a[row][g][kk] (column = 4 kk + g) read with ds_read_b128; W_i is pre-permuted
// on the host into MFMA fragment order wf[i][jt][k4][lane][4], so a wave's B operand
// for a whole step is w/16 coalesced 16-B-per-lane loads, all issued before the first
// MFMA of the step (the weights of all steps, <= 1.4 MB, stay in L2).
#include "common.h"

namespace fgr {
namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kRows = 32;

template <int KT>   // KT = w / 16 (7 for w = 112, 14 for w = 224)
__global__ void __launch_bounds__(64 * KT)
res2net_chain_kernel(const float* __restrict__ h, int64_t n, int scale, int nums,
                     const float* __restrict__ wf, const float* __restrict__ bias,
                     const float* __restrict__ x, int cin, float* __restrict__ cat, int64_t ld) {
    constexpr int W = 16 * KT, AK = W / 4 + 4;
    __shared__ float a_img[kRows * 4 * AK];
    const int tid = threadIdx.x, nth = 64 * KT;
    const int wv = tid / 64, lane = tid % 64, g = lane >> 4, c = lane & 15;
    const int64_t r0 = (int64_t)blockIdx.x * kRows;
    const int64_t hw = (int64_t)scale * W;
    const int col = wv * 16 + c;                      // this lane's output column (C layout)

    for (int i = 0; i < nums; ++i) {
        // B fragments of this wave's column tile for the whole step (in flight during the
        // A-image build below)
        float4 b4[KT];
        const float* wb = wf + (((int64_t)i * KT + wv) * KT) * 256 + lane * 4;
#pragma unroll
        for (int k4 = 0; k4 < KT; ++k4) b4[k4] = *reinterpret_cast<const float4*>(wb + k4 * 256);
        const float bc = bias[i * W + col];
        // A image = sp_{i-1} (already in a_img) + h_i; kRows*W/nth = 8 elements per thread,
        // all global loads issued before the LDS read-modify-writes
        constexpr int PER = kRows * W / (64 * KT);
        float hv[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int e = tid + j * nth;
            const int row = e / W, cc = e - row * W;
            hv[j] = (r0 + row < n) ? h[(r0 + row) * hw + (int64_t)i * W + cc] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int e = tid + j * nth;
            const int row = e / W, cc = e - row * W;
            float* ap = a_img + (row * 4 + (cc & 3)) * AK + (cc >> 2);
            *ap = i > 0 ? hv[j] + *ap : hv[j];
        }
        __syncthreads();
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < KT; ++k4) {
            const float4 a0 = *reinterpret_cast<const float4*>(a_img + (c * 4 + g) * AK + k4 * 4);
            const float4 a1 = *reinterpret_cast<const float4*>(a_img + ((16 + c) * 4 + g) * AK + k4 * 4);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b4[k4].x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b4[k4].x, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b4[k4].y, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b4[k4].y, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b4[k4].z, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b4[k4].z, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b4[k4].w, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b4[k4].w, acc1, 0, 0, 0);
        }
        __syncthreads();                              // every wave is done reading the A image
#pragma unroll
        for (int rg = 0; rg < 2; ++rg) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = rg * 16 + 4 * g + r;
                const float y = fmaxf((rg ? acc1[r] : acc0[r]) + bc, 0.f);
                if (r0 + row < n) cat[(r0 + row) * ld + (int64_t)i * W + col] = y;
                a_img[(row * 4 + (col & 3)) * AK + (col >> 2)] = y;   // sp_i for step i + 1
            }
        }
        __syncthreads();
    }
    // untouched chunks and the block input (downsample operand) into the cat buffer
    const int rest = (scale - nums) * W;
    for (int e = tid; e < kRows * rest; e += nth) {
        const int row = e / rest, cc = e - row * rest;
        if (r0 + row < n)
            cat[(r0 + row) * ld + (int64_t)nums * W + cc] = h[(r0 + row) * hw + (int64_t)nums * W + cc];
    }
    if (x) {
        for (int e = tid; e < kRows * cin; e += nth) {
            const int row = e / cin, cc = e - row * cin;
            if (r0 + row < n) cat[(r0 + row) * ld + hw + cc] = x[(r0 + row) * cin + cc];
        }
    }
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_res2net_chain(const float* h, int64_t n, int32_t w, int32_t scale,
                                 const float* w_frag, const float* bias, const float* x,
                                 int32_t cin, float* cat, int64_t ld_cat, void* stream) {
    FGR_REQUIRE(n >= 0 && scale >= 2 && (w == 112 || w == 224) && cin >= 0,
                "fgr_res2net_chain: unsupported width %d / scale %d (needs 112 or 224)", w, scale);
    FGR_REQUIRE(ld_cat >= (int64_t)scale * w + (x ? cin : 0), "fgr_res2net_chain: ld_cat too small");
    FGR_REQUIRE(n == 0 || (h && w_frag && bias && cat), "fgr_res2net_chain: null pointer");
    if (n == 0) return FGR_OK;
    const dim3 grid((unsigned)ceil_div(n, kRows));
    hipStream_t st = as_stream(stream);
    if (w == 112)
        hipLaunchKernelGGL(res2net_chain_kernel<7>, grid, dim3(64 * 7), 0, st, h, n, scale,
                           scale - 1, w_frag, bias, x, cin, cat, ld_cat);
    else
        hipLaunchKernelGGL(res2net_chain_kernel<14>, grid, dim3(64 * 14), 0, st, h, n, scale,
                           scale - 1, w_frag, bias, x, cin, cat, ld_cat);
    FGR_CHECK_LAUNCH("res2net_chain_kernel");
    return FGR_OK;
}
