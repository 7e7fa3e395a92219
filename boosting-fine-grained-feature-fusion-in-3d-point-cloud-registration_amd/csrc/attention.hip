// Fused multi-head attention (flash-style, online softmax) on packed, unpadded
// segments, fp32 in / fp32 accumulate on the CDNA4 matrix cores
// (v_mfma_f32_16x16x4_f32: exact fp32 products, one rounding per FMA).
//
// Replaces the core of nn.MultiheadAttention as used by the reference's cross
// encoder (transformers.py:95-96, 197-226): o = softmax((q * scale) k^T + mask) v
// with the key padding mask expressed as the end of the key segment.
//
// Work decomposition: block = 4 waves = 64 query rows of one (segment, head);
// each wave owns 16 rows. K/V tiles of 64 keys are staged in LDS and shared by the
// 4 waves. S = Q K^T and O += P V run on 16x16x4 MFMAs; P crosses LDS once to be
// re-read in the A-operand layout.
//
// MFMA 16x16x4 f32 lane maps (lane l, g = l >> 4, c = l & 15):
//   A[i = c][k = g], B[k = g][j = c], C/D[row = 4g + r][col = c], r = 0..3.
#include "common.h"

namespace fgr {
namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kBQ = 64;   // query rows per block
constexpr int kBK = 64;   // keys per tile

template <int DH>
__global__ void __launch_bounds__(256)
attn_fwd_kernel(const float* __restrict__ q, int64_t ld_q, const float* __restrict__ k,
                int64_t ld_k, const float* __restrict__ v, int64_t ld_v, float* __restrict__ o,
                int64_t ld_o, const int64_t* __restrict__ q_off, const int64_t* __restrict__ kv_off,
                const int32_t* __restrict__ kv_seg, float scale) {
    constexpr int KS = DH / 4;                       // k-steps of S
    constexpr int NT = DH < 16 ? 1 : DH / 16;        // 16-wide output column tiles
    constexpr int LDK = DH + 1;
    constexpr int LDP = kBK + 4;
    __shared__ float k_lds[kBK * LDK];
    __shared__ float v_lds[kBK * LDK];
    __shared__ float p_lds[4][16 * LDP];

    const int seg = blockIdx.z, head = blockIdx.y;
    const int64_t qb = q_off[seg], qe = q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)blockIdx.x * kBQ;
    if (q0 >= qe) return;                              // block-uniform
    const int ks = kv_seg[seg];
    const int64_t kb = kv_off[ks], ke = kv_off[ks + 1];
    const int nk = (int)(ke - kb);

    const int tid = threadIdx.x, wv = tid / 64, lane = tid % 64;
    const int g = lane >> 4, c = lane & 15;
    const int64_t my_q = q0 + wv * 16 + c;             // A-operand row of this lane
    const bool q_ok = my_q < qe;

    // Q fragment (pre-scaled like the reference's q * sqrt(1/E))
    float qf[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
        qf[kk] = q_ok ? q[my_q * ld_q + head * DH + kk * 4 + g] * scale : 0.f;

    f32x4 acc_o[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc_o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run[4], l_run[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { m_run[r] = -INFINITY; l_run[r] = 0.f; }

    for (int k0 = 0; k0 < nk; k0 += kBK) {
        const int nt = min(kBK, nk - k0);
        __syncthreads();
        for (int e = tid; e < kBK * DH; e += 256) {
            const int key = e / DH, d = e - key * DH;
            float kv = 0.f, vv = 0.f;
            if (key < nt) {
                const int64_t row = kb + k0 + key;
                kv = k[row * ld_k + head * DH + d];
                vv = v[row * ld_v + head * DH + d];
            }
            k_lds[key * LDK + d] = kv;
            v_lds[key * LDK + d] = vv;
        }
        __syncthreads();

        // S tile (16 rows x 64 keys per wave) = 4 MFMA column tiles
        f32x4 s[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
                const float b = k_lds[(n * 16 + c) * LDK + kk * 4 + g];
                s[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[kk], b, s[n], 0, 0, 0);
            }
        }
        // key padding -> -inf; online softmax per row 4g + r
        float alpha[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float mx = -INFINITY;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                if (n * 16 + c >= nt) s[n][r] = -INFINITY;
                mx = fmaxf(mx, s[n][r]);
            }
#pragma unroll
            for (int o2 = 8; o2 > 0; o2 >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
            const float m_new = fmaxf(m_run[r], mx);
            const float m_use = m_new == -INFINITY ? 0.f : m_new;
            alpha[r] = expf(m_run[r] - m_use);
            float rs = 0.f;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const float p = expf(s[n][r] - m_use);
                s[n][r] = p;
                rs += p;
            }
#pragma unroll
            for (int o2 = 8; o2 > 0; o2 >>= 1) rs += __shfl_xor(rs, o2, 64);
            l_run[r] = l_run[r] * alpha[r] + rs;
            m_run[r] = m_new;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc_o[t][r] *= alpha[r];

        // P: C layout -> LDS -> A layout
        float* pw = p_lds[wv];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) pw[(4 * g + r) * LDP + n * 16 + c] = s[n][r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int kk = 0; kk < kBK / 4; ++kk) {
            const float a = pw[c * LDP + kk * 4 + g];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int col = t * 16 + c;
                const float b = col < DH ? v_lds[(kk * 4 + g) * LDK + col] : 0.f;
                acc_o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc_o[t], 0, 0, 0);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }

    // O / l -> rows 4g + r, cols t*16 + c
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t row = q0 + wv * 16 + 4 * g + r;
        if (row >= qe) continue;
        const float inv = 1.0f / l_run[r];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int col = t * 16 + c;
            if (col < DH) o[row * ld_o + head * DH + col] = acc_o[t][r] * inv;
        }
    }
}

// ------------------------------------------------------------------------------------
// v2 (DH in {16, 32, 64}): each wave owns RG x 16 query rows sharing every K/V operand
// read; LDS images are laid out so that each lane's operands for 4 consecutive k-steps
// are contiguous (one ds_read_b128 per 4 MFMAs); the next K/V tile is prefetched into
// registers while the current one is consumed; softmax in base 2 on a log2(e)-prescaled Q.
//   K image  k_lds[key][g][kk]      (d = 4 kk + g),           row pad 4
//   V image  v_lds[g][dim][kk]      (key = 4 kk + g),         row pad 4
//   P image  p_lds[wave][row][g][kk] (key = 4 kk + g),        row pad 4
// ------------------------------------------------------------------------------------
template <int DH, int RG>
__global__ void __launch_bounds__(256)
attn_fwd_v2(const float* __restrict__ q, int64_t ld_q, const float* __restrict__ k,
            int64_t ld_k, const float* __restrict__ v, int64_t ld_v, float* __restrict__ o,
            int64_t ld_o, const int64_t* __restrict__ q_off, const int64_t* __restrict__ kv_off,
            const int32_t* __restrict__ kv_seg, float scale_log2) {
    constexpr int KS = DH / 4;             // k-steps of S (multiple of 4)
    constexpr int NT = DH / 16;            // output column tiles
    constexpr int KROW = DH + 4;           // K image row (floats)
    constexpr int VROW = kBK / 4 + 4;      // V image (g, dim) row: 16 kk + pad
    constexpr int PROW = kBK + 4;          // P image row
    constexpr int BQ = 64 * RG;            // query rows per block
    constexpr int F4 = kBK * DH / 4 / 256; // float4 per thread per tile (K and V each)
    static_assert(KS % 4 == 0 && F4 >= 1, "DH must be a multiple of 16");
    __shared__ float k_lds[kBK * KROW];
    __shared__ float v_lds[4 * DH * VROW];
    __shared__ float p_lds[4][16 * PROW];

    const int seg = blockIdx.z, head = blockIdx.y;
    const int64_t qb = q_off[seg], qe = q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)blockIdx.x * BQ;
    if (q0 >= qe) return;                              // block-uniform
    const int ks = kv_seg[seg];
    const int64_t kb = kv_off[ks];
    const int nk = (int)(kv_off[ks + 1] - kb);
    const int tid = threadIdx.x, wv = tid / 64, lane = tid % 64;
    const int g = lane >> 4, c = lane & 15;

    float qf[RG][KS];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
        const int64_t row = q0 + wv * 16 * RG + rg * 16 + c;
        const bool ok = row < qe;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
            qf[rg][kk] = ok ? q[row * ld_q + head * DH + kk * 4 + g] * scale_log2 : 0.f;
    }
    f32x4 acc[RG][NT];
    float m_run[RG][4], l_run[RG][4];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[rg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; ++r) { m_run[rg][r] = -INFINITY; l_run[rg][r] = 0.f; }
    }

    // tile staging: thread handles F4 float4 of K and of V per tile
    float4 kr[F4], vr[F4];
    auto load_tile = [&](int k0) {
#pragma unroll
        for (int i = 0; i < F4; ++i) {
            const int e = tid + 256 * i;             // float4 index in the 64 x DH tile
            const int key = e / (DH / 4), d0 = (e % (DH / 4)) * 4;
            if (k0 + key < nk) {
                const int64_t row = kb + k0 + key;
                kr[i] = *reinterpret_cast<const float4*>(k + row * ld_k + head * DH + d0);
                vr[i] = *reinterpret_cast<const float4*>(v + row * ld_v + head * DH + d0);
            } else {
                kr[i] = make_float4(0.f, 0.f, 0.f, 0.f);
                vr[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < F4; ++i) {
            const int e = tid + 256 * i;
            const int key = e / (DH / 4), d0 = (e % (DH / 4)) * 4;
            const int kk = d0 >> 2;                  // d = 4 kk + g, g = 0..3
            float* kp = k_lds + key * KROW + kk;
            kp[0 * KS] = kr[i].x; kp[1 * KS] = kr[i].y; kp[2 * KS] = kr[i].z; kp[3 * KS] = kr[i].w;
            const int vg = key & 3, vkk = key >> 2;  // key = 4 kk + g
            float* vp = v_lds + (vg * DH + d0) * VROW + vkk;
            vp[0 * VROW] = vr[i].x; vp[1 * VROW] = vr[i].y; vp[2 * VROW] = vr[i].z; vp[3 * VROW] = vr[i].w;
        }
    };

    load_tile(0);
    for (int k0 = 0; k0 < nk; k0 += kBK) {
        const int nt = min(kBK, nk - k0);
        __syncthreads();                             // previous tile fully consumed
        store_tile();
        __syncthreads();
        if (k0 + kBK < nk) load_tile(k0 + kBK);      // prefetch next tile (in flight)

#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
            // S = Q K^T (16 rows x 64 keys), base-2 logits
            f32x4 sv[4];
#pragma unroll
            for (int n = 0; n < 4; ++n) sv[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k4 = 0; k4 < KS; k4 += 4) {
                float4 b4[4];
#pragma unroll
                for (int n = 0; n < 4; ++n)
                    b4[n] = *reinterpret_cast<const float4*>(k_lds + (n * 16 + c) * KROW + g * KS + k4);
                // 4 independent accumulators interleaved (dependent-issue latency 40 > 32)
#pragma unroll
                for (int n = 0; n < 4; ++n) sv[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[rg][k4 + 0], b4[n].x, sv[n], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 4; ++n) sv[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[rg][k4 + 1], b4[n].y, sv[n], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 4; ++n) sv[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[rg][k4 + 2], b4[n].z, sv[n], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 4; ++n) sv[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[rg][k4 + 3], b4[n].w, sv[n], 0, 0, 0);
            }
            float alpha[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float mx = -INFINITY;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    if (n * 16 + c >= nt) sv[n][r] = -INFINITY;
                    mx = fmaxf(mx, sv[n][r]);
                }
                mx = row16_max(mx);
                const float m_new = fmaxf(m_run[rg][r], mx);
                const float m_use = m_new == -INFINITY ? 0.f : m_new;
                alpha[r] = __builtin_amdgcn_exp2f(m_run[rg][r] - m_use);
                float rs = 0.f;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const float p = __builtin_amdgcn_exp2f(sv[n][r] - m_use);
                    sv[n][r] = p;
                    rs += p;
                }
                rs = row16_sum(rs);
                l_run[rg][r] = l_run[rg][r] * alpha[r] + rs;
                m_run[rg][r] = m_new;
            }
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[rg][t][r] *= alpha[r];
            // P (C layout) -> p_lds[row][g][kk] -> A operand
            float* pw = p_lds[wv];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int pg = c & 3, pkk = n * 4 + (c >> 2);   // key n*16 + c = 4 pkk + pg
#pragma unroll
                for (int r = 0; r < 4; ++r) pw[(4 * g + r) * PROW + pg * 16 + pkk] = sv[n][r];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int k4 = 0; k4 < kBK / 4; k4 += 4) {
                const float4 a4 = *reinterpret_cast<const float4*>(pw + c * PROW + g * 16 + k4);
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const float4 b4 = *reinterpret_cast<const float4*>(
                        v_lds + (g * DH + t * 16 + c) * VROW + k4);
                    acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, acc[rg][t], 0, 0, 0);
                    acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, acc[rg][t], 0, 0, 0);
                    acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, acc[rg][t], 0, 0, 0);
                    acc[rg][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, acc[rg][t], 0, 0, 0);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = q0 + wv * 16 * RG + rg * 16 + 4 * g + r;
            if (row >= qe) continue;
            const float inv = 1.0f / l_run[rg][r];
#pragma unroll
            for (int t = 0; t < NT; ++t) o[row * ld_o + head * DH + t * 16 + c] = acc[rg][t][r] * inv;
        }
    }
}

template <int DH, int RG>
void launch_v2(int max_q_len, int n_head, int n_seg, hipStream_t st, const float* q, int64_t ld_q,
               const float* k, int64_t ld_k, const float* v, int64_t ld_v, float* o, int64_t ld_o,
               const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg, float scale) {
    dim3 grid((unsigned)ceil_div(max_q_len, 64 * RG), (unsigned)n_head, (unsigned)n_seg);
    hipLaunchKernelGGL((attn_fwd_v2<DH, RG>), grid, dim3(256), 0, st, q, ld_q, k, ld_k, v, ld_v,
                       o, ld_o, q_off, kv_off, kv_seg, scale * 1.4426950408889634f);
}

template <int DH>
void launch(dim3 grid, hipStream_t st, const float* q, int64_t ld_q, const float* k, int64_t ld_k,
            const float* v, int64_t ld_v, float* o, int64_t ld_o, const int64_t* q_off,
            const int64_t* kv_off, const int32_t* kv_seg, float scale) {
    hipLaunchKernelGGL(attn_fwd_kernel<DH>, grid, dim3(256), 0, st, q, ld_q, k, ld_k, v, ld_v, o,
                       ld_o, q_off, kv_off, kv_seg, scale);
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_attention(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                             const float* v, int64_t ld_v, float* o, int64_t ld_o,
                             const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                             int32_t n_seg, int32_t max_q_len, int32_t n_head, int32_t head_dim,
                             float scale, void* stream) {
    FGR_REQUIRE(q && k && v && o && q_off && kv_off && kv_seg && n_seg > 0 && n_head > 0 &&
                    max_q_len >= 0,
                "fgr_attention: bad arguments");
    FGR_REQUIRE(ld_q >= n_head * head_dim && ld_k >= n_head * head_dim &&
                    ld_v >= n_head * head_dim && ld_o >= n_head * head_dim,
                "fgr_attention: row stride smaller than n_head * head_dim");
    if (max_q_len == 0) return FGR_OK;
    dim3 grid((unsigned)ceil_div(max_q_len, kBQ), (unsigned)n_head, (unsigned)n_seg);
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    switch (head_dim) {
        case 4: launch<4>(grid, st, q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, scale); break;
        case 8: launch<8>(grid, st, q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, scale); break;
        case 16: launch_v2<16, 2>(max_q_len, n_head, n_seg, st, q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, scale); break;
        case 32: launch_v2<32, 2>(max_q_len, n_head, n_seg, st, q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, scale); break;
        case 64: launch_v2<64, 2>(max_q_len, n_head, n_seg, st, q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, scale); break;
        case 128: launch<128>(grid, st, q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, scale); break;
        case 256: launch<256>(grid, st, q, ld_q, k, ld_k, v, ld_v, o, ld_o, q_off, kv_off, kv_seg, scale); break;
        default:
            set_error("fgr_attention: head_dim %d unsupported (4, 8, 16, 32, 64, 128, 256)", head_dim);
            return FGR_E_ARG;
    }
    FGR_CHECK_LAUNCH("attn_fwd_kernel");
    return FGR_OK;
}


// ------------------------------------------------------------------------------------------
// CorrespondenceDecoder.simple_attention (finegrained_regtr.py:328-363), the soft
// correspondence head used with direct_regress_coor: False: one head of width d whose values
// are the partner cloud's coordinates (3 columns),
//   corr[q] = sum_j softmax_j((q . k_j) * scale) * xyz[j],
// for every (layer, cloud) query segment in ONE launch (segment i attends to key segment
// kv_seg[i]; the reference's key padding mask is the segment end). fp32 throughout: a block
// holds 32 queries x 8 lanes (each lane a d/8 slice of the dot product, reduced over its 8
// lanes with DPP), key rows are staged 32 at a time through LDS, and the softmax is online
// (running max / sum, the 3 value sums rescaled on each new max).
// ------------------------------------------------------------------------------------------
namespace fgr {
namespace {

constexpr int kCaQ = 32;      // queries per block
constexpr int kCaK = 32;      // keys per LDS tile

template <int D>
__global__ void __launch_bounds__(256)
corr_attention_kernel(const float* __restrict__ q, int64_t ld_q, const float* __restrict__ k,
                      int64_t ld_k, const float* __restrict__ xyz, float* __restrict__ out,
                      const int64_t* __restrict__ q_off, const int64_t* __restrict__ kv_off,
                      const int32_t* __restrict__ kv_seg, const int64_t* __restrict__ v_off,
                      float scale) {
    constexpr int DL = D / 8;                              // dims per lane
    __shared__ float kt[kCaK][D + 4];
    __shared__ float vt[kCaK][3];
    const int seg = blockIdx.y;
    const int64_t qb = q_off[seg], qe = q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)blockIdx.x * kCaQ;
    if (q0 >= qe) return;                                  // block-uniform
    const int ks = kv_seg[seg];
    const int64_t kb = kv_off[ks], ke = kv_off[ks + 1];
    const int64_t vb = v_off[ks];                          // value rows of key segment ks
    const int tid = threadIdx.x, qi = tid >> 3, sl = tid & 7;
    const int64_t row = q0 + qi;
    const bool active = row < qe;
    float qv[DL];
#pragma unroll
    for (int e = 0; e < DL; ++e) qv[e] = active ? q[row * ld_q + sl * DL + e] * scale : 0.f;
    float m = -INFINITY, l = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int64_t j0 = kb; j0 < ke; j0 += kCaK) {
        const int nk = (int)min((int64_t)kCaK, ke - j0);
        __syncthreads();
        for (int e = tid; e < kCaK * D; e += 256) {
            const int r = e / D, cc = e - r * D;
            kt[r][cc] = r < nk ? k[(j0 + r) * ld_k + cc] : 0.f;
        }
        if (tid < kCaK * 3) {
            const int r = tid / 3, cc = tid - r * 3;
            vt[r][cc] = r < nk ? xyz[(vb + (j0 - kb) + r) * 3 + cc] : 0.f;
        }
        __syncthreads();
        for (int r = 0; r < nk; ++r) {
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < DL; ++e) s = fmaf(qv[e], kt[r][sl * DL + e], s);
            s += dpp<0xB1>(s);                             // the 8 lanes of this query
            s += dpp<0x4E>(s);
            s += dpp<0x141>(s);
            if (s > m) {
                const float f = __expf(m - s);
                l *= f; a0 *= f; a1 *= f; a2 *= f;
                m = s;
            }
            const float p = __expf(s - m);
            l += p;
            a0 = fmaf(p, vt[r][0], a0);
            a1 = fmaf(p, vt[r][1], a1);
            a2 = fmaf(p, vt[r][2], a2);
        }
    }
    if (active && sl == 0) {
        const float inv = 1.0f / l;
        out[row * 3 + 0] = a0 * inv;
        out[row * 3 + 1] = a1 * inv;
        out[row * 3 + 2] = a2 * inv;
    }
}

// ---- num_neighbors > 0 (finegrained_regtr.py:353-357) ------------------------------------
// The reference builds neighbor_mask (L, B, Q, S) = -inf and then runs
//   neighbor_mask[:, :, topk(attn, k).indices] = 0,
// which indexes the QUERY dimension with the top-k KEY indices of every (layer, pair, query)
// row: query row j of every layer and pair keeps its plain softmax iff j is among the union of
// all top-k key indices of that direction, every other query row is all -inf and its softmax
// (hence its correspondence) is NaN. Restated here as: scores (the same q.k * scale as
// corr_attention_kernel) -> per-row top-k by successive maxima -> a byte flag per index of
// the direction's union -> NaN rows. Ties rank the lower key index first.

// scores[row * ld_s + (j - kb)] for every key j of the row's key segment.
template <int D>
__global__ void __launch_bounds__(256)
corr_scores_kernel(const float* __restrict__ q, int64_t ld_q, const float* __restrict__ k,
                   int64_t ld_k, const int64_t* __restrict__ q_off,
                   const int64_t* __restrict__ kv_off, const int32_t* __restrict__ kv_seg,
                   float scale, float* __restrict__ scores, int64_t ld_s) {
    constexpr int DL = D / 8;
    __shared__ float kt[kCaK][D + 4];
    const int seg = blockIdx.y;
    const int64_t qb = q_off[seg], qe = q_off[seg + 1];
    const int64_t q0 = qb + (int64_t)blockIdx.x * kCaQ;
    if (q0 >= qe) return;
    const int ks = kv_seg[seg];
    const int64_t kb = kv_off[ks], ke = kv_off[ks + 1];
    const int tid = threadIdx.x, qi = tid >> 3, sl = tid & 7;
    const int64_t row = q0 + qi;
    const bool active = row < qe;
    float qv[DL];
#pragma unroll
    for (int e = 0; e < DL; ++e) qv[e] = active ? q[row * ld_q + sl * DL + e] * scale : 0.f;
    for (int64_t j0 = kb; j0 < ke; j0 += kCaK) {
        const int nk = (int)min((int64_t)kCaK, ke - j0);
        __syncthreads();
        for (int e = tid; e < kCaK * D; e += 256) {
            const int r = e / D, cc = e - r * D;
            kt[r][cc] = r < nk ? k[(j0 + r) * ld_k + cc] : 0.f;
        }
        __syncthreads();
        for (int r = 0; r < nk; ++r) {
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < DL; ++e) s = fmaf(qv[e], kt[r][sl * DL + e], s);
            s += dpp<0xB1>(s);
            s += dpp<0x4E>(s);
            s += dpp<0x141>(s);
            if (active && sl == 0) scores[row * ld_s + (j0 - kb) + r] = s;
        }
    }
}

// (value, index) ordered by value descending, then index ascending: a ranks before b.
__device__ __forceinline__ bool rank_before(float va, int ia, float vb, int ib) {
    return va > vb || (va == vb && ia < ib);
}

// One wave per query row: n_top rounds, each taking the best-ranked key strictly after the
// previous round's winner (no writes to the scores), flagging its index in the direction's
// union (flags[dir * ld_f + j] = 1; concurrent writers store the same byte).
__global__ void __launch_bounds__(256)
corr_topk_flags_kernel(const float* __restrict__ scores, int64_t ld_s,
                       const int64_t* __restrict__ q_off, const int64_t* __restrict__ kv_off,
                       const int32_t* __restrict__ kv_seg, int32_t n_clouds, int32_t n_top,
                       uint8_t* __restrict__ flags, int64_t ld_f) {
    const int seg = blockIdx.y;
    const int64_t row = q_off[seg] + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= q_off[seg + 1]) return;                     // wave-uniform
    const int lane = threadIdx.x & 63;
    const int ks = kv_seg[seg];
    const int nk = (int)(kv_off[ks + 1] - kv_off[ks]);
    const int dir = (seg % n_clouds) >= n_clouds / 2;
    const float* sr = scores + row * ld_s;
    float pv = INFINITY;
    int pi = -1;                                           // previous winner: ranks before all
    for (int t = 0; t < n_top; ++t) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        for (int j = lane; j < nk; j += 64) {
            const float v = sr[j];
            if (rank_before(pv, pi, v, j) && rank_before(v, j, bv, bi)) { bv = v; bi = j; }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const float ov = __shfl_xor(bv, o);
            const int oi = __shfl_xor(bi, o);
            if (rank_before(ov, oi, bv, bi)) { bv = ov; bi = oi; }
        }
        if (bi == 0x7fffffff) break;                       // fewer than n_top keys (rejected on the host)
        if (lane == 0) flags[dir * ld_f + bi] = 1;
        pv = bv;
        pi = bi;
    }
}

// corr rows whose in-cloud index is not in their direction's union become NaN (the softmax of
// an all -inf row).
__global__ void __launch_bounds__(256)
corr_nan_rows_kernel(float* __restrict__ out, const int64_t* __restrict__ q_off,
                     int32_t n_clouds, const uint8_t* __restrict__ flags, int64_t ld_f) {
    const int seg = blockIdx.y;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = q_off[seg] + j;
    if (row >= q_off[seg + 1]) return;
    const int dir = (seg % n_clouds) >= n_clouds / 2;
    if (j >= ld_f || !flags[dir * ld_f + j]) {             // an index >= S is never in the union
        const float nan = __builtin_nanf("");
        out[row * 3 + 0] = nan;
        out[row * 3 + 1] = nan;
        out[row * 3 + 2] = nan;
    }
}

}  // namespace
}  // namespace fgr

extern "C" int fgr_corr_attention(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                  const float* xyz, float* out, const int64_t* q_off,
                                  const int64_t* kv_off, const int32_t* kv_seg,
                                  const int64_t* v_off, int32_t n_seg, int32_t max_q_len,
                                  int32_t d, float scale, void* stream) {
    FGR_REQUIRE(q && k && xyz && out && q_off && kv_off && kv_seg && v_off && n_seg > 0 &&
                    max_q_len >= 0 && ld_q >= d && ld_k >= d,
                "fgr_corr_attention: bad arguments");
    FGR_REQUIRE(d == 32 || d == 64 || d == 128 || d == 256 || d == 512,
                "fgr_corr_attention: d %d unsupported (32, 64, 128, 256, 512)", d);
    if (max_q_len == 0) return FGR_OK;
    hipStream_t st = as_stream(stream);
    TimedCall timed_(st);
    const dim3 grid((unsigned)ceil_div(max_q_len, kCaQ), (unsigned)n_seg);
#define FGR_CA(DD)                                                                              \
    case DD:                                                                                    \
        hipLaunchKernelGGL(corr_attention_kernel<DD>, grid, dim3(256), 0, st, q, ld_q, k, ld_k, \
                           xyz, out, q_off, kv_off, kv_seg, v_off, scale);                      \
        break;
    switch (d) {
        FGR_CA(32)
        FGR_CA(64)
        FGR_CA(128)
        FGR_CA(256)
        FGR_CA(512)
    }
#undef FGR_CA
    FGR_CHECK_LAUNCH("corr_attention_kernel");
    return FGR_OK;
}

extern "C" int fgr_corr_topk_workspace(int64_t n_rows, int32_t max_kv_len, size_t* bytes) {
    FGR_REQUIRE(bytes && n_rows >= 0 && max_kv_len >= 0, "fgr_corr_topk_workspace: bad arguments");
    *bytes = (size_t)n_rows * (size_t)max_kv_len * sizeof(float);
    return FGR_OK;
}

extern "C" int fgr_corr_topk_mask(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                                  float* out, const int64_t* q_off, const int64_t* kv_off,
                                  const int32_t* kv_seg, int32_t n_seg, int32_t n_clouds,
                                  int64_t n_rows, int32_t max_q_len, int32_t max_kv_len, int32_t d,
                                  float scale, int32_t n_top, uint8_t* flags, void* ws,
                                  size_t ws_bytes, void* stream) {
    FGR_REQUIRE(q && k && out && q_off && kv_off && kv_seg && flags && n_seg > 0 && n_rows >= 0 &&
                    n_clouds > 0 && n_clouds % 2 == 0 && max_q_len >= 0 && max_kv_len >= 0 &&
                    n_top > 0 && ld_q >= d && ld_k >= d,
                "fgr_corr_topk_mask: bad arguments");
    FGR_REQUIRE(d == 32 || d == 64 || d == 128 || d == 256 || d == 512,
                "fgr_corr_topk_mask: d %d unsupported (32, 64, 128, 256, 512)", d);
    size_t need = 0;
    fgr_corr_topk_workspace(n_rows, max_kv_len, &need);
    FGR_REQUIRE(ws && ws_bytes >= need, "fgr_corr_topk_mask: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    FGR_REQUIRE(hipMemsetAsync(flags, 0, 2 * (size_t)max_kv_len, st) == hipSuccess,
                "fgr_corr_topk_mask: memset failed");
    if (max_q_len == 0 || max_kv_len == 0) return FGR_OK;
    float* scores = (float*)ws;
    const dim3 grid((unsigned)ceil_div(max_q_len, kCaQ), (unsigned)n_seg);
#define FGR_CS(DD)                                                                                \
    case DD:                                                                                      \
        hipLaunchKernelGGL(corr_scores_kernel<DD>, grid, dim3(256), 0, st, q, ld_q, k, ld_k,      \
                           q_off, kv_off, kv_seg, scale, scores, (int64_t)max_kv_len);            \
        break;
    switch (d) {
        FGR_CS(32)
        FGR_CS(64)
        FGR_CS(128)
        FGR_CS(256)
        FGR_CS(512)
    }
#undef FGR_CS
    FGR_CHECK_LAUNCH("corr_scores_kernel");
    hipLaunchKernelGGL(corr_topk_flags_kernel, dim3((unsigned)ceil_div(max_q_len, 4), (unsigned)n_seg),
                       dim3(256), 0, st, scores, (int64_t)max_kv_len, q_off, kv_off, kv_seg, n_clouds,
                       n_top, flags, (int64_t)max_kv_len);
    FGR_CHECK_LAUNCH("corr_topk_flags_kernel");
    hipLaunchKernelGGL(corr_nan_rows_kernel, dim3((unsigned)ceil_div(max_q_len, 256), (unsigned)n_seg),
                       dim3(256), 0, st, out, q_off, n_clouds, flags, (int64_t)max_kv_len);
    FGR_CHECK_LAUNCH("corr_nan_rows_kernel");
    return FGR_OK;
}
