// "g5" GEMM structure for the dense layers (f16x3 and bf16 modes):
//
//   C[M, N] = act(A[M, K] . W[N, K]^T + bias[N] (+ R[M, N]))
//
// Why a new structure. The forward's GEMMs are short and skinny (M ~ 2k-57k activation rows,
// K = 64..3840, N = 64..1792); at K = 256 a block runs 8 k32-steps. The register-staged
// kernels of gemm16.hip split A once per block into an LDS image and keep one k-step in
// flight, so each k-step waits a full HBM / L2 round trip (~1-2 us under load) and the
// ds_write_b128 pass of the split image (13 cycles per wave-instruction) sits on the
// critical path: 9544 x 768 x 256 ran at 27 us where the fp16 pipe needs 4.5 us.
//
// Structure:
//   * both operands travel global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR
//     destination), S stages in flight (counted vmcnt, raw s_barrier: one barrier per stage),
//     KS k32-steps per stage;
//   * A is staged as raw fp32 (full 128-B row lines, 16-B chunks XOR-swizzled by row bits 1
//     and 3 on the SOURCE address so the fragment reads are bank-conflict-free) and split
//     into fp16 terms in registers after the read. Every wave owns BM / 4 distinct rows, so
//     each A element is read and split exactly once per block (no LDS write pass at all);
//   * W images (fgr_split_weights_h3 / _bf16) are DMA'd as they lie (already in fragment
//     order) and shared by the 4 waves;
//   * swapped orientation as gemm16.hip: W fragments are the MFMA A operand, activations the
//     B operand, so each lane's 4 accumulators belong to ONE activation row -- the f16x3
//     per-row scale (and its rare in-flight lowering) is lane-local, the epilogue stores
//     16-B float4s.
// f16x3 precision contract: identical to gemm16.hip (row scales chosen per 32-wide chunk
// into [2^7, 2^8) and lowered only on overflow risk, two fp16 terms per operand, the three
// significant products hh, hm, mh in fp32 accumulation).
// Lane maps of v_mfma_f32_16x16x32_{f16,bf16} (lane l, g = l >> 4, c = l & 15): A[i = c][k =
// 8g + e], B[k = 8g + e][j = c], C[i = 4g + r][j = c].
#include "common.h"

namespace fgr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int SH_UNSET = 0x3fff;

// 16 zero bytes: the DMA source of A chunks past K (the LDS image gets exact zeros, so no
// register-side masking is needed)
__device__ __attribute__((aligned(16))) float g5_zero[4];

struct G5Args {
    const float* A; int64_t lda;
    const float* zero;                // g5_zero's device address (no GOT load in the loop)
    const u32x4* W; int ksteps;       // image [panel][kstep][term][g 4][16] x 16 B
    const float* wsc;                 // f16x3: per n 2^-e_n (padded to 16); bf16: unused
    float* C; int64_t ldc;
    const float* bias;
    const float* R; int64_t ldr;
    int M, N, K, act, vec_out;
    int ksplit; float* part;          // split-K: partials [ksplit][M][N] (scaled, no epilogue)
    // K / V attention images (head dim 64, staged-epilogue 64 x 128 tiles only): columns >=
    // kv_col0 go to the f16x3 images of their GLOBAL 64-row tile and head (attention16.hip
    // layout) instead of C; the k | v columns are the last 128 n_head
    char* kv_img; int2* kv_sc; int n_head; int kv_col0;
};

// f16x3 attention image geometry for head dim 64 (attention16.hip units<64>, unit_v<64>,
// v_swz<64>): 2048 16-B units per (tile, head), V from unit 1024
constexpr int kKv64Units = 2048;
constexpr int kKv64UnitV = 1024;

// chunk swizzle of A row r (16-B chunk q of a 128-B row line lands at q ^ swz(r)): rows
// {0-3, 12-15} and {4-11} of one ds_read_b128 lane group hit 16 distinct 16-B bank slots
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 5; }

// s_waitcnt vmcnt(n) (expcnt / lgkmcnt: no wait) -- gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
// s_waitcnt vmcnt(n) lgkmcnt(0)
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}

__device__ __forceinline__ float xg_max(float v) {        // max over lanes c, c^16, c^32, c^48
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float finish5(float y, float b, float r, int act) {
    if (act == FGR_ACT_RELU_RES_LEAKY) {
        const float t = fmaxf(y + b, 0.f) + r;
        return t > 0.f ? t : 0.1f * t;
    }
    const float t = y + b + r;
    return act == FGR_ACT_RELU ? fmaxf(t, 0.f) : t;
}

// TERMS 2: f16x3 (W image with hi / lo terms + row scales); 1: bf16 (single-term image).
// KW k-groups of 4 waves (intra-block split-K): group h computes the k32-steps ks = h, h + KW,
// ... of every stage for the same rows, so a block of a short-M GEMM (~1 block per CU) keeps
// KW waves per SIMD and one wave's convert / LDS-read VALU work overlaps another's MFMAs; the
// groups' accumulators are merged through LDS at the end (fixed order, deterministic).
// WC waves across the columns (1: every wave owns BM / 4 rows x all BN columns; 2: a 2 x 2
// layout, BM / 2 rows x BN / 2 columns per wave -- a third less LDS read traffic per MFMA,
// each A row split by the two waves that share it).
template <int BM, int BN, int KS, int S, int TERMS, bool PIPE, int KW = 1, int WC = 1,
          bool EPI_LDS = false>
__global__ void __launch_bounds__(256 * KW) gemm_g5(G5Args p) {
    constexpr int NW = 4 * KW;                 // waves per block
    constexpr int RW = 4 / WC;                 // waves across the rows
    constexpr int WR = BM / RW;                // rows per wave
    constexpr int TM = WR / 16;                // 16-row fragments per wave
    constexpr int TN = BN / 16;                // W panels per block
    constexpr int TNW = TN / WC;               // W panels per wave
    constexpr int A_UNITS = BM * 8 * KS;       // [ks][row][8 chunks] x 16 B
    constexpr int W_PANEL = TERMS * 64;        // units of one (panel, kstep)
    constexpr int W_UNITS = TN * KS * W_PANEL;
    constexpr int ST = A_UNITS + W_UNITS;      // units per stage
    constexpr int NP = ST / 64;                // DMA wave-instructions per stage
    constexpr int A_PIECES = A_UNITS / 64;
    static_assert(TM >= 1 && TNW >= 1 && TN % WC == 0 && NP % NW == 0 && KS % KW == 0, "tile");
    static_assert(!PIPE || KW == 1, "pipelined g5: one k-group");
    constexpr int P = NP / NW;                 // per wave per stage
    __shared__ u32x4 lds[S * ST];

    const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
    const int nwg = nbm * nbn, ntot = nwg * p.ksplit;
    int t = blockIdx.x;
    {   // XCD-aware bijective remap: consecutive tiles (n fastest) on one XCD
        const int q = ntot / 8, r = ntot % 8, x = t % 8, lo = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lo;
    }
    const int kz = t / nwg;                    // split-K part (0 without split)
    t %= nwg;
    const int bm = t / nbn, bn = t % nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform
    const int w4 = wv & 3, kg = wv >> 2;                     // wave in its k-group, k-group
    const int rw = w4 / WC, cw = w4 % WC;                    // row slice, column slice
    const int g = lane >> 4, c = lane & 15;
    const int npanel = (p.N + 15) / 16;
    // stages: [sb, sb + nk) of the K range (split-K: this block's share)
    const int nk_all = (p.K + 32 * KS - 1) / (32 * KS);
    const int sb = (int)((int64_t)kz * nk_all / p.ksplit);
    const int nk = (int)((int64_t)(kz + 1) * nk_all / p.ksplit) - sb;

    // ---- DMA sources of this wave's P pieces (per stage: + stage * KS * 32 floats / units)
    // (A_PIECES % NW == 0: piece j of every wave is an A piece iff j < A_PIECES / NW)
    static_assert(A_PIECES % NW == 0, "A pieces");
    const float* asrc[P];
    int akoff[P];                                            // k offset of the chunk in its step
    const u32x4* wsrc[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int q = wv + NW * j;
        if (j < A_PIECES / NW) {
            const int ks = q / (BM / 8);
            const int row = (q % (BM / 8)) * 8 + (lane >> 3);
            const int ch = (lane & 7) ^ swz(row);
            akoff[j] = ks * 32 + 4 * ch;
            asrc[j] = p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + akoff[j];
            wsrc[j] = nullptr;
        } else {
            const int w = q - A_PIECES;
            const int panel = w / (KS * TERMS), rem = w % (KS * TERMS);
            const int ks = rem / TERMS, term = rem % TERMS;
            const int pg = min(n0 / 16 + panel, npanel - 1);
            wsrc[j] = p.W + ((int64_t)pg * p.ksteps + ks) * W_PANEL + term * 64 + lane;
            asrc[j] = nullptr;
            akoff[j] = 0;
        }
    }
    auto issue = [&](int sl) {
        lds_void* base = (lds_void*)(lds + (sl % S) * ST);
        const int s = sb + sl;                                 // global stage
        const int k0 = s * KS * 32;
        if (k0 + KS * 32 <= p.K) {                              // wave-uniform: no K tail
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int q = wv + NW * j;
                lds_void* dst = (lds_void*)((__attribute__((address_space(3))) char*)base + q * 1024);
                const void* src = j < A_PIECES / NW ? (const void*)(asrc[j] + k0)
                                                    : (const void*)(wsrc[j] + (int64_t)s * KS * W_PANEL);
                __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int q = wv + NW * j;
                lds_void* dst = (lds_void*)((__attribute__((address_space(3))) char*)base + q * 1024);
                const void* src;
                if (j < A_PIECES / NW) {
                    src = k0 + akoff[j] < p.K ? (const void*)(asrc[j] + k0) : (const void*)p.zero;
                } else {
                    src = wsrc[j] + (int64_t)s * KS * W_PANEL;
                }
                __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
            }
        }
    };

    f32x4 acc[TNW][TM];
#pragma unroll
    for (int j = 0; j < TNW; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int sh[TM];
    float scv[TM];                             // 2^sh (1 while unset)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        sh[i] = SH_UNSET;
        scv[i] = 1.f;
    }

    // fragment reads of one k32-step: this wave's W panels (A operand) and raw fp32 rows
    auto read_frags = [&](const u32x4* st, int ks, u32x4 (&ua)[TM][2], u32x4 (&wf)[TNW][TERMS]) {
#pragma unroll
        for (int j = 0; j < TNW; ++j)
#pragma unroll
            for (int tt = 0; tt < TERMS; ++tt)
                wf[j][tt] = st[A_UNITS + ((cw * TNW + j) * KS + ks) * W_PANEL + tt * 64 + lane];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row = rw * WR + 16 * i + c;
            const u32x4* ar = st + (ks * BM + row) * 8;
            ua[i][0] = ar[(2 * g) ^ swz(row)];
            ua[i][1] = ar[(2 * g + 1) ^ swz(row)];
        }
    };
    // activation fragments (B operand): f16x3 row scaling + two-term split, or bf16 rounding
    auto convert = [&](const u32x4 (&ua)[TM][2], u32x4 (&bh)[TM], u32x4 (&bl)[TM]) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const u32x4 u0 = ua[i][0], u1 = ua[i][1];
            const float x[8] = {__uint_as_float(u0[0]), __uint_as_float(u0[1]),
                                __uint_as_float(u0[2]), __uint_as_float(u0[3]),
                                __uint_as_float(u1[0]), __uint_as_float(u1[1]),
                                __uint_as_float(u1[2]), __uint_as_float(u1[3])};
            if constexpr (TERMS == 2) {
                // the lowering test is monotone in the row max, so a lane whose own 8 values
                // do not trigger it cannot make the row trigger: the exact row max (2
                // permlane swaps) is only formed when some lane's values do (first chunk of
                // a row, or a chunk that grows past the current scale)
                float cm = max3_abs(x[0], x[1], x[2]);
                cm = max3_abs(x[3], x[4], cm);
                cm = fmaxf(cm, max3_abs(x[5], x[6], x[7]));
                const bool may = cm > 0.f && __builtin_amdgcn_frexp_expf(cm) + sh[i] > 15;
                if (__builtin_amdgcn_ballot_w64(may)) {
                    cm = xg_max(cm);
                    const bool lower = cm > 0.f && __builtin_amdgcn_frexp_expf(cm) + sh[i] > 15;
                    const int nsh = lower ? min(8 - __builtin_amdgcn_frexp_expf(cm), 127) : sh[i];
                    const float f = (sh[i] == SH_UNSET || !lower) ? 1.f
                                                                   : __builtin_ldexpf(1.f, nsh - sh[i]);
#pragma unroll
                    for (int j = 0; j < TNW; ++j) acc[j][i] *= f;
                    sh[i] = nsh;
                    scv[i] = __builtin_ldexpf(1.f, sh[i] == SH_UNSET ? 0 : sh[i]);
                }
                // hi = f16(x sc), lo = f16(x sc - hi) by v_fma_mix (x sc exact: power of two;
                // x sc - hi exact in fp32): one VALU per term and element
                split8_f16(x, scv[i], bh[i], bl[i]);
            } else {
                bf16x8 h;
#pragma unroll
                for (int e = 0; e < 8; ++e) h[e] = (__bf16)x[e];
                bh[i] = __builtin_bit_cast(u32x4, h);
                bl[i] = bh[i];
            }
        }
    };
    auto mma = [&](const u32x4 (&wf)[TNW][TERMS], const u32x4 (&bh)[TM], const u32x4 (&bl)[TM]) {
#pragma unroll
        for (int j = 0; j < TNW; ++j) {
            if constexpr (TERMS == 2) {
                const f16x8 wh = __builtin_bit_cast(f16x8, wf[j][0]);
                const f16x8 wl = __builtin_bit_cast(f16x8, wf[j][1]);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const f16x8 ah = __builtin_bit_cast(f16x8, bh[i]);
                    const f16x8 al = __builtin_bit_cast(f16x8, bl[i]);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, al, acc[j][i], 0, 0, 0);
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, acc[j][i], 0, 0, 0);
                }
            } else {
                const bf16x8 wb = __builtin_bit_cast(bf16x8, wf[j][0]);
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        wb, __builtin_bit_cast(bf16x8, bh[i]), acc[j][i], 0, 0, 0);
            }
        }
    };

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nk) issue(s);

    if constexpr (!PIPE) {
        for (int s = 0; s < nk; ++s) {
            // this wave's DMAs of stage s retired (later stages may stay in flight), then the
            // barrier makes every wave's pieces visible and retires all reads of the buffer
            // that is refilled next
            const int ahead = min(S - 2, nk - 1 - s);
            if constexpr (S >= 4) {
                if (ahead >= 2) wait_vm_lgkm0<2 * P>();
                else if (ahead == 1) wait_vm_lgkm0<P>();
                else wait_vm_lgkm0<0>();
            } else {
                if (ahead >= 1) wait_vm_lgkm0<P>();
                else wait_vm_lgkm0<0>();
            }
            __builtin_amdgcn_s_barrier();
            if (s + S - 1 < nk) issue(s + S - 1);
            const u32x4* st = lds + (s % S) * ST;
#pragma unroll
            for (int kk = 0; kk < KS / KW; ++kk) {
                const int ks = kk * KW + kg;
                u32x4 ua[TM][2], wf[TNW][TERMS], bh[TM], bl[TM];
                read_frags(st, ks, ua, wf);
                convert(ua, bh, bl);
                mma(wf, bh, bl);
            }
        }
    } else {
        // software-pipelined (KS == 1): the fragments of stage s + 1 are read and split while
        // the MFMAs of stage s run from registers
        static_assert(KS == 1 && S >= 3, "pipelined g5: one k32-step per stage, >= 3 stages");
        {
            const int ahead = min(S - 2, nk - 1);
            if (ahead >= 2) wait_vm_lgkm0<2 * P>();
            else if (ahead == 1) wait_vm_lgkm0<P>();
            else wait_vm_lgkm0<0>();
        }
        __builtin_amdgcn_s_barrier();
        u32x4 ua[TM][2], wf[TNW][TERMS], bh[TM], bl[TM];
        read_frags(lds, 0, ua, wf);
        convert(ua, bh, bl);
        for (int s = 0; s < nk; ++s) {
            if (s + 1 < nk) {
                // stage s + 1 landed (stages up to s + S - 2 were issued; keep the later ones
                // in flight); the barrier also retires every wave's reads of stage s
                const int ahead = min(S - 3, nk - 2 - s);
                if constexpr (S >= 5) {
                    if (ahead >= 2) wait_vm_lgkm0<2 * P>();
                    else if (ahead == 1) wait_vm_lgkm0<P>();
                    else wait_vm_lgkm0<0>();
                } else if constexpr (S == 4) {
                    if (ahead >= 1) wait_vm_lgkm0<P>();
                    else wait_vm_lgkm0<0>();
                } else {
                    wait_vm_lgkm0<0>();
                }
                __builtin_amdgcn_s_barrier();
                if (s + S - 1 < nk) issue(s + S - 1);
                u32x4 ua2[TM][2], wf2[TNW][TERMS];
                read_frags(lds + ((s + 1) % S) * ST, 0, ua2, wf2);
                mma(wf, bh, bl);
                convert(ua2, bh, bl);
#pragma unroll
                for (int j = 0; j < TNW; ++j)
#pragma unroll
                    for (int tt = 0; tt < TERMS; ++tt) wf[j][tt] = wf2[j][tt];
            } else {
                mma(wf, bh, bl);
            }
        }
    }

    if constexpr (KW == 2) {
        // merge the k-groups: group 1 parks its accumulators (+ f16x3 row exponents) in the
        // drained stage buffers, group 0 adds them at the common (smaller) row scale; every
        // DMA retired at the last stage (vmcnt 0), the barrier retires every stage read
        static_assert(S * ST * 16 >= 4 * TNW * TM * 64 * 16 + 4 * TM * 64 * 4, "merge space");
        __syncthreads();
        f32x4* xa = reinterpret_cast<f32x4*>(lds);
        int* xs = reinterpret_cast<int*>(xa + 4 * TNW * TM * 64);
        if (kg == 1) {
#pragma unroll
            for (int j = 0; j < TNW; ++j)
#pragma unroll
                for (int i = 0; i < TM; ++i) xa[((w4 * TNW + j) * TM + i) * 64 + lane] = acc[j][i];
#pragma unroll
            for (int i = 0; i < TM; ++i) xs[(w4 * TM + i) * 64 + lane] = sh[i];
        }
        __syncthreads();
        if (kg == 1) return;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            float f0 = 1.f, f1 = 1.f;
            if constexpr (TERMS == 2) {
                // an unset exponent means that group saw only zeros (its accumulators are 0)
                const int s1 = xs[(w4 * TM + i) * 64 + lane];
                if (s1 != SH_UNSET) {
                    if (sh[i] == SH_UNSET) {
                        sh[i] = s1;
                    } else {
                        const int s0 = min(sh[i], s1);
                        f0 = __builtin_ldexpf(1.f, s0 - sh[i]);
                        f1 = __builtin_ldexpf(1.f, s0 - s1);
                        sh[i] = s0;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < TNW; ++j)
                acc[j][i] = acc[j][i] * f0 + xa[((w4 * TNW + j) * TM + i) * 64 + lane] * f1;
        }
    }

    if (p.ksplit > 1) {
        // split-K: this part's scaled product, no bias / residual / activation (applied by
        // g5_splitk_reduce after summing the parts in order)
        float* pk = p.part + (int64_t)kz * p.M * p.N;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int m = m0 + rw * WR + 16 * i + c;
            if (m >= p.M) continue;
            const float rs = TERMS == 2 ? __builtin_ldexpf(1.f, -sh[i]) : 1.f;
#pragma unroll
            for (int j = 0; j < TNW; ++j) {
                const int n = n0 + 16 * (cw * TNW + j) + 4 * g;
                if (n >= p.N) continue;
                float4 ws = make_float4(1.f, 1.f, 1.f, 1.f);
                if constexpr (TERMS == 2) ws = *reinterpret_cast<const float4*>(p.wsc + n);
                const float y[4] = {acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                    acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w};
                float* prow = pk + (int64_t)m * p.N;
                if ((p.N & 3) == 0 && n + 3 < p.N) {
                    *reinterpret_cast<float4*>(prow + n) = make_float4(y[0], y[1], y[2], y[3]);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (n + e < p.N) prow[n + e] = y[e];
                }
            }
        }
        return;
    }

    if constexpr (KW == 1 && WC == 1) {
        if (p.vec_out && EPI_LDS) {
            // staged epilogue: each wave parks its scaled WR x BN tile in the drained stage
            // buffers and writes it back row-major, 16-B per lane over whole 256 / 512-B row
            // slices (the MFMA layout stores 64-B pieces of 16 rows per instruction); bias,
            // residual and activation applied in the row-major pass (coalesced R reads)
            constexpr int RS_ = BN + 4;                         // padded row stride (floats)
            static_assert(S * ST * 16 >= 4 * WR * RS_ * 4, "epilogue staging space");
            __syncthreads();                                    // every stage read retired
            float* buf = reinterpret_cast<float*>(lds) + wv * (WR * RS_);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float rs = TERMS == 2 ? __builtin_ldexpf(1.f, -sh[i]) : 1.f;
#pragma unroll
                for (int j = 0; j < TNW; ++j) {
                    const int n = min(n0 + 16 * j + 4 * g, ((p.N + 15) / 16) * 16 - 4);
                    float4 ws = make_float4(1.f, 1.f, 1.f, 1.f);
                    if constexpr (TERMS == 2) ws = *reinterpret_cast<const float4*>(p.wsc + n);
                    *reinterpret_cast<float4*>(buf + (16 * i + c) * RS_ + 16 * j + 4 * g) =
                        make_float4(acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                    acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w);
                }
            }
            __syncthreads();
            if constexpr (BM == 64 && BN == 128 && TERMS == 2) {
                if (p.kv_img && n0 >= p.kv_col0) {              // block-uniform: 2 K or V heads
                    // the staged 64 x 128 tile (wave w's rows at buf_w = lds + w * WR * RS_) is
                    // two heads of the global 64-row tile bm: bias added, rows past M zero, per
                    // head max |.| -> power-of-two exponent (max in [2^14, 2^15), as
                    // attn_kv_image16_kernel), split terms into the image units
                    __shared__ float kvred[2][4];
                    const float* tile = reinterpret_cast<const float*>(lds);
                    float v[4][8];
                    float hm[2] = {0.f, 0.f};
#pragma unroll
                    for (int it = 0; it < 4; ++it) {                // items: (key, 8-dim group)
                        const int item = tid + 256 * it;            // 0 .. 1023
                        const int hh = item >> 9, key = (item >> 3) & 63, gg = item & 7;
                        const int col = 64 * hh + 8 * gg;
                        const float* src = tile + (key / WR) * (WR * RS_) + (key % WR) * RS_ + col;
                        const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n0 + col);
                        const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n0 + col + 4);
                        const float4 x0 = *reinterpret_cast<const float4*>(src);
                        const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                        const bool ok = m0 + key < p.M;
                        v[it][0] = ok ? x0.x + b0.x : 0.f; v[it][1] = ok ? x0.y + b0.y : 0.f;
                        v[it][2] = ok ? x0.z + b0.z : 0.f; v[it][3] = ok ? x0.w + b0.w : 0.f;
                        v[it][4] = ok ? x1.x + b1.x : 0.f; v[it][5] = ok ? x1.y + b1.y : 0.f;
                        v[it][6] = ok ? x1.z + b1.z : 0.f; v[it][7] = ok ? x1.w + b1.w : 0.f;
                        float mx = 0.f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf(v[it][e]));
                        hm[hh] = fmaxf(hm[hh], mx);             // it 0-1: head 0, 2-3: head 1
                    }
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        float m = hm[hh];
#pragma unroll
                        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
                        if (lane == 0) kvred[hh][wv] = m;
                    }
                    __syncthreads();
                    const int rel = n0 - p.kv_col0;
                    const int isv = rel >= 64 * p.n_head ? 1 : 0;
                    const int head0 = (rel - isv * 64 * p.n_head) / 64;
#pragma unroll
                    for (int it = 0; it < 4; ++it) {
                        const int item = tid + 256 * it;
                        const int hh = item >> 9, key = (item >> 3) & 63, gg = item & 7;
                        const float tm = fmaxf(fmaxf(kvred[hh][0], kvred[hh][1]),
                                               fmaxf(kvred[hh][2], kvred[hh][3]));
                        const int e = tm > 0.f ? min(15 - __builtin_amdgcn_frexp_expf(tm), 127) : 0;
                        const float sc = __builtin_ldexpf(1.f, e);
                        const int64_t ti = (int64_t)bm * p.n_head + head0 + hh;
                        if (tid == 0 && it == 0) reinterpret_cast<int*>(p.kv_sc + ti)[isv] = e;
                        if (tid == 0 && it == 2) reinterpret_cast<int*>(p.kv_sc + ti)[isv] = e;
                        _Float16 th[8], tl[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const float x = v[it][j] * sc;
                            th[j] = (_Float16)x;
                            tl[j] = (_Float16)(x - (float)th[j]);
                        }
                        char* base = p.kv_img + ti * (int64_t)(kKv64Units * 16);
                        char *d0, *d1;
                        if (isv) {                          // [term][key][64] f16, chunk ^ v_swz<64>
                            const int ch = gg ^ (((key >> 1) & 3) << 1);
                            d0 = base + kKv64UnitV * 16 + key * 128 + ch * 16;
                            d1 = d0 + 128 * 64;
                        } else {                            // [ks][term][g'][key] x 8 dims
                            const int ks = gg >> 2, gq = gg & 3;
                            d0 = base + (((ks * 2 + 0) * 4 + gq) * 64 + key) * 16;
                            d1 = base + (((ks * 2 + 1) * 4 + gq) * 64 + key) * 16;
                        }
                        *reinterpret_cast<uint4*>(d0) = *reinterpret_cast<const uint4*>(th);
                        *reinterpret_cast<uint4*>(d1) = *reinterpret_cast<const uint4*>(tl);
                    }
                    return;
                }
            }
            constexpr int LPRW = BN / 4, RPI = 64 / LPRW;       // lanes per row, rows per pass
            const int col = 4 * (lane % LPRW);
            const int n = n0 + col;
#pragma unroll
            for (int it = 0; it < WR / RPI; ++it) {
                const int row = it * RPI + lane / LPRW;
                const int m = m0 + rw * WR + row;
                if (m >= p.M || n >= p.N) continue;
                const float4 y = *reinterpret_cast<const float4*>(buf + row * RS_ + col);
                float* crow = p.C + (int64_t)m * p.ldc;
                const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
                if (n + 3 < p.N) {
                    float4 bb = make_float4(0.f, 0.f, 0.f, 0.f), rr = bb;
                    if (p.bias) bb = *reinterpret_cast<const float4*>(p.bias + n);
                    if (rrow) rr = *reinterpret_cast<const float4*>(rrow + n);
                    *reinterpret_cast<float4*>(crow + n) =
                        make_float4(finish5(y.x, bb.x, rr.x, p.act), finish5(y.y, bb.y, rr.y, p.act),
                                    finish5(y.z, bb.z, rr.z, p.act), finish5(y.w, bb.w, rr.w, p.act));
                } else {
                    const float yv[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if (n + e >= p.N) break;
                        crow[n + e] = finish5(yv[e], p.bias ? p.bias[n + e] : 0.f,
                                              rrow ? rrow[n + e] : 0.f, p.act);
                    }
                }
            }
            return;
        }
    }

    // epilogue: lane holds C[m = m0 + rw WR + 16i + c][n = n0 + 16 (cw TNW + j) + 4g + r]
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + rw * WR + 16 * i + c;
        if (m >= p.M) continue;
        const float rs = TERMS == 2 ? __builtin_ldexpf(1.f, -sh[i]) : 1.f;   // 0: all-zero row
        float* crow = p.C + (int64_t)m * p.ldc;
        const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
#pragma unroll
        for (int j = 0; j < TNW; ++j) {
            const int n = n0 + 16 * (cw * TNW + j) + 4 * g;
            if (n >= p.N) continue;
            float4 ws = make_float4(1.f, 1.f, 1.f, 1.f);
            if constexpr (TERMS == 2) ws = *reinterpret_cast<const float4*>(p.wsc + n);
            const float y[4] = {acc[j][i][0] * rs * ws.x, acc[j][i][1] * rs * ws.y,
                                acc[j][i][2] * rs * ws.z, acc[j][i][3] * rs * ws.w};
            if (p.vec_out && n + 3 < p.N) {
                float4 bb = make_float4(0.f, 0.f, 0.f, 0.f), rr = bb;
                if (p.bias) bb = *reinterpret_cast<const float4*>(p.bias + n);
                if (rrow) rr = *reinterpret_cast<const float4*>(rrow + n);
                *reinterpret_cast<float4*>(crow + n) =
                    make_float4(finish5(y[0], bb.x, rr.x, p.act), finish5(y[1], bb.y, rr.y, p.act),
                                finish5(y[2], bb.z, rr.z, p.act), finish5(y[3], bb.w, rr.w, p.act));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (n + e >= p.N) break;
                    crow[n + e] = finish5(y[e], p.bias ? p.bias[n + e] : 0.f,
                                          rrow ? rrow[n + e] : 0.f, p.act);
                }
            }
        }
    }
}

template <int BM, int BN, int KS, int S, int TERMS, bool PIPE = false, int KW = 1, int WC = 1,
          bool EPI = false>
void launch_g5(const G5Args& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    hipLaunchKernelGGL((gemm_g5<BM, BN, KS, S, TERMS, PIPE, KW, WC, EPI>),
                       dim3((unsigned)(nbm * nbn * a.ksplit)), dim3(256 * KW), 0, st, a);
}

// split-K epilogue: C = act(sum_z part[z] + bias (+ R)), parts summed in order z = 0, 1, ...
// (deterministic); 4 columns per thread
__global__ void __launch_bounds__(256) g5_splitk_reduce(G5Args p) {
    const int nq = (p.N + 3) / 4;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)p.M * nq) return;
    const int m = (int)(t / nq), n = (int)(t % nq) * 4;
    const int64_t mn = (int64_t)p.M * p.N;
    const float* pp = p.part + (int64_t)m * p.N + n;
    float* crow = p.C + (int64_t)m * p.ldc;
    const float* rrow = p.R ? p.R + (int64_t)m * p.ldr : nullptr;
    if ((p.N & 3) == 0 && p.vec_out) {
        float4 y = *reinterpret_cast<const float4*>(pp);
        for (int z = 1; z < p.ksplit; ++z) {
            const float4 v = *reinterpret_cast<const float4*>(pp + z * mn);
            y.x += v.x; y.y += v.y; y.z += v.z; y.w += v.w;
        }
        float4 bb = make_float4(0.f, 0.f, 0.f, 0.f), rr = bb;
        if (p.bias) bb = *reinterpret_cast<const float4*>(p.bias + n);
        if (rrow) rr = *reinterpret_cast<const float4*>(rrow + n);
        *reinterpret_cast<float4*>(crow + n) =
            make_float4(finish5(y.x, bb.x, rr.x, p.act), finish5(y.y, bb.y, rr.y, p.act),
                        finish5(y.z, bb.z, rr.z, p.act), finish5(y.w, bb.w, rr.w, p.act));
        return;
    }
    for (int e = 0; e < 4 && n + e < p.N; ++e) {
        float y = pp[e];
        for (int z = 1; z < p.ksplit; ++z) y += pp[z * mn + e];
        crow[n + e] = finish5(y, p.bias ? p.bias[n + e] : 0.f, rrow ? rrow[n + e] : 0.f, p.act);
    }
}

const float* g5_zero_ptr() {
    static const float* z = [] {
        void* p = nullptr;
        return hipGetSymbolAddress(&p, HIP_SYMBOL(g5_zero)) == hipSuccess ? (const float*)p : nullptr;
    }();
    return z;
}

template <int TERMS>
bool dispatch_g5_tile(char cfg, const G5Args& a, hipStream_t st);

template <int TERMS>
bool dispatch_g5(char cfg, const G5Args& a, hipStream_t st) {
    if (!a.zero) return false;
    if (!dispatch_g5_tile<TERMS>(cfg, a, st)) return false;
    if (a.ksplit > 1) {
        const int64_t nthr = (int64_t)a.M * ((a.N + 3) / 4);
        hipLaunchKernelGGL(g5_splitk_reduce, dim3((unsigned)ceil_div(nthr, 256)), dim3(256), 0, st, a);
    }
    return true;
}

template <int TERMS>
bool dispatch_g5_tile(char cfg, const G5Args& a, hipStream_t st) {
    switch (cfg) {
        case 'A': launch_g5<64, 64, 1, 4, TERMS>(a, st); break;
        case 'B': launch_g5<64, 128, 1, 3, TERMS>(a, st); break;
        case 'C': launch_g5<64, 64, 2, 3, TERMS>(a, st); break;
        case 'D': launch_g5<64, 128, 2, 3, TERMS>(a, st); break;
        case 'E': launch_g5<128, 64, 1, 4, TERMS>(a, st); break;
        case 'F': launch_g5<128, 128, 1, 3, TERMS>(a, st); break;
        case 'G': launch_g5<64, 256, 1, 3, TERMS>(a, st); break;
        case 'H': launch_g5<128, 128, 2, 2, TERMS>(a, st); break;
        case 'I': launch_g5<64, 64, 1, 3, TERMS>(a, st); break;
        case 'J': launch_g5<128, 64, 2, 3, TERMS>(a, st); break;
        // software-pipelined: K..R
        case 'K': launch_g5<64, 64, 1, 4, TERMS, true>(a, st); break;
        case 'L': launch_g5<64, 128, 1, 4, TERMS, true>(a, st); break;
        case 'M': launch_g5<64, 64, 1, 5, TERMS, true>(a, st); break;
        case 'N': launch_g5<128, 64, 1, 4, TERMS, true>(a, st); break;
        case 'O': launch_g5<128, 128, 1, 3, TERMS, true>(a, st); break;
        case 'P': launch_g5<64, 256, 1, 3, TERMS, true>(a, st); break;
        case 'Q': launch_g5<64, 128, 1, 3, TERMS, true>(a, st); break;
        case 'R': launch_g5<128, 128, 1, 4, TERMS, true>(a, st); break;
        // two k-groups (512 threads): S..W
        case 'S': launch_g5<64, 64, 2, 3, TERMS, false, 2>(a, st); break;
        case 'T': launch_g5<64, 128, 2, 3, TERMS, false, 2>(a, st); break;
        case 'U': launch_g5<64, 64, 2, 4, TERMS, false, 2>(a, st); break;
        case 'V': launch_g5<128, 64, 2, 3, TERMS, false, 2>(a, st); break;
        case 'W': launch_g5<64, 64, 2, 2, TERMS, false, 2>(a, st); break;
        // 2 x 2 wave layout: 0..7
        case '0': launch_g5<64, 128, 1, 3, TERMS, false, 1, 2>(a, st); break;
        case '1': launch_g5<64, 64, 1, 3, TERMS, false, 1, 2>(a, st); break;
        case '2': launch_g5<128, 128, 1, 3, TERMS, false, 1, 2>(a, st); break;
        case '3': launch_g5<128, 64, 1, 3, TERMS, false, 1, 2>(a, st); break;
        case '4': launch_g5<64, 128, 2, 3, TERMS, false, 2, 2>(a, st); break;
        case '5': launch_g5<64, 64, 2, 2, TERMS, false, 2, 2>(a, st); break;
        case '6': launch_g5<64, 256, 1, 3, TERMS, false, 1, 2>(a, st); break;
        case '7': launch_g5<128, 128, 1, 4, TERMS, false, 1, 2>(a, st); break;
        // 128 x 128, deeper pipelines (L2 / MALL traffic per MFMA halves vs 64 x 64): 8, 9
        case '8': launch_g5<128, 128, 1, 4, TERMS, false>(a, st); break;
        case '9': launch_g5<128, 128, 1, 5, TERMS, false>(a, st); break;
        // staged (row-major) epilogue: X, Y, Z = I, B, G with it
        case 'X': launch_g5<64, 64, 1, 3, TERMS, false, 1, 1, true>(a, st); break;
        case 'Y': launch_g5<64, 128, 1, 3, TERMS, false, 1, 1, true>(a, st); break;
        case 'Z': launch_g5<64, 256, 1, 3, TERMS, false, 1, 1, true>(a, st); break;
        default: return false;
    }
    return true;
}

}  // namespace

// A 16-B aligned with lda % 4 == 0 and K % 8 == 0 (checked by the callers).
// ksplit > 1: split-K over ksplit parts with `part` = ksplit * M * N floats of workspace
bool gemm_g5_f16x3(char cfg, const float* A, int64_t lda, const void* W, int ksteps,
                   const float* wsc, float* C, int64_t ldc, const float* bias, const float* R,
                   int64_t ldr, int M, int N, int K, int act, int vec_out, hipStream_t st,
                   int ksplit, float* part) {
    G5Args a{A, lda, g5_zero_ptr(), (const u32x4*)W, ksteps, wsc, C, ldc, bias, R, ldr, M, N, K,
             act, vec_out, ksplit > 1 && part ? ksplit : 1, part, nullptr, nullptr, 0, 0};
    return dispatch_g5<2>(cfg, a, st);
}

// the in_proj with the K / V images of every global 64-row tile (head dim 64) in the staged
// epilogue: g5 'Y' (64 x 128 tiles, 3 stages, staged epilogue), q columns to C
bool gemm_g5_f16x3_qkv(const float* A, int64_t lda, const void* W, int ksteps, const float* wsc,
                       float* q, int64_t ld_q, const float* bias, int M, int d, int n_head,
                       char* kv_img, int2* kv_sc, hipStream_t st) {
    G5Args a{A, lda, g5_zero_ptr(), (const u32x4*)W, ksteps, wsc, q, ld_q, bias, nullptr, 0, M,
             3 * d, d, FGR_ACT_NONE, 1, 1, nullptr, kv_img, kv_sc, n_head, d};
    return dispatch_g5<2>('Y', a, st);
}

bool gemm_g5_bf16(char cfg, const float* A, int64_t lda, const void* W, int ksteps, float* C,
                  int64_t ldc, const float* bias, const float* R, int64_t ldr, int M, int N, int K,
                  int act, int vec_out, hipStream_t st, int ksplit, float* part) {
    G5Args a{A, lda, g5_zero_ptr(), (const u32x4*)W, ksteps, nullptr, C, ldc, bias, R, ldr, M, N,
             K, act, vec_out, ksplit > 1 && part ? ksplit : 1, part, nullptr, nullptr, 0, 0};
    return dispatch_g5<1>(cfg, a, st);
}

// tile of a g5 variant (BM x BN), false for an unknown variant
bool g5_tile(char cfg, int* bm, int* bn) {
    static const char* k64x64 = "ACIKMSUW15X";
    static const char* k64x128 = "BDLQT04Y";
    static const char* k128x64 = "EJNV3";
    static const char* k128x128 = "FHOR2789";
    static const char* k64x256 = "GP6Z";
    auto in = [cfg](const char* set) { for (; *set; ++set) if (*set == cfg) return true; return false; };
    if (in(k64x64)) { *bm = 64; *bn = 64; }
    else if (in(k64x128)) { *bm = 64; *bn = 128; }
    else if (in(k128x64)) { *bm = 128; *bn = 64; }
    else if (in(k128x128)) { *bm = 128; *bn = 128; }
    else if (in(k64x256)) { *bm = 64; *bn = 256; }
    else return false;
    return true;
}

// split-K factor for an M x N x K g5 GEMM on BM x BN tiles: enough blocks to fill the chip
// twice when the tile grid alone does not (<= 8 parts, >= 4 k32-steps each); FGR_GEMM_KSPLIT
// forces a factor (tuning)
int g5_ksplit(int M, int N, int K, int BM, int BN) {
    const char* f = getenv("FGR_GEMM_KSPLIT");
    const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    const int kst = (K + 31) / 32;
    int ks;
    if (f && f[0]) {
        ks = atoi(f);
    } else {
        ks = 1;
        while (ks < 8 && tiles * ks < 512 && kst / (2 * ks) >= 4) ks *= 2;
    }
    return ks < 1 ? 1 : (ks > kst ? kst : ks);
}

}  // namespace fgr
