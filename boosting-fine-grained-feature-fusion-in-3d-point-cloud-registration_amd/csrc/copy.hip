// Batched device-to-device copies: up to kMaxCopies (src, dst, bytes) triples in ONE launch.
// The HIP-graph replay of the forward (fgreg/regtr.py) refreshes its static kpconv_meta inputs
// and clones its outputs every step -- ~10-30 small copies, each a separate blit dispatch
// (~4-5 us apiece in the trace) -- so they go through this kernel instead.
#include "common.h"

namespace fgr {
namespace {

constexpr int kMaxCopies = 32;

constexpr int64_t kChunk = 256 * 64;   // bytes per block: 256 threads x 4 x 16 B

struct CopyBatch {
    const char* src[kMaxCopies];
    char* dst[kMaxCopies];
    int64_t bytes[kMaxCopies];
    int first[kMaxCopies + 1];         // copy k owns blocks [first[k], first[k + 1])
    int m;
};

// one flat grid over every copy's chunks (no idle blocks for the short copies); 16-B
// accesses when both ends allow
__global__ void __launch_bounds__(256) copy_batch_kernel(CopyBatch b) {
    int k = 0;
    while (k + 1 < b.m && b.first[k + 1] <= (int)blockIdx.x) ++k;     // block-uniform
    const char* s = b.src[k];
    char* d = b.dst[k];
    const int64_t n = b.bytes[k];
    const int64_t chunk = (int64_t)(blockIdx.x - b.first[k]) * kChunk;
    if (chunk >= n) return;
    const bool vec = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0;
    if (vec) {
        const int64_t n16 = n / 16;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = chunk / 16 + threadIdx.x + 256 * u;
            if (i < n16)
                reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
        }
        const int64_t tail = n16 * 16;
        if (chunk == 0 && threadIdx.x < n - tail) d[tail + threadIdx.x] = s[tail + threadIdx.x];
    } else {
        for (int64_t i = chunk + threadIdx.x; i < min(n, chunk + kChunk); i += 256) d[i] = s[i];
    }
}

}  // namespace
}  // namespace fgr

using namespace fgr;

extern "C" int fgr_copy_batch(int32_t n, const void* const* src, void* const* dst,
                              const int64_t* bytes, void* stream) {
    FGR_REQUIRE(n >= 0 && (n == 0 || (src && dst && bytes)), "fgr_copy_batch: bad arguments");
    hipStream_t st = as_stream(stream);
    for (int32_t i0 = 0; i0 < n; i0 += kMaxCopies) {
        const int m = n - i0 < kMaxCopies ? n - i0 : kMaxCopies;
        CopyBatch b{};
        int64_t nblk = 0;
        for (int j = 0; j < m; ++j) {
            FGR_REQUIRE(bytes[i0 + j] >= 0 && (bytes[i0 + j] == 0 || (src[i0 + j] && dst[i0 + j])),
                        "fgr_copy_batch: copy %d: bad pointer / size", i0 + j);
            b.src[j] = static_cast<const char*>(src[i0 + j]);
            b.dst[j] = static_cast<char*>(dst[i0 + j]);
            b.bytes[j] = bytes[i0 + j];
            b.first[j] = (int)nblk;
            nblk += ceil_div(bytes[i0 + j], kChunk);
        }
        FGR_REQUIRE(nblk < (int64_t)1 << 30, "fgr_copy_batch: %lld blocks", (long long)nblk);
        b.first[m] = (int)nblk;
        b.m = m;
        if (nblk == 0) continue;
        hipLaunchKernelGGL(copy_batch_kernel, dim3((unsigned)nblk), dim3(256), 0, st, b);
        FGR_CHECK_LAUNCH("copy_batch_kernel");
    }
    return FGR_OK;
}

namespace fgr {
namespace {
// off[0] = 0, off[i + 1] = off[i] + len[i]: one wave, a running sum over 64-entry chunks
__global__ void __launch_bounds__(64) lengths_to_offsets_kernel(const int64_t* __restrict__ len,
                                                                int n, int64_t* __restrict__ off) {
    const int lane = threadIdx.x;
    int64_t carry = 0;
    if (lane == 0) off[0] = 0;
    for (int b = 0; b < n; b += 64) {
        int64_t v = b + lane < n ? len[b + lane] : 0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {                 // inclusive scan over the wave
            const int64_t u = __shfl_up(v, d, 64);
            if (lane >= d) v += u;
        }
        if (b + lane < n) off[b + lane + 1] = carry + v;
        carry += __shfl(v, 63, 64);
    }
}
}  // namespace
}  // namespace fgr

extern "C" int fgr_lengths_to_offsets(const int64_t* lengths, int32_t n, int64_t* offsets,
                                      void* stream) {
    FGR_REQUIRE(n >= 0 && offsets && (n == 0 || lengths), "fgr_lengths_to_offsets: bad arguments");
    hipLaunchKernelGGL(lengths_to_offsets_kernel, dim3(1), dim3(64), 0, as_stream(stream), lengths, n,
                       offsets);
    FGR_CHECK_LAUNCH("lengths_to_offsets_kernel");
    return FGR_OK;
}
