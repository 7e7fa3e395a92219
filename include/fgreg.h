/* fgreg.h -- C ABI of libfgreg.so, the MI355X (gfx950) kernels of the per-pair
 * registration forward of "Boosting Fine-grained Feature Fusion in 3D Point
 * Cloud Registration" (a REGTR fork: KPConv + Res2Net backbone, cross-attention
 * transformer, weighted-Procrustes pose).
 *
 * Conventions (every entry point):
 *  - all array arguments are DEVICE pointers allocated by the caller; nothing
 *    is allocated inside (data-dependent sizes use a count call + a fill call,
 *    scratch comes from a caller-provided workspace sized by *_workspace());
 *  - `stream` is a hipStream_t passed as void*; all work is stream-ordered,
 *    no call synchronises the device or the host;
 *  - return 0 on success, a negative FGR_E* code on error; the message of the
 *    last error on the calling thread is returned by fgr_last_error();
 *  - no C++ exception crosses the ABI; no mutable global state besides a
 *    per-thread error string.
 *
 * Packed layout: clouds are stacked along rows in the reference's order
 * src_0..src_{B-1}, tgt_0..tgt_{B-1} (models/finegrained_regtr.py:121), with
 * int64 row offsets `off[n_clouds + 1]`. A neighbour table is (Nq, width)
 * int64 whose missing entries hold the "shadow" index Ns_total
 * (finegrained_kpconv.py:288-291).
 */
#ifndef FGREG_H
#define FGREG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FGR_ABI_VERSION 2

enum {
    FGR_OK = 0,
    FGR_E_ARG = -1,      /* invalid argument / shape            */
    FGR_E_LAUNCH = -2,   /* HIP launch or runtime error          */
    FGR_E_WORKSPACE = -3 /* workspace too small                  */
};

/* radius-search row semantics */
enum {
    FGR_NB_INDEX = 0, /* PyTorch3D ball_query: first `width` supports in index order
                         (finegrained_kpconv.py:266-293, PreprocessorGPU)          */
    FGR_NB_DIST = 1   /* nanoflann radiusSearch(sorted) + [:, :K]: the `width`
                         nearest, ties by index (neighbors.cpp:211-332, :260-261)  */
};

/* activation codes; FGR_ACT_RELU_RES_LEAKY (the f16x3 GEMMs only) applies the residual AFTER
 * the ReLU: C = LeakyReLU_0.1(ReLU(A.W + bias) + R) -- a Res2Net block output plus its
 * identity shortcut (finegrained_kpconv_blocks.py:715-725) in one epilogue. */
enum { FGR_ACT_NONE = 0, FGR_ACT_LEAKY = 1, FGR_ACT_RELU = 2, FGR_ACT_RELU_RES_LEAKY = 3 };

int fgr_abi_version(void);
const char* fgr_last_error(void);

/* Opt-in instrumentation (bench.py's per-kernel rooflines; not part of the reference's
 * interface): arms two caller-created hipEvent_t for the NEXT timed entry point called on
 * this thread (fgr_kpconv_gather, fgr_attention*, fgr_gemm_f16x3, fgr_gemm_bf16,
 * fgr_grid_subsample_count / _fill, fgr_radius_search,
 * fgr_radius_grid_build, fgr_radius_search_grid, fgr_instnorm, fgr_layernorm,
 * fgr_pair_pose). That call records `start_event` on its stream right before its
 * first kernel launch and `end_event` after its last one, then disarms; (NULL, NULL)
 * disarms explicitly. Thread-local like the error string. */
int fgr_time_next_call(void* start_event, void* end_event);

/* ---- grid subsampling ------------------------------------------------------------
 * Replaces batch_grid_subsampling_kpconv_gpu (finegrained_kpconv.py:218-245; ME
 * UNWEIGHTED_AVERAGE) and its CPU twin subsample_batch
 * (cpp_subsampling/wrapper.cpp:62-333 -> grid_subsampling.cpp:5-211).
 * Voxel key and barycentre follow grid_subsampling.cpp bit for bit; voxels are
 * emitted in ascending key order per cloud, members summed in ascending point index.
 * `max_cells`: a counting sort over a dense voxel-key histogram of that many counters (the
 * clouds' key spaces nx*ny*nz laid end to end; 0 = the default 8 n_points + 2^20; < 0 is
 * rejected: the round-1 radix-sort path was removed in round 5). The same max_cells must be
 * passed to all three calls.
 * 1) fgr_grid_subsample_count: writes counts[c] (voxels of cloud c) and
 *    counts[n_clouds] (total) as int64; keeps the sorted state in `ws`. Dense path only:
 *    if the key space exceeds max_cells, counts[n_clouds] = -(cells needed) and nothing else
 *    is valid -- call again with a larger max_cells.
 * 2) fgr_grid_subsample_fill: writes out_points (total, 3) and optionally the
 *    voxel keys (total) from the same `ws` (must follow the count call). */
int fgr_grid_subsample_workspace(int64_t n_points, int32_t n_clouds, int64_t max_cells,
                                 size_t* bytes);
int fgr_grid_subsample_count(const float* points, const int64_t* off, int32_t n_clouds,
                             int64_t n_points, float dl, int64_t max_cells, void* ws,
                             size_t ws_bytes, int64_t* counts, void* stream);
int fgr_grid_subsample_fill(int64_t n_points, int32_t n_clouds, int64_t max_cells, int64_t n_out,
                            void* ws, size_t ws_bytes, const float* points, float* out_points,
                            int64_t* out_keys, void* stream);

/* ---- radius neighbour search -----------------------------------------------------
 * Replaces batch_neighbors_kpconv_gpu (ball_query, finegrained_kpconv.py:266-293)
 * and batch_neighbors_kpconv (cpp_neighbors.batch_query, :248-263).
 * d2 = ((qx-sx)^2 + (qy-sy)^2) + (qz-sz)^2 in fp32 without FMA, kept iff d2 < r*r.
 * fgr_radius_count: uncapped neighbour count per query + the max (int32 scalar);
 * fgr_radius_search: fills out (nq, width) int64 (mode FGR_NB_*; DIST needs width <= 64). */
int fgr_radius_count(const float* q, const int64_t* q_off, const float* s, const int64_t* s_off,
                     int32_t n_clouds, int64_t nq, int32_t max_q_len, float radius,
                     int32_t* counts, int32_t* max_count, void* stream);
int fgr_radius_search(const float* q, const int64_t* q_off, const float* s, const int64_t* s_off,
                      int32_t n_clouds, int64_t nq, int64_t ns, int32_t max_q_len, float radius,
                      int32_t mode, int32_t width, int64_t* out, void* stream);

/* Cell-binned radius search for large clouds (same rows as fgr_radius_search, both modes):
 * fgr_radius_grid_build bins the supports of every cloud into cubic cells of edge
 * >= 1.0625 * radius (a counting sort; the grid workspace, fgr_radius_grid_workspace() bytes,
 * depends on ns and n_clouds only); fgr_radius_search_grid then scans the 27 cells around
 * each query. One grid serves every query set searched with a radius <= the build radius
 * over the same supports (the conv and pool tables of a pyramid level). width <= 256.
 * With counts != NULL it writes the uncapped counts + their max instead (fgr_radius_count). */
int fgr_radius_grid_workspace(int64_t ns, int32_t n_clouds, size_t* bytes);
int fgr_radius_grid_build(const float* s, const int64_t* s_off, int32_t n_clouds, int64_t ns,
                          float radius, void* grid, size_t grid_bytes, void* stream);
int fgr_radius_search_grid(const float* q, const int64_t* q_off, int32_t n_clouds, int64_t nq,
                           int32_t max_q_len, const float* s, const int64_t* s_off, int64_t ns,
                           const void* grid, size_t grid_bytes, float radius, int32_t mode,
                           int32_t width, int64_t* out, int32_t* counts, int32_t* max_count,
                           void* stream);

/* ---- KPConv ------------------------------------------------------------------------
 * The gather-weight stage of KPConv.forward (finegrained_kpconv_blocks.py:296-381,
 * rigid, linear influence, sum aggregation):
 *   wf[q, k, c] = sum_{valid h} max(0, 1 - |(s[idx[q,h]] - q) - kp[k]| / extent) * x[idx[q,h], c]
 * and the normaliser of :395-399: nnorm[q] = max(1, #{valid h : sum_c x[idx[q,h], c] > 0}).
 * The caller finishes with (wf.view(nq, K*cin) @ W.view(K*cin, cout)) / nnorm.
 * workspace: fgr_kpconv_gather_workspace() bytes (per-source-row flags of the normaliser). */
int fgr_kpconv_gather_workspace(int64_t ns, int32_t cin, size_t* bytes);
int fgr_kpconv_gather(const float* q, const float* s, int64_t nq, int64_t ns, const int64_t* idx,
                      int32_t width, const float* x, int32_t cin, const float* kp, int32_t n_kp,
                      float extent, float* wf, float* nnorm, void* workspace, size_t ws_bytes,
                      void* stream);

/* max_pool (finegrained_kpconv_blocks.py:125-141): out[q, c] = max over the row of
 * x[idx[q, h], c], shadow entries contributing 0 (the appended zero row). */
int fgr_max_pool(const float* x, int64_t ns, int32_t c, const int64_t* idx, int64_t nq,
                 int32_t width, float* out, void* stream);

/* ---- normalisation -----------------------------------------------------------------
 * Segmented instance norm, nn.InstanceNorm1d(affine=False) applied per cloud
 * (BatchNormBlock, finegrained_kpconv_blocks.py:498-507), fused with:
 *   v   = row_div ? x[r, c] / row_div[r] : x[r, c]       (KPConv normaliser, :399)
 *   y   = act((v - mean_seg,c) / sqrt(var_seg,c + eps))   (biased variance)
 *   out = residual ? post_act(y + residual[r, c]) : y     (bottleneck sum, :725)
 * Segments of up to 1024 rows are normalised from registers in one launch; longer
 * ones need a workspace of fgr_instnorm_workspace() bytes (two launches). */
int fgr_instnorm_workspace(int64_t max_seg_len, int32_t c, int32_t n_seg, size_t* bytes);
int fgr_instnorm(const float* x, int64_t n, int32_t c, const int64_t* seg_off, int32_t n_seg,
                 int64_t max_seg_len, const float* row_div, float eps, int32_t act,
                 const float* residual, int32_t post_act, float* out, void* ws, size_t ws_bytes,
                 void* stream);

/* Row LayerNorm (nn.LayerNorm, transformers.py:105-107) with an optional added
 * tensor (the positional embedding, transformers.py:194-195): out = LN(x)*g + b (+ add).
 * If pre_bias is given, x += pre_bias is applied first and written back to x (the
 * deferred bias of the Linear that produced the residual stream). */
int fgr_layernorm(float* x, int64_t n, int32_t d, const float* gamma, const float* beta,
                  float eps, const float* add, const float* pre_bias, float* out, void* stream);
/* Two LayerNorms of the same rows in one pass (same eps, shared statistics):
 * out = LN(x)*gamma + beta (+ add), out2 = LN(x)*gamma2 + beta2 (+ add2). The cross encoder's
 * per-layer output norm (transformers.py:43-44, return_intermediate) of layer l and norm1 +
 * with_pos_embed of layer l + 1 (:193-195) read the same residual stream. x is not written. */
int fgr_layernorm_dual(const float* x, int64_t n, int32_t d, const float* gamma,
                       const float* beta, const float* add, float* out, const float* gamma2,
                       const float* beta2, const float* add2, float* out2, float eps,
                       void* stream);

/* out = a + b over n floats: the post-norm layer's with_pos_embed (transformers.py:121-124,
 * pre_norm: False; the pre-norm path fuses this add into fgr_layernorm). */
int fgr_add(const float* a, const float* b, int64_t n, float* out, void* stream);

/* PositionEmbeddingCoordsSine (position_embedding.py:29-49) for 3-D input. */
int fgr_sine_pos_embed(const float* xyz, int64_t n, int32_t d_model, float temperature,
                       float scale, float* out, void* stream);

/* ---- Res2Net hierarchy ----------------------------------------------------------------
 * The fine-grained fusion core of my_Bottle2neck (res2net.py:126-148), eval BatchNorm
 * folded into the Linears: for i < scale - 1,
 *   sp_i = ReLU(W_i (sp_{i-1} + h_i) + b_i)          (sp_{-1} = 0)
 * writing cat = [sp_0 .. sp_{scale-2} | h_{scale-1} | x] (the conv3 / downsample operand).
 * h (n, scale*w), x (n, cin) or NULL, cat (n, ld_cat); bias (scale-1, w).
 * fgr_res2net_chain6 (fp32-accurate split bf16: three exact bf16 terms, six products; w = 112
 * or 224, dispatched at w = 224 where it measured faster): w_img = the (scale-1, w, w) folded
 * weights K-padded to a multiple of 32, split into three bf16 terms and laid out in 16x16x32
 * fragment order [i][jt][ks][term][g][c][8] (fgreg.ops.res2net_fragments3); h 16-B aligned. */
int fgr_res2net_chain6(const float* h, int64_t n, int32_t w, int32_t scale, const void* w_img,
                       const float* bias, const float* x, int32_t cin, float* cat,
                       int64_t ld_cat, void* stream);

/* fp32-accurate f16x3 variant (scaled two-term fp16 splits, see fgr_gemm_f16x3): rows of
 * a = sp_{i-1} + h_i scaled exactly per row, W_i rows pre-scaled per output column.
 * w_img = fgreg.ops.res2net_fragments_h3 image [i][jt][ks][term 2][g][c][8] (fp16), w_scale
 * (scale-1, w) the inverse column scales; h, cat, w_scale, bias 16-B aligned, ld_cat % 4 == 0. */
int fgr_res2net_chain_h3(const float* h, int64_t n, int32_t w, int32_t scale, const void* w_img,
                         const float* w_scale, const float* bias, const float* x, int32_t cin,
                         float* cat, int64_t ld_cat, void* stream);

/* ---- dense layers ----------------------------------------------------------------------
 * Every Linear / KPConv-weight product of the forward:
 *   C[m, n] = act(A[m, :] . W[n, :] + bias[n] (+ R[m, n]))
 * W is given as an image built once per weight (element (i, j) read from
 * w[i * stride_n + j * stride_k], so a (K, Cin, Cout) KPConv weight needs no transpose copy);
 * A fp32 row-major, 16-B aligned with lda % 4 == 0 when k % 8 == 0.
 *
 * fp32-accurate scaled split-fp16 GEMM ("f16x3", the default mode):
 * W rows are scaled by powers of two (row max in [2^14, 2^15)) and A rows on the fly (per
 * row, lowered only when a later k chunk would overflow fp16, with an exact rescale of the
 * partial sums); each operand is then split into two fp16 terms (2^-22 relative) and the
 * three significant term products accumulate in fp32 on v_mfma_f32_16x16x32_f16: <= ~3 *
 * 2^-22 relative per product (fp32's own rounding is 2^-24). The image (built once by
 * fgr_split_weights_h3, fgr_split_weights_h3_bytes() bytes, 16-B aligned) holds the split W
 * in tile order followed by the per-row inverse scales. */
int fgr_split_weights_h3_bytes(int32_t n, int32_t k, size_t* bytes);
int fgr_split_weights_h3(const float* w, int32_t n, int32_t k, int64_t stride_n,
                         int64_t stride_k, void* img, void* stream);
/* Many fgr_split_weights_h3 images in one launch (training re-splits every weight after each
 * optimizer step): descs = a DEVICE array of count descriptors, panel0 = the running sum of
 * the earlier descriptors' (n + 15) / 16, total_panels = the sum over all; every image
 * bit-equal to fgr_split_weights_h3's. */
typedef struct {
    const float* w;       /* element (i, j) at w[i * stride_n + j * stride_k] */
    void* img;            /* fgr_split_weights_h3_bytes(n, k) bytes, 16-B aligned */
    int64_t stride_n;
    int64_t stride_k;
    int64_t panel0;
    int32_t n;
    int32_t k;
} fgr_split_desc;
int fgr_split_weights_h3_batch(const void* descs, int32_t count, int64_t total_panels,
                               void* stream);
int fgr_gemm_f16x3(const float* a, int64_t lda, const void* w_img, float* c, int64_t ldc,
                   const float* bias, const float* r, int64_t ldr, int32_t m, int32_t n,
                   int32_t k, int32_t act, void* stream);

/* bf16 GEMM (the bf16 compute mode, BASELINE configs[4] -- 3DLoMatch with bf16 features),
 * same contract as fgr_gemm_f16x3 (act includes FGR_ACT_RELU_RES_LEAKY):
 *   C[m, n] = act(bf16(A[m, :]) . bf16(W[n, :]) + bias[n] (+ R[m, n]))
 * One v_mfma_f32_16x16x32_bf16 product per product: operands rounded to bf16 (RNE, ~2^-9
 * relative), fp32 accumulation, fp32 epilogue and output. Replaces the same nn.Linear /
 * KPConv-weight products as fgr_gemm_f16x3 (finegrained_regtr.py:47-105 via its layers) at a
 * third of the matrix-core work. W image built once by fgr_split_weights_bf16
 * (fgr_split_weights_bf16_bytes() bytes, 16-B aligned; element (i, j) read from
 * w[i * stride_n + j * stride_k]); A 16-B aligned with lda % 4 == 0 when k % 8 == 0. */
/* Split-K forms of fgr_gemm_f16x3 / fgr_gemm_bf16 (same contract plus a caller workspace):
 * where the tile grid alone cannot fill the chip (few activation rows, long K) the g5 kernel
 * runs ksplit parts over disjoint k ranges into the workspace and one launch sums them in a
 * fixed order and applies the epilogue (deterministic). fgr_gemm_workspace (mode 0 = f16x3,
 * 1 = bf16) returns the bytes the dispatcher wants for a shape (0: no split); a smaller or
 * NULL workspace runs unsplit. */
int fgr_gemm_workspace(int32_t m, int32_t n, int32_t k, int32_t mode, size_t* bytes);
int fgr_gemm_f16x3_ws(const float* a, int64_t lda, const void* w_img, float* c, int64_t ldc,
                      const float* bias, const float* r, int64_t ldr, int32_t m, int32_t n,
                      int32_t k, int32_t act, void* ws, size_t ws_bytes, void* stream);
int fgr_gemm_bf16_ws(const float* a, int64_t lda, const void* w_img, float* c, int64_t ldc,
                     const float* bias, const float* r, int64_t ldr, int32_t m, int32_t n,
                     int32_t k, int32_t act, void* ws, size_t ws_bytes, void* stream);

/* Pre-norm transformer sub-layer input, fused (transformers.py:193-196 norm1 ->
 * with_pos_embed -> self_attn in_proj; :213-221 norm2 -> multihead_attn in_proj; :231-232
 * norm3 -> linear1):
 *   C[m, n] = act(A[m, :] . W[n, :] + bias[n]),  A = LayerNorm_eps(X) * gamma + beta (+ add)
 * with the LayerNorm over the k features of each row (biased variance, as nn.LayerNorm) and
 * the f16x3 product of fgr_gemm_f16x3 (w_img from fgr_split_weights_h3). act: FGR_ACT_NONE or
 * FGR_ACT_RELU; add (optional, e.g. the positional embedding) has row stride ld_add. All
 * pointers 16-B aligned, row strides multiples of 4. Only for shapes where
 * fgr_gemm_f16x3_ln_supported(m, n, k) returns 1 (the row-stationary kernel: k <= 256,
 * k % 8 == 0, n % 16 == 0, many rows); FGR_E_ARG otherwise. */
int fgr_gemm_f16x3_ln_supported(int32_t m, int32_t n, int32_t k);
int fgr_gemm_f16x3_ln(const float* x, int64_t ldx, const float* gamma, const float* beta,
                      float eps, const float* add, int64_t ld_add, const void* w_img, float* c,
                      int64_t ldc, const float* bias, int32_t m, int32_t n, int32_t k,
                      int32_t act, void* stream);
/* fgr_gemm_f16x3_ln plus a second LayerNorm output of the same rows, written once:
 *   out2 = LayerNorm_eps(X) * gamma2 + beta2   (row stride ld_out2, 16-B aligned)
 * -- the cross encoder's per-layer output norm of layer l (transformers.py:43-44) computed in
 * the prologue of layer l + 1's in_proj, which normalises the same rows. Requires `add`. */
int fgr_gemm_f16x3_ln_out2(const float* x, int64_t ldx, const float* gamma, const float* beta,
                           float eps, const float* add, int64_t ld_add, const void* w_img,
                           float* c, int64_t ldc, const float* bias, int32_t m, int32_t n,
                           int32_t k, int32_t act, const float* gamma2, const float* beta2,
                           float* out2, int64_t ld_out2, void* stream);

/* Pre-norm position-wise feed-forward sub-layer in one launch (transformers.py:231-238):
 *   out = x + linear2(ReLU(linear1(LayerNorm_eps(x) * gamma + beta)))
 * x, out (m, d) (out may be x itself), linear1 (f, d) + b1, linear2 (d, f) + b2, the f16x3
 * products of fgr_gemm_f16x3; the (m, f) hidden activations never leave the chip.
 * w1_img: fgr_split_weights_h3 of linear1.weight; w2_img: fgr_split_weights_ffn2 of
 * linear2.weight (the chunk-major image in the k order the fused kernel consumes; bytes from
 * fgr_split_weights_ffn2_bytes(d, f), f % 32 == 0); bound (device, 2 floats) = {max_j
 * ||linear1.weight[j]||_2, max_j |b1[j]|} (sets the hidden values' fp16 scale). All pointers
 * 16-B aligned, row strides multiples of 4. fgr_ffn_f16x3_supported(m, d, f): d = 256,
 * 64 <= f <= 2048, f % 64 == 0 (the ModelNet transformer). Replaces the two-launch
 * linear1 (fgr_gemm_f16x3_ln) -> linear2 (fgr_gemm_f16x3_ws, residual) sequence. */
int fgr_split_weights_ffn2_bytes(int32_t n, int32_t k, size_t* bytes);
int fgr_split_weights_ffn2(const float* w, int32_t n, int32_t k, int64_t stride_n,
                           int64_t stride_k, void* img, void* stream);
int fgr_ffn_f16x3_supported(int32_t m, int32_t d, int32_t f);
int fgr_ffn_f16x3(const float* x, int64_t ldx, const float* gamma, const float* beta, float eps,
                  const void* w1_img, const float* b1, const void* w2_img, const float* b2,
                  const float* bound, float* out, int64_t ldo, int32_t m, int32_t d, int32_t f,
                  void* stream);

int fgr_split_weights_bf16_bytes(int32_t n, int32_t k, size_t* bytes);
int fgr_split_weights_bf16(const float* w, int32_t n, int32_t k, int64_t stride_n,
                           int64_t stride_k, void* img, void* stream);
int fgr_gemm_bf16(const float* a, int64_t lda, const void* w_img, float* c, int64_t ldc,
                  const float* bias, const float* r, int64_t ldr, int32_t m, int32_t n, int32_t k,
                  int32_t act, void* stream);

/* ---- attention ---------------------------------------------------------------------
 * Multi-head scaled-dot-product attention core of nn.MultiheadAttention
 * (transformers.py:95-96, 197-226) on packed, unpadded segments: query segment
 * i (rows q_off[i]..q_off[i+1]) attends to key segment kv_seg[i] (rows
 * kv_off[j]..kv_off[j+1]); the reference's key padding mask is the segment end.
 * Head h reads columns [h*dh, (h+1)*dh) of q/k/v rows (row strides ld_*).
 * o = softmax((q * scale) k^T) v, fp32 in/out, fp32 MFMA (v_mfma_f32_16x16x4_f32); any
 * head_dim in {4, 8, 16, 32, 64, 128, 256} (the forward dispatches head_dim 32 / 64 -- every
 * reference config -- to fgr_attention_f16x3 / _bf16 below). */
int fgr_attention(const float* q, int64_t ld_q, const float* k, int64_t ld_k, const float* v,
                  int64_t ld_v, float* o, int64_t ld_o, const int64_t* q_off,
                  const int64_t* kv_off, const int32_t* kv_seg, int32_t n_seg,
                  int32_t max_q_len, int32_t n_head, int32_t head_dim, float scale, void* stream);

/* fp32-accurate attention on the fp16 matrix cores (head_dim 32 -- ModelNet's d 256 / 8 heads --
 * or 64 -- 3DMatch's d 512 / 8 heads), same semantics and arguments as fgr_attention plus
 * the key segment count / row count / longest key segment and a caller workspace: K/V are
 * scaled per (64-key tile, head), Q per query and P by 2^14 into fp16's normal range (exact
 * powers of two), split into two fp16 terms and the three significant term products
 * accumulate in fp32 (<= ~3 * 2^-22 per product); q/k/v/o 16-B aligned, row strides
 * multiples of 4. Workspace: fgr_attention_f16x3_workspace() bytes (split
 * K/V images + per-tile scale exponents), 16-B aligned. */
int fgr_attention_f16x3_workspace(int64_t n_kv_rows, int32_t n_kv_seg, int32_t n_head,
                                  size_t* bytes);
int fgr_attention_f16x3(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                        const float* v, int64_t ld_v, float* o, int64_t ld_o,
                        const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                        int32_t n_seg, int32_t n_kv_seg, int64_t n_kv_rows, int32_t max_q_len,
                        int32_t max_kv_len, int32_t n_head, int32_t head_dim, float scale,
                        void* workspace, int64_t ws_bytes, void* stream);

/* bf16 attention (the bf16 compute mode; head_dim 32 or 64), same semantics and arguments as
 * fgr_attention_f16x3: q * scale * log2(e), K, V and the softmax numerators P rounded to bf16
 * (RNE) where they enter v_mfma_f32_16x16x32_bf16; scores, the online softmax, accumulation
 * and the output stay fp32. Workspace: fgr_attention_bf16_workspace() bytes (bf16 K/V
 * images), 16-B aligned. */
int fgr_attention_bf16_workspace(int64_t n_kv_rows, int32_t n_kv_seg, int32_t n_head,
                                 size_t* bytes);
int fgr_attention_bf16(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                       const float* v, int64_t ld_v, float* o, int64_t ld_o,
                       const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                       int32_t n_seg, int32_t n_kv_seg, int64_t n_kv_rows, int32_t max_q_len,
                       int32_t max_kv_len, int32_t n_head, int32_t head_dim, float scale,
                       void* workspace, int64_t ws_bytes, void* stream);

/* CorrespondenceDecoder.simple_attention (finegrained_regtr.py:328-363; the soft
 * correspondence head of direct_regress_coor: False): single-head attention of width d whose
 * values are the partner cloud's coordinates, for all (layer, cloud) segments in one launch:
 *   out[r] = sum_j softmax_j(scale * q[r] . k[j]) * xyz[v_off[s'] + (j - kv_off[s'])]
 * for query row r of segment s (rows q_off[s]..q_off[s+1]), s' = kv_seg[s], keys j in
 * kv_off[s']..kv_off[s'+1]. fp32; d in {32, 64, 128, 256, 512}; out (rows, 3). */
int fgr_corr_attention(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                       const float* xyz, float* out, const int64_t* q_off, const int64_t* kv_off,
                       const int32_t* kv_seg, const int64_t* v_off, int32_t n_seg,
                       int32_t max_q_len, int32_t d, float scale, void* stream);

/* CorrespondenceDecoder with num_neighbors > 0 (finegrained_regtr.py:353-357), applied to the
 * output of fgr_corr_attention (same q, k, segments and scale). The reference's
 * `neighbor_mask[:, :, topk(attn, k).indices] = 0` indexes the QUERY dimension with top-k KEY
 * indices, so a query row j keeps its unmasked softmax iff j is in the union U_dir of the
 * top-k key indices of every (layer, pair, query) row of its direction (src->tgt, tgt->src);
 * every other row is NaN (softmax of an all -inf row). Segments i with (i % n_clouds) <
 * n_clouds / 2 are the src direction. flags (2 * max_kv_len bytes, device) receive U as
 * bytes, direction-major, for the caller's index-range check (an index >= Q raises in the
 * reference). Ties rank the lower key index first. Workspace: fgr_corr_topk_workspace. */
int fgr_corr_topk_workspace(int64_t n_rows, int32_t max_kv_len, size_t* bytes);
int fgr_corr_topk_mask(const float* q, int64_t ld_q, const float* k, int64_t ld_k, float* out,
                       const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                       int32_t n_seg, int32_t n_clouds, int64_t n_rows, int32_t max_q_len,
                       int32_t max_kv_len, int32_t d, float scale, int32_t n_top, uint8_t* flags,
                       void* ws, size_t ws_bytes, void* stream);

/* Batched device-to-device copies: n (src[i] -> dst[i], bytes[i]) triples (host arrays of device
 * pointers) in one launch per 32 copies; 16-B accesses where both ends are 16-B aligned. Not a
 * reference interface: the HIP-graph replay of the forward refreshes its static inputs and
 * clones its outputs with it (one dispatch instead of one blit per tensor). */
int fgr_copy_batch(int32_t n, const void* const* src, void* const* dst, const int64_t* bytes,
                   void* stream);

/* Device-side row offsets from device-side lengths (int64, n entries -> n + 1 offsets,
 * offsets[0] = 0), so a pyramid level's segment table is built without a host round trip
 * (replaces the host-list -> device copy of fgreg.ops.offsets after grid subsampling;
 * reference: the stack_lengths / batch offsets of PreprocessorGPU,
 * finegrained_kpconv.py:422-542). One launch, asynchronous. */
int fgr_lengths_to_offsets(const int64_t* lengths, int32_t n, int64_t* offsets, void* stream);

/* ---- pose ----------------------------------------------------------------------------
 * fast_compute_rigid_transform (utils/se3_torch.py:226-273; threshold < 0 gives the
 * unthresholded compute_rigid_transform, :131-173) on n_batch independent problems
 * a, b (n_batch, n_pts, 3), w (n_batch, n_pts) -> out (n_batch, 3, 4). */
int fgr_procrustes(const float* a, const float* b, const float* w, int64_t n_batch, int64_t n_pts,
                   float threshold, float* out, void* stream);

/* The forward's pose stage (models/finegrained_regtr.py:198-218) straight from the
 * packed tensors: for pair p and layer l, a = [src_kp ; tgt_corr_l], b = [src_corr_l ;
 * tgt_kp], w = sigmoid([src_logit_l ; tgt_logit_l]) thresholded at `threshold`.
 * xyz (n_tot, 3) coarse points, corr (n_layers, n_tot, 3), logits (n_layers, n_tot),
 * seg_off (2*n_pairs + 1) -> out (n_layers, n_pairs, 3, 4). */
int fgr_pair_pose(const float* xyz, const float* corr, const float* logits, int64_t n_tot,
                  const int64_t* seg_off, int32_t n_pairs, int32_t n_layers, float threshold,
                  float* out, void* stream);

/* ---- test-step tail --------------------------------------------
 * What GenericRegModel.test_step runs after the forward (generic_reg_model.py:128-132),
 * on packed tensors (clouds src_0..src_{B-1}, tgt_0..tgt_{B-1}):
 *  fgr_overlap_pool     compute_overlaps, one level (finegrained_kpconv.py:560-569):
 *                       out[q] = clamp(mean_{h: idx[q,h] < n_prev} prev[idx[q,h]], 0, 1),
 *                       NaN for a row without valid entries (as the reference);
 *  fgr_bce_logits_mean  nn.BCEWithLogitsLoss() on x[i * stride_x] vs y[i] (:264-267);
 *  fgr_transform_points se3_transform_list (se3_torch.py:70-90): rows of segment s get
 *                       pose[s] (3 x 4), or se3_inv(pose[s]) when inverse != 0;
 *  fgr_infonce_rows     InfoNCELossFull.compute_infonce (feature_loss.py:268-296) per anchor
 *                       row, given the match logits (n_anchor, ld) over ALL positive rows
 *                       (columns of pair b: p_off[b]..p_off[b+1]): nearest positive by
 *                       torch.cdist's matrix-multiply distance (lowest index on ties),
 *                       row_mask = (its distance < r_p), points closer than r_n ignored,
 *                       row_loss = logsumexp - positive logit;
 *  fgr_infonce_reduce   sum(loss[mask]) / sum(mask) per pair, mean over pairs (:295, 314);
 *  fgr_circle_loss      CircleLossFull.forward (feature_loss.py:160-243) with Euclidean feature
 *                       distances (feature_loss_type: circle, finegrained_regtr.py:86-88) over
 *                       n_pairs pairs packed along rows (anchor rows a_off[b]..a_off[b+1] of
 *                       anchor_feat (n_anchor, d) / axyz, positive rows p_off[b]..p_off[b+1]);
 *                       fd_off[b] = sum_{b' < b} n_a(b') n_p(b') (int64, device), fd_elems its
 *                       total; max_anchor / max_pos the largest per-pair counts; the workspace
 *                       holds the per-pair distance matrices and per-line losses
 *                       (fgr_circle_loss_workspace bytes); out = the 0-d loss (NaN for a pair
 *                       with no row or no column holding both a positive and a negative, as
 *                       the reference's mean over an empty selection);
 *  fgr_pair_cdist       the circle loss's first stage alone: fd (packed per pair at fd_off[b],
 *                       row-major n_a(b) x n_p(b)) = sqrt(sum_k (a_ik - p_jk)^2 + 1e-12), the
 *                       reference's cdist 'euclidean' by direct differences
 *                       (feature_loss.py:11-36): the training CircleLoss forward;
 *  fgr_corr_loss        CorrCriterion('mae') for src (pose) + tgt (se3_inv(pose)) directions
 *                       with overlap weights w (corr_loss.py:18-38, finegrained_regtr.py:283-296);
 *  fgr_se3_compare      se3_compare(pred[l, b], gt[b]) (se3_torch.py:117-129) -> rotation
 *                       error in degrees and translation error, (n_layers, n_pairs) each.
 * The single-block reductions are deterministic. */
int fgr_overlap_pool(const float* prev, int64_t n_prev, const int64_t* idx, int64_t nq,
                     int32_t width, float* out, void* stream);
int fgr_bce_logits_mean(const float* x, int64_t stride_x, const float* y, int64_t n, float* out,
                        void* stream);
int fgr_transform_points(const float* xyz, int64_t n, const int64_t* seg_off, int32_t n_seg,
                         const float* pose, int32_t inverse, float* out, void* stream);
int fgr_infonce_rows(const float* logits, int64_t ld, const float* axyz, const float* pxyz,
                     const int64_t* a_off, const int64_t* p_off, int32_t n_pairs, int64_t n_anchor,
                     float r_p, float r_n, float* row_loss, float* row_mask, void* stream);
/* Training (loss.backward() through the InfoNCE above): dlogits (n_anchor, n_cols over all
 * pairs' positive rows) = grad[0] * row_weight[i] * (softmax_ij - [j == positive]) over the
 * row's pair block, ignored columns and other pairs' columns 0; row_weight[i] =
 * row_mask[i] / (kept rows of the pair * n_pairs) makes it the gradient of
 * fgr_infonce_reduce's output. The positive / ignore mask / log-sum-exp are recomputed as
 * fgr_infonce_rows does. */
int fgr_infonce_rows_bwd(const float* logits, int64_t ld, const float* axyz, const float* pxyz,
                         const int64_t* a_off, const int64_t* p_off, int32_t n_pairs,
                         int64_t n_anchor, int64_t n_cols, float r_n, const float* row_weight,
                         const float* grad, float* dlogits, int64_t ld_d, void* stream);
int fgr_infonce_reduce(const float* row_loss, const float* row_mask, const int64_t* a_off,
                       int32_t n_pairs, float* out, void* stream);
int fgr_circle_loss_workspace(int64_t fd_elems, int64_t n_anchor, int64_t n_pos, size_t* bytes);
int fgr_circle_loss(const float* anchor_feat, const float* pos_feat, int32_t d, const float* axyz,
                    const float* pxyz, const int64_t* a_off, const int64_t* p_off,
                    const int64_t* fd_off, int32_t n_pairs, int64_t n_anchor, int64_t n_pos,
                    int32_t max_anchor, int32_t max_pos, int64_t fd_elems, float r_p, float r_n,
                    void* ws, size_t ws_bytes, float* out, void* stream);
int fgr_pair_cdist(const float* anchor_feat, const float* pos_feat, int32_t d, const int64_t* a_off,
                   const int64_t* p_off, const int64_t* fd_off, int32_t n_pairs, int32_t max_anchor,
                   int32_t max_pos, float* fd, void* stream);
int fgr_corr_loss(const float* xyz, const float* corr, const float* w, const int64_t* seg_off,
                  int32_t n_pairs, const float* pose, float* out, void* stream);
int fgr_se3_compare(const float* pred, const float* gt, int32_t n_layers, int32_t n_pairs,
                    float* rot_deg, float* trans, void* stream);

/* ---- ModelNet evaluation metrics (benchmark/benchmark_modelnet.py:33-82 compute_metrics, the
 * ModelNet branch of GenericRegModel.test_step, generic_reg_model.py:138-147) -------------------
 * pred, gt (n_pairs, 3, 4) fp32 poses; src, ref (n_pairs, n_pts, 3) the input clouds; raw
 * (n_pairs, n_raw, 3) the clean reference clouds (points_raw); all contiguous.
 * out (n_pairs, 7) fp64 = r_mse, r_mae (the 'xyz' Euler angles in degrees, scipy's from_matrix
 * orthogonalisation restated), t_mse, t_mae, err_r_deg, err_t (isotropic), chamfer_dist (the
 * modified Chamfer distance over the raw cloud). Workspace: fgr_modelnet_metrics_workspace
 * bytes (the per-point squared minima). Two launches, deterministic. */
int fgr_modelnet_metrics_workspace(int32_t n_pairs, int32_t n_pts, size_t* bytes);
int fgr_modelnet_metrics(const float* pred, const float* gt, const float* src, const float* ref,
                         const float* raw, int32_t n_pairs, int32_t n_pts, int32_t n_raw, void* ws,
                         size_t ws_bytes, double* out, void* stream);

/* ---- Input side: the ModelNet crop test pipeline on the GPU ----------
 * Replaces, for a batch of samples, the geometry of data_loaders/modelnet_transforms.py
 * RandomCrop (:176-246), RandomTransformSE3_euler (:300-355), Resampler (:92-148),
 * RandomJitter (:151-173) and ShufflePoints (:374-397) as chained by
 * data_loaders/modelnet.py:111-117; the random draws stay in NumPy's stream on the host
 * (fgreg/transforms_gpu.py). Pair b's raw cloud is rows [offsets[b], offsets[b+1]) of `raw`
 * (ld floats per row, xyz first; at most fgr_crop_max_points rows); cloud 0 = source,
 * 1 = reference.
 *  fgr_crop_pairs_mask      per (pair, cloud): d = (p - mean(p)) . dirs[b, c] and the
 *                           percentile threshold (order statistics crop_k[b], crop_k[b]+1 of d,
 *                           NumPy's lerp with gamma[b]; crop_k[b] < 0: threshold 0, the
 *                           p_keep = 0.5 rule) -> mask (2, Ntot) u8, keep (2, Ntot) i32 (kept
 *                           raw indices, in order, at the pair's offset) and count (n_pairs, 2).
 *  fgr_crop_pairs_assemble  per pair: output row i of cloud c is raw row keep[c][sel[b, c, i]]
 *                           (Resampler's choice composed with ShufflePoints' permutation by
 *                           the host), the source moved by rt[b] (3x4 float32), plus
 *                           noise[b, c, i] (float64, clipped); overlap[b, c, i] = the other
 *                           cloud's mask at that raw index; corr (2, Ntot) i64 gets the
 *                           correspondence pairs (raw-index order) at the pair's offset and
 *                           n_corr[b] their count. sel must hold distinct values < count.
 * Outputs equal fgreg.transforms.modelnet_crop_test bit for bit (tests/test_gpu_transforms.py). */
int fgr_crop_max_points(int32_t* n_max);
int fgr_crop_pairs_mask(const float* raw, int32_t ld, const int64_t* offsets, int32_t n_pairs,
                        const double* dirs, const int32_t* crop_k, const double* gamma,
                        uint8_t* mask, int32_t* keep, int32_t* count, void* stream);
int fgr_crop_pairs_assemble(const float* raw, int32_t ld, const int64_t* offsets, int32_t n_pairs,
                            const uint8_t* mask, const int32_t* keep, const int32_t* sel,
                            const double* noise, const float* rt, int32_t m, float* xyz,
                            uint8_t* overlap, int64_t* corr, int32_t* n_corr, void* stream);

/* The pre-norm layer's in_proj with the attention's K / V images written in its epilogue
 * (transformers.py:193-196 / :213-221 + the image building of fgr_attention_f16x3, head dim 32):
 * qkv = (LayerNorm(x) * gamma + beta + add) W^T + bias as fgr_gemm_f16x3_ln, but only the q
 * columns [0, d) go to q (m, d; ld_q) as fp32 -- the k and v columns go straight into kv_img:
 * the f16x3 K / V images of every GLOBAL 64-row tile and head, then their int2 scale exponents
 * (fgr_kv_image_bytes(m, n_head, 32) bytes). Optional side output out2 = LayerNorm(x) * gamma2 +
 * beta2 as fgr_gemm_f16x3_ln_out2. fgr_gemm_f16x3_ln_qkv_supported(m, d, n_head): d = 32 n_head =
 * 256 and the row-stationary kernel for (m, 3d, d).
 * fgr_attention_f16x3_img: fgr_attention_f16x3 (head dim 32) reading those images (kv rows = the
 * same packed rows, n_kv_rows = m) instead of building its own. */
int fgr_kv_image_bytes(int64_t n_rows, int32_t n_head, int32_t head_dim, size_t* bytes);
int fgr_gemm_f16x3_ln_qkv_supported(int32_t m, int32_t d, int32_t n_head);
int fgr_gemm_f16x3_ln_qkv(const float* x, int64_t ldx, const float* gamma, const float* beta,
                          float eps, const float* add, int64_t ld_add, const void* w_img, float* q,
                          int64_t ld_q, const float* bias, int32_t m, int32_t d, int32_t n_head,
                          void* kv_img, const float* gamma2, const float* beta2, float* out2,
                          int64_t ld_out2, void* stream);
/* fgr_gemm_f16x3_qkv: the same for an in_proj without the LayerNorm prologue, head dim 64
 * (qkv = a W^T + bias, a (m, d); the staged 64 x 128-tile g5 epilogue writes the images):
 * fgr_gemm_f16x3_qkv_supported(m, d, n_head): d = 64 n_head, d % 128 == 0. fgr_kv_image_bytes
 * takes head_dim 32 or 64, fgr_attention_f16x3_img reads either. */
int fgr_gemm_f16x3_qkv_supported(int32_t m, int32_t d, int32_t n_head);
int fgr_gemm_f16x3_qkv(const float* a, int64_t lda, const void* w_img, float* q, int64_t ld_q,
                       const float* bias, int32_t m, int32_t d, int32_t n_head, void* kv_img,
                       void* stream);
/* bf16 mode: fgr_gemm_bf16_qkv writes q (fp32) and the bf16 K / V images (head dim 64, no
 * scales; fgr_kv_image_bf16_bytes) of every global 64-row tile from the register-staged 64 x
 * 128 bf16 kernel's epilogue, fgr_attention_bf16_img reads them. */
int fgr_kv_image_bf16_bytes(int64_t n_rows, int32_t n_head, int32_t head_dim, size_t* bytes);
int fgr_gemm_bf16_qkv_supported(int32_t m, int32_t d, int32_t n_head);
int fgr_gemm_bf16_qkv(const float* a, int64_t lda, const void* w_img, float* q, int64_t ld_q,
                      const float* bias, int32_t m, int32_t d, int32_t n_head, void* kv_img,
                      void* stream);
int fgr_attention_bf16_img(const float* q, int64_t ld_q, const void* kv_img, int64_t n_kv_rows,
                           float* o, int64_t ld_o, const int64_t* q_off, const int64_t* kv_off,
                           const int32_t* kv_seg, int32_t n_seg, int32_t max_q_len,
                           int32_t n_head, int32_t head_dim, float scale, void* stream);
int fgr_attention_f16x3_img(const float* q, int64_t ld_q, const void* kv_img, int64_t n_kv_rows,
                            float* o, int64_t ld_o, const int64_t* q_off, const int64_t* kv_off,
                            const int32_t* kv_seg, int32_t n_seg, int32_t max_q_len,
                            int32_t n_head, int32_t head_dim, float scale, void* stream);

/* The CorrespondenceRegressor head (finegrained_regtr.py:411-455, direct_regress_coor: True) on
 * the (m, d) stacked layer outputs f in two row-stationary f16x3 launches:
 *   hidden = ReLU(f W0^T + b0), logits = f Wc^T + bc   -- ONE product over the image of the
 *            stacked (d + 16, d) weight [W0; Wc; 0] (fgr_split_weights_h3) with bias
 *            b0c = [b0; bc; 0] (d + 16 floats); hidden (m, d) is caller scratch;
 *   corr   = ReLU(hidden W2^T + b2) W4^T + b4           -- the 3-wide coor_mlp[4] formed in the
 *            second product's epilogue from its fp32 outputs (w4 (3, d) and b4 (3) fp32).
 * corr (m, 3), logits (m) contiguous. fgr_corr_head_supported(m, d): d % 16 == 0, d <= 256;
 * other widths use fgr_gemm_f16x3 per layer. */
int fgr_corr_head_supported(int32_t m, int32_t d);
int fgr_corr_head_f16x3(const float* f, int64_t ldf, int32_t m, int32_t d, const void* w0c_img,
                        const float* b0c, const void* w2_img, const float* b2, const float* w4,
                        const float* b4, float* hidden, float* corr, float* logits, void* stream);

/* ---- Training backward (train.py -> trainer.py:110-125 backward) -------
 * The dense products' gradients run on the GEMM entry points above with transposed weight
 * images (fgreg/autograd.py); these cover the rest. Every entry point is deterministic: no
 * floating-point atomics, every reduction in a fixed order (ABI 2; ABI 1's two scatters added
 * with fp32 atomics).
 *  fgr_nbr_inverse      the inverse (CSR) of an (nq, width) neighbour table over ns support rows:
 *                       start[ns + 1], and for support row s the entries e = q * width + h with
 *                       idx[e] == s in ascending e at ent[start[s] .. start[s + 1]); pos[e] = the
 *                       CSR slot of entry e, -1 where idx[e] names no support row (shadow index
 *                       / negative). ent and pos hold nq * width ints; workspace
 *                       fgr_nbr_inverse_workspace bytes. Built once per table, read by both
 *                       scatters below (the reference's gather(method=2) transpose,
 *                       finegrained_kpconv_blocks.py:66-97, as a gather over the inverse).
 *  fgr_kpconv_scatter   KPConv gather-weight backward: dx[s, c] = sum over the entries (q, h)
 *                       naming s, in CSR order, of sum_k w(q,h,k) dwf[q,k,c] with the forward's
 *                       influences (finegrained_kpconv_blocks.py:296-381). dx (ns, cin) is
 *                       WRITTEN (rows nobody names get 0); start / pos from fgr_nbr_inverse of
 *                       idx; workspace fgr_kpconv_scatter_workspace bytes (one cin-row per
 *                       table entry).
 *  fgr_max_pool_bwd     max_pool (:125-141): dx[s, c] = sum of dy[q, c] over the entries (q, h)
 *                       naming s whose slot h is the row's first maximum of channel c (shadow
 *                       entries read 0 and pass nothing on). dx (ns, c) is WRITTEN; start / ent
 *                       from fgr_nbr_inverse of idx; workspace fgr_max_pool_bwd_workspace.
 *  fgr_segnorm_stats    per-(segment, channel) mean / rstd / biased var of v = x / row_div:
 *                       InstanceNorm1d per cloud (:498-507) or BatchNorm1d batch statistics
 *                       (one segment, res2net.py:126-159 in train()); workspace
 *                       fgr_segnorm_workspace bytes.
 *  fgr_segnorm_apply    out = post(act((v - mean) rstd (* gamma + beta)) + residual).
 *  fgr_segnorm_bwd      its backward from (y = out, dy): dx, dres (= d residual), dgamma / dbeta
 *                       (NULL without gamma); workspace fgr_segnorm_workspace + 8 n_seg c bytes.
 *  fgr_layernorm_bwd    nn.LayerNorm backward (transformers.py:105-107): dx, and
 *                       dgamma_dbeta[0..d) = sum dy xhat, [d..2d) = sum dy; d <= 1024.
 *  fgr_colsum           out[c] = sum_r x[r, c] (fp64 partials; bias gradients).
 *  fgr_attention_bwd    softmax attention backward over packed segments (the layout of
 *                       fgr_attention*): dq, dk, dv (each may alias column slices of one
 *                       tensor), head dim 4 / 8 / 16 / 32 / 64, fp32; key segments may be attended by any
 *                       number of query segments.
 *  fgr_corr_attention_bwd  backward of fgr_corr_attention (CorrespondenceDecoder.simple_attention,
 *                       finegrained_regtr.py:328-363): from dout (n_rows, 3) = d corr, writes
 *                       dq = scale dS K and dk = scale dS^T Q (dS = P (dout . xyz_j - dout .
 *                       corr_i)) over the same segment tables; xyz gets no gradient (the
 *                       reference's values are coordinates). Key rows no query segment attends
 *                       get dk = 0; d 32 / 64 / 128 / 256 / 512, fp32; workspace
 *                       fgr_corr_attention_bwd_workspace(n_rows) bytes. */
int fgr_nbr_inverse_workspace(int64_t nq, int32_t width, int64_t ns, size_t* bytes);
int fgr_nbr_inverse(const int64_t* idx, int64_t nq, int32_t width, int64_t ns, int32_t* start,
                    int32_t* pos, int32_t* ent, void* ws, size_t ws_bytes, void* stream);
int fgr_kpconv_scatter_workspace(int64_t nq, int32_t width, int32_t cin, size_t* bytes);
int fgr_kpconv_scatter(const float* q, const float* s, int64_t nq, int64_t ns, const int64_t* idx,
                       int32_t width, const float* dwf, int32_t cin, const float* kernel_points,
                       int32_t n_kp, float extent, const int32_t* start, const int32_t* pos,
                       float* dx, void* ws, size_t ws_bytes, void* stream);
int fgr_max_pool_bwd_workspace(int64_t nq, int32_t c, size_t* bytes);
int fgr_max_pool_bwd(const float* x, int64_t ns, int32_t c, const int64_t* idx, int64_t nq,
                     int32_t width, const float* dy, const int32_t* start, const int32_t* ent,
                     float* dx, void* ws, size_t ws_bytes, void* stream);
int fgr_corr_attention_bwd_workspace(int64_t n_rows, size_t* bytes);
int fgr_corr_attention_bwd(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                           const float* xyz, const float* dout, float* dq, int64_t ld_dq, float* dk,
                           int64_t ld_dk, const int64_t* q_off, const int64_t* kv_off,
                           const int32_t* kv_seg, const int64_t* v_off, int32_t n_seg,
                           int32_t n_kv_seg, int64_t n_rows, int32_t max_q_len, int32_t max_kv_len,
                           int32_t d, float scale, void* ws, size_t ws_bytes, void* stream);
int fgr_segnorm_workspace(int64_t max_seg_len, int32_t c, int32_t n_seg, size_t* bytes);
int fgr_segnorm_stats(const float* x, int64_t n, int32_t c, const int64_t* seg_off, int32_t n_seg,
                      int64_t max_seg_len, const float* row_div, float eps, float* mean, float* rstd,
                      float* var, void* ws, size_t ws_bytes, void* stream);
int fgr_segnorm_apply(const float* x, int64_t n, int32_t c, const int64_t* seg_off, int32_t n_seg,
                      const float* row_div, const float* mean, const float* rstd, const float* gamma,
                      const float* beta, int32_t act, const float* residual, int32_t post_act,
                      float* out, void* stream);
/* fgr_segnorm_stats then fgr_segnorm_apply in one call (the training forward). */
int fgr_segnorm_fwd(const float* x, int64_t n, int32_t c, const int64_t* seg_off, int32_t n_seg,
                    int64_t max_seg_len, const float* row_div, float eps, float* mean, float* rstd,
                    float* var, const float* gamma, const float* beta, int32_t act,
                    const float* residual, int32_t post_act, float* out, void* ws, size_t ws_bytes,
                    void* stream);
int fgr_segnorm_bwd(const float* x, int64_t n, int32_t c, const int64_t* seg_off, int32_t n_seg,
                    int64_t max_seg_len, const float* row_div, const float* mean, const float* rstd,
                    const float* gamma, const float* beta, int32_t act, int32_t has_residual,
                    int32_t post_act, const float* y, const float* dy, float* dx, float* dres,
                    float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);
int fgr_colsum_workspace(int64_t n, int32_t c, size_t* bytes);
int fgr_colsum(const float* x, int64_t n, int32_t c, int64_t ldx, float* out, void* ws,
               size_t ws_bytes, void* stream);
int fgr_layernorm_bwd_workspace(int64_t n, int32_t d, size_t* bytes);
int fgr_layernorm_bwd(const float* x, int64_t n, int32_t d, const float* gamma, float eps,
                      const float* dy, float* dx, float* dgamma_dbeta, void* ws, size_t ws_bytes,
                      void* stream);
int fgr_attention_bwd_workspace(int64_t nq, int32_t nhead, size_t* bytes);
int fgr_attention_bwd(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                      int64_t ldv, const float* o, int64_t ldo, const float* dout, int64_t lddo,
                      float* dq, int64_t lddq, float* dk, int64_t lddk, float* dv, int64_t lddv,
                      const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                      int32_t n_seg, int32_t n_kv_seg, int64_t nq, int64_t max_q_len,
                      int64_t max_kv_len, int32_t nhead, int32_t dh, float scale, void* ws,
                      size_t ws_bytes, void* stream);
/* Training with nn.MultiheadAttention(dropout = p > 0): the same forward / backward with the
 * attention weights of the PV product dropped by a counter-based hash of (seed, head, query
 * row, key row) -- kept with probability 1 - p and scaled by 1 / (1 - p), the softmax sum
 * over every weight (transformers.py:95-96; common.h attn_drop_hash). The backward with the
 * same seed / p reproduces the forward's mask; head dim 16 / 32 / 64 (the forward: 32 / 64),
 * 16-B aligned rows. Masks are not torch's Philox draws (same distribution). */
int fgr_attention_f16x3_drop(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                             const float* v, int64_t ld_v, float* o, int64_t ld_o,
                             const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                             int32_t n_seg, int32_t n_kv_seg, int64_t n_kv_rows, int32_t max_q_len,
                             int32_t max_kv_len, int32_t n_head, int32_t head_dim, float scale,
                             void* workspace, int64_t ws_bytes, uint32_t seed, float p,
                             void* stream);
/* Training pair (dropout p >= 0 as the _drop pair): the forward also writes, per (row, head),
 * the log2-sum-exp of the scaled scores to lse (n_rows * n_head floats); the backward reads it
 * back and skips its own max / sum pass over the keys (head dim 16 / 32 / 64, 16-B aligned
 * rows; other shapes recompute it). */
int fgr_attention_f16x3_train(const float* q, int64_t ld_q, const float* k, int64_t ld_k,
                              const float* v, int64_t ld_v, float* o, int64_t ld_o,
                              const int64_t* q_off, const int64_t* kv_off, const int32_t* kv_seg,
                              int32_t n_seg, int32_t n_kv_seg, int64_t n_kv_rows, int32_t max_q_len,
                              int32_t max_kv_len, int32_t n_head, int32_t head_dim, float scale,
                              void* workspace, int64_t ws_bytes, uint32_t seed, float p, float* lse,
                              void* stream);
int fgr_attention_bwd_train(const float* q, int64_t ldq, const float* k, int64_t ldk,
                            const float* v, int64_t ldv, const float* o, int64_t ldo,
                            const float* dout, int64_t lddo, float* dq, int64_t lddq, float* dk,
                            int64_t lddk, float* dv, int64_t lddv, const int64_t* q_off,
                            const int64_t* kv_off, const int32_t* kv_seg, int32_t n_seg,
                            int32_t n_kv_seg, int64_t nq, int64_t max_q_len, int64_t max_kv_len,
                            int32_t nhead, int32_t dh, float scale, void* ws, size_t ws_bytes,
                            uint32_t seed, float p, const float* lse, int64_t n_kv_rows,
                            void* stream);
/* fgr_attention_bwd_train's workspace over nq query rows in n_seg segments and n_kv_rows packed
 * key rows in n_kv_seg segments: lse / D per (row, head) and, at head dim 32 / 64, the K / V /
 * Q / dO tile images of the dQ and dK / dV kernels on the f16 matrix cores (split-fp16 x3
 * products, as fgr_attention_f16x3). A workspace of fgr_attention_bwd_workspace's size runs the
 * fp32-MFMA kernels instead. */
int fgr_attention_bwd_train_workspace(int64_t nq, int32_t n_seg, int64_t n_kv_rows,
                                      int32_t n_kv_seg, int32_t nhead, int32_t dh, size_t* bytes);
int fgr_attention_bwd_drop(const float* q, int64_t ldq, const float* k, int64_t ldk,
                           const float* v, int64_t ldv, const float* o, int64_t ldo,
                           const float* dout, int64_t lddo, float* dq, int64_t lddq, float* dk,
                           int64_t lddk, float* dv, int64_t lddv, const int64_t* q_off,
                           const int64_t* kv_off, const int32_t* kv_seg, int32_t n_seg,
                           int32_t n_kv_seg, int64_t nq, int64_t max_q_len, int64_t max_kv_len,
                           int32_t nhead, int32_t dh, float scale, void* ws, size_t ws_bytes,
                           uint32_t seed, float p, void* stream);

/* Weight gradient of a dense product, dW = dY^T X (every nn.Linear / KPConv weight of the
 * backward, trainer.py:110-125), read straight from the two row-major activations:
 *   dw[i][j] = sum_{r < rows} dy[r * ld_dy + i] * x[r * ld_x + j]      (i < m, j < n)
 * and, when db is not NULL, the bias gradient db[i] = sum_r dy[r * ld_dy + i] (fp64 sums).
 * fp32-accurate (f16x3: per-chunk column scales, three fp16 products, fp32 accumulation);
 * m, n, the row strides and ld_dw multiples of 4, dy / x / dw 16-B aligned. Rows are split
 * into chunks whose partials are summed in chunk order (deterministic); the workspace
 * fgr_gemm_wgrad_workspace(rows, m, n, db != NULL) bytes holds them (0 when one chunk
 * suffices). rows == 0 writes zeros. */
int fgr_gemm_wgrad_workspace(int64_t rows, int32_t m, int32_t n, int32_t with_bias, size_t* bytes);
int fgr_gemm_f16x3_wgrad(const float* dy, int64_t ld_dy, const float* x, int64_t ld_x,
                         int64_t rows, int32_t m, int32_t n, float* dw, int64_t ld_dw, float* db,
                         void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FGREG_H */
