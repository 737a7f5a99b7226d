/*
 * gdino_amd.h — C-ABI of the MI355X-native Grounding DINO hot path.
 *
 * Every entry point takes plain device pointers, sizes and a HIP stream
 * (gd_stream_t is layout-compatible with hipStream_t; pass NULL for the null
 * stream).  No torch types cross this boundary: the Python host side hands
 * over tensor.data_ptr() and torch.cuda.current_stream().cuda_stream.
 *
 * Status convention (replaces the reference's printf-only launch errors,
 * ops/src/cuda/ms_deform_im2col_cuda.cuh:948-952 and :1321-1325): every call
 * returns GD_OK or an error code, and gd_last_error() gives the message of the
 * most recent failure on the calling thread.
 *
 * Entry points and the reference interface each one replaces:
 *
 *   gd_msda_forward   <- ms_deform_attn_forward
 *                        models/GroundingDINO/ops/src/vision.cpp:14,
 *                        ops/src/ms_deform_attn.h:21-39,
 *                        ops/src/cuda/ms_deform_attn_cuda.cu:20-80
 *   gd_msda_backward  <- ms_deform_attn_backward
 *                        models/GroundingDINO/ops/src/vision.cpp:15,
 *                        ops/src/ms_deform_attn.h:41-61,
 *                        ops/src/cuda/ms_deform_attn_cuda.cu:83-153
 *   gd_msda_backward_geom  the same, given a host copy of the level shapes
 *                        (enables the pixel-block tiling of the encoder
 *                        backward; no reference counterpart)
 *   gd_runtime_info   <- get_cuda_version
 *                        models/GroundingDINO/csrc/vision.cpp:11-51,
 *                        models/GroundingDINO/csrc/cuda_version.cu
 *   gd_biattn_softmax_fwd / _bwd / _workspace_bytes
 *                     <- BiMultiHeadAttention.forward softmax chain (global
 *                        max shift, +-5e4 clamps, column max, -inf masks, the
 *                        two softmaxes) and its autograd backward
 *                        models/GroundingDINO/fuse_modules.py:174-217
 *   gd_window_attn_forward / _backward
 *                     <- WindowAttention.forward core (q.scale.k^T, relative
 *                        position bias gather, shift mask, softmax, attn.v)
 *                        and its autograd backward incl. the scatter into
 *                        relative_position_bias_table
 *                        models/GroundingDINO/backbone/swin_transformer.py:134-174
 *   gd_window_attn_image_forward / _backward
 *                     <- the same plus SwinTransformerBlock.forward's zero
 *                        pad, cyclic shift, window partition, window reverse,
 *                        roll back and crop
 *                        models/GroundingDINO/backbone/swin_transformer.py:238-292
 *
 *   gd_attn_forward / _backward
 *                     <- the attention cores the reference runs as eager
 *                        matmul / softmax / matmul: BERT self-attention (HF
 *                        BertSelfAttention via bertwarper.py:31-166), the
 *                        text enhancer's and the decoder's
 *                        nn.MultiheadAttention (transformer_vanilla.py:83,
 *                        transformer.py:839,844)
 *   gd_msda_prologue_forward / _backward
 *                     <- the MSDA module's softmax over L*P and sampling-
 *                        location math (reference_points + offsets /
 *                        normalizer) models/GroundingDINO/ms_deform_attn.py:274-363
 *   gd_wgrad / gd_wgrad_splits / gd_wgrad_workspace_bytes
 *                     <- the weight / bias gradient of the token-heavy
 *                        nn.Linear layers (autograd's dW = dY^T X GEMM), as a
 *                        split-K fp32 reduction (no reference counterpart:
 *                        torch autograd in the reference)
 *   gd_add_layernorm_forward / _forward2 / _backward / _workspace_bytes
 *                     <- the post-norm `norm(src + dropout(src2))` of the
 *                        deformable encoder / decoder layers and the text
 *                        enhancer (transformer.py:789-808, 877-936,
 *                        transformer_vanilla.py:83-110) and its backward
 *   gd_add_scaled_forward / _backward / _workspace_bytes
 *                     <- the layer-scale / drop-path residual endings
 *                        `v = v + drop_path(gamma_v * delta_v)` of the
 *                        BiAttention fusion block (fuse_modules.py:285-286)
 *                        and `x = shortcut + drop_path(x)` of the Swin blocks
 *                        (swin_transformer.py:295-296) and their backward
 *   gd_graph_memsets_to_kernels
 *                     <- no reference counterpart: the step graph's memset
 *                        nodes as kernel nodes (PyTorch's reductions zero
 *                        their semaphores with a memset)
 *   gd_contrastive_forward
 *                     <- ContrastiveEmbed.forward (x . text^T, -inf on padded
 *                        tokens, -inf right padding to max_text_len)
 *                        models/GroundingDINO/utils.py:242-273, and the
 *                        two-stage score enc_outputs_class_unselected.max(-1)
 *                        models/GroundingDINO/transformer.py:292-296
 *   gd_linear_sum_assignment
 *                     <- HungarianMatcher.forward's C.cpu() + per-image
 *                        scipy.optimize.linear_sum_assignment
 *                        models/GroundingDINO/matcher.py:104-110 (scipy 1.15
 *                        rectangular_lsap: same algorithm, operation order and
 *                        tie-breaking, on the device)
 */
#ifndef GDINO_AMD_H
#define GDINO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* gd_stream_t;

typedef enum {
  GD_OK = 0,
  GD_ERR_INVALID = 1,     /* bad argument (shape, null pointer, dtype) */
  GD_ERR_UNSUPPORTED = 2, /* valid but not implemented combination */
  GD_ERR_LAUNCH = 3,      /* HIP launch / runtime error */
  GD_ERR_DEVICE = 4,      /* a device-side check failed (gd_device_status) */
} gd_status;

typedef enum {
  GD_F32 = 0,
  GD_F64 = 1,
  GD_BF16 = 2,
  GD_F16 = 3,
} gd_dtype;

/* ------------------------------------------------------------------------ */
/* Multi-scale deformable attention                                          */
/* ------------------------------------------------------------------------ */
/*
 * value            [N, S, M, D]        value_dtype (F32, F64, BF16)
 * spatial_shapes   [L, 2] int64 (H, W), device memory
 * level_start_index[L]    int64,        device memory
 * sampling_loc     [N, Lq, M, L, P, 2] loc_dtype = F64 if value is F64, else F32
 * attn_weight      [N, Lq, M, L, P]    loc_dtype
 * output           [N, Lq, M*D]        value_dtype; fully overwritten
 *
 * Semantics: ms_deformable_im2col_gpu_kernel, ms_deform_im2col_cuda.cuh:238-299
 * (sample at loc*(W,H) - 0.5, bilinear, zero outside -1 < h < H, -1 < w < W).
 */
gd_status gd_msda_forward(gd_dtype value_dtype, const void* value,
                          const int64_t* spatial_shapes,
                          const int64_t* level_start_index,
                          const void* sampling_loc, const void* attn_weight,
                          int batch, int spatial_size, int num_heads,
                          int channels, int num_levels, int num_query,
                          int num_point, void* output, gd_stream_t stream);

/*
 * grad_output      [N, Lq, M*D]        value_dtype
 * grad_value       [N, S, M, D]        accumulation dtype: F64 for F64 value,
 *                                      else F32 (zeroed by this call)
 * grad_sampling_loc[N, Lq, M, L, P, 2] loc_dtype (fully overwritten)
 * grad_attn_weight [N, Lq, M, L, P]    loc_dtype (fully overwritten)
 *
 * Semantics: ms_deform_attn_col2im_bilinear, ms_deform_im2col_cuda.cuh:88-159.
 * grad_value is accumulated with float atomics, so its low bits depend on
 * arrival order (as in the reference).
 */
gd_status gd_msda_backward(gd_dtype value_dtype, const void* value,
                           const int64_t* spatial_shapes,
                           const int64_t* level_start_index,
                           const void* sampling_loc, const void* attn_weight,
                           const void* grad_output, int batch,
                           int spatial_size, int num_heads, int channels,
                           int num_levels, int num_query, int num_point,
                           void* grad_value, void* grad_sampling_loc,
                           void* grad_attn_weight, gd_stream_t stream);
/* gd_msda_backward with a HOST copy of spatial_shapes ([num_levels][2]
 * int64, or NULL = gd_msda_backward).  When the levels tile the queries
 * exactly (num_query == spatial_size == sum H*W: the encoder), the backward
 * takes 4 x 8 pixel blocks of each level as its LDS pre-aggregation tiles
 * instead of 32 consecutive queries; results are the same sums. */
gd_status gd_msda_backward_geom(gd_dtype value_dtype, const void* value,
                                const int64_t* spatial_shapes,
                                const int64_t* level_start_index,
                                const void* sampling_loc, const void* attn_weight,
                                const void* grad_output, int batch,
                                int spatial_size, int num_heads, int channels,
                                int num_levels, int num_query, int num_point,
                                void* grad_value, void* grad_sampling_loc,
                                void* grad_attn_weight, const int64_t* spatial_shapes_host,
                                gd_stream_t stream);

/* The same backward without float atomics ("sorted": a per-sample pass for
 * grad_sampling_loc / grad_attn_weight, then grad_value as a sum per
 * destination row over an inverted index of the samples; csrc/msda_sorted.inc).
 * Replaces the same reference entry (ms_deform_attn_cuda.cu:83-153,
 * ms_deform_attn.h:46-61).  Requirements (else GD_ERR_UNSUPPORTED):
 * value F32 or BF16, channels 32, num_levels 4, num_point 4, the HOST level
 * shapes, level_start_index their cumulative sums (as the model builds it)
 * and spatial_size == sum H*W.
 *   grad_value_dtype  F32, or BF16 when value is BF16 (written directly:
 *                     every row is written exactly once, no zero fill)
 *   workspace         device memory of gd_msda_backward_workspace_bytes()
 *   flags             GD_MSDA_DETERMINISTIC: every output bitwise
 *                     reproducible (each grad_value row summed in sample
 *                     order); 0: same sums, order of arrival inside a cell.
 * gd_msda_backward_workspace_bytes returns 0 when the sorted backward does
 * not apply to these sizes. */
#define GD_MSDA_DETERMINISTIC 1
size_t gd_msda_backward_workspace_bytes(gd_dtype value_dtype, int batch, int spatial_size, int num_heads,
                                        int channels, int num_levels, int num_query, int num_point,
                                        const int64_t* spatial_shapes_host, int flags);
gd_status gd_msda_backward_sorted(gd_dtype value_dtype, const void* value,
                                  const int64_t* spatial_shapes,
                                  const int64_t* level_start_index,
                                  const void* sampling_loc, const void* attn_weight,
                                  const void* grad_output, int batch,
                                  int spatial_size, int num_heads, int channels,
                                  int num_levels, int num_query, int num_point,
                                  void* grad_value, gd_dtype grad_value_dtype,
                                  void* grad_sampling_loc, void* grad_attn_weight,
                                  const int64_t* spatial_shapes_host, void* workspace,
                                  size_t workspace_bytes, int flags, gd_stream_t stream);

/*
 * MSDA prologue (ms_deform_attn.py:274-363): offsets [N, Lq, M*L*P*2] and
 * attention logits [N, Lq, M*L*P] (F32 or BF16, contiguous rows with the
 * given row strides in elements), reference_points [N, Lq, L, ref_dim] F32
 * (ref_dim 2: + offsets / (W_l, H_l); 4: + offsets / P * wh * 0.5),
 * spatial_shapes [L][2] int64 on the device; L*P == 16.
 * -> sampling_loc [N, Lq, M, L, P, 2] F32, attn_weight [N, Lq, M, L, P] F32
 *    (softmax over each unit's L*P logits).
 * Backward -> grad_offsets / grad_logits, contiguous, in the input dtype;
 * the reference points get no gradient.
 */
gd_status gd_msda_prologue_forward(gd_dtype dtype, const void* offsets, int64_t offsets_row_stride,
                                   const void* logits, int64_t logits_row_stride,
                                   const float* reference_points, int ref_dim,
                                   const int64_t* spatial_shapes, int N, int Lq, int M, int L, int P,
                                   float* sampling_loc, float* attn_weight, gd_stream_t stream);
gd_status gd_msda_prologue_backward(gd_dtype dtype, const float* grad_loc, const float* grad_attn,
                                    const float* attn_weight, const float* reference_points,
                                    int ref_dim, const int64_t* spatial_shapes, int N, int Lq, int M,
                                    int L, int P, void* grad_offsets, void* grad_logits,
                                    gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* BiAttention bidirectional softmax (fuse_modules.py:174-217)               */
/* ------------------------------------------------------------------------ */
/*
 * s        [B, H, S, T]  scores q.k^T (dtype F32 or BF16), T <= 1024
 * pad_v    [B, S] uint8 (1 = padded image token) or NULL
 * pad_l    [B, T] uint8 (1 = padded text token) or NULL
 * pv       [B, H, S, T]  softmax over T (image -> text attention)
 * pl       [B, H, S, T]  softmax over S, column-normalised (text -> image)
 * workspace gd_biattn_workspace_bytes(B, H, S, T) bytes of device memory
 */
size_t gd_biattn_workspace_bytes(int B, int H, int S, int T);
gd_status gd_biattn_softmax_fwd(gd_dtype dtype, const void* s, const uint8_t* pad_v,
                                const uint8_t* pad_l, int B, int H, int S, int T, void* pv,
                                void* pl, void* workspace, gd_stream_t stream);
/* ds = pv * (dpv - rowsum(dpv * pv)) + pl * (dpl - colsum(dpl * pl)) */
gd_status gd_biattn_softmax_bwd(gd_dtype dtype, const void* pv, const void* pl, const void* dpv,
                                const void* dpl, int B, int H, int S, int T, void* ds,
                                void* workspace, gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Swin window attention (swin_transformer.py:134-174)                       */
/* ------------------------------------------------------------------------ */
/*
 * qkv       [B_, N, 3, nH, head_dim] the qkv Linear output (F32 or BF16,
 *           16-byte aligned), windows of one image consecutive
 * table     [(2Wh-1)(2Ww-1), nH] F32 relative_position_bias_table
 * rel_index [N*N] int64 relative_position_index
 * mask      [nW, N, N] F32 shift mask (0 / -100) or NULL; window b uses
 *           mask[b % nW]; B_ % nW == 0
 * out       [B_, N, nH*head_dim] (qkv dtype);  lse [B_, nH, N] F32 (softmax
 *           log-sum-exp, input of the backward)
 * N <= 64, head_dim == 32 (every Swin-T/S/B/L head); scale = head_dim^-0.5
 * unless qk_scale is set.
 */
gd_status gd_window_attn_forward(gd_dtype dtype, const void* qkv, const float* table,
                                 const int64_t* rel_index, const float* mask, int B_, int N,
                                 int nH, int head_dim, int nW, float scale, void* out, float* lse,
                                 gd_stream_t stream);
/* grad_qkv [B_, N, 3, nH, head_dim] is written (every real token);
 * grad_table [(2Wh-1)(2Ww-1), nH] F32 is ACCUMULATED into (zero it first). */
gd_status gd_window_attn_backward(gd_dtype dtype, const void* qkv, const float* table,
                                  const int64_t* rel_index, const float* mask, const void* out,
                                  const void* grad_out, const float* lse, int B_, int N, int nH,
                                  int head_dim, int nW, float scale, void* grad_qkv,
                                  float* grad_table, gd_stream_t stream);
/*
 * The same on the UNPARTITIONED image: qkv [B, H*W, 3, nH, head_dim] (the qkv
 * Linear of the normed tokens, row-major over (y, x)) -> out [B, H*W, nH*head_dim].
 * The image is zero-padded to Hp x Wp (multiples of `window`), rolled by
 * -shift and cut into B * (Hp/window) * (Wp/window) windows of N = window^2
 * tokens, exactly as the reference; a pad position's q/k/v is qkv_bias
 * [3, nH, head_dim] (same dtype as qkv; the Linear of a zero row), or zeros
 * when qkv_bias is NULL.  mask (NULL when shift == 0) is [nW_image, N, N].
 * lse is [B * nW_image, nH, N].
 */
gd_status gd_window_attn_image_forward(gd_dtype dtype, const void* qkv, const void* qkv_bias,
                                       const float* table, const int64_t* rel_index, const float* mask,
                                       int B, int H, int W, int window, int shift, int nH, int head_dim,
                                       float scale, void* out, float* lse, gd_stream_t stream);
/* grad_qkv [B, H*W, 3, nH, head_dim] is written; grad_qkv_bias [3, nH,
 * head_dim] F32 (the pad positions' share of the qkv bias gradient; ignored
 * when qkv_bias is NULL) and grad_table are ACCUMULATED into. */
gd_status gd_window_attn_image_backward(gd_dtype dtype, const void* qkv, const void* qkv_bias,
                                        const float* table, const int64_t* rel_index, const float* mask,
                                        const void* out, const void* grad_out, const float* lse, int B,
                                        int H, int W, int window, int shift, int nH, int head_dim,
                                        float scale, void* grad_qkv, float* grad_qkv_bias,
                                        float* grad_table, gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Masked multi-head attention (flash-style; scores never reach HBM)         */
/* ------------------------------------------------------------------------ */
/*
 * q [B, H, Lq, head_dim], k / v [B, H, Lk, head_dim] and out (and the
 * gradients) are addressed through host arrays of 3 element strides
 * (b, h, l); channels are contiguous and every row is 16-byte aligned.
 * mask (mask_kind 1: uint8 keep-mask, 1 = attend; 2: additive F32; 0: none)
 * is indexed [b, h, q, k] through 3 host strides (b, h, q), 0 for a
 * broadcast dimension, and is contiguous along k.
 * dtype F32 or BF16, head_dim 32 or 64, Lq, Lk > 0, B*H < 65536.
 * lse [B, H, Lq] F32: per-row log-sum-exp (+inf for a row with every key
 * masked, whose output is 0), input of the backward.
 * dropout_p in [0, 1): attention-probability dropout after the softmax
 * normaliser; element (b, h, q, k) is dropped when
 * lowbias32(k*0x9E3779B1 ^ q*0x85EBCA77 ^ (b*H+h)*0xC2B2AE3D ^ seed)
 * < dropout_p * 2^32 (the backward must get the same seed).
 */
gd_status gd_attn_forward(gd_dtype dtype, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                          const int64_t* q_strides, const void* k, const int64_t* k_strides,
                          const void* v, const int64_t* v_strides, const void* mask, int mask_kind,
                          const int64_t* mask_strides, float scale, float dropout_p, uint32_t seed,
                          void* out, const int64_t* out_strides, float* lse, gd_stream_t stream);
/* The same with the dropout seed also read from device memory: the kernels
 * use seed ^ *seed_dev (seed_dev NULL: seed alone).  A captured HIP graph
 * bakes a host seed into every replay; a seed tensor the graph refills each
 * step (a graph-safe torch.randint) gives every replay its own mask, and the
 * backward reads the same word. */
gd_status gd_attn_forward_dev(gd_dtype dtype, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                              const int64_t* q_strides, const void* k, const int64_t* k_strides,
                              const void* v, const int64_t* v_strides, const void* mask, int mask_kind,
                              const int64_t* mask_strides, float scale, float dropout_p, uint32_t seed,
                              const uint32_t* seed_dev, void* out, const int64_t* out_strides, float* lse,
                              gd_stream_t stream);
gd_status gd_attn_backward_dev(gd_dtype dtype, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                               const int64_t* q_strides, const void* k, const int64_t* k_strides,
                               const void* v, const int64_t* v_strides, const void* mask, int mask_kind,
                               const int64_t* mask_strides, float scale, float dropout_p, uint32_t seed,
                               const uint32_t* seed_dev, const void* out, const int64_t* out_strides,
                               const void* grad_out, const int64_t* grad_out_strides, const float* lse,
                               float* dsum, void* grad_q, const int64_t* grad_q_strides, void* grad_k,
                               const int64_t* grad_k_strides, void* grad_v, const int64_t* grad_v_strides,
                               gd_stream_t stream);
/* dsum: [B, H, Lq] F32 workspace (rowsum(dO . O)); grad_q / grad_k / grad_v
 * are fully written. */
gd_status gd_attn_backward(gd_dtype dtype, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                           const int64_t* q_strides, const void* k, const int64_t* k_strides,
                           const void* v, const int64_t* v_strides, const void* mask, int mask_kind,
                           const int64_t* mask_strides, float scale, float dropout_p, uint32_t seed,
                           const void* out, const int64_t* out_strides, const void* grad_out,
                           const int64_t* grad_out_strides, const float* lse, float* dsum,
                           void* grad_q, const int64_t* grad_q_strides, void* grad_k,
                           const int64_t* grad_k_strides, void* grad_v,
                           const int64_t* grad_v_strides, gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Contrastive text-alignment head (utils.py:242-273)                        */
/* ------------------------------------------------------------------------ */
/*
 * x [B, Q, C] and text [B, T, C] (F32 or BF16) through host arrays of two
 * element strides (b, row); rows contiguous and 16-byte aligned; C % 32 == 0.
 * text_mask [B, T] uint8 (1 = real token), contiguous.  T <= Tout.
 * logits [B, Q, Tout] F32 (or NULL): x . text^T, -inf where text_mask is 0
 *        and for T <= t < Tout.
 * rowmax [B, Q] F32 (or NULL): max over t of logits (-inf if no token).
 */
gd_status gd_contrastive_forward(gd_dtype dtype, const void* x, const int64_t* x_strides,
                                 const void* text, const int64_t* text_strides,
                                 const uint8_t* text_mask, int B, int Q, int T, int C, int Tout,
                                 float* logits, float* rowmax, gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Split-K weight gradient of token-heavy Linear layers                      */
/* ------------------------------------------------------------------------ */
/*
 * grad_y [T, O] and x [T, I] (F32 or BF16) row-major with row strides ldy /
 * ldx (elements, 16-byte aligned rows); O, I multiples of 64.
 * grad_w [O, I] F32 = grad_y^T x;  grad_b [O] F32 = column sums of grad_y
 * (or NULL).  Both are overwritten.  splits: token splits (gd_wgrad_splits
 * gives the default); workspace: gd_wgrad_workspace_bytes(O, I, splits)
 * bytes of device memory.  Deterministic (fixed-order reduction).
 */
int gd_wgrad_splits(int T, int O, int I);
/* the same policy for `batch` independent products (gd_wgrad_batched) */
int gd_wgrad_splits_batched(int T, int O, int I, int batch);
/* Batched form: out[b] = grad_y[b]^T x[b] for b < batch (batch strides in
 * elements), written in out_dtype (F32 or BF16) with batch stride
 * batch_stride_out; grad_b only for batch == 1.  Used for the
 * image-token-long products of BiAttention (P_l^T v_v, P_v^T dO_v, dS^T q).
 * workspace: gd_wgrad_workspace_bytes(O, I, batch * splits) bytes. */
gd_status gd_wgrad_batched(gd_dtype dtype, const void* grad_y, int64_t ldy, int64_t batch_stride_y,
                           const void* x, int64_t ldx, int64_t batch_stride_x, int T, int O, int I,
                           int batch, int splits, void* workspace, gd_dtype out_dtype, void* out,
                           int64_t batch_stride_out, float* grad_b, gd_stream_t stream);
size_t gd_wgrad_workspace_bytes(int O, int I, int splits);
gd_status gd_wgrad(gd_dtype dtype, const void* grad_y, int64_t ldy, const void* x, int64_t ldx, int T,
                   int O, int I, int splits, void* workspace, float* grad_w, float* grad_b,
                   gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Residual add + LayerNorm                                                  */
/* ------------------------------------------------------------------------ */
/*
 * x, r [rows, C] (F32 or BF16 each; r may be NULL), weight / bias [C] F32,
 * C in {64, 96, 128, 192, 256, 384, 512, 768, 1024, 1536, 2048}.
 * y [rows, C] F32 = LayerNorm(x + r) * weight + bias; mean / rstd [rows] F32.
 * _forward2 also writes y_bf16 [rows, C] BF16 = y rounded to nearest even
 * (when not NULL): the copy a bf16 GEMM consumer would otherwise cast.
 * Backward: grad_y F32 -> grad_x (x dtype), grad_r (r dtype, or NULL),
 * grad_weight / grad_bias [C] F32 (both or neither; overwritten, need
 * gd_add_layernorm_workspace_bytes(C) bytes of workspace).  Deterministic.
 */
size_t gd_add_layernorm_workspace_bytes(int C);
gd_status gd_add_layernorm_forward(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                   const float* weight, const float* bias, int64_t rows, int C,
                                   float eps, float* y, float* mean, float* rstd, gd_stream_t stream);
gd_status gd_add_layernorm_forward2(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                    const float* weight, const float* bias, int64_t rows, int C,
                                    float eps, float* y, void* y_bf16, float* mean, float* rstd,
                                    gd_stream_t stream);
gd_status gd_add_layernorm_backward(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                    const float* weight, const float* grad_y, const float* mean,
                                    const float* rstd, int64_t rows, int C, void* grad_x, void* grad_r,
                                    float* grad_weight, float* grad_bias, void* workspace,
                                    gd_stream_t stream);
/* The same with grad_y2 (optional, fp32 [rows, C]): the gradient of a second
 * consumer of y, summed with grad_y inside the kernel (the accumulation add
 * autograd would run for an output read by two layers).  Python:
 * gdino_amd.layernorm.add_norm(..., taps=2). */
gd_status gd_add_layernorm_backward2(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                     const float* weight, const float* grad_y, const float* grad_y2,
                                     const float* mean, const float* rstd, int64_t rows, int C, void* grad_x,
                                     void* grad_r, float* grad_weight, float* grad_bias, void* workspace,
                                     gd_stream_t stream);

/* Three-input add + LayerNorm of the deformable layers' attention sublayer,
 * C = 256: y = LayerNorm(x + (r + dropout(r2))) -- x the fp32 residual
 * stream, r the fp32 identity the MSDA module adds and r2 its bf16 output
 * (reference ms_deform_attn.py `self.dropout(output) + identity`, then
 * transformer.py:789-808 `norm1(src + dropout1(src2))` with dropout1 = 0).
 * Dropout keeps (row, col) by a counter-based hash of seed ^ *seed_dev
 * (seed_dev NULL: seed alone), kept values bf16(v / (1 - p)); the backward
 * regenerates the mask.  Backward: grad_x = the gradient of x and of r (the
 * same values), grad_r2 (bf16, optional) = bf16(bf16(ds) / (1 - p)) where
 * kept; grad_weight / grad_bias fp32 (workspace:
 * gd_add_layernorm_workspace_bytes(256)).  grad_y2 (optional): the gradient of a
 * second consumer of y, summed in the kernel.  Python:
 * gdino_amd.layernorm.add_norm3. */
gd_status gd_add_layernorm3_forward(const float* x, const float* r, const void* r2_bf16, const float* weight,
                                    const float* bias, int64_t rows, int C, float eps, float drop_p, uint32_t seed,
                                    const uint32_t* seed_dev, float* y, void* y_bf16, float* mean, float* rstd,
                                    gd_stream_t stream);
gd_status gd_add_layernorm3_backward(const float* x, const float* r, const void* r2_bf16, const float* weight,
                                     const float* grad_y, const float* grad_y2, const float* mean, const float* rstd,
                                     int64_t rows, int C,
                                     float drop_p, uint32_t seed, const uint32_t* seed_dev, float* grad_x,
                                     void* grad_r2_bf16, float* grad_weight, float* grad_bias, void* workspace,
                                     gd_stream_t stream);

/* Pre-norm residual step (Swin blocks, reference swin_transformer.py
 * :295-296): sum = x + branch * scale, y = LayerNorm(sum) (y_bf16: optional
 * bf16 twin), x / sum / y fp32 [rows, C], branch fp32 or bf16, scale fp32:
 * scale[row / tokens_per_sample] when per_sample, else scale[0] (the
 * drop-path factor).  C in {96, 192, 256, 384, 768}.  Backward sums the two
 * incoming gradients in the kernel: ds = grad_sum (NULL: 0) + LN'(grad_y);
 * grad_x = ds, grad_branch = ds * scale (branch dtype, optional), gamma /
 * beta gradients fp32 (workspace: gd_add_layernorm_workspace_bytes(C)).
 * Python: gdino_amd.layernorm.add_scaled_norm. */
gd_status gd_add_scaled_layernorm_forward(const float* x, gd_dtype branch_dtype, const void* branch,
                                          const float* scale, int64_t tokens_per_sample, int per_sample,
                                          const float* weight, const float* bias, int64_t rows, int C, float eps,
                                          float* sum, float* y, void* y_bf16, float* mean, float* rstd,
                                          gd_stream_t stream);
gd_status gd_add_scaled_layernorm_backward(const float* grad_sum, const float* grad_y, const float* sum,
                                           gd_dtype branch_dtype, const float* scale, int64_t tokens_per_sample,
                                           int per_sample, const float* weight, const float* mean, const float* rstd,
                                           int64_t rows, int C, float* grad_x, void* grad_branch,
                                           float* grad_weight, float* grad_bias, void* workspace,
                                           gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Scaled residual ending (fuse_modules.py:285-286, swin_transformer.py:295-296) */
/* ------------------------------------------------------------------------ */
/*
 * x, branch, out [B, N, C] contiguous (F32 or BF16 each, vector aligned:
 * 16 B for F32, 8 B for BF16), C % 4 == 0, C <= 1024; s F32 with
 * s[b][c] at s + b * s_bstride + c * s_cstride (s_cstride 0 or 1; strides 0
 * broadcast).  out = x + branch * s in fp32, rounded to out's dtype.
 * Backward: grad_out (F32 or BF16) -> grad_branch = grad_out * s in
 * branch's dtype (or NULL) and grad_s_bc [B, C] F32 = sum over the N tokens
 * of grad_out * branch (or NULL; needs gd_add_scaled_workspace_bytes(B, N, C)
 * bytes of workspace; the caller folds it to s's broadcast shape).
 * Deterministic.
 */
size_t gd_add_scaled_workspace_bytes(int64_t B, int64_t N, int C);
gd_status gd_add_scaled_forward(gd_dtype x_dtype, const void* x, gd_dtype branch_dtype, const void* branch,
                                const float* s, int64_t s_bstride, int s_cstride, int64_t B, int64_t N, int C,
                                gd_dtype out_dtype, void* out, gd_stream_t stream);
gd_status gd_add_scaled_backward(gd_dtype g_dtype, const void* grad_out, gd_dtype branch_dtype,
                                 const void* branch, const float* s, int64_t s_bstride, int s_cstride,
                                 int64_t B, int64_t N, int C, void* grad_branch, float* grad_s_bc,
                                 void* workspace, gd_stream_t stream);
/* out[n] = a + b (fp32, n % 4 == 0, 16-B aligned) with the bf16 copies of out
 * and of a (each optional, NULL) written in the same pass: the encoder's
 * with_pos_embed (reference transformer.py:780-781, query = src + pos) feeding
 * the bf16 sampling-offset / attention-weight and value projections
 * (ms_deform_attn.py:290-297 under autocast).  Python:
 * gdino_amd.misc.add_with_twins. */
gd_status gd_add_twin_forward(const float* a, const float* b, int64_t n, float* out, void* out_bf16, void* a_bf16,
                              gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Box refinement: out = sigmoid(delta + inverse_sigmoid(ref))               */
/* ------------------------------------------------------------------------ */
/*
 * Replaces the composition `delta + inverse_sigmoid(ref)` then `.sigmoid()`
 * of the decoder's anchor update (reference transformer.py:728-731) and the
 * per-layer box heads (reference groundingdino.py:325-327), inverse_sigmoid
 * as reference util/misc.py:614-618 (clamp to [0, 1], then log(max(x, eps) /
 * max(1 - x, eps))).  Python: gdino_amd.misc.box_refine.
 *
 * delta [n0, n1, n2] fp32 / bf16 and ref fp32, each with its own element
 * strides (ds*, rs*); out fp32 contiguous [n0, n1, n2].  Backward: grad_out
 * and out (the forward's result) contiguous fp32; grad_delta (delta's dtype)
 * and grad_ref (fp32) contiguous, either may be NULL.  The gradients are
 * autograd's for the composition (clamp masks inclusive; NaN ref -> 0).
 */
gd_status gd_box_refine_forward(gd_dtype delta_dtype, const void* delta, int64_t ds0, int64_t ds1, int64_t ds2,
                                const float* ref, int64_t rs0, int64_t rs1, int64_t rs2, int64_t n0, int64_t n1,
                                int64_t n2, float eps, float* out, gd_stream_t stream);
gd_status gd_box_refine_backward(gd_dtype delta_dtype, const float* grad_out, const float* out, const float* ref,
                                 int64_t rs0, int64_t rs1, int64_t rs2, int64_t n0, int64_t n1, int64_t n2,
                                 float eps, void* grad_delta, float* grad_ref, gd_stream_t stream);

/* Decoder query anchors of one layer (reference transformer.py:660-672,
 * utils.py:204-230 gen_sineembed_for_position): ref [nq, bs, 4] fp32 (element
 * strides rs0..rs2), valid_ratios [bs, L, 4] fp32 contiguous, dim_t [128]
 * (10000^(2 (j / 2) / 128)) -> ref_input [nq, bs, L, 4] = ref * valid_ratios,
 * sine [nq, bs, 512] = the (y, x, w, h) sine / cosine embedding of
 * ref_input[:, :, 0].  Forward only (the anchors carry no gradient).
 * Python: models/GroundingDINO/utils.query_anchors. */
gd_status gd_query_anchor_forward(const float* ref, int64_t rs0, int64_t rs1, int64_t rs2, int64_t nq, int64_t bs,
                                  const float* valid_ratios, int L, const float* dim_t, float* ref_input,
                                  float* sine, gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Captured-graph surgery (the train step as one HIP graph)                  */
/* ------------------------------------------------------------------------ */
/*
 * graph: a captured, not yet instantiated hipGraph_t.  Every memset node is
 * replaced by a kernel node (the library's fill kernels, same destination,
 * value and dependencies): on ROCm 7.0 a replayed graph's memset nodes stop
 * taking effect once eager device-to-device copies have run between
 * replays.  Returns the number of nodes replaced, or -1 when a memset node
 * cannot be expressed (element size not 1 / 2 / 4, a pitched 2-D memset, a
 * destination not aligned to its element); all nodes are validated before
 * any is edited, so on -1 the graph is unchanged.
 */
int gd_graph_memsets_to_kernels(void* graph);
/*
 * stream: a hipStream_t whose capture failed part-way (an operation the
 * capture refused, e.g. a synchronisation): ends the invalidated capture and
 * destroys its graph so the stream runs work again.  -> 1 when a capture
 * was ended, 0 when the stream was not capturing, -1 on a HIP error.
 */
int gd_stream_abort_capture(void* stream);

/* ------------------------------------------------------------------------ */
/* Hungarian matching (matcher.py:104-110)                                   */
/* ------------------------------------------------------------------------ */
/*
 * cost    [problems][Q][K] F32 (problem p at cost + p * problem_stride,
 *         row-major [Q, K]); problem p uses its first n_p = sizes[p] columns
 *         (the targets; device memory, int32).
 * Solves linear_sum_assignment(cost[p][:, :n_p]) exactly as scipy 1.15 does
 * (float64, same tie-breaking) and writes its min(Q, n_p) pairs in ascending
 * row (query) order: out_row[p][r] = query, out_col[p][r] = target, r <
 * min(Q, n_p); the remaining K - min(Q, n_p) slots get -1.  status[p] (or
 * NULL): 0, or 1 when scipy would raise (infeasible: +inf costs), in which
 * case the pairs are the reference's fallback (argmin query per target,
 * matcher.py:111-119).  Limits: max(Q, K) <= 2048, min(Q, K) or Q <= 1024.
 */
gd_status gd_linear_sum_assignment(const float* cost, int problems, int Q, int K, int64_t problem_stride,
                                   const int* sizes, int64_t* out_row, int64_t* out_col, int* status,
                                   gd_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Runtime                                                                   */
/* ------------------------------------------------------------------------ */
const char* gd_last_error(void);
/* "hip=<runtime version>;arch=<gcnArchName of current device>;build=<hipcc>" */
const char* gd_runtime_info(void);
/* Synchronises `stream`, then reads and clears the library's device-side
 * check word: GD_OK, or GD_ERR_DEVICE with the failed check in
 * gd_last_error().  The kernels never store out of bounds when a check fails
 * (e.g. the sorted MSDA backward drops a record whose slot lies past its
 * buffer instead of faulting); this call is how the host learns of it.
 * Not for use inside a graph capture (it synchronises). */
gd_status gd_device_status(gd_stream_t stream);
/* Token-linear forward GEMM (csrc/tlin.hip): y[M, N] = x[M, K] . W[N, K]^T
 * (+ bias[N]) (ReLU when relu != 0), bf16 x / W / bias / y, fp32
 * accumulation; x rows ldx apart, y rows ldy apart (elements, multiples of
 * 8, 16-B aligned), W contiguous.  K, N multiples of 8.  The forward of the
 * token-heavy Linear layers (reference F.linear under bf16 autocast:
 * transformer.py:784-808, fuse_modules.py:43-64, swin_transformer.py:30-46).
 * Python: gdino_amd.wgrad.TokenLinear. */
gd_status gd_token_linear_forward(const void* x, int64_t ldx, const void* weight, const void* bias, int M, int K,
                                  int N, int relu, void* y, int64_t ldy, gd_stream_t stream);
/* The same product with the backward of a ReLU folded into the store:
 * y = (x . W^T) where mask[M, N] > 0, else 0 (mask rows ldm apart, bf16) --
 * the input gradient of the FFN's second Linear, whose input is the first
 * Linear's ReLU output (reference transformer.py:784-790 forward_ffn:
 * linear2(dropout(relu(linear1(src))))), so the ReLU's threshold pass over
 * the [tokens, d_ffn] gradient is gone.  Python: gdino_amd.wgrad.TokenLinear. */
gd_status gd_token_linear_forward_masked(const void* x, int64_t ldx, const void* weight, int M, int K, int N,
                                         const void* mask, int64_t ldm, void* y, int64_t ldy, gd_stream_t stream);
/* ABI version: bumped when a signature changes. */
int gd_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GDINO_AMD_H */
