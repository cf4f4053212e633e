/* liblci — MI355X (gfx950) kernels for the long-context image-token mixers of
 * NHLBI/long_context_biomedical_imaging (the reference), exposed as a C ABI.
 *
 * Conventions
 *   - Plain device pointers, sizes and a hipStream_t passed as void*. No torch types.
 *   - Every entry point enqueues on `stream` and returns 0 on success; non-zero on failure with
 *     lci_last_error() describing it (1 = bad shape/alignment, 2 = HIP API error, 3 = launch error).
 *   - Memory is owned by the caller; the library never allocates or frees device memory. Buffers
 *     documented as "accumulated" must be zeroed by the caller.
 *   - dtype codes: 0 = f32, 1 = bf16 (IEEE bfloat16 stored as uint16). Row-major throughout.
 *   - "channels-last" = (B, L, C) with unit channel stride; "channel-major rows" = (rows, L).
 *
 * Reference interfaces replaced (file:line under /root/reference)
 *   lci_attn_*            SABlock.forward attention core, model/models/backbone_vit.py:191-203
 *   lci_window_attn_*     WindowAttention.forward, model/models/backbone_swin.py:339-359, and in grid mode the
 *                         pad/roll/window_partition/window_reverse/crop of SwinTransformerBlock.forward_part1
 *                         (:435-487) with compute_mask (:591-628)
 *   lci_selective_scan_*  mamba_ssm selective_scan_fn (mamba-ssm 1.2.0.post1) as called at model/models/mamba.py:125-134
 *   lci_dwconv_silu_*     MambaVisionMixer depthwise conv1d + SiLU, model/models/mamba.py:118-119
 *   lci_mamba_proj_*      MambaVisionMixer x_proj -> (dt, B, C) split -> dt_proj, model/models/mamba.py:120-124
 *   lci_fftconv_*         fftconv_ref (gelu=False), model/models/hyena.py:32-51 / Filter.forward :201-216
 *   lci_direct_conv_*     the same long convolution for Swin-window rows (L <= 512, backbone_swin.py:361-362)
 *   lci_hyena_pre/post_*  HyenaOperator short filter + gating, model/models/hyena.py:317-355
 *   lci_upsample2x_*      UperNet2D.forward's final bilinear re-sampling (align_corners=False, 2x), model/models/
 *                         seg_heads.py:138, into the head conv's channels-last bf16 operand
 *   lci_upsample3d_cl_fwd UperNet3D.forward's final trilinear re-sampling (seg_heads.py:273), same fusion;
 *   lci_resample1d_adj    its adjoint (deterministic gather), one axis at a time
 *   lci_hyena_filter_*    Filter.filter (implicit-filter MLP z -> Linear/Sin x3 -> Linear, ExponentialModulation),
 *                         model/models/hyena.py:54-117,190-199, called at :343
 *   lci_conv3_fwd         MONAI-1.3 UnetResBlock 3x3(x3) convs of the ViTUNETR / SwinUNETR heads, enhance_heads.py:30-356
 *   lci_inorm_*           MONAI-1.3 UnetResBlock InstanceNorm (+ LeakyReLU) of the same heads
 *   lci_patch_embed_*     MONAI-1.3 PatchEmbeddingBlock (backbone_vit.py:351-361) / PatchEmbed (backbone_swin.py:800-806)
 *   lci_layernorm_*       TransformerBlock / SwinTransformerBlock norm1, norm2 (nn.LayerNorm, backbone_vit.py:250-262,
 *                         backbone_swin.py:418,431) + the autocast cast
 *                         of its output to the next Linear's bf16 operand
 *   lci_gelu_*            MONAI MLPBlock's nn.GELU() between linear1 and linear2 (backbone_vit.py:249) under autocast
 *   lci_linear_*          the token-wise nn.Linear GEMMs: MLPBlock linear1 + GELU + linear2 with fused epilogues
 *                         (backbone_vit.py:249, MONAI MLPBlock) and the weight / bias gradient of (SABlock qkv / out_proj
 *                         backbone_vit.py:166-167, MONAI MLPBlock linear1/2, MambaVisionMixer in/x/dt/out_proj
 *                         mamba.py:60-64,90, HyenaOperator in/out_proj hyena.py:278-279, Swin qkv/proj/mlp)
 */
#ifndef LCI_H_
#define LCI_H_

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped whenever an entry point's argument list or buffer contract changes (3: lci_layernorm_bwd gained dres;
 * 4: lci_conv3_wgrad writes one partial per voxel split instead of one per split and wave; 5: lci_linear_wgrad;
 * 6: lci_hyena_filter; 7: lci_upsample2x; 8: lci_gelu;
 * 9: lci_layernorm_add_fwd; 10: lci_upsample2x_nhwc; 11: lci_fftconv Su; 12: lci_upsample3d_cl_fwd,
 * lci_resample1d_adj and the round-3 entry points below; 13: lci_conv3_fwd_split, lci_conv3_pack_weight,
 * lci_inorm_apply_res, lci_convup_interleave, lci_window_bias with either table optional; 14: lci_window_attn_fwd
 * takes the transposed table biasT, lci_window_attn_bwd's plain table only for windows of N > 384; 15:
 * lci_window_attn_bwd pad_ws; 16: lci_attn_bwd delta_ws is (B, H, 2, L): the negated row constants -lse2 | -delta; 17: lci_window_bwd_needs_plain;
 * 18: lci_attn_bwd delta_ws is lci_attn_bwd_ws_bytes(B, H, L) bytes; 19: selective-scan checkpoints in the I/O
 * dtype; 20: lci_attn_gen_fwd / lci_attn_gen_bwd; 21: lci_gemm_bt; 22: lci_linear_fwd removed, superseded by
 * lci_gemm_bt; 23: lci_fftconv_spectrum Dv; 24: lci_inorm_finalize; 25: lci_adam_step; 26: Hyena gate dx2 / gx2
 * in the activation dtype; 27: lci_layernorm_bwd dxb; 28: lci_resample_cl_fwd, lci_resample1d_adj_ac; 29: lci_bn_relu_*; 30: lci_gemm_bt_acc;
 * 31: lci_layernorm_bwd dres2; 32: one-chunk selective scan without end-state workspaces (xend / xinit / sdt null),
 * lci_selective_scan_bwd_plain_dbc); 33: lci_gemm_bt_small (+ _supported, _acc). */
#define LCI_ABI_VERSION 33
const char* lci_last_error(void);
int lci_abi_version(void);
/* sha256 prefix of the sources the library was built from (build_lib.source_hash); the Python binding refuses a
 * library whose hash differs from the sources beside it. */
const char* lci_build_hash(void);

/* ------------------------------------------------------------------ ViT full self-attention (flash)
 * qkv : (B, L, 3*H*64) bf16, the packed qkv Linear output, channel order (qkv, head, d)
 *       (backbone_vit.py:168 Rearrange "b h (qkv l d) -> qkv b l h d").
 * out : (B, L, H*64) bf16 = softmax(q k^T * scale) v in "b l (h d)" order (backbone_vit.py:169).
 * lse2: (B, H, L) f32 = log2 sum_y exp(scale q.k_y) per query row (consumed by the backward).
 * knorm_ws: lci_attn_fwd_ws_bytes(B, L, H) bytes of device memory (per-64-key-tile bounds max ||k||,
 *       written and read by this call; they let the forward skip the row max on provably safe tiles).
 * head_dim must be 64; pointers 16-byte aligned. */
int lci_attn_fwd(const void* qkv, void* out, float* lse2, float* knorm_ws, int B, int L, int H, int head_dim,
                 float scale, void* stream);
long long lci_attn_fwd_ws_bytes(int B, int L, int H);
/* dqkv (B, L, 3*H*64) bf16 <- dQ, dK, dV in the packed layout; dout (B, L, H*64) bf16;
 * delta_ws: 16-byte aligned workspace of lci_attn_bwd_ws_bytes(B, H, L) bytes, written by the call: the (B, H, 2, L)
 * f32 rows -lse2 | -delta (the backward kernels' row constants). No atomics: bitwise reproducible. */
int lci_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, void* dqkv,
                 float* delta_ws, int B, int L, int H, int head_dim, float scale, void* stream);
long long lci_attn_bwd_ws_bytes(int B, int H, int L);
/* Same as lci_attn_bwd, one launch at a time (stage 0 = delta, 1 = dK/dV, 2 = dQ; -1 = all)
 * for timing. */
int lci_attn_bwd_stage(int stage, const void* qkv, const void* out, const void* dout, const float* lse2,
                       void* dqkv, float* delta_ws, int B, int L, int H, int head_dim, float scale, void* stream);

/* ViT attention in exact f32 products (csrc/attention_gen.hip): the reference's fp32 (non-AMP) SABlock path
 * (backbone_vit.py:191-201: fp32 einsums + softmax) and head dims 65..256 (the `custom` preset,
 * backbone_vit.py:78-86) in either dtype. dtype 0 = f32, 1 = bf16 (I/O; f32 arithmetic on v_mfma_f32_16x16x4_f32).
 * qkv (B, L, 3*H*D), out (B, L, H*D), dqkv like qkv, dout like out, all in the I/O dtype; D = head_dim <= 256,
 * any L. lse: (B, H, L) f32, NATURAL-log row logsumexp of scale q.k. delta_ws: (B, H, L) f32 workspace.
 * Deterministic (no atomics). Replaces the same reference lines as lci_attn_fwd / lci_attn_bwd. */
int lci_attn_gen_fwd(int dtype, const void* qkv, void* out, float* lse, int B, int L, int H, int head_dim,
                     float scale, void* stream);
int lci_attn_gen_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                     float* delta_ws, int B, int L, int H, int head_dim, float scale, void* stream);

/* ------------------------------------------------------------------ Swin window attention (head_dim 32)
 * geo[16] = {mode, nd, S0, S1, S2, ws0, ws1, ws2, sh0, sh1, sh2, B_or_Bw, nW, N, C, H}
 *   mode 1 (grid): qkv (B, S0, S1[, S2], 3C) bf16 channels-last on the UN-padded grid; window ws, shift sh;
 *                  padded voxels take q/k/v = qkv_bias (f32, 3C, may be null = zeros); the -100 region mask
 *                  of compute_mask (backbone_swin.py:591-628) is part of the bias table; out (B, S.., C) bf16
 *                  is the un-shifted, cropped result.
 *   mode 0 (windows): qkv (Bw, N, 3C), optional mask (nW, N, N) f32 (has_mask), out (Bw, N, C).
 * Bias table: lci_window_bias(rpb (H, N, N) f32 = rpb_table[rp_index], mask or null) writes
 *   bias (T, H, Npad, Npad) bf16 = (rpb + mask) * log2(e), -1e30 at padded rows/columns (Npad = ceil(N/32)*32,
 *   T = lci_window_bias_elems(geo, has_mask) / (H Npad^2): window types), and its transpose biasT; either (not
 *   both) may be null; both 8-byte aligned.
 * lse2: (Bw, H, N) f32 (Bw = B * prod(ceil(S/ws)) in grid mode). N <= 768. */
long long lci_window_bias_elems(const int* geo, int has_mask);
int lci_window_bias(const float* rpb, const float* mask, void* bias, void* biasT, const int* geo, void* stream);
/* biasT: the transposed (key-major) table, 16-byte aligned. */
int lci_window_attn_fwd(const void* qkv, const float* qkv_bias, const void* biasT, int has_mask, void* out,
                        float* lse2, const int* geo, float scale, void* stream);
/* dqkv (same layout as qkv) <- dQ/dK/dV; dbias_pad (3C, accumulated) <- dK/dV of padded voxels, with pad_ws an f32
 * workspace of lci_window_pad_ws_elems(geo) elements (per-window partials, summed in a fixed order);
 * dS: optional bf16 workspace of lci_window_dS_elems(geo) elements; drpb (H, N, N) f32 written if dS given.
 * biasT required (16-byte aligned); bias (plain table) only read for windows of N > 384 (two-phase kernel), may be
 * null otherwise. */
int lci_window_attn_bwd(const void* qkv, const float* qkv_bias, const void* bias, const void* biasT, int has_mask,
                        const void* out, const void* dout, const float* lse2, void* dqkv, float* dbias_pad,
                        float* pad_ws, void* dS, float* drpb, const int* geo, float scale, void* stream);
long long lci_window_dS_elems(const int* geo);
long long lci_window_pad_ws_elems(const int* geo);
/* 1 if lci_window_attn_bwd needs the plain `bias` table for geo (the two-phase kernel: windows of more than 12 key
 * blocks of 32 tokens), 0 if biasT alone suffices; -1 for an invalid geo. */
int lci_window_bwd_needs_plain(const int* geo);
/* Index maps of the grid mode (test/inspection entry; same device functions as the kernels), per window w < Bw and
 * window token n < N, int32 (Bw, N): src_row = token row (b, s0, s1[, s2]) flattened that the window token reads
 * and the output scatters to, -1 for a padded voxel (F.pad + roll(-shift) + window_partition, and their inverse);
 * region = compute_mask region id (3 slices per shifted axis) of the token within its window type, rid = the same
 * derived from the padded coordinate; wtype (Bw) = the bias-table type of each window. */
int lci_window_index_map(const int* geo, int* src_row, int* region, int* rid, int* wtype, void* stream);

/* Grid-mode window partition for the Hyena / Mamba mixers inside Swin windows (backbone_swin.py:445-487, 361-365):
 * scatter = 0: win (Bw, N, C) <- grid (B, S0, S1[, S2], C): F.pad (zeros) -> roll(-shift) -> window_partition;
 * scatter = 1: grid <- win for the non-padded tokens: window_reverse -> roll(+shift) -> crop. Rows of C elements of
 * elem_bytes (2 or 4) bytes, C * elem_bytes % 16 == 0, 16-byte aligned; geo as above (mode 1, C in geo[14]). The
 * index map is win_row(), the one the attention kernels and lci_window_index_map use. */
int lci_window_gather(const void* src, void* dst, int elem_bytes, const int* geo, int scatter, void* stream);

/* ------------------------------------------------------------------ decoder-head 3x3(x3) convolution
 * Replaces the kernel-3 stride-1 convs of MONAI-1.3 UnetResBlock (get_conv_layer conv_only, bias=False) in the
 * ViTUNETR / SwinUNETR heads (model/models/enhance_heads.py:30-356).
 * x (B, D, H, W, Cin) bf16 channels-last; w (Cout, KD*9, Cin) bf16 (tap order kd, kh, kw); y (B, D, H, W, Cout)
 * bf16 = sum over taps/channels of x[p + (kd-1, kh-1, kw-1)] w (zero outside the volume), f32 accumulation.
 * KD = 3 (3-D) or 1 (2-D, D = 1). Cout % 32 == 0. The input gradient is the same call on dy with
 * w'[c, t, n] = w[n, c, KD*9-1-t]. */
int lci_conv3_fwd(const void* x, const void* w, void* y, int B, int D, int H, int W, int Cin, int Cout, int KD,
                  void* stream);
/* Split-K form for small volumes (few 512-voxel tiles): part (nsplit, B*D*H*W, Cout) f32 workspace holds the
 * partial sums of contiguous ranges of the (tap group, 32-channel chunk) slabs, summed in split order into y
 * (deterministic). nsplit = lci_conv3_fwd_splits(B*D*H*W, Cin, Cout, KD) (1: use lci_conv3_fwd); Cin % 32 == 0;
 * y and part 16-byte aligned. */
int lci_conv3_fwd_splits(long long V, int Cin, int Cout, int KD);
/* The kernels' weight operands from the f32 parameter w (Cout, Cin, KD*3*3) (nn.Conv layout), one pass:
 * mode 0: (Cout, T, Cin) bf16 for lci_conv3_fwd; mode 1: (Cin_pad, T, Cout) bf16 = w[n][c][T-1-t] (the flipped,
 * transposed weight of the data gradient), rows c >= Cin zero. */
int lci_conv3_pack_weight(const float* w, void* out, int Cout, int Cin, int KD, int mode, int Cin_pad, void* stream);
/* Transposed conv with kernel == stride (the UNETR heads' up-sampling, MONAI get_conv_layer(is_transposed=True),
 * enhance_heads.py:30-356) runs as one GEMM Y (B*D*H*W, taps*C) bf16 (columns tap-major, tap = (a*kh + b)*kw + c);
 * this moves Y to the channels-last output (B, D*kd, H*kh, W*kw, ld) (rows of ld >= C channels, the C written at the
 * row start: ld = 2C writes the first half of a channel concatenation) and, adjoint = 1, gathers the output-grid
 * rows back to Y's layout. C, ld multiples of 8; 16-byte aligned pointers. */
int lci_convup_interleave(const void* src, void* dst, int B, int D, int H, int W, int kd, int kh, int kw, int C, int ld,
                          int adjoint, void* stream);
int lci_conv3_fwd_split(const void* x, const void* w, void* y, float* part, int nsplit, int B, int D, int H, int W,
                        int Cin, int Cout, int KD, void* stream);
/* Weight gradient: part (lci_conv3_wgrad_splits(B*D*H*W, Cin, Cout, KD), KD*9, Cout, Cin) f32 <- per-voxel-split
 * partial sums of dy[p, n] * x[p + off(tap), c]; dW[n, c, tap] = sum over the first axis (caller). x (.., Cin),
 * dy (.., Cout) bf16 channels-last; Cin, Cout multiples of 32. Deterministic (no atomics). */
long long lci_conv3_wgrad_splits(long long V, int Cin, int Cout, int KD);
int lci_conv3_wgrad(const void* x, const void* dy, float* part, int B, int D, int H, int W, int Cin, int Cout,
                    int KD, void* stream);

/* ------------------------------------------------------------------ decoder-head instance norm (+ LeakyReLU)
 * Replaces MONAI-1.3 UnetResBlock norm1+lrelu / norm2 / norm3 (InstanceNorm, affine=False, eps 1e-5) in the UNETR
 * heads (enhance_heads.py:30-356), channels-last. x, dz, out: (B, V, C) bf16, C % 8 == 0, C <= 2048.
 * reduce: part (B, 2, C, lci_inorm_chunks(V, B)) f32 <- per-chunk sums of (x, x^2) when dz is null, else of
 *   (dn, dn*n) with n = (x - mean) * rstd, dn = dz * (act && n < 0 ? slope : 1); stats (B, 2, C) = mean, rstd.
 * apply: dz null -> out = act ? lrelu(n) : n;  else out = dx = rstd * (dn - coef0 - n * coef1), coef (B, 2, C)
 *   = voxel means of (dn, dn*n).
 * finalize: the partial sums (in f64, fixed order) -> out (B, 2, C): mode 0 the stats (mean, rstd with eps), mode 1
 *   the coefficients (the voxel means of both sums). */
int lci_inorm_chunks(long long V, int B);
int lci_inorm_reduce(const void* x, const void* dz, const float* stats, float* part, long long V, int B, int C,
                     int act, float slope, void* stream);
int lci_inorm_finalize(const float* part, float* out, long long V, int B, int C, int mode, float eps, void* stream);
/* Training BatchNorm + ReLU (UperNet PSPModule.bottleneck / FPN_fuse.conv_fusion, seg_heads.py:26-31, :60-63,
 * :158-163, :192-195) over x (V, C) bf16 channels-last = every voxel of the batch; stats (2, C) = (mean, rstd) from
 * lci_inorm_reduce / lci_inorm_finalize with B = 1. Forward y (V, C) f32 = relu((x - mean) rstd w + b). Backward:
 * part (2, C, lci_inorm_chunks(V, 1)) sums of g = dy [y > 0] and g xhat (dy f32 when dy_f32, else bf16), then
 * lci_inorm_finalize mode 1 -> coef (2, C) means, then dx (V, C) bf16 = (g - coef0 - xhat coef1) rstd w.
 * C % 8 == 0, C <= 2048, 16-byte aligned. */
int lci_bn_relu_fwd(const void* x, const float* stats, const float* w, const float* b, float* y, long long V, int C,
                    void* stream);
int lci_bn_relu_bwd_reduce(const void* x, const void* dy, int dy_f32, const float* stats, const float* w,
                           const float* b, float* part, long long V, int C, void* stream);
int lci_bn_relu_bwd_apply(const void* x, const void* dy, int dy_f32, const float* stats, const float* coef,
                          const float* w, const float* b, void* dx, long long V, int C, void* stream);
int lci_inorm_apply(const void* x, const void* dz, const float* stats, const float* coef, void* out, long long V,
                    int B, int C, int act, float slope, void* stream);
/* UnetResBlock's tail, lrelu(norm2(x) + r), in one pass with the unfused bf16 roundings: out (B, V, C) bf16 =
 * bf16(lrelu(bf16(bf16(n) + r))), n = (x - mean) * rstd from stats; r = bf16(norm(y; stats_y)) (the norm3 residual)
 * when stats_y is given, else y (a bf16 block input). */
int lci_inorm_apply_res(const void* x, const float* stats, const void* y, const float* stats_y, void* out,
                        long long V, int B, int C, float slope, void* stream);

/* ------------------------------------------------------------------ Mamba selective scan (d_state 8)
 * Channels-last: u, delta (B, L, Dx); Bm, Cm (B, L, 8) (e.g. column slices of x_proj's output); y (B, L, .).
 * strides[16] (elements) = {bu,tu, bd,td, bB,tB, bC,tC, by,ty, bdy,tdy, bdu,tdu, bdd,tdd} (batch, token).
 * A (Dx, 8), D (Dx), delta_bias (Dx) f32 (D, delta_bias may be null). delta' = softplus(delta + delta_bias)
 * when delta_softplus, else delta + delta_bias.
 * chunk: multiple of 8. Workspaces f32: xend, xinit (B*nch*Dx*8), sdt (B*nch*Dx), nch = ceil(L/chunk);
 * ckpt (B*ceil(L/8)*Dx*8) elements of the I/O dtype (bf16 I/O: bf16 states) or null (needed by the backward).
 * With one chunk (L <= chunk, e.g. Swin-window sequences) xend / xinit / sdt may all be null: only the output pass
 * runs (nothing is carried into the chunk) and the final state is not produced. */
int lci_selective_scan_fwd(int dtype, const void* u, const void* delta, const float* A, const void* Bm,
                           const void* Cm, const float* D, const float* delta_bias, void* y,
                           const long long* strides, int B, int L, int Dx, int N, int chunk, int delta_softplus,
                           float* xend, float* xinit, float* sdt, void* ckpt, void* stream);
/* du, ddelta (B, L, Dx) written; dBC (B, L, 16) f32 = [dB | dC], dA (Dx, 8), dD, ddelta_bias accumulated (dBC stored
 * instead, needing no zero fill, where lci_selective_scan_bwd_plain_dbc(L, Dx, chunk) returns 1).
 * sdt / ckpt from the forward with the same chunk (sdt null after a one-chunk forward without end states: the
 * adjoint aggregate and reverse carry are skipped); gl, gin: (B*nch*Dx*8) f32 workspaces. */
int lci_selective_scan_bwd(int dtype, const void* u, const void* delta, const float* A, const void* Bm,
                           const void* Cm, const float* D, const float* delta_bias, const void* dy, void* du,
                           void* ddelta, float* dBC, float* dA, float* dD, float* ddelta_bias,
                           const long long* strides, int B, int L, int Dx, int N, int chunk, int delta_softplus,
                           const float* sdt, const void* ckpt, float* gl, float* gin, void* stream);
int lci_selective_scan_bwd_plain_dbc(int L, int Dx, int chunk);

/* SiLU(depthwise conv1d(k = 3, 'same')) of both channel halves of in (B, L, 2C) (token stride in_ts):
 * ox (B, L, C) (token stride ox_ts) and oz at column offset zoff of a (B, L, oz_ts) buffer. */
int lci_dwconv_silu_fwd(int dtype, const void* in, const float* wx, const float* bx, const float* wz,
                        const float* bz, void* ox, void* oz, int B, int L, int C, int K, int in_ts, int ox_ts,
                        int oz_ts, int zoff, void* stream);
/* din (B, L, 2C) written. gx / gz: grads of ox / oz (same layouts). part (lci_dwconv_silu_bwd_part_rows(B, L), 2C, 4)
 * f32 written with per-(sequence, 256-token run) sums of (dw0, dw1, dw2, db) per channel (x half first); the caller
 * sums the first axis (deterministic; ABI 12 replaced the accumulated dwx/dbx/dwz/dbz float atomics). */
long long lci_dwconv_silu_bwd_part_rows(int B, int L);
int lci_dwconv_silu_bwd(int dtype, const void* in, const float* wx, const float* bx, const float* wz,
                        const float* bz, const void* gx, const void* gz, void* din, float* part, int B, int L, int C,
                        int K, int in_ts, int ox_ts, int oz_ts, int zoff, void* stream);

/* MambaVisionMixer x_proj -> split -> dt_proj (mamba.py:120-124) fused, bf16 autocast numerics. Per token:
 * x_dbl = bf16(xs Wx^T) (R + 2N columns), dt = bf16(x_dbl[:R] Wdt^T + bias), bc = x_dbl[R:] (B | C), dtl = x_dbl[:R].
 * Weight images (bf16, built by the caller; dims = lci_mamba_proj_dims -> {Dxp, nb1, ks2, nb3, ks4}):
 *   w1 (nb1*32, Dx) = Wx zero-padded; w2p (Dxp, ks2*16): w2p[d][16 s + 8 h + j] = Wdt[d][32 (s >> 1) + 16 (s & 1)
 *   + (j & 3) + 8 (j >> 2) + 4 h] (zero past R / Dx); w2t (nb3*32, Dx) = Wdt^T zero-padded; w1t (Dxp, ks4*16):
 *   w1t[d][r] = Wx[r][d] (zero past R + 2N / Dx). bias (Dx) f32.
 * fwd: xs (M, Dx) bf16 (token stride ts_x) -> dt (M, Dx) (stride ts_dt), bc (M, 2N) contiguous, dtl (M, ld_dtl).
 * bwd: ddt (M, Dx), dbc (M, 2N) bf16 -> dxs = bf16(d x_dbl Wx) (+ du when not null), dxdbl (M, ld_dxdbl) = d x_dbl
 *   with d x_dbl = [bf16(ddt Wdt) | dbc]; the weight gradients are lci_linear_wgrad calls on (dxdbl, xs) and
 *   (ddt, dtl). Dx % 16 == 0, 2N % 8 == 0, R + 2N <= 64; 16-byte aligned rows (dt / dxs / du 8). */
int lci_mamba_proj_dims(int Dx, int R, int N2, int* dims);
int lci_mamba_proj_fwd(const void* xs, long long ts_x, const void* w1, const void* w2p, const float* bias, void* dt,
                       long long ts_dt, void* bc, void* dtl, int ld_dtl, long long M, int Dx, int R, int N2,
                       void* stream);
int lci_mamba_proj_bwd(const void* ddt, long long ts_ddt, const void* dbc, const void* w2t, const void* w1t,
                       const void* du, long long ts_du, void* dxs, long long ts_dxs, void* dxdbl, int ld_dxdbl,
                       long long M, int Dx, int R, int N2, void* stream);

/* ------------------------------------------------------------------ Hyena long convolution (f32)
 * FFT size n = lci_fft_size(L) = pow2 >= 2L (L <= 262144). tw: n complex f32 (f32x2) from lci_fft_twiddles.
 * Rows are channel-major f32 (R, C, L); the filter of row r is r % C; k (C, L). */
long long lci_fft_size(int L);
int lci_fft_twiddles(void* tw, int n, void* stream);
/* K (C, n) complex f32 = filter spectra (scaled by 1/n); SK (C, n) complex scratch. Dv (C) or null: folded into the
 * spectra (K += D / n, the spectrum of D delta), so the convolution with K carries the + D u term (ABI 23). */
int lci_fftconv_spectrum(const float* k, const float* Dv, void* K, void* SK, const void* tw, int C, int L,
                         void* stream);
/* y = causal_conv(u, k) + D u; S: (C*ceil(R/2), n) complex scratch. Su (optional, same shape): receives the
 * column spectra of u, left intact for lci_fftconv_bwd (ABI 11). Dv (C) or null: D u added in the time domain (null
 * when K already carries D, lci_fftconv_spectrum with Dv). */
int lci_fftconv_fwd(const float* u, const void* K, const float* Dv, float* y, void* S, void* Su, const void* tw,
                    int R, int C, int L, void* stream);
/* du = corr(dy, k) + D dy (written; Dv (C) or null as in lci_fftconv_fwd); dk (C, L) = sum_rows corr(dy, u)
 * (written, optional); dD accumulated (optional): dk[:, 0] (the lag-0 correlation sum_rows sum_t dy u) when dk is
 * computed, else a row dot product. S, S2: (C*ceil(R/2), n) complex scratch (S2 only with dk and no Su); Su: the forward's kept
 * column spectra of u (optional: skips their recomputation); SK: (C, n) complex scratch. */
int lci_fftconv_bwd(const float* dy, const float* u, const void* K, const float* Dv, float* du, float* dk,
                    float* dD, void* S, void* S2, const void* Su, void* SK, const void* tw, int R, int C, int L,
                    void* stream);
/* Direct causal long convolution for short rows (L <= lci_direct_conv_max_len(): the Swin-window sequences of
 * backbone_swin.py:361-362), exact f32 products on the f32 MFMA instead of an FFT. u, y (R, C, L) f32 channel-major
 * rows (filter of row r*C + c is c), k (C, L), D (C) f32 or null.
 * fwd: adjoint = 0: y = causal_conv(u, k) + D u;  adjoint = 1: y = corr(u, k) + D u, i.e. du from dy (written).
 * dk: part (lci_direct_conv_dk_splits(R, C, L), C, ceil(L / 32), 64) f32 <- per-row-split diagonal-band sums of
 *     G = dy^T u (band d, slot e + 31: sum over rows and t - s = 32 d + e of dy[r][t] u[r][s], e in [-31, 31])
 *     (written); dk[32 d + e] = sum over splits of band[d][e + 31] + band[d + 1][e - 1] for e in [0, 32),
 *     dD[c] = dk[c][0] (caller). Deterministic. */
int lci_direct_conv_max_len(void);
int lci_direct_conv_fwd(const float* u, const float* k, const float* D, float* y, int R, int C, int L, int adjoint,
                        void* stream);
int lci_direct_conv_dk_splits(int R, int C, int L);
int lci_direct_conv_dk(const float* dy, const float* u, float* part, int R, int C, int L, void* stream);
/* z (BB, L, 3D) channels-last in_proj output; causal depthwise conv (w (3D, K), bias (3D)); per head h,
 * x1/x2/v = conv channels [h*3hd, +hd), [+hd, +2hd), [+2hd, +3hd). vg = v*x1 -> (BB, D, L) f32 rows;
 * x2 -> (BB, L, D) channels-last (z dtype). */
int lci_hyena_pre_fwd(int dtype, const void* z, const float* w, const float* bias, float* vg, void* x2, int BB,
                      int L, int H, int hd, int K, void* stream);
/* out (BB, L, D) = y (BB, D, L) f32 * x2, channels-last. */
int lci_hyena_post_fwd(int dtype, const float* y, const void* x2, void* out, int BB, int L, int D, void* stream);
/* dy (BB, D, L) f32 = dout * x2; dx2 (BB, L, D) = dout * y in the activation dtype (x2's). */
int lci_hyena_post_bwd(int dtype, const float* y, const void* x2, const void* dout, float* dy, void* dx2, int BB,
                       int L, int D, void* stream);
/* dz (BB, L, 3D) written; dw (3D, K), db (3D) accumulated. gx2: (BB, L, D) in the activation dtype, i.e. the
 * post backward's dx2 as it is (ABI 26: dx2 / gx2 were f32, so the autograd engine cast dx2 to x2's bf16 and the
 * caller cast it back). */
int lci_hyena_pre_bwd(int dtype, const void* z, const float* w, const float* bias, const float* dvg,
                      const void* gx2, void* dz, float* dw, float* db, int BB, int L, int H, int hd, int K,
                      void* stream);

/* ------------------------------------------------------------------ Hyena implicit filter (order = D = 64)
 * prep: the f32 parameters W1 (64, E), b1, freq (64), W2, b2, W3, b3 (64x64, 64), W4 (64, 64), deltas (64) ->
 * img (lci_hyena_filter_img_elems() bf16, 16-B aligned: MFMA weight fragments) and vec (320 f32).
 * fwd: z (L, E) f32 rows, t (L) f32 -> k (64, L) f32 = modulated filter, bf16-autocast rounding.
 * bwd: dk (64, L) f32 -> dh, s3, da3, s2, da2, s1 (L, 64) bf16 with permuted feature columns (feature of column c:
 * 32(c>>4>>1) + 16((c>>4)&1) + 8((c&7)>>2) + 4((c>>3)&1) + (c&3)) for the three 64x64 weight gradients,
 * dz (L, E) f32 (written), part (lci_hyena_filter_partials(L, E) f32: per-wave [2 + E][64] sums of
 * db1, dfreq, dW1[:, e] over positions, indexed by feature; the caller sums them). 1 <= E <= 8. */
/* ------------------------------------------------------------------ bilinear 2x up-sampling (align_corners=False)
 * fwd: x (B, C, H, W) f32 -> y (B, 2H, 2W, C) bf16 channels-last (16-B aligned); bwd: dy (B, 2H, 2W, C) bf16
 * channels-last -> dx (B, C, H, W) f32 (written). C % 8 == 0. */
int lci_upsample2x_fwd(const float* x, void* y, int B, int C, int H, int W, void* stream);
int lci_upsample2x_bwd(const void* dy, float* dx, int B, int C, int H, int W, void* stream);
/* the same for a channels-last input map: x (B, H, W, C) f32 -> y (B, 2H, 2W, C) bf16; dy -> dx (B, H, W, C) f32 */
int lci_upsample2x_nhwc_fwd(const float* x, void* y, int B, int C, int H, int W, void* stream);
int lci_upsample2x_nhwc_bwd(const void* dy, float* dx, int B, int C, int H, int W, void* stream);
/* ------------------------------------------------------------------ trilinear up-sampling (align_corners=False)
 * UperNet3D.forward's final F.interpolate(x, size=input_size, mode="trilinear") (seg_heads.py:273) into the head
 * conv's channels-last bf16 operand: x (B, D, H, W, C) f32 channels-last -> y (B, OD, OH, OW, C) bf16, any output
 * size (scale in/out per axis, torch's arithmetic). Its adjoint, one axis at a time: lci_resample1d_adj maps
 * dy (outer, n_out, inner) (bf16 if dy_bf16, else f32) to dx (outer, n_in, inner) f32 (written), deterministic.
 * C % 8 == 0, inner % 8 == 0, 16-byte aligned. */
int lci_upsample3d_cl_fwd(const float* x, void* y, int B, int C, int D, int H, int W, int OD, int OH, int OW,
                          void* stream);
int lci_resample1d_adj(const void* dy, int dy_bf16, float* dx, long long outer, int n_out, int n_in, long long inner,
                       void* stream);
/* ------------------------------------------------ linear re-sampling to any size, align_corners either way (ABI 28)
 * FPN_fuse's resize (seg_heads.py:49-50, :74 / :181-182, :206, F.interpolate(x, size, mode=(bi|tri)linear, align_corners=True))
 * and PSPModule's up-sampling of the pooled bins (seg_heads.py:44 / :176): x (B, D, H, W, C) channels-last (f32, or
 * bf16 when x_bf16) -> y (B, OD, OH, OW, C) f32 [+ add of y's shape (f32, or bf16 when add_bf16), summed in the same
 * pass]; bilinear when D = OD = 1. torch's scale and source-index arithmetic (area_pixel_compute_scale /
 * _source_index). lci_resample1d_adj_ac is the one-axis adjoint with the same align_corners choice (deterministic
 * gathers in place of torch's atomic upsample backward). C % 8 == 0, inner % 8 == 0, 16-byte aligned. */
int lci_resample_cl_fwd(const void* x, int x_bf16, const void* add, int add_bf16, float* y, int B, int C, int D, int H,
                        int W, int OD, int OH, int OW, int align_corners, void* stream);
int lci_resample1d_adj_ac(const void* dy, int dy_bf16, float* dx, long long outer, int n_out, int n_in,
                          long long inner, int align_corners, void* stream);

long long lci_hyena_filter_img_elems(void);
long long lci_hyena_filter_partials(int L, int E);
int lci_hyena_filter_prep(const float* W1, const float* b1, const float* freq, const float* W2, const float* b2,
                          const float* W3, const float* b3, const float* W4, const float* deltas, int E, void* img,
                          float* vec, void* stream);
int lci_hyena_filter_fwd(const float* z, const float* t, const void* img, const float* vec, int E, int L, float shift,
                         float* k, void* stream);
int lci_hyena_filter_bwd(const float* z, const float* t, const void* img, const float* vec, int E, int L, float shift,
                         const float* dk, void* dh, void* s3, void* da3, void* s2, void* da2, void* s1, float* dz,
                         float* part, void* stream);

/* ------------------------------------------------------------------ patch embedding (conv, k = stride = p)
 * x (B, C, S0, S1[, S2]) (dtype x_dtype), w (D, C*prod(p)) f32, bias (D) / pos (L, D) f32 or null;
 * channels_last = 1: y (B, L, D) (ViT, + pos); 0: y (B, D, G0, G1[, G2]) (Swin; right zero-pad to p). */
int lci_patch_embed_fwd(const void* x, int x_dtype, const float* w, const float* bias, const float* pos, void* y,
                        int y_dtype, int B, int C, int D, int nd, const int* img_size, const int* patch,
                        int channels_last, void* stream);
/* dw (D*K), db (D) accumulated; dpos (L, D) written (channels_last only). */
int lci_patch_embed_bwd(const void* x, int x_dtype, const void* dy, int dy_dtype, float* dw, float* db, float* dpos,
                        int B, int C, int D, int nd, const int* img_size, const int* patch, int channels_last,
                        void* stream);

/* ------------------------------------------------------------------ transformer-block LayerNorm
 * x (rows, C) f32 residual stream, C % 4 == 0, C <= 2048; gamma, beta (C) f32; eps as nn.LayerNorm's.
 * Pointers 16-byte aligned (8 for bf16 y / dy).
 * fwd: y (rows, C) = bf16 when bf16_out (the value autocast would hand the next Linear) else f32;
 *      mean, rstd (rows) f32 (biased variance, as torch).
 * bwd: dy (rows, C) bf16 when bf16_dy else f32; dx (rows, C) f32 written (+ dres (rows, C) f32, the residual
 *      path's gradient, when not null); part (lci_layernorm_bwd_blocks(rows),
 *      2, C) f32 written with per-workgroup partial sums of (dy * n, dy), n = (x - mean) * rstd: the caller sums
 *      them over the first axis for dgamma, dbeta. */
int lci_layernorm_bwd_blocks(long long rows);
int lci_layernorm_fwd(const float* x, const float* gamma, const float* beta, void* y, int bf16_out, float* mean,
                      float* rstd, long long rows, int C, float eps, void* stream);
/* xsum = h + add (f32; add bf16 if add_bf16 else f32), y = LayerNorm(xsum) as lci_layernorm_fwd (mean / rstd of xsum):
 * the block's mid residual add fused into norm2; the backward is lci_layernorm_bwd on xsum. */
int lci_layernorm_add_fwd(const float* h, const void* add, int add_bf16, float* xsum, const float* gamma,
                          const float* beta, void* y, int bf16_out, float* mean, float* rstd, long long rows, int C,
                          float eps, void* stream);
/* dxb (rows, C) bf16 or null: dx rounded to bf16 in the same pass, the gradient of a bf16 branch output added by
 * lci_layernorm_add_fwd (ABI 27). dres2 (rows, C) f32 or null (needs dres): a second residual gradient, summed with
 * dres first -- a recorded hidden state's decoder gradient, which autograd would otherwise add in a separate pass
 * (ABI 31). */
int lci_layernorm_bwd(const float* x, const void* dy, int bf16_dy, const float* gamma, const float* mean,
                      const float* rstd, const float* dres, const float* dres2, float* dx, void* dxb, float* part,
                      long long rows, int C, void* stream);

/* ------------------------------------------------------------------ token-wise Linear: weight / bias gradient
 * dy (M, ldy) bf16 row-major (columns [0, N) used), x (M, ldx) bf16 row-major (columns [0, K) used): the layer's
 * output gradient and (autocast) input. part (ns, N, K) f32 <- per-token-split partial sums of dy^T x and, when
 * dbpart is not null, dbpart (ns, N) f32 <- partial column sums of dy; ns = lci_linear_wgrad_splits(M, N, K)
 * (0: shape not supported). dW / db = sums over the first axis (caller). N, K, ldy, ldx multiples of 8, pointers
 * 16-byte aligned. Deterministic (no atomics). */
long long lci_linear_wgrad_splits(long long M, int N, int K);
int lci_linear_wgrad(const void* dy, long long ldy, const void* x, long long ldx, long long M, int N, int K,
                     float* part, float* dbpart, void* stream);
/* Narrow outputs (the UNETR heads' 1x1 conv to 1-8 channels, over channels-last voxel rows): y (M, N) bf16 =
 * x (M, ldx) . w^T + bias, w (N, K) bf16, bias (N) bf16 or null; N <= 8, K <= 256, K % 8 == 0.
 * bwd (N <= 4): dx (M, K) bf16 = dy . w (optional); part ((N K + N), lci_linear_small_threads()) f32 <- per-thread
 * partial sums of dy^T x (row-major N x K) and of dy; dW, db = sums over the last axis (caller). */
int lci_linear_small_threads(void);
int lci_linear_small_fwd(const void* x, long long ldx, const void* w, const void* bias, void* y, long long M, int N,
                         int K, void* stream);
int lci_linear_small_bwd(const void* x, long long ldx, const void* w, const void* dy, void* dx, float* part,
                         long long M, int N, int K, void* stream);
/* GELU (erf) of n bf16 elements (n % 8 == 0, 16-B aligned): y = gelu(x); dx = dy * gelu'(x). */
int lci_gelu_fwd(const void* x, void* y, long long n, void* stream);
int lci_gelu_bwd(const void* x, const void* dy, void* dx, long long n, void* stream);
/* Projection GEMM (csrc/gemm.hip): y (M, ldy) bf16 = x (M, ldx) . w^T + bias, w (N, K) bf16 contiguous, bias (N) bf16
 * or null; f32 accumulation, bias added in f32 and the sum rounded once (the autocast nn.Linear's arithmetic). The
 * forward and data-gradient GEMMs of the token-wise Linear layers: SABlock qkv / out_proj (backbone_vit.py:166-167),
 * MLPBlock (:249), Hyena in/out_proj (hyena.py:278-279), Mamba in/out_proj (mamba.py:60-64,90); the data gradient
 * is the call with the transposed weight. Supported when lci_gemm_bt_supported(N, K): N % 384 == 0 or N % 256 == 0, N <= 4096,
 * K % 32 == 0; ldx, ldy % 8 == 0; x / w / y 16-byte aligned; any M (per-tile 32-bit offsets). */
int lci_gemm_bt_supported(int N, int K);
/* y = bf16(y + bf16(x . w^T)) (no bias): the product added into an existing bf16 matrix in the epilogue -- UnetResBlock's
 * 1x1 residual data gradient summed into conv1's (the autograd sum, same roundings). Same support as lci_gemm_bt. */
int lci_gemm_bt_acc(const void* x, long long ldx, const void* w, void* y, long long ldy, long long M, int N, int K,
                    void* stream);
int lci_gemm_bt(const void* x, long long ldx, const void* w, const void* bias, void* y, long long ldy, long long M,
                int N, int K, void* stream);
/* The same product for the shapes lci_gemm_bt's 256 x 384 persistent tiles do not fill (round 6): the Swin stage-3 / 4
 * projections and data gradients (backbone_swin.py:339-359 qkv / proj, Mlp fc1 / fc2 at 4096 / 512 tokens) and the
 * decoder heads' 1x1 convolutions (N = 96 / 192 / 288 at up to 2^21 voxels: MONAI UnetResBlock conv3 / UnetOutBlock,
 * enhance_heads.py:30-356), which ran on hipBLASLt. Same arithmetic and argument meaning as lci_gemm_bt; supported
 * when lci_gemm_bt_small_supported(N, K): N % 32 == 0, K % 16 == 0; ldx, ldy % 8 == 0; x / w / y 16-byte aligned,
 * bias 8-byte; any M. */
int lci_gemm_bt_small_supported(int N, int K);
int lci_gemm_bt_small(const void* x, long long ldx, const void* w, const void* bias, void* y, long long ldy,
                      long long M, int N, int K, void* stream);
/* y = bf16(y + bf16(x . w^T)), lci_gemm_bt_acc's arithmetic with lci_gemm_bt_small's support (UnetResBlock's 1x1
 * residual data gradient at 96 / 192 / 288 channels). */
int lci_gemm_bt_small_acc(const void* x, long long ldx, const void* w, void* y, long long ldy, long long M, int N,
                          int K, void* stream);

/* ------------------------------------------------------------------ optimizer step (csrc/optim.hip)
 * Adam / AdamW update of nt <= lci_adam_max_tensors() f32 tensors in one launch (trainer_base.py:171-177 ->
 * torch.optim.Adam / AdamW, optim_base.py:87-89): p[i], g[i], m[i] (exp_avg), v[i]
 * (exp_avg_sq) of n[i] elements each; step[i] -> the tensor's device step count, already incremented for this update
 * (bias corrections 1 - beta^step evaluated on the device, so the call can sit in a captured graph). adamw = 1:
 * decoupled weight decay, 0: L2 (added to the gradient); maximize negates the gradient. The arithmetic is torch's
 * fused Adam's (f64 moment updates, f32 step size / denominator / update). The pointer arrays are host memory. */
int lci_adam_max_tensors(void);
int lci_adam_step(float* const* p, const float* const* g, float* const* m, float* const* v, const float* const* step,
                  const long long* n, int nt, double lr, double beta1, double beta2, double weight_decay, double eps,
                  int adamw, int maximize, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LCI_H_ */
