/* liblci — MI355X (gfx950) kernels for the long-context image-token mixers.
 *
 * C-ABI boundary: plain device pointers, sizes and a hipStream_t passed as void*. No torch types.
 * Every entry point enqueues on `stream` and returns 0 on success; on failure it returns non-zero and
 * lci_last_error() describes the problem (bad shape/alignment -> 1, HIP API error -> 2, launch -> 3).
 * Memory is owned by the caller: the library never allocates or frees device memory.
 * bf16 = IEEE bfloat16 stored as uint16. Row-major throughout.
 *
 * Reference interfaces replaced (file:line in NHLBI/long_context_biomedical_imaging):
 *   lci_attn_fwd / lci_attn_bwd
 *       SABlock.forward attention core, model/models/backbone_vit.py:191-203
 *       (einsum QK^T * scale -> softmax -> einsum AV; autograd backward of the same)
 */
#ifndef LCI_H_
#define LCI_H_

#ifdef __cplusplus
extern "C" {
#endif

const char* lci_last_error(void);
int lci_abi_version(void);

/* Flash attention forward.
 *   qkv  : (B, L, 3*H*head_dim) bf16 — the packed qkv Linear output, channel order (qkv, head, d)
 *          (backbone_vit.py:168 Rearrange "b h (qkv l d) -> qkv b l h d").
 *   out  : (B, L, H*head_dim) bf16 — softmax(q k^T * scale) v in "b l (h d)" order (backbone_vit.py:169).
 *   lse2 : (B, H, L) f32 — log2(sum_y exp(scale q.k_y)) per query row, consumed by lci_attn_bwd.
 *   head_dim must be 64; pointers 16-byte aligned. */
int lci_attn_fwd(const void* qkv, void* out, float* lse2, int B, int L, int H, int head_dim, float scale,
                 void* stream);

/* Flash attention backward: dqkv (B, L, 3*H*head_dim) bf16 receives dQ, dK, dV in the packed layout.
 *   dout: (B, L, H*head_dim) bf16; delta_ws: (B, H, L) f32 workspace. */
int lci_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, void* dqkv,
                 float* delta_ws, int B, int L, int H, int head_dim, float scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LCI_H_ */
