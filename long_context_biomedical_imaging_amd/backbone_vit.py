"""ViT backbone with attention / Hyena / Mamba token mixers — drop-in for
/root/reference/model/models/backbone_vit.py.

Same public names, constructor signatures, forward shapes, parameter-creation order and state_dict
keys as the reference (custom_ViT :45-116, SABlock :120-211, TransformerBlock :213-263,
ViT_with_alt_ops :265-397). The attention core runs the liblci flash-attention HIP kernels
(kernels.flash_attention); the L x L matrix is never formed, so `save_attn=True` recomputes the
attention matrix on demand instead of storing it every forward (see SABlock.attention_matrix).
"""
from __future__ import annotations

from collections.abc import Sequence

import torch
import torch.nn as nn
import torch.utils.checkpoint

from . import kernels
from .blocks import MLPBlock, OutLayerNorm, PatchEmbeddingBlock, TokenLayerNorm, TokenLinear
from .hyena import HyenaOperator
from .mamba import MambaVisionMixer


def custom_ViT(config, input_feature_channels):
    """Returns (ViT_with_alt_ops, [hidden_size]*13), sizes as backbone_vit.py:56-89."""
    v = config.ViT
    if v.size == "small":
        hidden_size, mlp_dim, num_layers, num_heads = 384, 1536, 12, 6
    elif v.size == "base":
        hidden_size, mlp_dim, num_layers, num_heads = 768, 3072, 12, 12
    elif v.size == "custom":
        hidden_size, mlp_dim, num_layers, num_heads = v.hidden_size, v.mlp_dim, v.num_layers, v.num_heads
    else:
        raise ValueError(f"Unknown model size {v.size} specified in config.")
    v.hidden_size, v.mlp_dim, v.num_layers, v.num_heads = hidden_size, mlp_dim, num_layers, num_heads

    if config.time == 1:
        spatial_dims = 2
        input_size = [config.height, config.width]
        mod_patch_size = v.patch_size[1:] if len(v.patch_size) == 3 else v.patch_size
    else:
        spatial_dims = 3
        input_size = [config.time, config.height, config.width]
        mod_patch_size = v.patch_size

    model = ViT_with_alt_ops(use_hyena=v.use_hyena, use_mamba=v.use_mamba, in_channels=input_feature_channels,
                             img_size=input_size, patch_size=mod_patch_size, hidden_size=hidden_size,
                             mlp_dim=mlp_dim, num_layers=num_layers, num_heads=num_heads, dropout_rate=0.0,
                             spatial_dims=spatial_dims, classification=config.task_type == "class",
                             hyena_l_max=getattr(v, "hyena_l_max", HYENA_L_MAX))
    return model, [hidden_size] * 13


# The reference hard-codes HyenaOperator(l_max=66000) (backbone_vit.py:172), so any sequence longer than 66000
# tokens raises (hyena.py:314) -- among them BASELINE configs[3] (1024^2 patch 2, L = 262144). `hyena_l_max`
# (config --ViT.hyena_l_max, default 66000 = the reference) is an opt-in deviation that sizes the implicit
# filter (and its positional-embedding Parameter, (1, l_max, 3)) for longer sequences.
HYENA_L_MAX = 66000




class SABlock(nn.Module):
    """Token mixer: full self-attention (flash, HIP), or HyenaOperator, or MambaVisionMixer."""

    def __init__(self, use_hyena: bool, use_mamba: bool, hidden_size: int, num_heads: int,
                 dropout_rate: float = 0.0, qkv_bias: bool = False, save_attn: bool = False, *,
                 hyena_l_max: int = HYENA_L_MAX) -> None:
        super().__init__()
        if not (0 <= dropout_rate <= 1):
            raise ValueError("dropout_rate should be between 0 and 1.")
        if hidden_size % num_heads != 0:
            raise ValueError("hidden size should be divisible by num_heads.")
        self.num_heads = num_heads
        self.use_hyena = use_hyena
        self.use_mamba = use_mamba
        if not use_hyena and not use_mamba:
            self.drop_output = nn.Dropout(dropout_rate)
            self.drop_weights = nn.Dropout(dropout_rate)
            self.head_dim = hidden_size // num_heads
            if self.head_dim > kernels.ATTN_GEN_MAX_HEAD_DIM:
                # head_dim <= 64 (every reference preset: small 384/6, base 768/12) runs on the placed bf16 kernels
                # (smaller dims zero-padded, exact), 65..256 on csrc/attention_gen.hip; larger `custom` splits
                # (backbone_vit.py:78-86) fail here, not mid-step
                raise ValueError(f"attention head_dim {self.head_dim} (hidden_size {hidden_size} / num_heads "
                                 f"{num_heads}) is not supported: the HIP attention kernels take head_dim "
                                 f"<= {kernels.ATTN_GEN_MAX_HEAD_DIM} (DESIGN.md §7)")
            self.scale = self.head_dim ** -0.5
            self.save_attn = save_attn
            self.att_mat = torch.Tensor()
            self.qkv = TokenLinear(hidden_size, hidden_size * 3, bias=qkv_bias)
            self.out_proj = TokenLinear(hidden_size, hidden_size)
        elif use_hyena and not use_mamba:
            self.hyena = HyenaOperator(d_model=hidden_size, l_max=hyena_l_max, filter_order=64, num_heads=num_heads,
                                       num_blocks=1, short_filter_order=5, bidrectional=True,
                                       dropout=dropout_rate, filter_dropout=dropout_rate, activation="id")
        elif not use_hyena and use_mamba:
            self.mamba = MambaVisionMixer(d_model=hidden_size, d_state=8, d_conv=3, expand=1)

    def forward(self, x):
        if not self.use_hyena and not self.use_mamba:
            if self.training and self.drop_weights.p > 0:
                raise NotImplementedError("attention-weight dropout > 0 is not fused into the flash kernel")
            qkv = self.qkv(x)
            o = kernels.flash_attention(qkv, self.num_heads, self.scale)
            if self.save_attn:
                self.att_mat = self.attention_matrix(qkv.detach())
            x = self.drop_output(self.out_proj(o))
        elif self.use_hyena and not self.use_mamba:
            x = self.hyena(x)
        elif not self.use_hyena and self.use_mamba:
            x = self.mamba(x)
        return x

    @torch.no_grad()
    def attention_matrix(self, qkv):
        """softmax(q k^T * scale), (B, H, L, L) — inspection only (save_attn), O(L^2) memory."""
        b, l, _ = qkv.shape
        t = qkv.reshape(b, l, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4).float()
        return (torch.einsum("blxd,blyd->blxy", t[0], t[1]) * self.scale).softmax(dim=-1)


class TransformerBlock(nn.Module):
    def __init__(self, use_hyena: bool, use_mamba: bool, hidden_size: int, mlp_dim: int, num_heads: int,
                 dropout_rate: float = 0.0, qkv_bias: bool = False, save_attn: bool = False, *,
                 hyena_l_max: int = HYENA_L_MAX) -> None:
        super().__init__()
        if not (0 <= dropout_rate <= 1):
            raise ValueError("dropout_rate should be between 0 and 1.")
        if hidden_size % num_heads != 0:
            raise ValueError("hidden_size should be divisible by num_heads.")
        self.mlp = MLPBlock(hidden_size, mlp_dim, dropout_rate)
        self.norm1 = TokenLayerNorm(hidden_size)
        self.use_hyena = use_hyena
        self.use_mamba = use_mamba
        self.attn = SABlock(use_hyena, use_mamba, hidden_size, num_heads, dropout_rate, qkv_bias, save_attn,
                            hyena_l_max=hyena_l_max)
        self.norm2 = TokenLayerNorm(hidden_size)

    def forward(self, x):
        # x + attn(norm1(x)); x + mlp(norm2(x)) (backbone_vit.py:261-262)
        _, h, m = self.forward_pair(x, None)
        return h + m

    def forward_pair(self, h, m, tap=False):
        """The block on the residual stream held as a pair: its input is h + m (m = the previous block's MLP output,
        bf16, or None), summed inside the norm1 LayerNorm kernel instead of by a separate add; returns (h + m, the
        stream after the attention residual, this block's MLP output). The residual gradient of each add is summed
        inside the LayerNorm backward kernels, which also write m's bf16 gradient (no cast passes)."""
        if m is None:
            x, xt, y = self.norm1.forward_residual(h, tap=True)
        else:
            x, xt, y = self.norm1.forward_residual_add(h, m, tap=True)
        h, y = self.norm2.forward_residual_add(x, self.attn(y))   # x + attn(.) summed inside the norm2 kernel
        # tap: the returned block input is a separate alias, so a consumer outside the block (a decoder reading the
        # hidden state) gets its gradient summed inside norm1's backward kernel rather than by an autograd add
        return (xt if tap else x), h, self.mlp(y)


class ViT_with_alt_ops(nn.Module):
    def __init__(self, use_hyena: bool, use_mamba: bool, in_channels: int, img_size: Sequence[int] | int,
                 patch_size: Sequence[int] | int, hidden_size: int = 768, mlp_dim: int = 3072,
                 num_layers: int = 12, num_heads: int = 12, pos_embed: str = "conv", proj_type: str = "conv",
                 pos_embed_type: str = "learnable", classification: bool = False, num_classes: int = 2,
                 dropout_rate: float = 0.0, spatial_dims: int = 3, post_activation="Tanh",
                 qkv_bias: bool = False, save_attn: bool = False, *, hyena_l_max: int = HYENA_L_MAX) -> None:
        super().__init__()
        if not (0 <= dropout_rate <= 1):
            raise ValueError("dropout_rate should be between 0 and 1.")
        if hidden_size % num_heads != 0:
            raise ValueError("hidden_size should be divisible by num_heads.")
        self.classification = classification
        self.spatial_dims = spatial_dims
        if use_hyena or use_mamba:
            pos_embed_type = "none"
        self.patch_embedding = PatchEmbeddingBlock(in_channels=in_channels, img_size=img_size,
                                                   patch_size=patch_size, hidden_size=hidden_size,
                                                   num_heads=num_heads, proj_type=proj_type,
                                                   pos_embed_type=pos_embed_type, dropout_rate=dropout_rate,
                                                   spatial_dims=spatial_dims)
        self.blocks = nn.ModuleList([
            TransformerBlock(use_hyena, use_mamba, hidden_size, mlp_dim, num_heads, dropout_rate, qkv_bias,
                             save_attn, hyena_l_max=hyena_l_max) for _ in range(num_layers)])
        self.norm = OutLayerNorm(hidden_size)
        # Not a reference option: per-block activation checkpointing (recompute each block's forward in the
        # backward) for token counts whose saved activations exceed one GPU (256^3 p2: ~35 GB per block).
        # True = every block; an int k = the first k blocks only (the rest keep their activations: less recompute
        # where the memory allows it).
        self.checkpoint_blocks = False
        if self.classification and not use_hyena and not use_mamba:
            self.cls_token = nn.Parameter(torch.zeros(1, 1, hidden_size))

    def forward(self, x, keep_hidden=None):
        """Returns hidden_states_out as the reference's (backbone_vit.py:379-397): [image, block outputs 1..L,
        LN(last)]. keep_hidden (not a reference argument; EncoderDecoderModel passes its decoder's `hidden_taps`):
        the hidden_states_out indices the caller reads; the other block outputs come back as None. The default
        (None) returns every entry, as the reference does, to any other caller."""
        if self.spatial_dims == 2:
            x = x.squeeze(2)
        hidden_states_out = [x]
        x = self.patch_embedding(x)
        if hasattr(self, "cls_token"):
            cls_token = self.cls_token.expand(x.shape[0], -1, -1)
            x = torch.cat((cls_token, x), dim=1)
        nck = len(self.blocks) if self.checkpoint_blocks is True else int(self.checkpoint_blocks or 0)
        # The residual stream between blocks is the pair (h, m): block i + 1's norm1 kernel forms block i's output
        # h + m, which is also what hidden_states_out records (the same tensor); only the last block's output is a
        # separate add. A checkpointed block saves its inputs, so where its input is also a recorded hidden state
        # the stream is materialised as one tensor there (the add; the checkpoint and the list share it) -- the pair
        # would hold h, m and the sum. keep_hidden (the decoder's taps, from EncoderDecoderModel) leaves the block
        # outputs no decoder reads as None, so untapped checkpoint boundaries keep the pair (+1 bf16 tensor per
        # boundary, 1.6 GB at 2^21 tokens) and skip the add, its recompute and its backward cast.
        def keep(idx):
            return keep_hidden is None or idx in keep_hidden

        train = self.training and torch.is_grad_enabled()
        h, m = x, None
        for i, blk in enumerate(self.blocks):
            tap = i > 0 and keep(i)
            if i < nck and train:
                xin, h, m = torch.utils.checkpoint.checkpoint(blk.forward_pair, h, m, tap, use_reentrant=False)
            else:
                xin, h, m = blk.forward_pair(h, m, tap)
            if i > 0:   # xin = block i - 1's output, hidden_states_out[i]
                hidden_states_out.append(xin if keep(i) else None)
            if i + 1 < min(nck, len(self.blocks)) and train and keep(i + 1):
                h, m = h + m, None   # a recorded input of a checkpointed block: one tensor
        if m is not None:
            x = h + m
        else:               # no blocks (the embedding, not recorded) or a materialised last output
            x = h
        if len(self.blocks):
            hidden_states_out.append(x)
        x = self.norm(x)
        hidden_states_out.append(x)
        return hidden_states_out
