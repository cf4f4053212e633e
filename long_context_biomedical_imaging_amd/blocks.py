"""Small building blocks the reference takes from MONAI 1.3 (requirements.txt:5), restated.

State-dict keys, constructor signatures and parameter-creation order match MONAI 1.3 so reference
checkpoints load and seeded initialisation reproduces the reference's weights:
  MLPBlock            backbone_vit.py:249 / backbone_swin.py:433  (linear1 -> GELU(erf) -> linear2)
  PatchEmbeddingBlock backbone_vit.py:351-361  (conv k=s=p -> flatten/transpose -> + position_embeddings)
  PatchEmbed          backbone_swin.py:800-806 (right pad to a patch multiple -> conv k=s=p)
The patch-embedding forward runs the HIP patch-embed kernels (kernels.patch_embed_*); TokenLayerNorm (an
nn.LayerNorm) runs the HIP LayerNorm kernels (kernels.layer_norm); TokenLinear (an nn.Linear) takes its weight / bias
gradient from the HIP split-token GEMM (kernels.linear, lci_linear_wgrad).
"""
from __future__ import annotations

import os
from collections.abc import Sequence

import numpy as np
import torch
import torch.nn as nn

from . import kernels


def ensure_tuple_rep(tup, dim):
    if not isinstance(tup, (list, tuple)):
        return (tup,) * dim
    if len(tup) == dim:
        return tuple(tup)
    raise ValueError(f"Sequence must have length {dim}, got {len(tup)}.")


def trunc_normal_(tensor, mean=0.0, std=1.0, a=-2.0, b=2.0):
    with torch.no_grad():
        return nn.init.trunc_normal_(tensor, mean=mean, std=std, a=a, b=b)


class TokenLayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters, state_dict keys and init) for the token blocks' norm1 / norm2
    (TransformerBlock backbone_vit.py:250,256,261-262; SwinTransformerBlock backbone_swin.py:418,431) on the HIP
    LayerNorm kernels. Under bf16 autocast the output is the bf16 operand the following Linear would cast it to
    (the same rounding of the same f32 result), so the f32 intermediate and the cast kernels drop out; outside
    autocast it returns f32 as nn.LayerNorm does. GPU only."""

    @staticmethod
    def _bf16_out():
        return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16

    def forward(self, x):
        return kernels.layer_norm(x, self.weight, self.bias, self.eps, self._bf16_out())

    def forward_residual_add(self, h, a, tap=False):
        """(h + a, self(h + a)) with the residual add inside the LayerNorm forward kernel; tap: (h + a, an alias of it
        for a consumer outside the block, self(h + a))."""
        return kernels.add_residual_layer_norm(h, a, self.weight, self.bias, self.eps, self._bf16_out(), tap)

    def forward_residual(self, x, tap=False):
        """(x, self(x)) for a residual block x + f(self(x)); the backward adds the residual gradient inside the
        LayerNorm kernel (one pass over the residual stream fewer); tap: (x, an alias of x, self(x)), whose gradient
        is summed in the same kernel."""
        return kernels.residual_layer_norm(x, self.weight, self.bias, self.eps, self._bf16_out(), tap)


class OutLayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters, keys, init) whose f32 result is a model output rather than a Linear operand:
    ViT_with_alt_ops.norm (backbone_vit.py:368, :390), run on the HIP LayerNorm kernels with f32 out (what nn.LayerNorm
    returns under autocast); torch's layer_norm on the CPU."""

    def forward(self, x):
        if x.is_cuda:
            return kernels.layer_norm(x, self.weight, self.bias, self.eps, False)
        return super().forward(x)


_UNIT_AFFINE = {}


def layer_norm_no_affine(x: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """F.layer_norm(x, [C]) without affine parameters (SwinTransformer.proj_out, backbone_swin.py:866-873), f32 out,
    on the HIP LayerNorm kernels (unit gamma / zero beta) on the GPU."""
    if not x.is_cuda:
        return torch.nn.functional.layer_norm(x, [x.shape[-1]], eps=eps)
    key = (x.shape[-1], x.device)
    wb = _UNIT_AFFINE.get(key)
    if wb is None:
        wb = (torch.ones(x.shape[-1], device=x.device), torch.zeros(x.shape[-1], device=x.device))
        _UNIT_AFFINE[key] = wb
    return kernels.layer_norm(x, wb[0], wb[1], eps, False)


class TokenLinear(nn.Linear):
    """nn.Linear (same parameters, state_dict keys and seeded init) for the token-wise projections. On the GPU
    (kernels.linear) the forward and data gradient run on lci_gemm_bt where it takes the shape (hipBLASLt otherwise),
    the weight and bias gradients, a reduction over all B*L tokens into a small N x K output, on lci_linear_wgrad."""

    def forward(self, x):
        if x.is_cuda:
            return kernels.linear(x, self.weight, self.bias)
        return super().forward(x)


class MLPBlock(nn.Module):
    def __init__(self, hidden_size: int, mlp_dim: int, dropout_rate: float = 0.0, act="GELU",
                 dropout_mode="vit") -> None:
        super().__init__()
        if not (0 <= dropout_rate <= 1):
            raise ValueError("dropout_rate should be between 0 and 1.")
        mlp_dim = mlp_dim or hidden_size
        self.linear1 = TokenLinear(hidden_size, mlp_dim)
        self.linear2 = TokenLinear(mlp_dim, hidden_size)
        if act != "GELU":
            raise NotImplementedError(f"act={act}: only GELU is used by the reference")
        self.fn = nn.GELU()
        self.drop1 = nn.Dropout(dropout_rate)
        if dropout_mode == "vit":
            self.drop2 = nn.Dropout(dropout_rate)
        elif dropout_mode == "swin":
            self.drop2 = self.drop1
        else:
            raise ValueError(f"dropout_mode {dropout_mode}")

    def forward(self, x):
        h = self.linear1(x)
        h = kernels.gelu(h) if kernels.gelu_supported(h) else self.fn(h)
        return self.drop2(self.linear2(self.drop1(h)))


class PatchEmbeddingBlock(nn.Module):
    """proj_type='conv' only (the reference never selects 'perceptron')."""

    def __init__(self, in_channels: int, img_size: Sequence[int] | int, patch_size: Sequence[int] | int,
                 hidden_size: int, num_heads: int, proj_type: str = "conv", pos_embed_type: str = "learnable",
                 dropout_rate: float = 0.0, spatial_dims: int = 3) -> None:
        super().__init__()
        if not (0 <= dropout_rate <= 1):
            raise ValueError("dropout_rate should be between 0 and 1.")
        if hidden_size % num_heads != 0:
            raise ValueError(f"hidden size {hidden_size} should be divisible by num_heads {num_heads}.")
        if proj_type != "conv":
            raise NotImplementedError("only proj_type='conv' is used by the reference")
        if pos_embed_type not in ("none", "learnable"):
            raise NotImplementedError(f"pos_embed_type={pos_embed_type}")
        self.proj_type, self.pos_embed_type = proj_type, pos_embed_type
        img_size = ensure_tuple_rep(img_size, spatial_dims)
        patch_size = ensure_tuple_rep(patch_size, spatial_dims)
        for m, p in zip(img_size, patch_size):
            if m < p:
                raise ValueError("patch_size should be smaller than img_size.")
        self.img_size, self.patch_size = tuple(img_size), tuple(patch_size)
        self.n_patches = int(np.prod([im_d // p_d for im_d, p_d in zip(img_size, patch_size)]))
        conv = nn.Conv2d if spatial_dims == 2 else nn.Conv3d
        self.patch_embeddings = conv(in_channels, hidden_size, kernel_size=patch_size, stride=patch_size)
        self.position_embeddings = nn.Parameter(torch.zeros(1, self.n_patches, hidden_size))
        self.dropout = nn.Dropout(dropout_rate)
        if pos_embed_type == "learnable":
            trunc_normal_(self.position_embeddings, mean=0.0, std=0.02, a=-2.0, b=2.0)
        self.apply(self._init_weights)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, mean=0.0, std=0.02, a=-2.0, b=2.0)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def forward(self, x):
        y = kernels.patch_embed(x, self.patch_embeddings.weight, self.patch_embeddings.bias,
                                self.position_embeddings, channels_last_tokens=True)
        return self.dropout(y)


class PatchEmbed(nn.Module):
    def __init__(self, patch_size: Sequence[int] | int = 2, in_chans: int = 1, embed_dim: int = 48,
                 norm_layer=nn.LayerNorm, spatial_dims: int = 3) -> None:
        super().__init__()
        if spatial_dims not in (2, 3):
            raise ValueError("spatial dimension should be 2 or 3.")
        patch_size = ensure_tuple_rep(patch_size, spatial_dims)
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        conv = nn.Conv2d if spatial_dims == 2 else nn.Conv3d
        self.proj = conv(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        if self.norm is not None:
            raise NotImplementedError("patch_norm=True is not used by the reference (backbone_swin.py:760)")
        return kernels.patch_embed(x, self.proj.weight, self.proj.bias, None, channels_last_tokens=False)
