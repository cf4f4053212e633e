"""Oracle: patch-embed conv (k = stride = patch), CPU restatement. Test infrastructure only.

MONAI-1.3 PatchEmbeddingBlock (proj_type='conv') as used by ViT_with_alt_ops
(/root/reference/model/models/backbone_vit.py:351-361, forward :383):
    conv(k=s=p) -> flatten(2).transpose(-1,-2) -> + position_embeddings -> dropout(p=0)
MONAI-1.3 PatchEmbed as used by SwinTransformer_with_alt_ops (backbone_swin.py:800-806, :885):
    right-pad each spatial dim to a multiple of p -> conv(k=s=p); no norm (patch_norm=False, :760)
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def vit_patch_embed(x, weight, bias, pos):
    """x (B, C, *S) -> (B, L, D)."""
    conv = F.conv2d if x.dim() == 4 else F.conv3d
    p = weight.shape[2:]
    y = conv(x, weight, bias, stride=p)
    return y.flatten(2).transpose(-1, -2) + pos


def swin_patch_embed(x, weight, bias):
    """x (B, C, *S) -> (B, D, *S/p) with right zero-padding to a patch multiple."""
    p = weight.shape[2:]
    pads = []
    for s, pp in zip(reversed(x.shape[2:]), reversed(p)):
        pads += [0, (pp - s % pp) % pp]
    x = F.pad(x, pads)
    conv = F.conv2d if x.dim() == 4 else F.conv3d
    return conv(x, weight, bias, stride=p)
