"""Oracle: ViT_with_alt_ops encoder forward, CPU restatement over a state_dict. Test infra only.

Follows /root/reference/model/models/backbone_vit.py:
  :379-397  squeeze T (2-D) -> patch_embedding -> [cls token] -> blocks -> final LN; 14 outputs
  :260-263  TransformerBlock: x += attn(LN1 x); x += MLP(LN2 x)   (MONAI MLPBlock: Linear-GELU-Linear)
  :189-211  SABlock dispatch: attention / hyena / mamba
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import attention, hyena, patch_embed, selective_scan


def _sub(sd, prefix):
    n = len(prefix)
    return {k[n:]: v for k, v in sd.items() if k.startswith(prefix)}


def block_forward(x, sd, num_heads, mode="attention", q_chunk=None):
    h = F.layer_norm(x, (x.shape[-1],), sd["norm1.weight"], sd["norm1.bias"])
    if mode == "attention":
        a = attention.sablock_attention(h, sd["attn.qkv.weight"], sd.get("attn.qkv.bias"),
                                        sd["attn.out_proj.weight"], sd["attn.out_proj.bias"], num_heads,
                                        q_chunk)
    elif mode == "hyena":
        a = hyena.hyena_forward(h, _sub(sd, "attn.hyena."), num_heads)
    else:
        a = selective_scan.mamba_mixer(h, _sub(sd, "attn.mamba."))
    x = x + a
    h = F.layer_norm(x, (x.shape[-1],), sd["norm2.weight"], sd["norm2.bias"])
    h = F.linear(F.gelu(F.linear(h, sd["mlp.linear1.weight"], sd["mlp.linear1.bias"])),
                 sd["mlp.linear2.weight"], sd["mlp.linear2.bias"])
    return x + h


def vit_forward(x, sd, num_layers, num_heads, spatial_dims=2, mode="attention", q_chunk=None):
    if spatial_dims == 2:
        x = x.squeeze(2)
    outs = [x]
    x = patch_embed.vit_patch_embed(x, sd["patch_embedding.patch_embeddings.weight"],
                                    sd["patch_embedding.patch_embeddings.bias"],
                                    sd["patch_embedding.position_embeddings"])
    if "cls_token" in sd:
        x = torch.cat((sd["cls_token"].expand(x.shape[0], -1, -1), x), dim=1)
    for i in range(num_layers):
        x = block_forward(x, _sub(sd, f"blocks.{i}."), num_heads, mode, q_chunk)
        outs.append(x)
    outs.append(F.layer_norm(x, (x.shape[-1],), sd["norm.weight"], sd["norm.bias"]))
    return outs
