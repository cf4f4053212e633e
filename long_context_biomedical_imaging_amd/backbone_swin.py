"""Swin backbone with shifted-window attention / Hyena / Mamba mixers — drop-in for
/root/reference/model/models/backbone_swin.py.

Same public names, constructor signatures, parameter-creation order and state_dict keys as the
reference (custom_Swin :44-129, window ops :135-224, WindowAttention :227-367, SwinTransformerBlock
:370-537, PatchMergingV2 :540-585, compute_mask :591-628, BasicLayer :631-733,
SwinTransformer_with_alt_ops :736-911).

Attention blocks run the liblci window-attention kernel in *grid mode*: the qkv Linear is applied to the
un-padded channels-last token grid, and the kernel does the reference's F.pad -> torch.roll(-shift) ->
window_partition gather, the relative-position-bias add, the -100 region mask (computed from region ids,
bit-identical to compute_mask), the softmax and AV, and the window_reverse -> roll(+shift) -> crop scatter
as address arithmetic — none of the ~6 full-tensor copies per block are made. Padded tokens take the qkv
bias as their q/k/v, exactly what Linear(0) gives the reference's zero-padded LayerNorm output.
WindowAttention.forward(x, mask) keeps the reference signature (pre-partitioned windows) for direct callers.
"""
from __future__ import annotations

from collections.abc import Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels
from .blocks import MLPBlock as Mlp
from .blocks import PatchEmbed, TokenLayerNorm, TokenLinear, layer_norm_no_affine, trunc_normal_
from .hyena import HyenaOperator
from .mamba import MambaVisionMixer


def custom_Swin(config, input_feature_channels):
    s = config.Swin
    presets = {"unetr": (48, [2, 2, 2, 2], [3, 6, 12, 24]), "tiny": (96, [2, 2, 6, 2], [3, 6, 12, 24]),
               "small": (96, [2, 2, 18, 2], [3, 6, 12, 24]), "base": (128, [2, 2, 18, 2], [4, 8, 16, 32]),
               "large": (192, [2, 2, 18, 2], [6, 12, 24, 48])}
    if s.size in presets:
        embed_dim, depths, num_heads = presets[s.size]
        s.embed_dim, s.depths, s.num_heads = embed_dim, depths, num_heads
    elif s.size == "custom":
        embed_dim, depths, num_heads = s.embed_dim, s.depths, s.num_heads
    else:
        raise ValueError(f"Unknown model size {s.size} specified in config.")
    if config.time == 1:
        spatial_dims = 2
        if len(s.patch_size) == 3:
            mod_patch_size, mod_window_size = s.patch_size[1:], s.window_size[1:]
        else:
            mod_patch_size, mod_window_size = s.patch_size, s.window_size
    else:
        spatial_dims = 3
        mod_patch_size, mod_window_size = s.patch_size, s.window_size
    model = SwinTransformer_with_alt_ops(use_hyena=s.use_hyena, use_mamba=s.use_mamba,
                                         in_chans=input_feature_channels, embed_dim=embed_dim,
                                         window_size=mod_window_size, patch_size=mod_patch_size, depths=depths,
                                         num_heads=num_heads, spatial_dims=spatial_dims)
    n = len(depths)
    return model, [embed_dim * 2 ** (n - i) for i in range(n, 0, -1)] + [embed_dim * 2 ** n]


def window_partition(x, window_size):
    x_shape = x.size()
    if len(x_shape) == 5:
        b, d, h, w, c = x_shape
        x = x.view(b, d // window_size[0], window_size[0], h // window_size[1], window_size[1],
                   w // window_size[2], window_size[2], c)
        return x.permute(0, 1, 3, 5, 2, 4, 6, 7).contiguous().view(-1, window_size[0] * window_size[1] * window_size[2], c)
    b, h, w, c = x.shape
    x = x.view(b, h // window_size[0], window_size[0], w // window_size[1], window_size[1], c)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(-1, window_size[0] * window_size[1], c)


def window_reverse(windows, window_size, dims):
    if len(dims) == 4:
        b, d, h, w = dims
        x = windows.view(b, d // window_size[0], h // window_size[1], w // window_size[2], window_size[0],
                         window_size[1], window_size[2], -1)
        return x.permute(0, 1, 4, 2, 5, 3, 6, 7).contiguous().view(b, d, h, w, -1)
    b, h, w = dims
    x = windows.view(b, h // window_size[0], w // window_size[1], window_size[0], window_size[1], -1)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(b, h, w, -1)


def get_window_size(x_size, window_size, shift_size=None):
    use_window_size = list(window_size)
    if shift_size is not None:
        use_shift_size = list(shift_size)
    for i in range(len(x_size)):
        if x_size[i] <= window_size[i]:
            use_window_size[i] = x_size[i]
            if shift_size is not None:
                use_shift_size[i] = 0
    if shift_size is None:
        return tuple(use_window_size)
    return tuple(use_window_size), tuple(use_shift_size)


def relative_position_index(window_size) -> torch.Tensor:
    coords = torch.stack(torch.meshgrid(*[torch.arange(w) for w in window_size], indexing="ij"))
    cf = torch.flatten(coords, 1)
    rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
    for i, w in enumerate(window_size):
        rel[:, :, i] += w - 1
    if len(window_size) == 3:
        rel[:, :, 0] *= (2 * window_size[1] - 1) * (2 * window_size[2] - 1)
        rel[:, :, 1] *= 2 * window_size[2] - 1
    else:
        rel[:, :, 0] *= 2 * window_size[1] - 1
    return rel.sum(-1)


class _TableGather(torch.autograd.Function):
    """table[idx] whose backward scatters with index_add_ (float atomics): autograd's default index backward sorts
    the n^2 = 117649 indices of a 7^3 window on every call (a rocprim merge sort, ~2 ms per C3 step)."""

    @staticmethod
    def forward(ctx, table, idx):
        ctx.save_for_backward(idx)
        ctx.rows = table.shape[0]
        return table[idx]

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        gt = torch.zeros(ctx.rows, g.shape[-1], device=g.device, dtype=g.dtype)
        if torch.are_deterministic_algorithms_enabled():
            # fixed-order sum (autograd's sorted index backward); index_add_ below uses float atomics
            gt.index_put_((idx,), g, accumulate=True)
        else:
            gt.index_add_(0, idx, g)
        return gt, None


class WindowAttention(nn.Module):
    def __init__(self, use_hyena: bool, use_mamba: bool, dim: int, num_heads: int, window_size: Sequence[int],
                 qkv_bias: bool = False, attn_drop: float = 0.0, proj_drop: float = 0.0) -> None:
        super().__init__()
        self.dim = dim
        self.use_hyena = use_hyena
        self.use_mamba = use_mamba
        if not use_hyena and not use_mamba:
            self.window_size = window_size
            self.num_heads = num_heads
            head_dim = dim // num_heads
            if head_dim > kernels.WIN_HEAD_DIM:
                # csrc/window.hip is built for head_dim 32 (every Swin preset: 96/3 ... 768/24); smaller custom
                # splits run zero-padded to 32 (kernels.pad_heads, exact), larger ones fail here, not mid-step
                raise ValueError(f"window attention head_dim {head_dim} (dim {dim} / num_heads {num_heads}) is not "
                                 f"supported: the HIP window kernels take head_dim <= {kernels.WIN_HEAD_DIM} "
                                 f"(DESIGN.md §7)")
            self.scale = head_dim ** -0.5
            n_tab = int(np.prod([2 * w - 1 for w in window_size]))
            self.relative_position_bias_table = nn.Parameter(torch.zeros(n_tab, num_heads))
            self.register_buffer("relative_position_index", relative_position_index(window_size))
            self.qkv = TokenLinear(dim, dim * 3, bias=qkv_bias)
            self.attn_drop = nn.Dropout(attn_drop)
            self.proj = TokenLinear(dim, dim)
            self.proj_drop = nn.Dropout(proj_drop)
            trunc_normal_(self.relative_position_bias_table, std=0.02)
            self.softmax = nn.Softmax(dim=-1)
        elif use_hyena and not use_mamba:
            self.hyena = HyenaOperator(d_model=self.dim, l_max=66000, filter_order=64, num_heads=num_heads,
                                       num_blocks=1, short_filter_order=5, bidrectional=False, dropout=attn_drop,
                                       filter_dropout=proj_drop, activation="id")
        elif not use_hyena and use_mamba:
            self.mamba = MambaVisionMixer(d_model=self.dim, d_state=8, d_conv=3, expand=1)

    def rel_bias(self, n):
        """(heads, n, n) f32 relative-position bias = table[index[:n, :n]] (backbone_swin.py:343-346)."""
        idx = self.relative_position_index[:n, :n].reshape(-1)
        g = _TableGather.apply(self.relative_position_bias_table, idx)
        return g.reshape(n, n, -1).permute(2, 0, 1).float().contiguous()

    def _check_drop(self):
        if self.training and (self.attn_drop.p > 0):
            raise NotImplementedError("attention dropout > 0 is not fused into the window kernel")

    def forward(self, x, mask):
        """Reference signature: x (B*nW, N, C) pre-partitioned windows, mask (nW, N, N) or None."""
        b, n, c = x.shape
        if not self.use_hyena and not self.use_mamba:
            self._check_drop()
            qkv = self.qkv(x)
            o = kernels.window_attention(qkv, self.rel_bias(n), mask, self.num_heads, self.scale)
            x = self.proj_drop(self.proj(o))
        elif self.use_hyena and not self.use_mamba:
            x = self.hyena(x)
        else:
            x = self.mamba(x)
        return x

    def forward_grid(self, xn, window_size, shift_size):
        """Fused path: xn = LN1 output on the un-padded grid (b, d, h, w, c) or (b, h, w, c)."""
        self._check_drop()
        n = int(np.prod(window_size))
        qkv = self.qkv(xn)
        bias = self.qkv.bias
        o = kernels.window_attention_grid(qkv, bias, self.rel_bias(n), self.num_heads, self.scale,
                                          tuple(window_size), tuple(shift_size))
        return self.proj_drop(self.proj(o))


class SwinTransformerBlock(nn.Module):
    def __init__(self, use_hyena: bool, use_mamba: bool, dim: int, num_heads: int, window_size: Sequence[int],
                 shift_size: Sequence[int], mlp_ratio: float = 4.0, qkv_bias: bool = True, drop: float = 0.0,
                 attn_drop: float = 0.0, drop_path: float = 0.0, act_layer: str = "GELU",
                 norm_layer: type[nn.LayerNorm] = nn.LayerNorm, use_checkpoint: bool = False) -> None:
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        self.use_checkpoint = use_checkpoint
        if norm_layer is nn.LayerNorm:   # same parameters and init, HIP kernels (bf16 autocast operand out)
            norm_layer = TokenLayerNorm
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(use_hyena, use_mamba, dim, window_size=self.window_size, num_heads=num_heads,
                                    qkv_bias=qkv_bias, attn_drop=attn_drop, proj_drop=drop)
        if drop_path > 0.0:
            raise NotImplementedError("drop_path > 0 is not used by the reference (drop_path_rate=0.0)")
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(hidden_size=dim, mlp_dim=int(dim * mlp_ratio), act=act_layer, dropout_rate=drop,
                       dropout_mode="swin")

    def forward_part1(self, x, mask_matrix):
        x_shape = x.size()
        x = self.norm1(x)
        dims_sp = tuple(x.shape[1:-1])
        window_size, shift_size = get_window_size(dims_sp, self.window_size, self.shift_size)
        if not self.attn.use_hyena and not self.attn.use_mamba:
            return self.attn.forward_grid(x, window_size, shift_size)
        if any(i > 0 for i in shift_size):
            raise NotImplementedError("shifted windows with hyena/mamba do not occur in the reference")
        if x.is_cuda and kernels.window_gather_supported(x):
            # Hyena / Mamba inside windows (shift 0, backbone_swin.py:674): F.pad + window_partition as one gather,
            # window_reverse + crop as one scatter (lci_window_gather)
            xw = kernels.window_partition_grid(x, window_size, shift_size)
            return kernels.window_reverse_grid(self.attn(xw, mask=None), x.shape, window_size, shift_size)
        c = x.shape[-1]
        pads = [(window_size[i] - s % window_size[i]) % window_size[i] for i, s in enumerate(dims_sp)]
        padarg = []
        for p in reversed(pads):
            padarg += [0, p]
        x = F.pad(x, [0, 0] + padarg)
        dims = [x.shape[0], *x.shape[1:-1]]
        if any(i > 0 for i in shift_size):
            raise NotImplementedError("shifted windows with hyena/mamba do not occur in the reference")
        x_windows = window_partition(x, window_size)
        attn_windows = self.attn(x_windows, mask=None)
        attn_windows = attn_windows.view(-1, *(tuple(window_size) + (c,)))
        x = window_reverse(attn_windows, window_size, dims)
        if len(x_shape) == 5:
            return x[:, :dims_sp[0], :dims_sp[1], :dims_sp[2], :].contiguous()
        return x[:, :dims_sp[0], :dims_sp[1], :].contiguous()

    def forward_part2(self, x):
        return self.drop_path(self.mlp(self.norm2(x)))

    def forward(self, x, mask_matrix):
        shortcut = x
        if self.use_checkpoint:
            x = torch.utils.checkpoint.checkpoint(self.forward_part1, x, mask_matrix, use_reentrant=False)
        else:
            x = self.forward_part1(x, mask_matrix)
        if (not self.use_checkpoint and isinstance(self.drop_path, nn.Identity) and x.is_cuda
                and isinstance(self.norm2, TokenLayerNorm)):
            # shortcut + attention summed inside the norm2 LayerNorm kernel (one pass over the stream fewer)
            x, y = self.norm2.forward_residual_add(shortcut, x)
            return x + self.mlp(y)
        x = shortcut + self.drop_path(x)
        if self.use_checkpoint:
            x = x + torch.utils.checkpoint.checkpoint(self.forward_part2, x, use_reentrant=False)
        else:
            x = x + self.forward_part2(x)
        return x


class PatchMergingV2(nn.Module):
    def __init__(self, dim: int, norm_layer: type[nn.LayerNorm] = nn.LayerNorm, spatial_dims: int = 3) -> None:
        super().__init__()
        self.dim = dim
        if norm_layer is nn.LayerNorm:   # same parameters and init; its output is the reduction's bf16 operand
            norm_layer = TokenLayerNorm
        if spatial_dims == 3:
            self.reduction = TokenLinear(8 * dim, 2 * dim, bias=False)
            self.norm = norm_layer(8 * dim)
        elif spatial_dims == 2:
            self.reduction = TokenLinear(4 * dim, 2 * dim, bias=False)
            self.norm = norm_layer(4 * dim)

    def forward(self, x):
        x_shape = x.size()
        if len(x_shape) == 5:
            b, d, h, w, c = x_shape
            if (h % 2 == 1) or (w % 2 == 1) or (d % 2 == 1):
                x = F.pad(x, (0, 0, 0, w % 2, 0, h % 2, 0, d % 2))
            # = torch.cat([x[:, i::2, j::2, k::2, :] for i, j, k in product(range(2), repeat=3)], -1) as one
            # permuted copy: the eight strided slices' backward accumulated eight full-size gradients (seven adds)
            b, d, h, w, c = x.shape
            x = (x.view(b, d // 2, 2, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 5, 2, 4, 6, 7)
                 .reshape(b, d // 2, h // 2, w // 2, 8 * c))
        elif len(x_shape) == 4:
            b, h, w, c = x_shape
            if (h % 2 == 1) or (w % 2 == 1):
                x = F.pad(x, (0, 0, 0, w % 2, 0, h % 2))
            # = torch.cat([x[:, j::2, i::2, :] for i, j in product(range(2), range(2))], -1) (block = 2 (w parity)
            # + h parity) as one permuted copy
            b, h, w, c = x.shape
            x = x.view(b, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 4, 2, 5).reshape(b, h // 2, w // 2, 4 * c)
        return self.reduction(self.norm(x))


MERGING_MODE = {"mergingv2": PatchMergingV2}


def compute_mask(dims, window_size, shift_size, device):
    """(nW, N, N) mask, -100 across regions (backbone_swin.py:591-628). Kept for API parity; the fused
    kernel evaluates the same region test in-register."""
    cnt = 0
    if len(dims) == 3:
        d, h, w = dims
        img_mask = torch.zeros((1, d, h, w, 1), device=device)
        for d in slice(-window_size[0]), slice(-window_size[0], -shift_size[0]), slice(-shift_size[0], None):
            for h in slice(-window_size[1]), slice(-window_size[1], -shift_size[1]), slice(-shift_size[1], None):
                for w in slice(-window_size[2]), slice(-window_size[2], -shift_size[2]), slice(-shift_size[2], None):
                    img_mask[:, d, h, w, :] = cnt
                    cnt += 1
    elif len(dims) == 2:
        h, w = dims
        img_mask = torch.zeros((1, h, w, 1), device=device)
        for h in slice(-window_size[0]), slice(-window_size[0], -shift_size[0]), slice(-shift_size[0], None):
            for w in slice(-window_size[1]), slice(-window_size[1], -shift_size[1]), slice(-shift_size[1], None):
                img_mask[:, h, w, :] = cnt
                cnt += 1
    mask_windows = window_partition(img_mask, window_size).squeeze(-1)
    attn_mask = mask_windows.unsqueeze(1) - mask_windows.unsqueeze(2)
    return attn_mask.masked_fill(attn_mask != 0, float(-100.0)).masked_fill(attn_mask == 0, float(0.0))


class BasicLayer(nn.Module):
    def __init__(self, use_hyena: bool, use_mamba: bool, dim: int, depth: int, num_heads: int,
                 window_size: Sequence[int], drop_path: list, mlp_ratio: float = 4.0, qkv_bias: bool = False,
                 drop: float = 0.0, attn_drop: float = 0.0, norm_layer: type[nn.LayerNorm] = nn.LayerNorm,
                 downsample: nn.Module | None = None, use_checkpoint: bool = False) -> None:
        super().__init__()
        self.window_size = window_size
        if use_hyena or use_mamba:
            self.shift_size = tuple(0 for _ in window_size)
        else:
            self.shift_size = tuple(i // 2 for i in window_size)
        self.no_shift = tuple(0 for _ in window_size)
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(use_hyena=use_hyena, use_mamba=use_mamba, dim=dim, num_heads=num_heads,
                                 window_size=self.window_size,
                                 shift_size=self.no_shift if (i % 2 == 0) else self.shift_size,
                                 mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, drop=drop, attn_drop=attn_drop,
                                 drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer, use_checkpoint=use_checkpoint)
            for i in range(depth)])
        self.downsample = downsample
        if callable(self.downsample):
            self.downsample = downsample(dim=dim, norm_layer=norm_layer, spatial_dims=len(self.window_size))

    def forward(self, x):
        x_shape = x.size()
        nd = len(x_shape) - 2
        b, c = x_shape[:2]
        sp = tuple(x_shape[2:])
        x = x.permute(0, *range(2, 2 + nd), 1)          # b c ... -> b ... c
        for blk in self.blocks:
            x = blk(x, None)                            # the mask is evaluated inside the window kernel
        x = x.reshape(b, *sp, -1)
        if self.downsample is not None:
            x = self.downsample(x)
        return x.permute(0, nd + 1, *range(1, nd + 1))  # b ... c -> b c ...


class SwinTransformer_with_alt_ops(nn.Module):
    def __init__(self, use_hyena: bool, use_mamba: bool, in_chans: int, embed_dim: int,
                 window_size: Sequence[int], patch_size: Sequence[int], depths: Sequence[int],
                 num_heads: Sequence[int], mlp_ratio: float = 4.0, qkv_bias: bool = True, drop_rate: float = 0.0,
                 attn_drop_rate: float = 0.0, drop_path_rate: float = 0.0,
                 norm_layer: type[nn.LayerNorm] = nn.LayerNorm, patch_norm: bool = False,
                 use_checkpoint: bool = False, spatial_dims: int = 3, downsample="mergingv2",
                 use_v2=False) -> None:
        super().__init__()
        if use_v2:
            raise NotImplementedError("use_v2 (UnetrBasicBlock per stage) is never enabled by the reference")
        self.use_hyena = use_hyena
        self.use_mamba = use_mamba
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.patch_norm = patch_norm
        self.window_size = window_size
        self.patch_size = patch_size
        self.spatial_dims = spatial_dims
        self.patch_embed = PatchEmbed(patch_size=self.patch_size, in_chans=in_chans, embed_dim=embed_dim,
                                      norm_layer=norm_layer if self.patch_norm else None, spatial_dims=spatial_dims)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.use_v2 = use_v2
        self.layers1 = nn.ModuleList()
        self.layers2 = nn.ModuleList()
        self.layers3 = nn.ModuleList()
        self.layers4 = nn.ModuleList()
        down = MERGING_MODE[downsample] if isinstance(downsample, str) else downsample
        for i_layer in range(self.num_layers):
            layer = BasicLayer(use_hyena=use_hyena, use_mamba=use_mamba, dim=int(embed_dim * 2 ** i_layer),
                               depth=depths[i_layer], num_heads=num_heads[i_layer], window_size=self.window_size,
                               drop_path=dpr[sum(depths[:i_layer]): sum(depths[: i_layer + 1])],
                               mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, drop=drop_rate, attn_drop=attn_drop_rate,
                               norm_layer=norm_layer, downsample=down, use_checkpoint=use_checkpoint)
            [self.layers1, self.layers2, self.layers3, self.layers4][i_layer].append(layer)
        self.num_features = int(embed_dim * 2 ** (self.num_layers - 1))

    def proj_out(self, x, normalize=False):
        if normalize:
            nd = x.dim() - 2
            ch = x.shape[1]
            x = x.permute(0, *range(2, 2 + nd), 1)
            x = layer_norm_no_affine(x)
            x = x.permute(0, nd + 1, *range(1, nd + 1))
        return x

    def forward(self, x, normalize=True):
        if self.spatial_dims == 2:
            x = x.squeeze(2)
        hidden_states_out = [x]
        x0 = self.pos_drop(self.patch_embed(x))
        hidden_states_out += [self.proj_out(x0, normalize)]
        # the reference's x.contiguous() between stages (backbone_swin.py:891-906) is a pure layout copy: the
        # stages exchange channels-last views here, so each BasicLayer's b c ... -> b ... c permute is free
        x1 = self.layers1[0](x0)
        hidden_states_out += [self.proj_out(x1, normalize)]
        x2 = self.layers2[0](x1)
        hidden_states_out += [self.proj_out(x2, normalize)]
        x3 = self.layers3[0](x2)
        hidden_states_out += [self.proj_out(x3, normalize)]
        x4 = self.layers4[0](x3)
        hidden_states_out += [self.proj_out(x4, normalize)]
        if self.spatial_dims == 2:
            hidden_states_out = [t.unsqueeze(2) for t in hidden_states_out]
        return hidden_states_out
