"""Task heads the encoders feed (callers of the hot path, not part of it).

ViTLinear / SwinLinear restate /root/reference/model/models/class_heads.py (:13-79).
ViTUNETR restates enhance_heads.py:187-356 on top of MONAI-1.3 UNETR blocks (UnetResBlock,
UnetrBasicBlock, UnetrPrUpBlock, UnetrUpBlock, UnetOutBlock: conv + InstanceNorm + LeakyReLU, transposed
conv up-sampling); SwinUNETR restates enhance_heads.py:30-184. SURVEY.md §8(f) rank 2.

The convolutions keep the nn.Conv / nn.ConvTranspose parameters (names, shapes, seeded init) but not their
MIOpen kernels, which at 128^3 spend 70-120 s in solver search per shape and then run a 96->96 3x3x3 conv
fwd+bwd in ~390 ms (tools/conv3d_probe.py), and which refuse 256^3 inputs (32-bit size limit):
  - 3x3(x3) stride-1 convs: the HIP implicit-GEMM kernel (csrc/conv.hip, kernels.conv3), channels-last;
  - transposed convs with kernel == stride (the up-sampling): one GEMM (V x Cin).(Cin x Cout*k^nd) and an
    interleaving copy, i.e. exactly the non-overlapping scatter they compute;
  - 1x1 convs: one GEMM over channels-last voxels.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels

# A/B switch for the 2-D heads (the headline ViTUNETR at 512^2): HIP conv3 + inorm (default; same step time as
# MIOpen at 512^2, without its ~2 min first-call solver search) vs torch/MIOpen (LCI_HIP_CONV_2D=0)
HIP_CONV_2D = os.environ.get("LCI_HIP_CONV_2D", "1") != "0"
# 3-D: HIP always in the product (MIOpen 3-D is ~40x slower here and refuses 256^3); the switch exists so the
# parity tests can run the same modules through torch's fp32 / bf16 convolutions as references
HIP_CONV_3D = os.environ.get("LCI_HIP_CONV_3D", "1") != "0"


def _hip(x, flag):
    """The HIP conv / instance-norm path computes bf16 operands with f32 accumulation and returns bf16: it is the
    autocast (use_amp) path. An f32 model run on the GPU without autocast keeps the reference's f32 convolutions
    (torch); CPU tensors go to the HIP path too, which refuses them (no CPU path)."""
    return flag and (not x.is_cuda or x.dtype == torch.bfloat16 or torch.is_autocast_enabled("cuda"))


class Conv3x3(nn.Conv3d):
    """nn.Conv3d(cin, cout, 3, 1, padding=1, bias=False) computed by the HIP conv3 kernel."""

    def forward(self, x):
        if not _hip(x, HIP_CONV_3D):
            return super().forward(x)
        return kernels.conv3(x, self.weight)


class Conv3x3_2d(nn.Conv2d):
    """nn.Conv2d(cin, cout, 3, 1, padding=1, bias=False) computed by the HIP conv3 kernel (D = 1)."""

    def forward(self, x):
        if not _hip(x, HIP_CONV_2D):
            return super().forward(x)
        return kernels.conv3(x, self.weight)


_CL = {2: torch.channels_last, 3: torch.channels_last_3d}   # dense channels-last layout per spatial rank


def _pointwise(x, weight, bias):
    """1x1 conv as a GEMM over channels-last voxels; result (B, Cout, *S) with channels-last strides. Narrow outputs
    (the heads' Conv to 1-4 classes / channels) under bf16 autocast run on lci_linear_small_* (kernels.pointwise_small):
    a 2-column GEMM is a pure stream that hipBLASLt runs with tiny tiles far below the HBM rate."""
    xl = x.movedim(1, -1)
    Cout, Cin = weight.shape[0], weight.shape[1]
    if (x.is_cuda and Cout <= 4 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        x2 = xl.to(torch.bfloat16).reshape(-1, Cin)
        if kernels.pointwise_small_supported(x2, Cout):
            y = kernels.pointwise_small(x2, weight, bias)
            return y.view(*xl.shape[:-1], Cout).movedim(-1, 1)
    if x.is_cuda:   # hipBLASLt forward / data gradient, HIP weight gradient (kernels.linear, as TokenLinear)
        return kernels.linear(xl, weight.reshape(Cout, Cin), bias).movedim(-1, 1)
    y = F.linear(xl, weight.reshape(Cout, Cin), bias)
    return y.movedim(-1, 1)


class Conv1x1(nn.Conv3d):
    def forward(self, x):
        return _pointwise(x, self.weight, self.bias)


class Conv1x1_2d(nn.Conv2d):
    def forward(self, x):
        return _pointwise(x, self.weight, self.bias)


def _up_gemm(x, weight, bias, k, skip=None):
    """ConvTranspose with kernel == stride: y[.., s*k + i, ..] = sum_c x[.., s, .., c] w[c, :, i..].

    One GEMM (V x Cin) . (Cin x prod(k) Cout) with the weight columns ordered (tap, Cout) and the bias added per
    column inside it, so every tap's Cout channels are one contiguous run that the interleaving copy moves whole.
    On the GPU it is kernels.linear (hipBLASLt forward / data gradient, HIP weight gradient: the (Cin x k^3 Cout)
    reduction over all V voxels is the shape hipBLASLt tiles worst, 12 ms per call at 128^3)."""
    nd = x.dim() - 2
    B, Cin = x.shape[:2]
    S = x.shape[2:]
    Cout = weight.shape[1]
    taps = 1
    for kk in k:
        taps *= kk
    wt = weight.movedim(1, -1).reshape(Cin, taps * Cout).t()                       # (taps * Cout, Cin)
    bt = bias.repeat(taps) if bias is not None else None
    x2 = x.movedim(1, -1).reshape(-1, Cin)
    y = kernels.linear(x2, wt, bt) if x.is_cuda else F.linear(x2, wt, bt)         # (V, taps * Cout)
    sk = skip.movedim(1, -1) if skip is not None else None
    if kernels.convup_interleave_supported(y, Cout, sk):
        # HIP interleave straight to the channels-last grid (and into the cat buffer with the skip, UnetrUpBlock)
        return kernels.convup_interleave(y, B, S, k, Cout, sk).movedim(-1, 1)
    y = y.view(B, *S, *k, Cout)
    if nd == 3:
        y = y.permute(0, 1, 4, 2, 5, 3, 6, 7)
    else:
        y = y.permute(0, 1, 3, 2, 4, 5)
    y = y.reshape(B, *(s * kk for s, kk in zip(S, k)), Cout)
    y = y.movedim(-1, 1)
    return torch.cat((y, skip), dim=1) if skip is not None else y


class ConvUp(nn.ConvTranspose3d):
    def forward(self, x, skip=None):
        """skip given: torch.cat((self(x), skip), dim=1) (UnetrUpBlock) produced in one pass."""
        return _up_gemm(x, self.weight, self.bias, self.kernel_size, skip)


class ConvUp_2d(nn.ConvTranspose2d):
    def forward(self, x, skip=None):
        return _up_gemm(x, self.weight, self.bias, self.kernel_size, skip)


class Convolution(nn.Module):
    """MONAI 1.3 Convolution without act / norm / dropout: the conv layer under `.conv`, so the parameters carry the
    reference's state_dict keys (`<block>.conv1.conv.weight`, `<up>.transp_conv.conv.weight`, ...)."""

    def __init__(self, conv):
        super().__init__()
        self.conv = conv

    def forward(self, *args):
        return self.conv(*args)


def _conv(nd, cin, cout, k, s, transposed=False, bias=False):
    """MONAI get_conv_layer(conv_only=True): padding (k - s + 1) // 2, output_padding 2p + s - k (per axis), the
    layer wrapped as MONAI's Convolution."""
    return Convolution(_conv_layer(nd, cin, cout, k, s, transposed, bias))


def _conv_layer(nd, cin, cout, k, s, transposed=False, bias=False):
    if isinstance(k, (tuple, list)) or isinstance(s, (tuple, list)):
        k = tuple(k) if isinstance(k, (tuple, list)) else (k,) * nd
        s = tuple(s) if isinstance(s, (tuple, list)) else (s,) * nd
        pad = tuple((a - b + 1) // 2 for a, b in zip(k, s))
        opad = tuple(2 * p + b - a for p, a, b in zip(pad, k, s))
    else:
        pad = (k - s + 1) // 2
        opad = 2 * pad + s - k
    kt = k if isinstance(k, tuple) else (k,) * nd
    st = s if isinstance(s, tuple) else (s,) * nd
    if transposed:
        if kt == st:
            cls = ConvUp_2d if nd == 2 else ConvUp
        else:
            cls = nn.ConvTranspose2d if nd == 2 else nn.ConvTranspose3d
        return cls(cin, cout, k, s, padding=pad, output_padding=opad, bias=bias)
    if all(a == 3 for a in kt) and all(b == 1 for b in st) and not bias and cout % 32 == 0:
        cls = Conv3x3_2d if nd == 2 else Conv3x3
    elif all(a == 1 for a in kt) and all(b == 1 for b in st):
        cls = Conv1x1_2d if nd == 2 else Conv1x1
    else:
        cls = nn.Conv2d if nd == 2 else nn.Conv3d
    return cls(cin, cout, k, s, padding=pad, bias=bias)


def _inorm(nd, c):
    return (nn.InstanceNorm2d if nd == 2 else nn.InstanceNorm3d)(c)


class UnetResBlock(nn.Module):
    def __init__(self, nd, cin, cout, k, stride):
        super().__init__()
        self.conv1 = _conv(nd, cin, cout, k, stride)
        self.conv2 = _conv(nd, cout, cout, k, 1)
        self.lrelu = nn.LeakyReLU(negative_slope=0.01, inplace=True)
        self.norm1 = _inorm(nd, cout)
        self.norm2 = _inorm(nd, cout)
        self.downsample = cin != cout or stride != 1
        if self.downsample:
            self.conv3 = _conv(nd, cin, cout, 1, stride)
            self.norm3 = _inorm(nd, cout)

        # channels-last HIP path: the convs are the HIP conv3 / GEMM forms and the instance norms (+ LeakyReLU)
        # the lci_inorm kernels, so the block never round-trips through NCDHW (2-D: only with HIP_CONV_2D)
        self.fused = isinstance(self.conv1.conv, (Conv3x3, Conv3x3_2d)) and cout % 8 == 0

    def forward(self, inp):
        if self.fused and _hip(inp, HIP_CONV_3D if inp.dim() == 5 else HIP_CONV_2D):
            if (self.downsample and isinstance(self.conv3.conv, (Conv1x1, Conv1x1_2d)) and self.conv3.conv.bias is None
                    and self.conv3.conv.stride == (1,) * (inp.dim() - 2)
                    and kernels.res_convs_supported(inp, self.conv1.conv.weight, self.conv3.conv.weight)):
                # conv1 and the 1x1 residual conv read the same input: one backward node sums their input
                # gradients inside the GEMM
                c1, r = kernels.res_convs(inp, self.conv1.conv.weight, self.conv3.conv.weight)
                out = kernels.instance_norm_act(c1, True)
            else:
                out = kernels.instance_norm_act(self.conv1(inp), True)
                r = self.conv3(inp) if self.downsample else inp
            c2 = self.conv2(out)
            # norm2 (+ norm3) + residual add + LeakyReLU in one pass where the operands are bf16 channels-last
            z = kernels.inorm_add_lrelu(c2, r, self.downsample)
            if z is not None:
                return z
            res = kernels.instance_norm_act(r, False) if self.downsample else r
            return F.leaky_relu(kernels.instance_norm_act(c2, False) + res, 0.01)
        out = self.lrelu(self.norm1(self.conv1(inp)))
        out = self.norm2(self.conv2(out))
        res = self.norm3(self.conv3(inp)) if self.downsample else inp
        return self.lrelu(out + res)


class UnetrPrUpBlock(nn.Module):
    def __init__(self, nd, cin, cout, num_layer, k, us):
        super().__init__()
        self.transp_conv_init = _conv(nd, cin, cout, us, us, transposed=True)
        self.blocks = nn.ModuleList([nn.Sequential(_conv(nd, cout, cout, us, us, transposed=True),
                                                   UnetResBlock(nd, cout, cout, k, 1)) for _ in range(num_layer)])

    def forward(self, x):
        x = self.transp_conv_init(x)
        for b in self.blocks:
            x = b(x)
        return x


class UnetrUpBlock(nn.Module):
    def __init__(self, nd, cin, cout, k, us):
        super().__init__()
        self.transp_conv = _conv(nd, cin, cout, us, us, transposed=True)
        self.conv_block = UnetResBlock(nd, cout + cout, cout, k, 1)

    def forward(self, inp, skip):
        if isinstance(self.transp_conv.conv, (ConvUp, ConvUp_2d)):
            return self.conv_block(self.transp_conv.conv(inp, skip))   # up-sampling + cat in one pass
        return self.conv_block(torch.cat((self.transp_conv(inp), skip), dim=1))


class UnetOutBlock(nn.Module):
    def __init__(self, nd, cin, cout):
        super().__init__()
        self.conv = _conv(nd, cin, cout, 1, 1, bias=True)

    def forward(self, x):
        return self.conv(x)


class UnetrBasicBlock(nn.Module):
    """MONAI UnetrBasicBlock(res_block=True): one UnetResBlock under `.layer`."""

    def __init__(self, nd, cin, cout, k, stride):
        super().__init__()
        self.layer = UnetResBlock(nd, cin, cout, k, stride)

    def forward(self, x):
        return self.layer(x)


class SwinUNETR(nn.Module):
    """enhance_heads.py:30-184: UNETR-style decoder over the five Swin stage taps (features [96, 192, 384, 768,
    1536] for Swin-tiny) and the input image; instance-norm residual conv blocks, transposed-conv up-sampling, the
    last up-sampling by the patch size."""

    def __init__(self, config, input_feature_channels, output_feature_channels):
        super().__init__()
        f = input_feature_channels
        if f[0] % 12 != 0:
            raise ValueError("Features should be divisible by 12 to use current UNETR config.")
        if config.encoder_name != "Swin":
            raise ValueError(f"Invalid backbone component for SwinUNETR head: {config.encoder_name}")
        cin = config.no_in_channel
        if config.time == 1:
            nd, self.spatial_dims, up = 2, 2, 2
            patch = tuple(config.Swin.patch_size[1:])
        else:
            nd, self.spatial_dims, up = 3, 3, (2, 2, 2)
            patch = tuple(config.Swin.patch_size)
        self.encoder1 = UnetrBasicBlock(nd, cin, f[0], 3, 1)
        self.encoder2 = UnetrBasicBlock(nd, f[0], f[0], 3, 1)
        self.encoder3 = UnetrBasicBlock(nd, f[1], f[1], 3, 1)
        self.encoder4 = UnetrBasicBlock(nd, f[2], f[2], 3, 1)
        self.encoder10 = UnetrBasicBlock(nd, f[4], f[4], 3, 1)
        self.decoder5 = UnetrUpBlock(nd, f[4], f[3], 3, up)
        self.decoder4 = UnetrUpBlock(nd, f[3], f[2], 3, up)
        self.decoder3 = UnetrUpBlock(nd, f[2], f[1], 3, up)
        self.decoder2 = UnetrUpBlock(nd, f[1], f[0], 3, up)
        self.decoder1 = UnetrUpBlock(nd, f[0], f[0], 3, patch)
        self.out = UnetOutBlock(nd, f[0], output_feature_channels)

    def forward(self, input_data):
        if self.spatial_dims == 2:
            input_data = [i.squeeze(2) for i in input_data]
        x_in, feats = input_data[0], input_data[1:]
        enc0 = self.encoder1(x_in)
        enc1 = self.encoder2(feats[0])
        enc2 = self.encoder3(feats[1])
        enc3 = self.encoder4(feats[2])
        dec4 = self.encoder10(feats[4])
        dec3 = self.decoder5(dec4, feats[3])
        dec2 = self.decoder4(dec3, enc3)
        dec1 = self.decoder3(dec2, enc2)
        dec0 = self.decoder2(dec1, enc1)
        out = self.out(self.decoder1(dec0, enc0))
        if self.spatial_dims == 2:
            out = out.unsqueeze(2)
        return out


class ViTUNETR(nn.Module):
    """enhance_heads.py:187-356 (feature_size 32, taps h3/h6/h9 + final LN)."""

    hidden_taps = (4, 7, 10)   # hidden_states_out indices read besides [0] and [-1] (hs[3], hs[6], hs[9])

    def __init__(self, config, input_feature_channels, output_feature_channels):
        super().__init__()
        fs = 32
        cin = config.no_in_channel
        if config.encoder_name != "ViT":
            raise ValueError(f"Invalid encoder_name for ViTUNETR head: {config.encoder_name}")
        hidden = config.ViT.hidden_size
        if config.time == 1:
            self.spatial_dims = 2
            img_size = [config.height, config.width]
            patch = config.ViT.patch_size[1:]
        else:
            self.spatial_dims = 3
            img_size = [config.time, config.height, config.width]
            patch = config.ViT.patch_size
        nd = self.spatial_dims
        self.feat_size = tuple(i // p for i, p in zip(img_size, patch))
        self.hidden_size = hidden
        p3 = patch if len(patch) == 3 else (1,) + tuple(patch)
        table = {2: ((0, 0, 0), (1, 1, 1, 2)), 4: ((1, 1, 0), (1, 1, 2, 2)), 8: ((2, 1, 0), (1, 2, 2, 2)),
                 16: ((2, 1, 0), (2, 2, 2, 2)), 32: ((2, 1, 0), (4, 2, 2, 2))}
        if p3[1] != p3[2] or p3[1] not in table:
            raise ValueError(f"ViT UNETR patch size {p3} not yet supported")
        (n2, n3, n4), (d1, d2, d3, d4) = table[p3[1]]
        self.encoder1 = UnetrBasicBlock(nd, cin, fs, 3, 1)
        self.encoder2 = UnetrPrUpBlock(nd, hidden, fs * 2, n2, 3, 2)
        self.encoder3 = UnetrPrUpBlock(nd, hidden, fs * 4, n3, 3, 2)
        self.encoder4 = UnetrPrUpBlock(nd, hidden, fs * 8, n4, 3, 2)
        self.decoder5 = UnetrUpBlock(nd, hidden, fs * 8, 3, d4)
        self.decoder4 = UnetrUpBlock(nd, fs * 8, fs * 4, 3, d3)
        self.decoder3 = UnetrUpBlock(nd, fs * 4, fs * 2, 3, d2)
        self.decoder2 = UnetrUpBlock(nd, fs * 2, fs, 3, d1)
        self.out = UnetOutBlock(nd, fs, output_feature_channels)
        self.proj_axes = (0, nd + 1) + tuple(d + 1 for d in range(nd))
        self.proj_view_shape = list(self.feat_size) + [hidden]

    def proj_feat(self, x):
        # the (B, L, C) tokens are already the channels-last (B, *S, C) volume: return the (B, C, *S) permuted view
        # (channels-last strides, which the HIP convs consume in place) instead of the reference's NCDHW copy
        return x.view([x.size(0)] + self.proj_view_shape).permute(self.proj_axes).contiguous(
            memory_format=_CL[self.spatial_dims])

    def forward(self, input_data):
        x_in = input_data[0]
        if self.spatial_dims == 2:
            x_in = x_in.squeeze(2)
        hs = input_data[1:-1]
        x = input_data[-1]
        enc1 = self.encoder1(x_in)
        enc2 = self.encoder2(self.proj_feat(hs[3]))
        enc3 = self.encoder3(self.proj_feat(hs[6]))
        enc4 = self.encoder4(self.proj_feat(hs[9]))
        dec3 = self.decoder5(self.proj_feat(x), enc4)
        dec2 = self.decoder4(dec3, enc3)
        dec1 = self.decoder3(dec2, enc2)
        out = self.out(self.decoder2(dec1, enc1))
        if self.spatial_dims == 2:
            out = out.unsqueeze(2)
        return out


class ViTLinear(nn.Module):
    def __init__(self, config, input_feature_channels, output_feature_channels):
        super().__init__()
        if config.encoder_name != "ViT":
            raise ValueError("Invalid backbone component for ViTLinear head")
        self.cls_token = not (config.ViT.use_hyena or config.ViT.use_mamba)
        self.classification_head = nn.Sequential(nn.Linear(input_feature_channels[-1], output_feature_channels),
                                                 nn.Tanh())

    def forward(self, x):
        x = x[-1]
        x = x[:, 0] if self.cls_token else x.mean(1)
        return self.classification_head(x)


class SwinLinear(nn.Module):
    def __init__(self, config, input_feature_channels, output_feature_channels):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool3d(1)
        self.classification_head = nn.Sequential(nn.Linear(input_feature_channels[-1], output_feature_channels),
                                                 nn.Tanh())

    def forward(self, x):
        x = torch.flatten(self.avgpool(x[-1]), 1)
        return self.classification_head(x)


class Identity(nn.Module):
    def forward(self, x):
        return x


# ----------------------------------------------------------------------------------------- UperNet heads
# The UperNet convs return standard-layout tensors: BatchNorm / interpolate follow them, and torch's ROCm
# batch_norm crashed (SIGSEGV) on channels-last views of 1x1-pixel pyramid maps.
class ConvK3(nn.Conv3d):
    """nn.Conv3d(cin, cout, 3, padding=1[, bias]) on the HIP conv3 kernel (any cout, optional bias)."""

    def forward(self, x):
        if not _hip(x, HIP_CONV_3D):
            return super().forward(x)
        return kernels.conv3(x, self.weight, self.bias).contiguous()


class ConvK3_2d(nn.Conv2d):
    def forward(self, x):
        if not _hip(x, HIP_CONV_2D):
            return super().forward(x)
        y = kernels.conv3(x, self.weight, self.bias)
        return y if _is_cl(x) else y.contiguous()   # channels-last in -> channels-last out (UPERNET_CL)


class ConvPoint(nn.Conv3d):
    """nn.Conv3d(cin, cout, 1, padding=p[, bias]) as one GEMM over channels-last voxels (zero border first)."""

    def forward(self, x):
        p = self.padding[0]
        if p:
            x = F.pad(x, (p,) * 6)
        return _pointwise(x, self.weight, self.bias).contiguous()


class ConvPoint_2d(nn.Conv2d):
    def forward(self, x):
        p = self.padding[0]
        if _is_cl(x):   # channels-last map (UPERNET_CL): the GEMM reads it in place, the zero border goes on after
            if p and self.bias is not None:
                x = F.pad(x.permute(0, 2, 3, 1), (0, 0, p, p, p, p)).permute(0, 3, 1, 2)
                p = 0
            y = _pointwise(x, self.weight, self.bias)
            if p:   # no bias: the border of a 1x1 conv of a zero-padded map is zero
                y = F.pad(y.permute(0, 2, 3, 1), (0, 0, p, p, p, p)).permute(0, 3, 1, 2)
            return y
        if p:
            x = F.pad(x, (p,) * 4)
        return _pointwise(x, self.weight, self.bias).contiguous()


def _k3(nd, cin, cout, bias=True):
    return (ConvK3_2d if nd == 2 else ConvK3)(cin, cout, kernel_size=3, padding=1, bias=bias)


def _k1(nd, cin, cout, bias=True, padding=0):
    return (ConvPoint_2d if nd == 2 else ConvPoint)(cin, cout, kernel_size=1, padding=padding, bias=bias)


class BatchNorm2d(nn.BatchNorm2d):
    """BatchNorm in f32 whatever the input dtype (output f32). Under bf16 autocast torch's ROCm batch_norm
    segfaults on the 1x1-pixel maps of the PSP pyramid (bin 1); computing the statistics in f32 avoids that and
    is at least as accurate as the reference's bf16 batch_norm. Same parameters/buffers as nn.BatchNorm2d."""

    def forward(self, x):
        return super().forward(x.float())


class BatchNorm3d(nn.BatchNorm3d):
    def forward(self, x):
        return super().forward(x.float())


def _bn(nd, c):
    return (BatchNorm2d if nd == 2 else BatchNorm3d)(c)


HIP_BN = os.environ.get("LCI_HIP_BN", "1") != "0"


def _bf16_operands(ts):
    """The maps a following conv concatenates, cast to its autocast operand dtype first: the cast commutes with the
    cat (the same bf16 values), and the cat then moves 2 bytes per element instead of 4 (the FPN fusion's 1536-channel
    512^2 cat at C4: 3.2 GB f32) with no separate cast pass."""
    if ts and ts[0].is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16:
        return [t.to(torch.bfloat16) for t in ts]
    return ts


def _conv_bn_relu(seq, x):
    """seq = Sequential(conv, BatchNorm, ReLU[, Dropout]) (PSPModule.bottleneck seg_heads.py:26-31 / :158-163,
    FPN_fuse.conv_fusion :60-63 / :192-195): in training mode the BatchNorm + ReLU of the conv's bf16 channels-last
    output run as one HIP op (kernels.batch_norm_relu: f32 out, no f32 copy of the input; MIOpen's batch norm and
    torch's ReLU took 4.9 ms per C4 step)."""
    y = seq[0](x)
    if (HIP_BN and len(seq) >= 3 and isinstance(seq[2], nn.ReLU) and isinstance(seq[1], nn.modules.batchnorm._BatchNorm)
            and kernels.batch_norm_relu_supported(y, seq[1])):
        y = kernels.batch_norm_relu(y, seq[1])
        for m in list(seq)[3:]:
            y = m(y)
        return y
    for m in list(seq)[1:]:
        y = m(y)
    return y


# The PSP pyramid's adaptive average pooling (to 1-6 bins) and its align_corners bilinear / trilinear up-sampling
# back to the feature size are separable linear maps along each spatial axis. Applied as small matrices (f32,
# autocast off, so the arithmetic stays f32 as in torch's kernels) they become batched GEMMs whose backward is a
# GEMM too: torch's upsample backward scatters every output pixel into the 1-36 pooled pixels with atomics
# (13.7 ms per stage at 512^2 x 96 channels, C4) and its adaptive-pool backward takes ~10 ms per stage.
SEPARABLE_PSP = os.environ.get("LCI_SEPARABLE_PSP", "1") != "0"
_SEP_CACHE = {}

# UperNet2D on ViT taps keeps the big maps channels-last end to end (the token taps already are): no NCHW copies of
# the 512^2 x 384-1536 maps at C4. The PSP's pooled 1-36 pixel maps stay NCHW (torch's ROCm batch_norm crashed on
# channels-last views of 1x1 maps).
UPERNET_CL = os.environ.get("LCI_UPERNET_CL", "1") != "0"

# The FPN's align_corners re-sampling (up_and_add and the final resize to the finest level) and the PSP's
# up-sampling of the pooled bins on lci_resample_cl_fwd (one pass, the FPN's lateral add summed in it) with a
# deterministic one-axis-at-a-time adjoint (kernels.resample_cl): torch's upsample_bilinear2d_backward is an atomic
# scatter (3.2 ms per 514^2 -> 512^2 x 384 call at C4) and the separable GEMMs run as batched hipBLASLt calls on
# 4-36 element matrices at the 3-D shapes (~0.1-0.5 ms each, ~5 ms per Swin-recipe step).
HIP_RESAMPLE = os.environ.get("LCI_HIP_RESAMPLE", "1") != "0"


def _is_cl(x):
    """A 4-D map in channels-last memory that is not also plain-contiguous (and big enough to matter)."""
    return (UPERNET_CL and x.dim() == 4 and x.shape[2] * x.shape[3] > 64 and not x.is_contiguous()
            and x.is_contiguous(memory_format=torch.channels_last))


def _cat_channels(ts):
    """torch.cat(ts, dim=1); channels-last maps are concatenated as NHWC (one channels-last result, no copies)."""
    if all(_is_cl(t) for t in ts):
        return torch.cat([t.permute(0, 2, 3, 1) for t in ts], dim=-1).permute(0, 3, 1, 2)
    return torch.cat(ts, dim=1)


def _pool_cl(x, bins):
    """adaptive average pooling of a channels-last (B, C, H, W) map: GEMMs over the NHWC layout, NCHW result."""
    B, C, H, W = x.shape
    ah, aw = _avg_pool_matrix(bins, H, x.device), _avg_pool_matrix(bins, W, x.device)
    with torch.autocast(x.device.type, enabled=False):
        t = ah @ x.float().permute(0, 2, 3, 1).reshape(B, H, W * C)           # (B, b, W C)
        t = aw @ t.reshape(B * bins, W, C)                                     # (B b, b, C)
    return t.reshape(B, bins, bins, C).permute(0, 3, 1, 2).contiguous().to(x.dtype)


def _up_cl(y, size):
    """align_corners=True up-sampling of a small NCHW map into a channels-last (B, C, H, W) f32 map."""
    B, C, bh, bw = y.shape
    uh, uw = _lin_interp_matrix(size[0], bh, y.device), _lin_interp_matrix(size[1], bw, y.device)
    with torch.autocast(y.device.type, enabled=False):
        t = uw @ y.float().permute(0, 2, 3, 1).reshape(B * bh, bw, C)          # (B bh, W, C)
        t = uh @ t.reshape(B, bh, size[1] * C)                                 # (B, H, W C)
    return t.reshape(B, size[0], size[1], C).permute(0, 3, 1, 2)


def _lin_interp_matrix(out_size, in_size, device):
    """(out, in) f32 weights of 1-D linear interpolation with align_corners=True, computed as torch's
    upsample kernels do (scale = (in - 1) / (out - 1) in f32, src = scale * i, i0 = floor, lambda = src - i0)."""
    key = ("lin", out_size, in_size, str(device))
    m = _SEP_CACHE.get(key)
    if m is None:
        scale = torch.tensor((in_size - 1) / (out_size - 1) if out_size > 1 else 0.0, dtype=torch.float32)
        src = scale * torch.arange(out_size, dtype=torch.float32)
        i0 = src.floor().to(torch.long).clamp(max=in_size - 1)
        lam1 = src - i0.to(torch.float32)
        i1 = torch.clamp(i0 + 1, max=in_size - 1)
        m = torch.zeros(out_size, in_size, dtype=torch.float32)
        rows = torch.arange(out_size)
        m.index_put_((rows, i0), 1.0 - lam1, accumulate=True)
        m.index_put_((rows, i1), lam1, accumulate=True)
        m = m.to(device)
        _SEP_CACHE[key] = m
    return m


def _avg_pool_matrix(out_size, in_size, device):
    """(out, in) f32 weights of adaptive average pooling: bin i averages [floor(i in / out), ceil((i+1) in / out))."""
    key = ("pool", out_size, in_size, str(device))
    m = _SEP_CACHE.get(key)
    if m is None:
        m = torch.zeros(out_size, in_size, dtype=torch.float32)
        for i in range(out_size):
            a, b = (i * in_size) // out_size, -((-(i + 1) * in_size) // out_size)
            m[i, a:b] = 1.0 / (b - a)
        m = m.to(device)
        _SEP_CACHE[key] = m
    return m


def _separable(x, mats):
    """Apply mats[k] (out_k, in_k) along spatial axis k of x (N, C, *S), last axis first; f32 result."""
    nd = len(mats)
    with torch.autocast(x.device.type, enabled=False):
        y = x.float() @ mats[-1].t()                              # (N, C, ..., W_out)
        if nd >= 2:
            y = mats[-2] @ y                                      # (N, C, [D,] H_out, W_out)
        if nd == 3:
            n, c, d, h, w = y.shape
            y = (mats[0] @ y.reshape(n * c, d, h * w)).reshape(n, c, mats[0].shape[0], h, w)
    return y


def adaptive_avg_pool(x, bins):
    """nn.AdaptiveAvgPool{2,3}d(bins)(x) as separable GEMMs (x's dtype out)."""
    mats = [_avg_pool_matrix(bins, s, x.device) for s in x.shape[2:]]
    return _separable(x, mats).to(x.dtype)


def upsample_align_corners(x, size):
    """F.interpolate(x, size, mode=(bi|tri)linear, align_corners=True) as separable GEMMs (f32 out)."""
    mats = [_lin_interp_matrix(o, i, x.device) for o, i in zip(size, x.shape[2:])]
    return _separable(x, mats)


class PSPModule(nn.Module):
    """seg_heads.py:18-47 (2-D) / :153-182 (3-D): adaptive-average-pool pyramid (bins 1, 2, 4, 6) -> 1x1 conv ->
    BN -> ReLU, (bi|tri)linear up-sampling (align_corners=True), concat, and a 1x1 bottleneck conv whose
    padding=1 grows the map by one voxel per side (kept: the FPN re-samples it), BN, ReLU, Dropout(0.1)."""

    def __init__(self, nd, in_channels, bin_sizes=(1, 2, 4, 6)):
        super().__init__()
        self.nd = nd
        out_channels = in_channels // len(bin_sizes)
        pool = nn.AdaptiveAvgPool2d if nd == 2 else nn.AdaptiveAvgPool3d
        self.stages = nn.ModuleList([nn.Sequential(pool(output_size=b), _k1(nd, in_channels, out_channels, False),
                                                   _bn(nd, out_channels), nn.ReLU(inplace=True))
                                     for b in bin_sizes])
        self.bottleneck = nn.Sequential(
            _k1(nd, in_channels + out_channels * len(bin_sizes), in_channels, bias=False, padding=1),
            _bn(nd, in_channels), nn.ReLU(inplace=True), (nn.Dropout2d if nd == 2 else nn.Dropout3d)(0.1))

    def forward(self, features):
        size = features.shape[2:]
        mode = "bilinear" if self.nd == 2 else "trilinear"
        if SEPARABLE_PSP and features.is_cuda and self.nd == 2 and _is_cl(features):
            pyramids = [features]
            for stage in self.stages:
                y = _pool_cl(features, stage[0].output_size)
                for m in list(stage)[1:]:
                    y = m(y)
                if HIP_RESAMPLE and kernels.resample_cl_supported(y, size):
                    up = kernels.resample_cl(y, size, True)
                else:
                    up = _up_cl(y, size)
                pyramids.append(up if up.dtype == y.dtype else up.to(y.dtype))
            return _conv_bn_relu(self.bottleneck, _cat_channels(_bf16_operands(pyramids)))
        if SEPARABLE_PSP and features.is_cuda:
            pyramids = [features]
            for stage in self.stages:
                if features.numel() <= (1 << 21):
                    # a small map (Swin's last stage, 4^3 x 768 at 128^3): torch's own pooling kernel; the separable
                    # form runs as batched hipBLASLt calls on 4-36 element matrices (~0.15 ms each)
                    y = stage[0](features)
                else:
                    y = adaptive_avg_pool(features, stage[0].output_size)
                for m in list(stage)[1:]:
                    y = m(y)
                if HIP_RESAMPLE and kernels.resample_cl_supported(y, size):
                    up = kernels.resample_cl(y, size, True)
                else:
                    up = upsample_align_corners(y, size)
                pyramids.append(up if up.dtype == y.dtype else up.to(y.dtype))
        else:
            pyramids = [features] + [F.interpolate(stage(features), size=size, mode=mode, align_corners=True)
                                     for stage in self.stages]
        return _conv_bn_relu(self.bottleneck, torch.cat(pyramids, dim=1))


_INTERP_DTYPE = {}


def _interp_dtype(x, mode):
    """The dtype F.interpolate(x, mode=mode) returns in the current autocast state (probed once on a 2x2 map)."""
    dev = x.device.type
    key = (x.dtype, mode, dev, torch.is_autocast_enabled(dev), torch.get_autocast_dtype(dev))
    dt = _INTERP_DTYPE.get(key)
    if dt is None:
        probe = x.new_zeros((1, 1) + (2,) * (x.dim() - 2))
        dt = F.interpolate(probe, size=(2,) * (x.dim() - 2), mode=mode, align_corners=True).dtype
        _INTERP_DTYPE[key] = dt
    return dt


class FPN_fuse(nn.Module):
    """seg_heads.py:52-76 / :187-211: lateral 1x1 convs, top-down up-and-add, ONE 3x3 smoothing conv shared by
    the three levels (the reference lists the same module three times), up-sample all to the finest level,
    concat, 3x3 conv -> BN -> ReLU."""

    def __init__(self, nd, feature_channels, fpn_out):
        super().__init__()
        assert feature_channels[0] == fpn_out
        self.nd = nd
        self.conv1x1 = nn.ModuleList([_k1(nd, c, fpn_out) for c in feature_channels[1:]])
        self.smooth_conv = nn.ModuleList([_k3(nd, fpn_out, fpn_out)] * (len(feature_channels) - 1))
        self.conv_fusion = nn.Sequential(_k3(nd, len(feature_channels) * fpn_out, fpn_out, bias=False),
                                         _bn(nd, fpn_out), nn.ReLU(inplace=True))

    def forward(self, features):
        mode = "bilinear" if self.nd == 2 else "trilinear"
        features = list(features)
        features[1:] = [c(f) for f, c in zip(features[1:], self.conv1x1)]
        # align_corners=True re-sampling to the same size is the identity (src = dst, weights 1 / 0): skipped for
        # the ViT taps, which all share one grid (torch still runs an interpolation kernel and an atomic backward)
        def resize(x, size):
            if tuple(x.shape[2:]) == tuple(size):
                return x.to(_interp_dtype(x, mode))
            if HIP_RESAMPLE and kernels.resample_cl_supported(x, size):
                return kernels.resample_cl(x, size, True).to(_interp_dtype(x, mode))
            if SEPARABLE_PSP and x.is_cuda and not _is_cl(x):
                # separable GEMMs (f32, as torch's kernel) whose backward is a GEMM, not an atomic scatter
                return upsample_align_corners(x, size).to(_interp_dtype(x, mode))
            return F.interpolate(x, size=size, mode=mode, align_corners=True)

        def up_and_add(x, y):   # seg_heads.py:49-50 / :181-182
            size = y.shape[2:]
            if (tuple(x.shape[2:]) != tuple(size) and HIP_RESAMPLE and _interp_dtype(x, mode) == torch.float32
                    and kernels.resample_cl_supported(x, size, y)):
                return kernels.resample_cl(x, size, True, add=y)   # the f32 sum, in the re-sampling pass
            return resize(x, size) + y

        P = [up_and_add(features[i], features[i - 1]) for i in reversed(range(1, len(features)))]
        P = [sc(x) for sc, x in zip(self.smooth_conv, P)]
        P = list(reversed(P))
        P.append(features[-1])
        size = P[0].shape[2:]
        P[1:] = [resize(f, size) for f in P[1:]]
        return _conv_bn_relu(self.conv_fusion, _cat_channels(_bf16_operands(P)))


class _UperNet(nn.Module):
    def __init__(self, nd, config, input_feature_channels, output_feature_channels):
        super().__init__()
        if config.encoder_name == "Swin":
            self.upernet_feature_channels = [-4, -3, -2, -1]
        elif config.encoder_name == "ViT":
            self.upernet_feature_channels = [4, 7, 10, -1]
            self.hidden_taps = (4, 7, 10)   # the encoder's other block outputs are not read (keep_hidden)
        else:
            raise ValueError(f"encoder_name {config.encoder_name} not recognized or comaptible with UperNet3D")
        chans = [input_feature_channels[c] for c in self.upernet_feature_channels]
        self.nd = nd
        self.encoder_name = config.encoder_name
        self.fpn_out = chans[0]
        self.input_size = (config.height, config.width) if nd == 2 else (config.time, config.height, config.width)
        self.PPN = PSPModule(nd, chans[-1])
        self.FPN = FPN_fuse(nd, chans, self.fpn_out)
        self.head = _k3(nd, self.fpn_out, output_feature_channels)
        if config.encoder_name == "ViT":
            patch = list(config.ViT.patch_size[1:]) if nd == 2 else list(config.ViT.patch_size)
            self.feat_size = tuple(i // p for i, p in zip(self.input_size, patch))
            self.proj_axes = (0, nd + 1) + tuple(d + 1 for d in range(nd))

    def _reshape_vit_output(self, x):
        x = x.view([x.size(0)] + list(self.feat_size) + [x.shape[-1]]).permute(self.proj_axes)
        if self.nd == 2 and UPERNET_CL and x.is_cuda:
            return x   # the token taps are channels-last already (see UPERNET_CL)
        return x.contiguous()   # NCHW: UperNet's BatchNorm / pooling / interpolation paths

    def freeze_bn(self):
        for module in self.modules():
            if isinstance(module, (nn.BatchNorm2d, nn.BatchNorm3d)):
                module.eval()


class UperNet2D(_UperNet):
    """seg_heads.py:79-147: UperNet on the ViT token taps h4/h7/h10/final or the last four Swin stages (time axis
    dropped), bilinear up-sampling to the image size (align_corners=False), 3x3 head, time axis re-inserted."""

    def __init__(self, config, input_feature_channels, output_feature_channels):
        super().__init__(2, config, input_feature_channels, output_feature_channels)

    def forward(self, features):
        features = [features[c] for c in self.upernet_feature_channels]
        if self.encoder_name == "ViT":
            features = [self._reshape_vit_output(f) for f in features]
        else:
            features = [f[:, :, 0, :, :] for f in features]
        features[-1] = self.PPN(features[-1])
        x = self.FPN(features)
        if (HIP_CONV_2D and isinstance(self.head, ConvK3_2d) and kernels.upsample2x_supported(x, self.input_size)
                and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            # the head conv computes in bf16 from a channels-last operand: up-sample straight into it
            x = kernels.upsample2x_bilinear_cl(x)
        else:
            x = F.interpolate(x, size=self.input_size, mode="bilinear")
        return torch.unsqueeze(self.head(x), 2)


class UperNet3D(_UperNet):
    """seg_heads.py:214-277: the 3-D UperNet (trilinear), optional output_size."""

    def __init__(self, config, input_feature_channels, output_feature_channels):
        super().__init__(3, config, input_feature_channels, output_feature_channels)

    def forward(self, features, output_size=None):
        features = [features[c] for c in self.upernet_feature_channels]
        if self.encoder_name == "ViT":
            features = [self._reshape_vit_output(f) for f in features]
        features[-1] = self.PPN(features[-1])
        x = self.FPN(features)
        size = self.input_size if output_size is None else output_size
        if (HIP_CONV_3D and isinstance(self.head, ConvK3) and kernels.upsample3d_supported(x, size)
                and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            # the head conv computes in bf16 from a channels-last operand: up-sample straight into it
            x = kernels.upsample3d_trilinear_cl(x, size)
        else:
            x = F.interpolate(x, size=size, mode="trilinear")
        return self.head(x)
