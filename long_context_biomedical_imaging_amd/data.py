"""On-disk format + loader of the reference: `NumpyDataset` (data/data_base.py:20-124),
`custom_numpy_to_tensor` and `define_transforms` (data/data_utils.py:19-150), `RandomBrightnessContrast`
(data/augmentation_functions/brightness.py).

Layout: `<data_dir>/<id>/<id>_input.npy` stored H x W [x D/T] [x C] (float), `<id>_output.npy` likewise for seg
masks / enhancement targets, optional `<data_dir>/*_metadata.csv` (SubjectID, Label) for classification and a
split CSV (SubjectID, Split). Samples come out as (C, T, H, W) float tensors, seg labels as (T, H, W) long.

The reference resizes with OpenCV and augments with torchvision, neither of which is in this image; both are
restated from their published algorithms (parity unpinned against the libraries themselves):
  * cv2.resize INTER_LINEAR on float32 = half-pixel-centre bilinear without antialiasing (F.interpolate
    bilinear, align_corners=False); INTER_NEAREST = floor(dst * src / dst) (F.interpolate "nearest"); like
    OpenCV, a single-channel H x W x 1 array comes back H x W, and 4-D arrays cannot be resized;
  * torchvision 0.16.1 RandomApply / RandomAffine (inverse affine matrix about the centre, nearest grid_sample,
    zero fill) / GaussianBlur (separable kernel, reflect padding), with the same torch RNG draws in the same order,
    so one seed gives the image and its mask the same affine, as in the reference's __getitem__.
"""
from __future__ import annotations

import glob
import logging
import math
import os
import random

import numpy as np
import torch
import torch.nn.functional as F

INTER_LINEAR, INTER_NEAREST = "linear", "nearest"


# ------------------------------------------------------------------------------------ resizing (cv2 semantics)
def _cv2_resize(img: np.ndarray, new_shape, interp: str) -> np.ndarray:
    """cv2.resize(img, (new_w, new_h), interpolation) for a float H x W [x C] array (C <= 512)."""
    if img.ndim > 3:
        raise ValueError("cv2.resize: only 2-D images with an optional channel axis can be resized")
    t = torch.from_numpy(np.ascontiguousarray(img, dtype=np.float32))
    t = t.unsqueeze(-1) if t.dim() == 2 else t
    t = t.permute(2, 0, 1).unsqueeze(0)                                   # (1, C, H, W)
    if interp == INTER_NEAREST:
        out = F.interpolate(t, size=tuple(new_shape), mode="nearest")
    else:
        out = F.interpolate(t, size=tuple(new_shape), mode="bilinear", align_corners=False, antialias=False)
    out = out[0].permute(1, 2, 0).numpy()
    return out[..., 0] if out.shape[-1] == 1 else out                     # OpenCV drops a single channel


def custom_numpy_to_tensor(image, height, width, time, no_channels, interp=INTER_LINEAR):
    """data_utils.py:19-117: stored H x W [x D] [x C] -> tensor (C, T/D, H, W); resize H, W; centre pad/crop D."""

    def _resize_xy(img, new_shape):
        if (img.shape[0], img.shape[1]) == new_shape:
            return img
        return _cv2_resize(img, new_shape, interp)

    def _resize_depth(img, new_d):
        if len(img.shape) == 3:
            if img.shape[-1] < new_d:
                pad = new_d - img.shape[-1]
                img = np.pad(img, ((0, 0), (0, 0), (pad // 2, pad - pad // 2)))
            elif img.shape[-1] > new_d:
                crop = img.shape[-1] - new_d
                img = img[:, :, crop // 2:img.shape[-1] - (crop - crop // 2)]
        elif len(img.shape) == 4:
            if img.shape[-2] < new_d:
                pad = new_d - img.shape[-2]
                img = np.pad(img, ((0, 0), (0, 0), (pad // 2, pad - pad // 2), (0, 0)))
            elif img.shape[-2] > new_d:
                crop = img.shape[-2] - new_d
                # the reference bounds this crop by shape[-1] (the channel count), data_utils.py:43; kept
                img = img[:, :, crop // 2:img.shape[-1] - (crop - crop // 2), :]
        else:
            raise ValueError(f"Image shape should be H x W x D (x C), consisting of 3 or 4 dimensions when time>1. "
                             f"Got {len(image.shape)} dimensions.")
        return img

    if len(image.shape) not in [2, 3, 4]:
        raise ValueError(f"Image shape should be H x W (x D x C), consisting of 2, 3, or 4 dimensions. "
                         f"Got {len(image.shape)} dimensions.")
    hw = (height, width)
    if no_channels == 1 and time == 1:
        if len(image.shape) == 2:
            image = np.expand_dims(_resize_xy(image, hw), (2, 3))
        elif len(image.shape) == 3:
            assert image.shape[-1] == 1, \
                f"Single channel and depth/time specified, but third dimension has size {image.shape[-1]}"
            image = np.expand_dims(_resize_xy(image, hw), (3))
        else:
            assert image.shape[-1] == 1, f"Single channel specified, but fourth (C) dimension has size {image.shape[-1]}"
            assert image.shape[-2] == 1, \
                f"Single depth/time specified, but third (D/T) dimension has size {image.shape[-2]}"
            image = _resize_xy(image, hw)
    elif no_channels > 1 and time == 1:
        if len(image.shape) == 2:
            raise ValueError("More than one input channel specified, but stored image only has two dimensions.")
        assert image.shape[-1] == no_channels, (f"Channel dimension in stored numpy ({image.shape[-1]}) does not "
                                                f"match specified channel dimension ({no_channels})")
        if len(image.shape) == 3:
            image = np.expand_dims(_resize_xy(image, hw), (2))
        else:
            assert image.shape[-2] == 1, \
                f"Single depth/time specified, but third (D/T) dimension has size {image.shape[-2]}"
            image = _resize_xy(image, hw)
    elif no_channels == 1 and time > 1:
        if len(image.shape) == 2:
            raise ValueError("More than one time/depth dimension specified, but stored image only has two dimensions.")
        if len(image.shape) == 3:
            image = np.expand_dims(_resize_depth(_resize_xy(image, hw), time), (3))
        else:
            assert image.shape[-1] == 1, f"Single channel specified, but fourth (C) dimension has size {image.shape[-1]}"
            image = _resize_depth(_resize_xy(image, hw), time)
    elif no_channels > 1 and time > 1:
        if len(image.shape) == 2:
            raise ValueError("More than one time dimension specified, but stored image only has two dimensions.")
        if len(image.shape) == 3:
            raise ValueError("More than one time/depth dimension and channel specified, but stored image only has "
                             "three dimensions.")
        assert image.shape[-1] == no_channels, (f"Channel dimension in stored numpy ({image.shape[-1]}) does not "
                                                f"match specified channel dimension ({no_channels})")
        image = _resize_depth(_resize_xy(image, hw), time)
    else:
        raise ValueError(f"Expected no_input_channel and time to be >=1, got {no_channels} and {time}")
    return torch.permute(torch.from_numpy(np.ascontiguousarray(image)), (-1, -2, 0, 1))   # C, T/D, H, W


# ------------------------------------------------------------------------------ augmentations (torchvision)
class RandomApply:
    """torchvision.transforms.RandomApply: skip all with probability 1 - p (one torch.rand draw)."""

    def __init__(self, transforms, p=0.5):
        self.transforms, self.p = transforms, p

    def __call__(self, img):
        if self.p < torch.rand(1):
            return img
        for t in self.transforms:
            img = t(img)
        return img


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, img):
        for t in self.transforms:
            img = t(img)
        return img


def _inverse_affine_matrix(center, angle, translate, scale, shear):
    rot = math.radians(angle)
    sx, sy = math.radians(shear[0]), math.radians(shear[1])
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [x / scale for x in (d, -b, 0.0, -c, a, 0.0)]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


class RandomAffine:
    """torchvision.transforms.RandomAffine(degrees, translate, scale, shear), NEAREST, fill 0, centre pivot, on the
    last two axes of a (..., H, W) tensor (leading axes share one draw)."""

    def __init__(self, degrees, translate=None, scale=None, shear=None):
        self.degrees = (-degrees, degrees)
        self.translate, self.scale = translate, scale
        self.shear = (-shear, shear) if isinstance(shear, (int, float)) else shear

    def __call__(self, img):
        h, w = img.shape[-2], img.shape[-1]
        angle = float(torch.empty(1).uniform_(float(self.degrees[0]), float(self.degrees[1])).item())
        if self.translate is not None:
            max_dx, max_dy = float(self.translate[0] * w), float(self.translate[1] * h)
            tx = int(round(torch.empty(1).uniform_(-max_dx, max_dx).item()))
            ty = int(round(torch.empty(1).uniform_(-max_dy, max_dy).item()))
        else:
            tx = ty = 0
        scale = float(torch.empty(1).uniform_(self.scale[0], self.scale[1]).item()) if self.scale else 1.0
        shear_x = shear_y = 0.0
        if self.shear is not None:
            shear_x = float(torch.empty(1).uniform_(self.shear[0], self.shear[1]).item())
            if len(self.shear) == 4:
                shear_y = float(torch.empty(1).uniform_(self.shear[2], self.shear[3]).item())
        m = _inverse_affine_matrix([0.0, 0.0], angle, [float(tx), float(ty)], scale, (shear_x, shear_y))
        x = img if img.dim() >= 4 else img.reshape((1,) * (4 - img.dim()) + tuple(img.shape))
        lead = x.shape[:-3]
        x = x.reshape(-1, *x.shape[-3:])
        dt = x.dtype if x.is_floating_point() else torch.float32
        theta = torch.tensor(m, dtype=dt).reshape(1, 2, 3)
        base = torch.empty(1, h, w, 3, dtype=dt)
        base[..., 0].copy_(torch.linspace(-w * 0.5 + 0.5, w * 0.5 + 0.5 - 1, steps=w))
        base[..., 1].copy_(torch.linspace(-h * 0.5 + 0.5, h * 0.5 + 0.5 - 1, steps=h).unsqueeze_(-1))
        base[..., 2].fill_(1)
        grid = base.view(1, h * w, 3).bmm(theta.transpose(1, 2) / torch.tensor([0.5 * w, 0.5 * h], dtype=dt))
        grid = grid.view(1, h, w, 2).expand(x.shape[0], h, w, 2)
        out = F.grid_sample(x.to(dt), grid, mode="nearest", padding_mode="zeros", align_corners=False)
        return out.to(img.dtype).reshape(img.shape)


class GaussianBlur:
    """torchvision.transforms.GaussianBlur(kernel_size=(kx, ky), sigma=(lo, hi)) on the last two axes."""

    def __init__(self, kernel_size, sigma):
        self.kernel_size, self.sigma = kernel_size, sigma

    @staticmethod
    def _k1(ks, s):
        x = torch.linspace(-(ks - 1) * 0.5, (ks - 1) * 0.5, steps=ks)
        pdf = torch.exp(-0.5 * (x / s).pow(2))
        return pdf / pdf.sum()

    def __call__(self, img):
        s = torch.empty(1).uniform_(self.sigma[0], self.sigma[1]).item()
        kx, ky = self.kernel_size
        k2 = torch.mm(self._k1(ky, s)[:, None], self._k1(kx, s)[None, :]).to(img.dtype)
        x = img.reshape(-1, *img.shape[-3:]) if img.dim() >= 3 else img.reshape(1, 1, *img.shape)
        c = x.shape[-3]
        x = F.pad(x, [kx // 2, kx // 2, ky // 2, ky // 2], mode="reflect")
        x = F.conv2d(x, k2.expand(c, 1, ky, kx), groups=c)
        return x.reshape(img.shape)


class RandomBrightnessContrast:
    """data/augmentation_functions/brightness.py: img * alpha + beta * mean(img * alpha) (python `random`)."""

    def __init__(self, brightness_limit=0.3, contrast_limit=0.3):
        self.brightness_limit, self.contrast_limit = brightness_limit, contrast_limit

    def __call__(self, img):
        alpha = 1.0 + random.uniform(-self.contrast_limit, self.contrast_limit)
        beta = 0.0 + random.uniform(-self.brightness_limit, self.brightness_limit)
        timg = img.clone()
        timg *= alpha
        timg += beta * torch.mean(timg)
        return timg


def define_transforms(config, split):
    """data_utils.py:120-150."""
    inp, out = [], []
    if config.affine_aug and split == "train":
        inp += [RandomApply([RandomAffine(10, (0.1, 0.1), (0.95, 1.05), 10)], p=.9)]
        out += [RandomApply([RandomAffine(10, (0.1, 0.1), (0.95, 1.05), 10)], p=.9)]
    if config.brightness_aug and split == "train":
        inp += [RandomApply([RandomBrightnessContrast()], p=.9)]
        if config.task_type == "enhance":
            out += [RandomApply([RandomBrightnessContrast()], p=.9)]
    if config.gaussian_blur_aug and split == "train":
        inp += [RandomApply([GaussianBlur(kernel_size=(1, 3), sigma=(0.1, 5))], p=.15)]
    ident = torch.nn.Identity()
    return (Compose(inp) if inp else ident), (Compose(out) if out else ident)


# ------------------------------------------------------------------------------------------------- dataset
class NumpyDataset(torch.utils.data.Dataset):
    """data_base.py:20-124: (image (C, T, H, W) f32, target, subject id) per subject directory."""

    def __init__(self, config, split):
        import pandas as pd
        self.config, self.split = config, split
        self.data_loc = config.data_dir
        self.height, self.width, self.time = config.height, config.width, config.time
        self.no_in_channel, self.no_out_channel = config.no_in_channel, config.no_out_channel
        self.split_csv = config.split_csv_path
        self.task_type = config.task_type
        assert self.time >= 1, "Time arg should be greater than or equal to 1"
        assert self.no_in_channel >= 1, "Number of input channels arg should be greater than or equal to 1"
        assert self.no_out_channel >= 1, "Number of output channels arg should be greater than or equal to 1"
        self.input_transform, self.output_transform = define_transforms(config, split)
        if self.split_csv is not None:
            df = pd.read_csv(self.split_csv)
            self.split_subject_ids = list(df[df.Split.isin([self.split])].SubjectID)
        else:
            ids = [p.split("/")[-2] for p in glob.glob(os.path.join(self.data_loc, "*", "*_input.npy"))]
            n = len(ids)
            if split == "train":
                self.split_subject_ids = ids[:int(0.6 * n)]
            elif split == "val":
                self.split_subject_ids = ids[int(0.6 * n):int(0.8 * n)]
            elif split == "test":
                self.split_subject_ids = ids[int(0.8 * n):]
            else:
                raise ValueError(f"Unknown split {split} specified, should be train, val, or test")
        logging.info(f"Size of {split} dataset: {len(self.split_subject_ids)}")
        if self.task_type == "class":
            self.metadata = pd.read_csv(glob.glob(os.path.join(self.data_loc, "*_metadata.csv"))[0])

    def __getitem__(self, index):
        sid = self.split_subject_ids[index]
        path = os.path.join(self.data_loc, sid, sid + "_input.npy")
        image = np.load(path).astype("float32")
        image = custom_numpy_to_tensor(image, self.height, self.width, self.time, self.no_in_channel)
        seed = np.random.randint(2147483647)
        random.seed(seed)
        torch.manual_seed(seed)
        image = self.input_transform(image)
        if self.task_type == "seg":
            seg = np.load(path.replace("_input", "_output")).astype("float32")
            seg = custom_numpy_to_tensor(seg, self.height, self.width, self.time, 1, INTER_NEAREST)
            random.seed(seed)
            torch.manual_seed(seed)
            seg = self.output_transform(seg)[0]
            return image, seg.type(torch.LongTensor), sid
        if self.task_type == "enhance":
            out = np.load(path.replace("_input", "_output")).astype("float32")
            out = custom_numpy_to_tensor(out, self.height, self.width, self.time, self.no_out_channel)
            random.seed(seed)
            torch.manual_seed(seed)
            return image, self.output_transform(out).type(torch.FloatTensor), sid
        if self.task_type == "class":
            label = float(self.metadata[self.metadata.SubjectID.isin([sid])].Label.iloc[0])
            return image, torch.tensor(label, dtype=torch.long), sid
        raise ValueError("Unkown task type.")

    def __len__(self):
        return len(self.split_subject_ids)
