"""Loader restatement (long_context_biomedical_imaging_amd/data.py) of data/data_base.py + data/data_utils.py.

OpenCV and torchvision are absent here, so resizing and augmentation are checked against their published
semantics (hand-computed values, invariants), not against the libraries: parity unpinned for those two.
The layout handling (H x W [x D] [x C] -> (C, T, H, W)), centre pad/crop, split logic, task-type targets and the
shared-seed image/mask augmentation are checked directly."""
import numpy as np
import pandas as pd
import pytest
import torch

from long_context_biomedical_imaging_amd import config as lconfig
from long_context_biomedical_imaging_amd import data


def test_resize_cv2_linear_and_nearest():
    img = np.array([[0.0, 1.0], [2.0, 3.0]], dtype=np.float32)
    t = data.custom_numpy_to_tensor(img, 4, 4, 1, 1)
    assert t.shape == (1, 1, 4, 4)
    # half-pixel bilinear: source x = (dst + 0.5) / 2 - 0.5 -> -0.25, 0.25, 0.75, 1.25 (clamped)
    np.testing.assert_allclose(t[0, 0, 0].numpy(), [0.0, 0.25, 0.75, 1.0], atol=1e-6)
    np.testing.assert_allclose(t[0, 0, :, 0].numpy(), [0.0, 0.5, 1.5, 2.0], atol=1e-6)
    n = data.custom_numpy_to_tensor(img, 4, 4, 1, 1, data.INTER_NEAREST)
    np.testing.assert_array_equal(n[0, 0].numpy(), [[0, 0, 1, 1], [0, 0, 1, 1], [2, 2, 3, 3], [2, 2, 3, 3]])


@pytest.mark.parametrize("shape,h,w,t,c,out", [
    ((6, 5), 6, 5, 1, 1, (1, 1, 6, 5)),
    ((6, 5, 1), 6, 5, 1, 1, (1, 1, 6, 5)),
    ((6, 5, 1, 1), 6, 5, 1, 1, (1, 1, 6, 5)),
    ((6, 5, 3), 6, 5, 1, 3, (3, 1, 6, 5)),
    ((6, 5, 3), 12, 10, 1, 3, (3, 1, 12, 10)),
    ((6, 5, 4), 6, 5, 8, 1, (1, 8, 6, 5)),       # depth padded 4 -> 8 (2 + 2)
    ((6, 5, 9), 3, 4, 4, 1, (1, 4, 3, 4)),       # depth cropped 9 -> 4 (centre), H/W resized
    ((6, 5, 4, 2), 6, 5, 6, 2, (2, 6, 6, 5)),
])
def test_layouts(shape, h, w, t, c, out):
    rng = np.random.default_rng(0)
    img = rng.standard_normal(shape).astype(np.float32)
    r = data.custom_numpy_to_tensor(img, h, w, t, c)
    assert tuple(r.shape) == out
    if shape == (6, 5, 4):
        np.testing.assert_array_equal(r[0, 2:6].numpy(), np.moveaxis(img, 2, 0))
        assert float(r[0, :2].abs().sum()) == 0.0 and float(r[0, 6:].abs().sum()) == 0.0
    if shape == (6, 5, 3) and h == 6:
        np.testing.assert_array_equal(r[:, 0].numpy(), np.moveaxis(img, 2, 0))


def test_layout_errors_match_reference():
    with pytest.raises(ValueError):
        data.custom_numpy_to_tensor(np.zeros((4, 4), np.float32), 4, 4, 1, 3)
    with pytest.raises(ValueError):
        data.custom_numpy_to_tensor(np.zeros((4, 4, 2), np.float32), 4, 4, 2, 3)
    with pytest.raises(ValueError):                      # OpenCV cannot resize a 4-D array
        data.custom_numpy_to_tensor(np.zeros((4, 4, 2, 1), np.float32), 8, 8, 2, 1)


def _write(tmp, n, shape, seg=True):
    rng = np.random.default_rng(1)
    for i in range(n):
        d = tmp / f"s{i:02d}"
        d.mkdir()
        np.save(d / f"s{i:02d}_input.npy", rng.standard_normal(shape).astype(np.float32))
        if seg:
            np.save(d / f"s{i:02d}_output.npy", rng.integers(0, 3, shape).astype(np.float32))


def _cfg(tmp, *extra):
    return lconfig.parse_config(["--data_dir", str(tmp), "--height", "16", "--width", "16", "--time", "1",
                                 "--no_out_channel", "3", *extra])


def test_dataset_splits_and_seg_targets(tmp_path):
    _write(tmp_path, 10, (16, 16))
    cfg = _cfg(tmp_path, "--affine_aug", "False", "--brightness_aug", "False", "--gaussian_blur_aug", "False")
    sizes = {s: len(data.NumpyDataset(cfg, s)) for s in ("train", "val", "test")}
    assert sizes == {"train": 6, "val": 2, "test": 2}
    ds = data.NumpyDataset(cfg, "train")
    img, seg, sid = ds[0]
    assert img.shape == (1, 1, 16, 16) and img.dtype == torch.float32
    assert seg.shape == (1, 16, 16) and seg.dtype == torch.long
    ref = np.load(tmp_path / sid / f"{sid}_output.npy")
    np.testing.assert_array_equal(seg[0].numpy(), ref.astype(np.int64))
    with pytest.raises(ValueError):
        data.NumpyDataset(cfg, "holdout")


def test_split_csv_and_class_labels(tmp_path):
    _write(tmp_path, 4, (16, 16), seg=False)
    pd.DataFrame({"SubjectID": ["s00", "s01", "s02", "s03"], "Split": ["train", "val", "train", "test"]}).to_csv(
        tmp_path / "split.csv", index=False)
    pd.DataFrame({"SubjectID": ["s00", "s01", "s02", "s03"], "Label": [1, 0, 2, 1]}).to_csv(
        tmp_path / "x_metadata.csv", index=False)
    cfg = _cfg(tmp_path, "--split_csv_path", str(tmp_path / "split.csv"), "--task_type", "class")
    ds = data.NumpyDataset(cfg, "train")
    assert ds.split_subject_ids == ["s00", "s02"]
    assert int(ds[1][1]) == 2


def test_augmentation_shares_the_affine_between_image_and_mask(tmp_path):
    """With brightness/blur off, an image equal to its label map stays equal after the (shared-seed) affine."""
    d = tmp_path / "s00"
    d.mkdir()
    lab = np.random.default_rng(2).integers(0, 3, (16, 16)).astype(np.float32)
    np.save(d / "s00_input.npy", lab)
    np.save(d / "s00_output.npy", lab)
    for i in range(1, 5):                                 # 60 % of 5 subjects -> 3 in train, s00 among them
        (tmp_path / f"s{i:02d}").mkdir()
        np.save(tmp_path / f"s{i:02d}" / f"s{i:02d}_input.npy", lab)
        np.save(tmp_path / f"s{i:02d}" / f"s{i:02d}_output.npy", lab)
    cfg = _cfg(tmp_path, "--brightness_aug", "False", "--gaussian_blur_aug", "False")
    ds = data.NumpyDataset(cfg, "train")
    changed = 0
    np.random.seed(0)
    for _ in range(8):
        img, seg, _ = ds[0]
        assert torch.equal(img[0].long(), seg)
        changed += int(not torch.equal(seg[0], torch.from_numpy(lab).long()))
    assert changed > 0                                    # p = 0.9 per draw: the affine did apply


def test_affine_identity_and_blur_normalisation():
    torch.manual_seed(0)
    x = torch.rand(2, 3, 9, 11)
    aff = data.RandomAffine(0, (0.0, 0.0), (1.0, 1.0), 0)
    assert torch.equal(aff(x), x)                         # zero angle/shift/shear, unit scale: identity grid
    blur = data.GaussianBlur((1, 3), (0.1, 5))
    c = torch.full((2, 3, 9, 11), 2.5)
    assert torch.allclose(blur(c), c)                     # normalised kernel, reflect padding
