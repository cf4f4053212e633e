"""Config / flag surface — the subset of the reference's argparse surface that selects and sizes the mixers.

Mirrors /root/reference/setup/config_utils.py (Nestedspace :9-21, check_args :89-141) and
setup/parsers/model_parser.py (--ViT.*, --Swin.* :29-47), plus the general flags the model and the
training step read (--encoder_name, --decoder_name, --task_type, --height/--width/--time,
--no_in_channel/--no_out_channel, --batch_size, --use_amp, --ddp, --optim.*).
"""
from __future__ import annotations

import argparse
import os


class Nestedspace(argparse.Namespace):
    """Dotted names become nested namespaces: `--ViT.size small` -> config.ViT.size."""

    def __setattr__(self, name, value):
        if "." in name:
            group, name = name.split(".", 1)
            ns = getattr(self, group, Nestedspace())
            setattr(ns, name, value)
            self.__dict__[group] = ns
        else:
            self.__dict__[name] = value

    def __getattr__(self, name):
        if "." in name:
            group, name = name.split(".", 1)
            try:
                ns = self.__dict__[group]
            except KeyError:
                raise AttributeError(name)
            return getattr(ns, name)
        raise AttributeError(name)


def str_to_bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("Boolean value expected.")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("lcimg")
    p.add_argument("--encoder_name", type=str, default="ViT", choices=["ViT", "Swin", "Identity"])
    p.add_argument("--decoder_name", type=str, default="ViTUNETR")
    p.add_argument("--task_type", type=str, default="seg", choices=["class", "seg", "enhance"])
    p.add_argument("--loss_func", type=str, default="CrossEntropy", choices=["CrossEntropy", "MSE"])
    p.add_argument("--height", type=int, default=512)
    p.add_argument("--width", type=int, default=512)
    p.add_argument("--time", type=int, default=1)
    p.add_argument("--no_in_channel", type=int, default=1)
    p.add_argument("--no_out_channel", type=int, default=2)
    p.add_argument("--batch_size", type=int, default=2)
    # general_parser.py:31-32, 70-72 (data.NumpyDataset)
    p.add_argument("--data_dir", type=str, default="data")
    p.add_argument("--split_csv_path", type=lambda v: None if v in (None, "None", "none") else v, default=None)
    p.add_argument("--affine_aug", type=str_to_bool, default=True)
    p.add_argument("--brightness_aug", type=str_to_bool, default=True)
    p.add_argument("--gaussian_blur_aug", type=str_to_bool, default=True)
    p.add_argument("--use_amp", action="store_true")
    p.add_argument("--ddp", action="store_true")
    p.add_argument("--optim_type", type=str, default="adam", choices=["adam", "adamw", "sgd", "nadam"])
    p.add_argument("--optim.lr", type=float, default=1e-4)
    p.add_argument("--optim.weight_decay", type=float, default=0.0)
    p.add_argument("--optim.beta1", type=float, default=0.90)
    p.add_argument("--optim.beta2", type=float, default=0.95)
    # general_parser.py:109-110 (trainer_base.py:168-176)
    p.add_argument("--clip_grad_norm", type=float, default=0.0)
    p.add_argument("--iters_to_accumulate", type=int, default=1)
    # model_parser.py:29-37
    p.add_argument("--ViT.size", type=str, default="small", choices=["small", "base", "custom"])
    p.add_argument("--ViT.patch_size", nargs="+", type=int, default=[16, 16, 16])
    p.add_argument("--ViT.hidden_size", type=int, default=768)
    p.add_argument("--ViT.mlp_dim", type=int, default=3072)
    p.add_argument("--ViT.num_layers", type=int, default=12)
    p.add_argument("--ViT.num_heads", type=int, default=12)
    p.add_argument("--ViT.use_hyena", type=str_to_bool, default=False)
    p.add_argument("--ViT.use_mamba", type=str_to_bool, default=False)
    # not a reference flag: opt-in Hyena filter length (the reference hard-codes 66000, backbone_vit.py:172, and
    # raises for longer sequences, hyena.py:314); needed for configs[3] (1024^2 patch 2, L = 262144)
    p.add_argument("--ViT.hyena_l_max", type=int, default=66000)
    # model_parser.py:39-47
    p.add_argument("--Swin.size", type=str, default="tiny", choices=["unetr", "tiny", "small", "base", "large", "custom"])
    p.add_argument("--Swin.patch_size", nargs="+", type=int, default=[2, 2, 2])
    p.add_argument("--Swin.window_size", nargs="+", type=int, default=[8, 8, 8])
    p.add_argument("--Swin.embed_dim", type=int, default=24)
    p.add_argument("--Swin.depths", nargs="+", type=int, default=[2, 2, 6, 2])
    p.add_argument("--Swin.num_heads", nargs="+", type=int, default=[3, 6, 12, 24])
    p.add_argument("--Swin.use_hyena", type=str_to_bool, default=False)
    p.add_argument("--Swin.use_mamba", type=str_to_bool, default=False)
    return p


def check_args(config):
    """The parts of config_utils.check_args (:89-141) that affect the model."""
    if "LOCAL_RANK" in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        config.ddp = True
    for enc in ("ViT", "Swin"):
        ns = getattr(config, enc, None)
        if ns is None:
            continue
        if len(ns.patch_size) == 1:
            ns.patch_size = ns.patch_size * 3
        if enc == "Swin" and len(ns.window_size) == 1:
            ns.window_size = ns.window_size * 3
        if ns.use_hyena and ns.use_mamba:
            raise ValueError(f"Cannot use both hyena and mamba in {enc}")
    return config


def parse_config(argv=None):
    cfg = build_parser().parse_args(argv, namespace=Nestedspace())
    return check_args(cfg)
