"""Checkpoint save / load (model/model_utils.py:13-77): same file layout ({epoch, config, optim_state,
sched_state, model_state}, `<log_dir>/<run_name>/models/<name>.pth`) and the same DDP `module.` prefix
reconciliation, so checkpoints move between the reference and this package in both directions (state_dict keys
are identical, tests/test_modules_cpu.py).

One deliberate difference: the config is stored as a plain nested dict (the reference pickles its Namespace),
so `load_model` can use `torch.load(weights_only=True)` — nothing in the file is executed. A checkpoint written
by the reference itself holds a pickled Namespace; pass `weights_only=False` only for files you trust.
"""
from __future__ import annotations

import logging
import os

import torch


def _plain(obj):
    if hasattr(obj, "__dict__") and not isinstance(obj, torch.Tensor):
        return {k: _plain(v) for k, v in vars(obj).items()}
    if isinstance(obj, (list, tuple)):
        return [_plain(v) for v in obj]
    return obj


def save_model(config, model, save_dir=None, save_filename=None, epoch=None, optim=None, sched=None):
    if save_dir is None:
        save_dir = os.path.join(config.log_dir, config.run_name, "models")
    if save_filename is None:
        save_filename = f"model_epoch_{epoch}" if epoch is not None else "model"
    os.makedirs(save_dir, exist_ok=True)
    path = os.path.join(save_dir, save_filename + ".pth")
    logging.info(f"Saving entire model at {path}")
    save_dict = {"epoch": epoch, "config": _plain(config)}
    if optim is not None:
        save_dict["optim_state"] = optim.state_dict()
    if sched is not None:
        save_dict["sched_state"] = sched.state_dict()
    save_dict["model_state"] = model.state_dict()
    torch.save(save_dict, path)
    return path


def load_model(model, full_load_path, device=torch.device("cpu"), weights_only: bool = True):
    assert os.path.exists(full_load_path), f"Specified load path {full_load_path} does not exist"
    logging.info(f"Loading model weights from {full_load_path}")
    saved = torch.load(full_load_path, map_location=device, weights_only=weights_only)
    state = saved["model_state"]
    ex_saved, ex_cur = next(iter(state)), next(iter(model.state_dict()))
    if "module" in ex_cur and "module" not in ex_saved:
        state = {f"module.{k}": v for k, v in state.items()}
    elif "module" not in ex_cur and "module" in ex_saved:
        state = {k.replace("module.", ""): v for k, v in state.items()}
    model.load_state_dict(state)
    return model
