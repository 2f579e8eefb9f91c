"""Checkpoints that carry the pruner's masks.

The reference saves {epoch, arch, state_dict, best_miou, optimizer, dataset} with torch.save and
copies the best one (semantic_seg.py:286-290, called at :1085-1092) but never the masks: a resumed
SRMB run (unseeded np.random, SRMBRepMasker.py:102-334) or pr_static run re-draws different masks.
Here the masks go next to the checkpoint in the compact form of Pruner.save_masks (SRMB masks as
their period-tile factors, everything else 1 bit per weight), and resume() restores both.

  save_checkpoint(state, is_best, save_dir=".", filename="checkpoint.pth.tar", pruner=None)
  resume(path, model, optimizer=None, pruner=None) -> state
"""
from __future__ import annotations

import os
import shutil

import torch


def mask_path(checkpoint_path: str) -> str:
    return checkpoint_path + ".masks.npz"


def save_checkpoint(state, is_best, save_dir=".", filename="checkpoint.pth.tar", pruner=None):
    """semantic_seg.py:286-290, plus the pruner's masks (<checkpoint>.masks.npz); the best copy
    (checkpoint_best.pth.tar) gets its masks copied too."""
    fpath = os.path.join(save_dir, filename)
    torch.save(state, fpath)
    if pruner is not None:
        pruner.save_masks(mask_path(fpath))
    if is_best:
        best = os.path.join(save_dir, "checkpoint_best.pth.tar")
        shutil.copyfile(fpath, best)
        if pruner is not None:
            shutil.copyfile(mask_path(fpath), mask_path(best))


def resume(path, model, optimizer=None, pruner=None):
    """The reference's --resume (semantic_seg.py:973-990) with the masks restored instead of
    re-drawn: loads the state dict (weights_only -- no code runs from the file), the optimizer
    state if given, and the pruner's masks if the checkpoint has them.  Returns the state."""
    state = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(state["state_dict"])
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    if pruner is not None:
        mp = mask_path(path)
        if not os.path.exists(mp):
            raise FileNotFoundError(f"{mp}: this checkpoint was saved without masks")
        pruner.load_masks(mp)
    return state


__all__ = ["save_checkpoint", "resume", "mask_path"]
