"""Checkpoint loading, drop-in for utils/ckpt_utils.py:8-68.

``load_ckpt(model, ckpt_dir_or_file, 'model')`` fills the GPU modules of this
package (``ProDiffTeacher``, ``GaussianDiffusion``/``WaveNet``, ...) from the
reference's training checkpoints: the newest ``model_ckpt_steps_<N>.ckpt`` of a
directory (or an explicit file), ``checkpoint['state_dict']`` either flat with
``<model_name>.`` prefixes (Lightning-style, stripped here) or nested
``{model_name: state_dict}``, optional ``strict=False`` shape filtering.  The
parameters are then packed into the HIP kernels' layouts on the next call (the
modules re-pack whenever a parameter tensor changes).

Difference from the reference: files load with ``torch.load(weights_only=True)``
(tensors and plain containers only, nothing unpickled is executed); a checkpoint
that needs arbitrary unpickling is refused with the loader's error.  The only
non-container globals allowed are numpy's scalar reconstructor and dtypes: the
reference trainer stores ``checkpoint_callback_best`` as a numpy scalar once it
resumes (``np.load(best_valid.npy)[0]``, utils/pl_utils.py:321,751), and such a
value is data, not code.
The vocoder layouts live beside their vocoders: FastDiff ``config.yaml`` +
``['state_dict']['model']`` (prodiff_amd.vocoder.load_fastdiff_model, reference
component/vocoder/fastdiff.py:17-41) and NSF-HiFiGAN ``config.json`` +
``['generator']`` (prodiff_amd.nsf_hifigan.load_model, modules/nsf_hifigan/models.py:21-36).
"""
from __future__ import annotations

import glob
import logging
import os
import re

import torch


def _numpy_safe_globals():
    import numpy as np
    try:
        from numpy._core.multiarray import scalar
    except ImportError:                     # numpy < 2
        from numpy.core.multiarray import scalar
    dtypes = [np.dtype] + [type(np.dtype(t)) for t in (np.float64, np.float32, np.float16, np.int64, np.int32,
                                                         np.int16, np.int8, np.uint8, np.bool_)]
    return [scalar] + dtypes


def _load(path):
    with torch.serialization.safe_globals(_numpy_safe_globals()):
        return torch.load(path, map_location="cpu", weights_only=True)


def get_all_ckpts(work_dir, steps=None):
    """ckpt_utils.py:20-26: newest step first."""
    pat = f"{work_dir}/model_ckpt_steps_*.ckpt" if steps is None else f"{work_dir}/model_ckpt_steps_{steps}.ckpt"
    return sorted(glob.glob(pat), key=lambda x: -int(re.findall(r".*steps_(\d+)\.ckpt", x)[0]))


def get_last_checkpoint(work_dir, steps=None):
    """ckpt_utils.py:8-17."""
    paths = get_all_ckpts(work_dir, steps)
    if not paths:
        return None, None
    logging.info(f"load module from checkpoint: {paths[0]}")
    return _load(paths[0]), paths[0]


def extract_state_dict(checkpoint, model_name="model"):
    """The sub-state-dict of ``model_name`` (ckpt_utils.py:37-48)."""
    sd = checkpoint["state_dict"]
    if any("." in k for k in sd):
        return {k[len(model_name) + 1:]: v for k, v in sd.items() if k.startswith(f"{model_name}.")}
    if "." not in model_name:
        return sd[model_name]
    base = model_name.split(".")[0]
    rest = model_name[len(base) + 1:]
    return {k[len(rest) + 1:]: v for k, v in sd[base].items() if k.startswith(f"{rest}.")}


def load_ckpt(cur_model, ckpt_base_dir, model_name="model", force=True, strict=True):
    """ckpt_utils.py:28-68."""
    if os.path.isfile(ckpt_base_dir):
        base_dir, ckpt_path = os.path.dirname(ckpt_base_dir), ckpt_base_dir
        checkpoint = _load(ckpt_base_dir)
    else:
        base_dir = ckpt_base_dir
        checkpoint, ckpt_path = get_last_checkpoint(ckpt_base_dir)
    if checkpoint is None:
        msg = f"| ckpt not found in {base_dir}."
        if force:
            raise AssertionError(msg)
        print(msg)
        return
    state_dict = extract_state_dict(checkpoint, model_name)
    if not strict:
        cur = cur_model.state_dict()
        bad = [k for k, p in state_dict.items() if k in cur and cur[k].shape != p.shape]
        for k in bad:
            print("| Unmatched keys: ", k, cur[k].shape, state_dict[k].shape)
        state_dict = {k: v for k, v in state_dict.items() if k not in bad}
    cur_model.load_state_dict(state_dict, strict=strict)
    print(f"| load '{model_name}' from '{ckpt_path}'.")
