"""Checkpoint / resume of the device-resident learner state.

The reference declares ``--save_interval`` / ``--model_dir`` but its save step is empty
(offpolicy/runner/shared/base_runner.py:207-209) and nothing is ever loaded, so there is no file
format to match: checkpoints here are one safetensors file (tensors only, loaded without
executing anything from the file) holding every component's named device tensors, plus a JSON
metadata string (component kinds and scalar counters).

Supported components (``checkpoint_tensors()`` / ``restore_tensors()`` protocol):
  QLearner      behavior [agent | mixer] parameters, target agent / mixer, Adam m / v / step
  OffQMix       behavior + target [agent | mixer], Adam m / v / step
  MappoTrainer  actor / critic parameters, both Adam states, ValueNorm running statistics
"""
import json

import torch
from safetensors.torch import load_file, save_file


def save_checkpoint(path, **components):
    """save_checkpoint("run.safetensors", learner=ql, offq=tr, mappo=mt)."""
    tensors, meta = {}, {}
    for name, obj in components.items():
        ts, scalars = obj.checkpoint_tensors()
        for k, v in ts.items():
            tensors[f"{name}/{k}"] = v.detach().contiguous().cpu()
        meta[name] = {"kind": type(obj).__name__, "scalars": scalars}
    save_file(tensors, path, metadata={"minimarl": json.dumps(meta)})


def load_checkpoint(path, **components):
    """Restore the named components in place (shapes and kinds must match the saved ones)."""
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        meta = json.loads(f.metadata()["minimarl"])
    tensors = load_file(path)
    for name, obj in components.items():
        if name not in meta:
            raise KeyError(f"checkpoint has no component {name!r} (has {sorted(meta)})")
        if meta[name]["kind"] != type(obj).__name__:
            raise TypeError(f"component {name!r} was saved from {meta[name]['kind']}, not {type(obj).__name__}")
        pre = name + "/"
        obj.restore_tensors({k[len(pre):]: v for k, v in tensors.items() if k.startswith(pre)},
                            meta[name]["scalars"])
    return meta


def copy_into(dst: torch.Tensor, src: torch.Tensor, what: str):
    if tuple(dst.shape) != tuple(src.shape):
        raise ValueError(f"checkpoint tensor {what}: shape {tuple(src.shape)} != {tuple(dst.shape)}")
    dst.copy_(src.to(device=dst.device, dtype=dst.dtype))
