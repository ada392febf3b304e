"""CPU: the checkpoint container (safetensors + JSON metadata) round-trips component tensors and
rejects mismatched components (no GPU needed)."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
from minimarl.checkpoint import load_checkpoint, save_checkpoint  # noqa: E402


class Comp:
    def __init__(self, n, fill):
        self.a = torch.full((n,), float(fill))
        self.s = torch.zeros(1)
        self.count = 0

    def checkpoint_tensors(self):
        return {"a": self.a, "s": self.s}, {"count": self.count}

    def restore_tensors(self, ts, scalars):
        from minimarl.checkpoint import copy_into
        copy_into(self.a, ts["a"], "a")
        copy_into(self.s, ts["s"], "s")
        self.count = scalars["count"]


class Other(Comp):
    pass


def test_round_trip(tmp_path):
    a = Comp(10, 3.5)
    a.s += 7
    a.count = 42
    p = str(tmp_path / "c.safetensors")
    save_checkpoint(p, x=a)
    b = Comp(10, 0)
    meta = load_checkpoint(p, x=b)
    assert meta["x"]["kind"] == "Comp"
    assert torch.equal(a.a, b.a) and torch.equal(a.s, b.s) and b.count == 42


def test_mismatch_rejected(tmp_path):
    p = str(tmp_path / "c.safetensors")
    save_checkpoint(p, x=Comp(10, 1))
    with pytest.raises(ValueError):
        load_checkpoint(p, x=Comp(11, 0))
    with pytest.raises(TypeError):
        load_checkpoint(p, x=Other(10, 0))
    with pytest.raises(KeyError):
        load_checkpoint(p, y=Comp(10, 0))
