"""CPU-side checks of the C ABI library: it loads and exports every declared symbol (no GPU calls)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "minimarl.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from minimarl._lib import LIB_PATH, lib, symbols
    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    L = lib()
    declared = _header_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), f"{name} declared in include/minimarl.h but not exported"
    # every ctypes signature we bind must exist too
    for name in symbols():
        assert hasattr(L, name), name
    assert L.mm_version() >= 100


def test_qnet_offsets_match_python_layout():
    from minimarl._lib import LIB_PATH, QnetDims, c_i64, lib
    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built")
    d = QnetDims(8, 47, 64, 64, 64, 5)
    offs = (c_i64 * 11)()
    assert lib().mm_qnet_param_offsets(ctypes.byref(d), offs) == 0
    N, D, F1, G, H, A = 8, 47, 64, 64, 64, 5
    sizes = [N * F1 * D, N * F1, N * G * F1, N * G, N * 3 * H * G, N * 3 * H * H, N * 3 * H, N * 3 * H, N * A * H, N * A]
    acc = 0
    for i, s in enumerate(sizes):
        assert offs[i] == acc
        acc += s
    assert offs[10] == acc
    assert lib().mm_qnet_packed_count(ctypes.byref(d)) > acc


def test_invalid_dims_report_error():
    from minimarl._lib import LIB_PATH, QnetDims, c_i64, lib
    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built")
    d = QnetDims(8, 47, 60, 64, 64, 5)       # F1 not a multiple of 32
    offs = (c_i64 * 11)()
    assert lib().mm_qnet_param_offsets(ctypes.byref(d), offs) < 0
    assert b"multiples of 32" in lib().mm_last_error()


def test_torch_op_library_registers_every_op():
    """libminimarl_torch.so (TORCH_LIBRARY(minimarl)) loads on the CPU and registers the hot-path ops
    and the Env / PER custom classes (no GPU calls)."""
    import torch
    from minimarl.ops import TORCH_LIB_PATH, load
    if not os.path.exists(TORCH_LIB_PATH):
        pytest.skip("torch op library not built")
    ops = load()
    for name in ("qnet_pack", "agent_q_fwd", "agent_q_act", "agent_q_max", "td_error", "gae_scan", "qmix_mixer_fwd",
                 "qmix_mixer_bwd", "td_target_loss", "vdn_sum", "mappo_get_actions", "mappo_evaluate_actions"):
        schema = str(getattr(ops, name).default._schema)
        assert schema.startswith(f"minimarl::{name}("), schema
        assert "(a!)" in schema          # outputs are caller-allocated mutable arguments
    assert torch.classes.minimarl.Env is not None and torch.classes.minimarl.PER is not None
    # workspace size queries run on the host (no tensors): Mix_Net of qmix/_network.py at the golden shapes
    # (N 8, state 8 x 47, Hm 32, k1 32) and evaluate_actions of 7 chunks x 5 steps
    ws = ops.qmix_mixer_workspace([8, 376, 32, 32], 32)
    assert ws >= 32 * (6 * 32 + 8 * 32 + 3 * 32 + 1)
    assert ops.mappo_evaluate_workspace([47, 32, 5], 35) >= 2 * 64 * (8 + 8 * 32 + 1)
