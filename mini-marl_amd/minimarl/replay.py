"""Device-resident prioritized chunk replay (csrc/per.hip).

Mirrors ``Prioritized_Experience_Replay`` (vdn/replay_buffer/buffer.py:10-90,
qmix/replay_buffer/per.py:10-81): ``collect_sample`` / ``sample`` / ``update`` with
the sum tree kept in HBM (f64, reference heap layout). Chunk payloads live in a
``ChunkStore`` (engine.py); this class manages priorities and slot -> row mapping.
"""
import ctypes

import torch

from ._lib import release, MM_PER_QMIX, MM_PER_VDN, c_vp, check, lib
from .qnet import ptr, stream_handle


class DevicePER:
    def __init__(self, capacity, flavor="vdn", alpha=0.4, beta=0.4, eps=1e-6, step_weight=0.99,
                 use_step_weight=True, update_alpha_beta=True, max_episodes=30000, update_iter=10,
                 device="cuda"):
        self.capacity = int(capacity)
        self.device = torch.device(device)
        fl = MM_PER_VDN if flavor == "vdn" else MM_PER_QMIX
        if update_alpha_beta:
            ai = (1 - alpha) / (max_episodes * update_iter)
            bi = (1 - beta) / (max_episodes * update_iter)
        else:
            ai = bi = 0.0
        h = c_vp()
        check(lib().mm_per_create(self.capacity, fl, alpha, beta, eps, step_weight, int(use_step_weight), ai, bi,
                                  ctypes.byref(h)), "per_create")
        self._h = h

    @classmethod
    def from_args(cls, args, flavor, device="cuda"):
        """Build from a reference-style args namespace (buffer_limit, alpha, beta, eps, ...)."""
        return cls(args.buffer_limit, flavor, args.alpha, args.beta, args.eps, getattr(args, "step_weight", 0.99),
                   getattr(args, "use_step_weight", flavor == "vdn"), args.update_alpha_beta, args.max_episodes,
                   args.update_iter, device)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._h = None
            try:
                release("mm_per_destroy", h)   # deferred while a graph capture is running
            except Exception:   # interpreter shutdown: module globals already gone
                pass

    @property
    def alpha(self):
        """Current alpha (the device value: graph-replayed sample calls anneal it on the device)."""
        return self.device_scalars()[1]

    @property
    def beta(self):
        return self.device_scalars()[2]

    def device_scalars(self):
        """(fill count, alpha, beta, alpha_inc, beta_inc, sample calls) read from the device (syncs)."""
        ts, sc = self.checkpoint_tensors()
        return [float(x) for x in ts["scalars"]]

    # ------------------------------------------------------------------ checkpoint (minimarl.checkpoint)
    def checkpoint_tensors(self):
        tree = torch.empty(2 * self.capacity - 1, dtype=torch.float64, device=self.device)
        rows = torch.empty(self.capacity, dtype=torch.int64, device=self.device)
        sc = (ctypes.c_double * 6)()
        check(lib().mm_per_save_state(self._h, ptr(tree), ptr(rows), sc, stream_handle(self.device)), "per_save_state")
        return {"tree": tree, "slot_rows": rows, "scalars": torch.tensor(list(sc), dtype=torch.float64)}, {}

    def restore_tensors(self, ts, scalars=None):
        from .checkpoint import copy_into
        tree = torch.empty(2 * self.capacity - 1, dtype=torch.float64, device=self.device)
        rows = torch.empty(self.capacity, dtype=torch.int64, device=self.device)
        copy_into(tree, ts["tree"], "tree")
        copy_into(rows, ts["slot_rows"], "slot_rows")
        sc = (ctypes.c_double * 6)(*[float(x) for x in ts["scalars"]])
        check(lib().mm_per_load_state(self._h, ptr(tree), ptr(rows), sc, stream_handle(self.device)), "per_load_state")

    def __len__(self):
        return int(lib().mm_per_size(self._h))

    def n_mirror_add(self, k):
        """Keep the host mirror of the fill count in step after graph-replayed inserts."""
        lib().mm_per_set_size_host(self._h, min(self.capacity, len(self) + int(k)))

    def tree(self):
        """Copy of the sum tree [2*cap-1] f64 (device)."""
        out = torch.empty(2 * self.capacity - 1, dtype=torch.float64, device=self.device)
        check(lib().mm_per_copy_tree(self._h, ptr(out), stream_handle(self.device)), "per_copy_tree")
        return out

    def slot_rows(self):
        """Copy of the slot -> chunk-store row table [cap] int64 (device)."""
        out = torch.empty(self.capacity, dtype=torch.int64, device=self.device)
        check(lib().mm_per_copy_slot_rows(self._h, ptr(out), stream_handle(self.device)), "per_copy_rows")
        return out

    def error_word(self, clear=False):
        """Sticky device error bits (synchronous): 1 = a priority update named a node outside the
        leaves; the kernel skipped it (the reference's tree write would raise / corrupt a node)."""
        out = ctypes.c_int32(0)
        check(lib().mm_per_error_word(self._h, ctypes.byref(out), int(bool(clear)), stream_handle(self.device)),
              "per_error_word")
        return int(out.value)

    def check_errors(self):
        """Raise IndexError if a device-side priority update was given an out-of-range node."""
        e = self.error_word(clear=True)
        if e & 1:
            raise IndexError("PER update: tree node outside the leaf range [cap-1, 2cap-1) (skipped on device)")

    def slot_rows_ptr(self):
        return lib().mm_per_slot_rows(self._h)

    def add(self, td, rows_inout=None):
        """Insert K chunks (td [K] f32 device) -> data slots [K] (int64 device)."""
        td = td.to(self.device, torch.float32).contiguous()
        slots = torch.empty(td.numel(), dtype=torch.int64, device=self.device)
        check(lib().mm_per_insert(self._h, ptr(td), td.numel(), ptr(rows_inout), ptr(slots),
                                  stream_handle(self.device)), "per_insert")
        return slots

    def sample(self, batch, fracs=None, seed=0, counter=0):
        """-> (tree nodes [B], data slots [B], IS weights [B]) all on device."""
        nodes = torch.empty(batch, dtype=torch.int64, device=self.device)
        slots = torch.empty(batch, dtype=torch.int64, device=self.device)
        w = torch.empty(batch, dtype=torch.float32, device=self.device)
        if fracs is not None:
            fr = torch.as_tensor(fracs, dtype=torch.float64).to(self.device).contiguous()
            check(lib().mm_per_sample(self._h, batch, ptr(fr), ptr(nodes), ptr(slots), ptr(w),
                                      stream_handle(self.device)), "per_sample")
        else:
            check(lib().mm_per_sample_rng(self._h, batch, seed, counter, ptr(nodes), ptr(slots), ptr(w),
                                          stream_handle(self.device)), "per_sample_rng")
        return nodes, slots, w

    def update(self, nodes, td):
        td = td.to(self.device, torch.float32).contiguous().view(-1)
        check(lib().mm_per_update(self._h, ptr(nodes), ptr(td), td.numel(), stream_handle(self.device)),
              "per_update")
