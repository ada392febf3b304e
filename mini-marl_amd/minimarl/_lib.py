"""ctypes binding of libminimarl.so (the C ABI declared in include/minimarl.h).

This is the product path: it loads the in-tree HIP library and fails loudly if it
is missing — there is no CPU fallback anywhere in ``minimarl``.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libminimarl.so")
# (A/B tools that load another build of the library assign LIB_PATH before the first lib() call)

c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_vp = ctypes.c_void_p

MM_Q_NONE, MM_Q_ACT, MM_Q_MAX, MM_Q_GATHER = 0, 1, 2, 3
MM_PER_VDN, MM_PER_QMIX = 0, 1
MM_LOSS_MIX_SUM, MM_LOSS_HUBER, MM_LOSS_TARGET_SUM = 1, 2, 4


class QnetDims(ctypes.Structure):
    _fields_ = [("n_agents", c_i32), ("obs_dim", c_i32), ("f1", c_i32), ("g", c_i32), ("h", c_i32),
                ("n_actions", c_i32)]


class QFwdIO(ctypes.Structure):
    _fields_ = [
        ("obs", c_vp), ("obs_se", c_i64), ("obs_sa", c_i64), ("obs_off", c_i64),
        ("obs_row", c_vp), ("reset_obs", c_vp),
        ("h_in", c_vp), ("hin_se", c_i64), ("hin_sa", c_i64), ("hin_sf", c_i64),
        ("h_out", c_vp), ("hout_se", c_i64), ("hout_sa", c_i64), ("hout_sf", c_i64),
        ("reset", c_vp),
        ("q_out", c_vp), ("q_se", c_i64), ("q_sa", c_i64),
        ("mode", c_i32),
        ("epsilon", c_f32), ("u", c_vp), ("rand_act", c_vp), ("seed", c_u64), ("counter", c_u64),
        ("act_out", c_vp),
        ("act_in", c_vp), ("act_se", c_i64),
        ("qsel_out", c_vp),
        ("eps_ptr", c_vp), ("counter_ptr", c_vp),
        ("save", c_vp),
        ("gi", c_vp),
    ]


class RollStepIO(ctypes.Structure):
    """mm_rollout_step_io (include/minimarl.h)"""
    _fields_ = [
        ("act", c_vp), ("store_obs", c_vp), ("row_stride", c_i64), ("slot", c_i32), ("chunk_len", c_i32),
        ("begin", c_i32), ("staging", c_vp), ("cur_row", c_vp), ("rew", c_vp), ("done", c_vp),
        ("state_in", c_i32), ("counter", c_vp),
        ("td_on", c_i32), ("td_slot", c_i32), ("gamma", c_f32),
        ("td_rew", c_vp), ("td_done", c_vp), ("td_qsel", c_vp), ("td_maxq", c_vp), ("td_act", c_vp),
        ("chunk_td", c_vp), ("store_act", c_vp), ("store_rew", c_vp), ("store_done", c_vp),
        ("n_rows", c_i64), ("err", c_vp),
    ]


class RollChunkIO(ctypes.Structure):
    """mm_rollout_chunk_io (include/minimarl.h)"""
    _fields_ = [
        ("store_obs", c_vp), ("row_stride", c_i64), ("n_rows", c_i64), ("staging", c_vp), ("cur_row", c_vp),
        ("c0", c_i32), ("n_steps", c_i32), ("chunk_len", c_i32), ("n_sets", c_i32),
        ("set0", c_i32), ("ring_len", c_i32), ("ring_pos", c_i32), ("handoff_len", c_i32),
        ("act0", c_vp), ("done_prev", c_vp), ("rew", c_vp), ("done", c_vp),
        ("counter", c_vp), ("ctl", c_vp), ("handoff", c_vp), ("err", c_vp),
    ]


class EnvCfg(ctypes.Structure):
    _fields_ = [("n_agents", c_i32), ("max_steps", c_i32), ("full_observable", c_i32), ("cols", c_i32),
                ("step_cost", c_f32)]


# (name, restype, argtypes) for every entry point of include/minimarl.h (+ extended ones)
_SIGS = [
    ("mm_last_error", ctypes.c_char_p, []),
    ("mm_version", c_i32, []),
    ("mm_qnet_param_offsets", c_i32, [ctypes.POINTER(QnetDims), ctypes.POINTER(c_i64)]),
    ("mm_qnet_packed_count", c_i64, [ctypes.POINTER(QnetDims)]),
    ("mm_qnet_pack", c_i32, [ctypes.POINTER(QnetDims), c_vp, c_vp, c_vp]),
    ("mm_qnet_pack_f32", c_i32, [ctypes.POINTER(QnetDims), c_vp, c_vp, c_vp]),
    ("mm_agent_q_fwd", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_i64, c_vp]),
    ("mm_agent_q_fwd2", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_i64, c_vp,
                                ctypes.POINTER(QFwdIO), c_i64, c_vp]),
    ("mm_agent_q_fwd_simple", c_i32, [ctypes.POINTER(QnetDims), c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    ("mm_env_create", c_i32, [ctypes.POINTER(EnvCfg), c_i64, c_u64, ctypes.POINTER(c_vp)]),
    ("mm_env_destroy", None, [c_vp]),
    ("mm_env_obs_dim", c_i32, [c_vp]),
    ("mm_env_reset", c_i32, [c_vp, c_vp, c_vp]),
    ("mm_env_step", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_env_step_rows", c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_env_step_rows_td", c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_env_reset_obs", c_vp, [c_vp]),
    ("mm_env_step_rows_begin", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_env_get_state", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_env_get_state_buf", c_i32, [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_env_set_state_buf", c_i32, [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_rollout_step_supported", c_i32, [c_vp, ctypes.POINTER(QnetDims), c_i64]),
    ("mm_rollout_step", c_i32, [c_vp, ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_vp,
                                ctypes.POINTER(QFwdIO), c_i64, ctypes.POINTER(RollStepIO), c_vp]),
    ("mm_rollout_chunk_supported", c_i32, [c_vp, ctypes.POINTER(QnetDims), c_i64]),
    ("mm_rollout_chunk", c_i32, [c_vp, ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_vp,
                                 ctypes.POINTER(QFwdIO), c_i64, ctypes.POINTER(RollChunkIO), c_vp]),
    ("mm_learner_set_multi_sample", c_i32, [c_i32, c_i32]),
    ("mm_hold_cus", c_i32, [c_i32, c_i64, c_vp, c_i64, ctypes.c_uint32, c_vp, c_vp]),
    ("mm_td_fold_range", c_i32, [c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32,
                                 c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    ("mm_env_grid_shape", c_i32, [c_vp, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)]),
    ("mm_td_chunk_step", c_i32, [c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp,
                                 c_vp, c_vp, c_i64, c_vp]),
    ("mm_td_chunk_step_rows", c_i32, [c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32,
                                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_chunk_begin", c_i32, [c_i64, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp]),
    ("mm_chunk_begin_rows", c_i32, [c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    ("mm_per_create", c_i32, [c_i64, c_i32, c_f64, c_f64, c_f64, c_f64, c_i32, c_f64, c_f64,
                              ctypes.POINTER(c_vp)]),
    ("mm_per_destroy", None, [c_vp]),
    ("mm_per_add_batch", c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    ("mm_per_insert", c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    ("mm_per_insert_fold", c_i32, [c_vp, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    ("mm_per_insert_td", c_i32, [c_vp, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_per_sample", c_i32, [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_per_sample_rng", c_i32, [c_vp, c_i32, c_u64, c_u64, c_vp, c_vp, c_vp, c_vp]),
    ("mm_per_update", c_i32, [c_vp, c_vp, c_vp, c_i32, c_vp]),
    ("mm_per_tree_ptr", c_vp, [c_vp]),
    ("mm_per_slot_rows", c_vp, [c_vp]),
    ("mm_per_size", c_i64, [c_vp]),
    ("mm_per_capacity", c_i64, [c_vp]),
    ("mm_per_alpha", c_f64, [c_vp]),
    ("mm_per_beta", c_f64, [c_vp]),
    ("mm_per_set_size", None, [c_vp, c_i64]),
    ("mm_per_set_size_host", None, [c_vp, c_i64]),
    ("mm_per_copy_tree", c_i32, [c_vp, c_vp, c_vp]),
    ("mm_per_copy_slot_rows", c_i32, [c_vp, c_vp, c_vp]),
    ("mm_per_error_word", c_i32, [c_vp, c_vp, c_i32, c_vp]),
]

_lib = None


def lib():
    """Load (once) and return the HIP library. Raises if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"minimarl: HIP library not built ({LIB_PATH}); run `make -C mini-marl_amd` "
                              "or __graft_entry__.build() — there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIGS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def symbols():
    return [s[0] for s in _SIGS]


_pending_destroy = []


def release(fn_name, h):
    """Destroy a native handle (``mm_env_destroy`` / ``mm_per_destroy``) from a ``__del__``.

    A garbage collection can run a ``__del__`` while some stream is being captured into a graph, where
    a device synchronisation or a free would invalidate the capture (and can abort). Such releases are
    deferred to the next call made outside a capture."""
    import torch
    try:
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    except Exception:
        capturing = False
    _pending_destroy.append((fn_name, h))
    if capturing:
        return
    while _pending_destroy:
        name, hh = _pending_destroy.pop()
        try:
            torch.cuda.synchronize()
        except Exception:
            pass
        getattr(lib(), name)(hh)


def check(rc, what=""):
    if rc != 0:
        msg = lib().mm_last_error().decode(errors="replace")
        raise RuntimeError(f"minimarl {what} failed (rc={rc}): {msg}")


class MixNetIO(ctypes.Structure):
    _fields_ = [("P", c_vp), ("gi", c_vp), ("q", c_vp), ("s_off", c_vp), ("h_in", c_vp), ("reset", c_vp),
                ("h_out", c_vp), ("qtot", c_vp), ("save", c_vp)]


class OuterArgs(ctypes.Structure):
    _fields_ = [("U", c_vp), ("u_g", c_i64), ("u_m", c_i64),
                ("V", c_vp), ("v_g", c_i64), ("v_m", c_i64), ("v_off", c_vp), ("v_reset", c_vp),
                ("dW", c_vp), ("w_g", c_i64), ("db", c_vp), ("b_g", c_i64),
                ("M", c_i32), ("R", c_i32), ("Cc", c_i32), ("accumulate", c_i32), ("groups", c_i32)]


class TmvArgs(ctypes.Structure):
    _fields_ = [("W", c_vp), ("w_g", c_i64), ("X", c_vp), ("x_g", c_i64), ("x_m", c_i64),
                ("Z", c_vp), ("z_g", c_i64), ("z_m", c_i64), ("Y", c_vp), ("y_g", c_i64), ("y_m", c_i64),
                ("M", c_i32), ("R", c_i32), ("Cc", c_i32), ("groups", c_i32)]


_SIGS += [
    ("mm_mixer_param_count", c_i32, [c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(c_i64)]),
    ("mm_mixer_save_dim", c_i32, [c_i32, c_i32, c_i32]),
    ("mm_mixer_delta_dim", c_i32, [c_i32, c_i32, c_i32]),
    ("mm_lrn_gather", c_i32, [c_i32, c_i32, c_i32, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                              c_vp, c_vp, c_vp, c_vp]),
    ("mm_mixer_fwd", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, ctypes.POINTER(MixNetIO), c_i32, c_vp]),
    ("mm_mixer_gi", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                            c_vp]),
    ("mm_mixer_gi_f16", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                            c_vp]),
    ("mm_lrn_loss", c_i32, [c_i32, c_i32, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp,
                            c_vp, c_vp, c_vp, c_vp]),
    ("mm_lrn_loss_ex", c_i32, [c_i32, c_i32, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp,
                               c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_mixer_bwd", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_vp]),
    ("mm_mixer_wgrad_partial_count", c_i64, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    ("mm_mixer_wgrad", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                               c_vp]),
    ("mm_vdn_sum", c_i32, [c_i64, c_i32, c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    ("mm_agent_bwd", c_i32, [ctypes.POINTER(QnetDims), c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_vp, c_vp, c_vp, c_vp]),
    ("mm_agent_bwd_seq", c_i32, [ctypes.POINTER(QnetDims), c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_vp, c_i32, c_vp]),
    ("mm_agent_mixer_bwd_seq", c_i32, [ctypes.POINTER(QnetDims), c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp,
                                       c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp,
                                       c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_outer_reduce", c_i32, [ctypes.POINTER(OuterArgs), c_vp]),
    ("mm_agent_q_pre2", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_i64, c_vp,
                                ctypes.POINTER(QFwdIO), c_i64, c_vp]),
    ("mm_agent_q_pre2_h3", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_i64, c_vp,
                                ctypes.POINTER(QFwdIO), c_i64, c_vp]),
    ("mm_agent_q_rec_seq2", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_i64, c_vp,
                                    ctypes.POINTER(QFwdIO), c_i64, c_i32, c_vp, c_vp]),
    ("mm_mixer_bwd_seq", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp, c_i32, c_vp]),
    ("mm_agent_q_rec2", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_i64, c_vp,
                                ctypes.POINTER(QFwdIO), c_i64, c_vp]),
    ("mm_outer_reduce_batch_partial", c_i64, [ctypes.POINTER(OuterArgs), c_i32]),
    ("mm_outer_reduce_batch", c_i32, [ctypes.POINTER(OuterArgs), c_i32, c_vp, c_i64, c_vp]),
    ("mm_outer_reduce_batch_bf3", c_i32, [ctypes.POINTER(OuterArgs), c_i32, c_vp, c_i64, c_vp]),
    ("mm_tmv", c_i32, [ctypes.POINTER(TmvArgs), c_vp]),
    ("mm_clip_adam", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp,
                             c_vp, c_f32, c_vp]),
    ("mm_clip_adam_pack", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_f32, c_f32, c_f32, c_f32, c_f32,
                                  c_vp, c_vp, c_vp, c_f32, ctypes.POINTER(QnetDims), c_vp, c_vp, c_vp, c_vp, c_i32,
                                  c_vp, c_u64, c_u64, c_vp, c_vp, c_vp, c_vp]),
    ("mm_clip2_adam", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp,
                              c_vp, c_f32, c_vp]),
    ("mm_per_sample_uniform", c_i32, [c_vp, c_i32, c_u64, c_u64, c_vp, c_vp, c_vp]),
    ("mm_eval_accum", c_i32, [c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_env_set_state", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_per_save_state", c_i32, [c_vp, c_vp, c_vp, ctypes.POINTER(c_f64), c_vp]),
    ("mm_per_load_state", c_i32, [c_vp, c_vp, c_vp, ctypes.POINTER(c_f64), c_vp]),
    ("mm_debug_trace", c_i32, [c_vp, c_i32]),
    ("mm_chunk_score", c_i32, [c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_mixer_fwd_seq_fits", c_i32, [c_i32, c_i32, c_i32, c_i32]),
    ("mm_mixer_fwd_seq", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(MixNetIO), c_i32, c_i32, c_vp,
                                 c_vp]),
    ("mm_mixer_fwd_seq_rec", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(MixNetIO), c_i32, c_i32, c_vp,
                                     c_vp]),
    ("mm_mixer_fwd_seq_hyper", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(MixNetIO), c_i32, c_i32,
                                       c_vp, c_vp]),
    ("mm_mixer_bwd_seq_hyper", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                       c_vp, c_vp, c_vp, c_i32, c_vp]),
    ("mm_mixer_bwd_seq_hyper_per", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp]),
    ("mm_mixer_bwd_seq_rec", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_vp, c_vp, c_i32, c_vp]),
    ("mm_mixer_seq_split", c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32]),
    ("mm_agent_mixer_pair_supported", c_i32, [ctypes.POINTER(QnetDims), c_i32, c_i32, c_i32, c_i32, c_i32, c_i32]),
    ("mm_agent_mixer_pre", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_vp,
                                   ctypes.POINTER(QFwdIO), c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                   c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_agent_mixer_rec_seq", c_i32, [ctypes.POINTER(QnetDims), c_vp, ctypes.POINTER(QFwdIO), c_vp,
                                       ctypes.POINTER(QFwdIO), c_i32, c_i32, c_vp, c_i32, c_i32, c_i32, c_i32,
                                       ctypes.POINTER(MixNetIO), c_i32, c_vp, c_vp]),
]


# ------------------------------------------------------------------ MAPPO (include/minimarl.h)
MM_MAPPO_ROLLOUT, MM_MAPPO_VALUES, MM_MAPPO_TRAIN = 0, 1, 2
MM_MST_ADV_MEAN, MM_MST_ADV_STD, MM_MST_ACTIVE_SUM, MM_MST_RET_MEAN, MM_MST_RET_SQ_MEAN, MM_MST_VN_MEAN, \
    MM_MST_VN_STD = range(7)
MM_MLOSS_POLICY, MM_MLOSS_ENTROPY, MM_MLOSS_VALUE, MM_MLOSS_RATIO = range(4)


class MappoDims(ctypes.Structure):
    _fields_ = [("obs_dim", c_i32), ("hidden", c_i32), ("n_actions", c_i32)]


class MappoNetIO(ctypes.Structure):
    _fields_ = [("P", c_vp), ("h_in", c_vp), ("h_out", c_vp), ("out", c_vp), ("save", c_vp)]


class MappoFwdArgs(ctypes.Structure):
    _fields_ = [("net", MappoNetIO * 2), ("obs", c_vp), ("mask", c_vp), ("act_in", c_vp), ("act_out", c_vp),
                ("u", c_vp), ("seed", c_u64), ("counter_ptr", c_vp), ("counter", c_u64), ("rows", c_i64),
                ("en", c_i64), ("T", c_i32), ("L", c_i32), ("rs", c_i64), ("mode", c_i32),
                ("deterministic", c_i32)]


class MappoBwdArgs(ctypes.Structure):
    _fields_ = [("P", c_vp * 2), ("save", c_vp * 2), ("gsoa", c_vp * 2), ("obs", c_vp), ("mask", c_vp),
                ("active", c_vp), ("act", c_vp), ("adv", c_vp), ("old_logp", c_vp), ("old_value", c_vp),
                ("returns", c_vp), ("stats", c_vp), ("loss_acc", c_vp), ("clip", c_f32), ("huber_delta", c_f32),
                ("entropy_coef", c_f32), ("value_coef", c_f32), ("en", c_i64), ("T", c_i32), ("L", c_i32),
                ("rs", c_i64)]


_MD = ctypes.POINTER(MappoDims)
_SIGS += [
    ("mm_mappo_param_count", c_i64, [_MD, c_i32]),
    ("mm_mappo_param_offsets", c_i32, [_MD, c_i32, ctypes.POINTER(c_i64)]),
    ("mm_mappo_save_fields", c_i32, [_MD, c_i32]),
    ("mm_mappo_grad_fields", c_i32, [_MD, c_i32]),
    ("mm_mappo_fwd", c_i32, [_MD, ctypes.POINTER(MappoFwdArgs), c_vp]),
    ("mm_mappo_bwd", c_i32, [_MD, ctypes.POINTER(MappoBwdArgs), c_vp]),
    ("mm_mappo_evaluate_actions", c_i32, [_MD, ctypes.POINTER(MappoFwdArgs), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                          c_vp, c_vp]),
    ("mm_mappo_wgrad_partial_count", c_i64, [_MD, c_i64]),
    ("mm_mappo_wgrad", c_i32, [_MD, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp]),
    ("mm_mappo_grad_scratch_count", c_i64, [_MD, c_i32, c_i32, c_i64]),
    ("mm_mappo_grad", c_i32, [_MD, ctypes.POINTER(MappoBwdArgs), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_mappo_gae", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i64, c_f32, c_f32, c_vp]),
    ("mm_mappo_adv_stats", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    ("mm_mappo_vn_update", c_i32, [c_vp, c_vp, c_f64, c_vp]),
    ("mm_mappo_stats_from_sums", c_i32, [c_vp, c_i64, c_vp, c_vp]),
    ("mm_mappo_insert", c_i32, [c_vp, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
]


# ------------------------------------------------------------------ offpolicy episode QMix / VDN
MM_OFFQ_VDN, MM_OFFQ_QMIX = 0, 1


class OffqDims(ctypes.Structure):
    _fields_ = [("n_agents", c_i32), ("obs_dim", c_i32), ("hidden", c_i32), ("n_actions", c_i32), ("mixer", c_i32),
                ("state_dim", c_i32), ("mixer_hidden", c_i32), ("hyper_hidden", c_i32)]


class OffqBatch(ctypes.Structure):
    _fields_ = [("obs", c_vp), ("share_obs", c_vp), ("acts", c_vp), ("rewards", c_vp), ("dones_env", c_vp),
                ("is_weight", c_vp), ("T", c_i32), ("B", c_i32), ("double_q", c_i32), ("huber", c_i32),
                ("gamma", c_f32), ("huber_delta", c_f32), ("per_nu", c_f32), ("per_eps", c_f32)]


_OD = ctypes.POINTER(OffqDims)
_SIGS += [
    ("mm_offq_param_counts", c_i32, [_OD, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    ("mm_offq_mixer_offsets", c_i32, [_OD, ctypes.POINTER(c_i64)]),
    ("mm_offq_workspace_bytes", c_i64, [_OD, c_i32, c_i32]),
    ("mm_offq_loss_grad", c_i32, [_OD, ctypes.POINTER(OffqBatch), c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    ("mm_offq_qvals_workspace_bytes", c_i64, [_OD, c_i32, c_i64]),
    ("mm_offq_q_values", c_i32, [_OD, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i64, c_vp, c_i64, c_vp]),
    ("mm_offq_soft_update", c_i32, [c_vp, c_vp, c_i64, c_f64, c_vp]),
]


# ------------------------------------------------------------------ offpolicy episode replay (mm_erb_*)
class ErbDims(ctypes.Structure):
    _fields_ = [("T", c_i32), ("N", c_i32), ("D", c_i32), ("S", c_i32), ("A", c_i32), ("same_share", c_i32),
                ("prioritized", c_i32), ("leaf_mode", c_i32)]


class ErbFields(ctypes.Structure):
    _fields_ = [("obs", c_vp), ("share_obs", c_vp), ("acts", c_vp), ("rewards", c_vp), ("dones", c_vp),
                ("dones_env", c_vp)]


_ED = ctypes.POINTER(ErbDims)
_SIGS += [
    ("mm_erb_create", c_i32, [_ED, c_i64, c_f64, ctypes.POINTER(c_vp)]),
    ("mm_erb_destroy", None, [c_vp]),
    ("mm_erb_insert", c_i32, [c_vp, c_i32, ctypes.POINTER(ErbFields), c_vp, c_vp]),
    ("mm_erb_len", c_i64, [c_vp]),
    ("mm_erb_current", c_i64, [c_vp]),
    ("mm_erb_it_capacity", c_i64, [c_vp]),
    ("mm_erb_sample_prioritized", c_i32, [c_vp, c_i32, c_f64, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp, c_vp]),
    ("mm_erb_sample_uniform", c_i32, [c_vp, c_i32, c_u64, c_u64, c_vp, c_vp]),
    ("mm_erb_gather", c_i32, [c_vp, c_i32, c_vp, ctypes.POINTER(ErbFields), c_vp]),
    ("mm_erb_update_priorities", c_i32, [c_vp, c_vp, c_vp, c_i32, c_vp]),
    ("mm_erb_sum_tree", c_vp, [c_vp]),
    ("mm_erb_min_tree", c_vp, [c_vp]),
    ("mm_erb_max_priority", c_vp, [c_vp]),
    ("mm_erb_error_word", c_vp, [c_vp]),
    ("mm_erb_copy_state", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
]


# ------------------------------------------------------------------ ma_gym Switch env (mm_switch_*)
class SwitchCfg(ctypes.Structure):
    _fields_ = [("n_agents", c_i32), ("max_steps", c_i32), ("full_observable", c_i32), ("clock", c_i32),
                ("step_cost", c_f32)]


_SIGS += [
    ("mm_switch_create", c_i32, [ctypes.POINTER(SwitchCfg), c_i64, ctypes.POINTER(c_vp)]),
    ("mm_switch_destroy", None, [c_vp]),
    ("mm_switch_obs_dim", c_i32, [c_vp]),
    ("mm_switch_reset", c_i32, [c_vp, c_vp, c_vp]),
    ("mm_switch_step", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_switch_get_state", c_i32, [c_vp, c_vp, c_vp, c_vp]),
    ("mm_switch_set_state", c_i32, [c_vp, c_vp, c_vp, c_vp]),
    ("mm_switch_reset_obs", c_vp, [c_vp]),
    ("mm_switch_step_rows", c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_switch_step_rows_begin", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("mm_switch_step_rows_td", c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp,
                                       c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
]
