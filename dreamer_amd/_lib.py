"""ctypes binding of libdreamer_hip.so (include/dreamer_hip.h).

The product path has no CPU fallback: if the library is missing or fails to
load, every hot-path call raises.  Build with ``python -m dreamer_amd.build``.
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdreamer_hip.so")
# kernel A/B runs only (tools/build_variant.py): another build of the same
# library, e.g. with a -D knob; never set on the product path
if os.environ.get("DREAMER_LIB_VARIANT"):
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "tools", "variants",
                            f"libdreamer_hip_{os.environ['DREAMER_LIB_VARIANT']}.so")

fp = C.c_void_p  # device pointers


class dr_linear(C.Structure):
    _fields_ = [("w", fp), ("b", fp)]


class dr_mlp3(C.Structure):
    _fields_ = [("l0", dr_linear), ("n1", dr_linear), ("l3", dr_linear), ("n4", dr_linear), ("l6", dr_linear)]


class dr_dims(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "hidden", "rows", "cols", "action", "img_h", "img_w", "enc_f1", "enc_f2", "enc_hidden",
        "prior_h1", "prior_h2", "rew_h1", "rew_h2", "cont_h1", "cont_h2",
        "actor_h1", "actor_h2", "critic_h1", "critic_h2", "buckets", "dec_f1", "dec_f2", "dec_hidden", "precision", "obs_dim", "enc_depth",
        "launch_form")] + [("fault", fp), ("fault_host", fp)]

DR_MAX_DEPTH = 5  # include/dreamer_hip.h: conv / convt slots (dr_dims.enc_depth <= 5)


class dr_world_model(C.Structure):
    _fields_ = [("conv", dr_linear * DR_MAX_DEPTH), ("map0", dr_linear), ("map1", dr_linear), ("map3", dr_linear),
                ("w_ih", fp), ("w_hh", fp), ("b_ih", fp), ("b_hh", fp),
                ("prior", dr_mlp3), ("reward", dr_mlp3), ("cont", dr_mlp3), ("buckets_rew", fp)]


class dr_decoder(C.Structure):
    _fields_ = [("up0", dr_linear), ("up1", dr_linear), ("up3", dr_linear), ("convt", dr_linear * DR_MAX_DEPTH)]


class dr_wm_batch(C.Structure):
    _fields_ = [("actions", fp), ("act_sb", C.c_longlong), ("act_st", C.c_longlong), ("rewards", fp),
                ("continues", fp), ("rc_sb", C.c_longlong), ("rc_st", C.c_longlong)]


class dr_wm_loss_cfg(C.Structure):
    _fields_ = [("beta_pred", C.c_float), ("beta_dyn", C.c_float), ("beta_rep", C.c_float)]


class dr_actor(C.Structure):
    _fields_ = [("l0", dr_linear), ("n1", dr_linear), ("l3", dr_linear), ("n4", dr_linear),
                ("mu", dr_linear), ("ls", dr_linear)]


class dr_critic(C.Structure):
    _fields_ = [("net", dr_mlp3), ("buckets", fp)]


class dr_noise(C.Structure):
    _fields_ = [("q", fp), ("eps", fp), ("rng", fp), ("row0", C.c_int), ("stream", C.c_int)]


class dr_frames(C.Structure):
    _fields_ = [("ring", fp), ("ring_cap", C.c_longlong), ("starts", fp), ("obs", fp),
                ("stride_b", C.c_longlong), ("stride_t", C.c_longlong), ("raw255", C.c_int), ("t0", C.c_int)]


_P = C.POINTER
_sz = C.c_size_t
_i = C.c_int
_ll = C.c_longlong
_f = C.c_float
_d = C.c_double

_SIGS = {
    "dr_last_error": (C.c_char_p, []),
    "dr_version": (_i, []),
    "dr_encoder_workspace_bytes": (_sz, [_P(dr_dims), _i]),
    "dr_encoder_features": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_frames), _i, _i, fp, fp, _sz, fp]),
    "dr_observe_workspace_bytes": (_sz, [_P(dr_dims), _i]),
    "dr_observe_scan": (_i, [_P(dr_dims), _P(dr_world_model), _i, _i, fp, fp, _ll, _ll, fp, fp, dr_noise,
                             fp, fp, fp, fp, _sz, fp]),
    "dr_imagine_tape_bytes": (_sz, [_P(dr_dims), _i, _i]),
    "dr_imagine_workspace_bytes": (_sz, [_P(dr_dims), _i, _i]),
    "dr_imagine_fwd": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_actor), _i, _i, fp, fp, dr_noise, _i,
                            fp, fp, fp, fp, fp, fp, fp, fp, fp, _sz, fp]),
    "dr_imagine_bwd": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_actor), _i, _i, fp, fp, fp, fp, fp,
                            fp, fp, fp, fp, _P(dr_actor), fp, _sz, fp]),
    "dr_imagine_bwd_prep": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_actor), _i, _i, fp, fp, fp, fp, _sz, fp]),
    "dr_imagine_bwd_main": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_actor), _i, _i, fp, fp, fp, fp, fp, _i,
                                 fp, _P(dr_actor), fp, _sz, fp]),
    "dr_step_workspace_bytes": (_sz, [_P(dr_dims), _i]),
    "dr_imagine_step": (_i, [_P(dr_dims), _P(dr_world_model), _i, fp, fp, fp, dr_noise, fp, fp, fp, fp,
                             fp, _sz, fp]),
    "dr_actor_act_workspace_bytes": (_sz, [_P(dr_dims), _i]),
    "dr_actor_act": (_i, [_P(dr_dims), _P(dr_actor), _i, fp, fp, dr_noise, _i, fp, fp, fp, fp, _sz, fp]),
    "dr_act_step_workspace_bytes": (_sz, [_P(dr_dims)]),
    "dr_act_step": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_actor), fp, _i, fp, fp, fp, dr_noise, _i,
                         fp, fp, fp, fp, fp, fp, fp, fp, _sz, fp]),
    "dr_gru_cell": (_i, [_P(dr_dims), _P(dr_world_model), _i, fp, fp, fp, fp, fp, _sz, fp]),
    "dr_categorical_sample": (_i, [_i, _i, _i, fp, dr_noise, fp, fp, fp, fp]),
    "dr_mlp3_fwd": (_i, [_P(dr_mlp3), _i, _i, fp, _ll, _i, fp, _ll, _i, _i, _i, fp, _ll, fp, _sz, fp]),
    "dr_bucket_value": (_i, [_i, _i, fp, fp, fp, fp]),
    "dr_critic_tape_bytes": (_sz, [_P(dr_dims), _i]),
    "dr_critic_workspace_bytes": (_sz, [_P(dr_dims), _i, _i]),
    "dr_critic_fwd": (_i, [_P(dr_dims), _P(dr_critic), _i, fp, _ll, fp, _ll, fp, fp, fp, fp, _sz, fp]),
    "dr_lambda_returns": (_i, [_i, _i, fp, fp, fp, _f, _f, fp, fp]),
    "dr_update_S": (_i, [_i, fp, fp, fp, fp, _sz, fp]),
    "dr_actor_loss_grad": (_i, [_i, _i, _i, fp, fp, fp, fp, fp, fp, _f, _f, fp, fp, fp, fp]),
    "dr_critic_loss_bwd": (_i, [_P(dr_dims), _P(dr_critic), _i, _i, fp, fp, fp, fp, _f, fp, _P(dr_critic),
                                fp, _sz, fp]),
    "dr_sqnorm": (_i, [_ll, fp, fp, fp]),
    "dr_sqnorm_multi": (_i, [_ll, fp, fp, fp, fp]),
    "dr_clip_stats": (_i, [_ll, fp, _ll, fp, _i, fp, fp, fp, fp, fp]),
    "dr_adamw": (_i, [_ll, fp, fp, fp, fp, fp, _f, _d, _d, _d, _d, _d, fp, fp, fp, fp]),
    "dr_ema": (_i, [_ll, fp, fp, _f, _f, fp, fp]),
    "dr_ac_optimiser_step": (_i, [_ll, fp, fp, fp, fp, fp, fp, _d, _d, _d, _d, _d,
                                  _ll, fp, fp, fp, fp, fp, fp, _d, _d, _d, _d, _d,
                                  _f, fp, _f, _f, _i, fp, fp, fp, fp, fp]),
    "dr_nonfinite": (_i, [_ll, fp, fp, fp]),
    "dr_replay_gather": (_i, [_ll, _i, _i, _i, _i, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp]),
    "dr_rng_advance": (_i, [fp, C.c_ulonglong, fp]),
    "dr_persistent_kernels": (_i, [_P(dr_dims), _i, _i, _i]),
    "dr_stream_create_cumask": (_i, [_i, _P(C.c_uint), _P(fp)]),
    "dr_stream_destroy": (_i, [fp]),
    "dr_device_cus": (_i, [_P(_i)]),
    "dr_host_device_ptr": (_i, [fp, _P(fp)]),
    "dr_wm_train_workspace_bytes": (_sz, [_P(dr_dims), _i, _i]),
    "dr_decoder_workspace_bytes": (_sz, [_P(dr_dims), _i]),
    "dr_decoder_fwd": (_i, [_P(dr_dims), _P(dr_decoder), _i, fp, _ll, fp, _ll, fp, fp, _sz, fp]),
    "dr_wm_train_phase": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_decoder), _i, _i, _P(dr_frames),
                               _P(dr_wm_batch), dr_noise, dr_wm_loss_cfg, _i, fp, _i, fp, fp, _P(dr_world_model),
                               _P(dr_decoder), fp, fp, fp, fp, _sz, fp]),
    "dr_wm_train_grads": (_i, [_P(dr_dims), _P(dr_world_model), _P(dr_decoder), _i, _i, _P(dr_frames),
                               _P(dr_wm_batch), dr_noise, dr_wm_loss_cfg, fp, fp, _P(dr_world_model),
                               _P(dr_decoder), fp, fp, fp, fp, _sz, fp]),
}

EXPORTED = sorted(_SIGS)

_lib = None
_load_error = None


def load():
    """Load the HIP library (no GPU needed to load it)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        _load_error = f"{LIB_PATH} not built (run: python -m dreamer_amd.build)"
        raise RuntimeError("dreamer_amd: HIP library missing: " + _load_error)
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


# include/dreamer_hip.h error codes
DR_E_INVALID, DR_E_HIP, DR_E_WORKSPACE, DR_E_UNSUPPORTED = 1001, 1002, 1003, 1004


class HipError(RuntimeError):
    """A libdreamer_hip entry point returned a non-zero code (``.code``)."""

    def __init__(self, name, code, msg):
        super().__init__(f"{name} failed ({code}): {msg}")
        self.code = code


def call(name, *args):
    """Call an int-returning entry point; raise HipError on a non-zero code."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.dr_last_error().decode(errors="replace")
        raise HipError(name, rc, msg)


def query(name, *args):
    return getattr(load(), name)(*args)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("dreamer_amd: tensors must live on the GPU (this framework is MI355X-only)")
    return t.data_ptr()


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(t):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError("dreamer_amd: hot-path ops run only on the GPU (MI355X); "
                           "move the model and tensors to 'cuda'")
