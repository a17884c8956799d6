"""ctypes binding of liblzmcts.so (C ABI: include/lzmcts.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).
There is no CPU fallback: if the library is missing or no GPU is visible, every entry
point raises. torch is imported first so that the library binds to the HIP runtime torch
already loaded (same soname, libamdhip64.so.7), and torch streams / device pointers are
valid inside it.
"""
import atexit
import ctypes
import os
import weakref

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LZM_LIB") or os.path.join(HERE, "liblzmcts.so")  # override: build experiments

LZM_OK = 0
LZM_ERR_ARG = -1
LZM_ERR_HIP = -2
LZM_ERR_CAPACITY = -3
LZM_ERR_STATE = -4
LZM_ERR_RESIDENCY = -5
LZM_ERR_RANGE = -6
LZM_ERR_WORDS = 8  # sticky error words per tree handle (lzm_check_errors)
LZM_TREE_EZ = 1
LZM_RNG_FAST = 2

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_d = ctypes.c_double

# name -> argtypes (all return int status unless listed in _RESTYPE)
SIGNATURES = {
    "lzm_create": [_i, _i, _i, _i, ctypes.POINTER(_vp)],
    "lzm_destroy": [_vp],
    "lzm_reserve": [_vp, _i],
    "lzm_num_roots": [_vp],
    "lzm_sims_capacity": [_vp],
    "lzm_action_space": [_vp],
    "lzm_flags": [_vp],
    "lzm_last_error": [],
    "lzm_set_pb_c": [_vp, _i, _f],
    "lzm_copy_tree": [_vp, _vp, _vp],
    "lzm_minmax_init": [_vp, _i, _f, _vp],
    "lzm_roots_prepare": [_vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp],
    "lzm_traverse": [_vp, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_gather_latent": [_vp, _vp, _i64, _vp, _vp, _vp],
    "lzm_backprop": [_vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_decode_backprop": [_vp, _i, _f, _vp, _vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i64, _vp, _vp],
    "lzm_inverse_scalar_transform": [_vp, _i, _i, _i, _vp, _vp],
    "lzm_get_distributions": [_vp, _vp, _vp],
    "lzm_get_values": [_vp, _vp, _vp],
    "lzm_get_trajectories": [_vp, _vp, _i, _vp],
    "lzm_last_traverse_passes": [_vp, _vp, _vp],
    "lzm_mlp_packed_floats": [_i, _i, _i, _i, _i],
    "lzm_mlp_kernel_floats": [_i, _i, _i, _i, _i],
    "lzm_search_mlp_kind": [_i, _i, _i, _i, _i, _i],
    "lzm_decode_backprop_traverse": [_vp, _i, _f, _vp, _vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i64, _vp, _i, _f,
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_mlp_initial_inference": [_i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_mlp_initial_inference_prepare": [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _f, _vp, _vp, _vp],
    "lzm_set_reuse": [_vp, _vp, _vp],
    "lzm_ez_lstm_input": [_i, _i, _i, _vp, _vp, _vp, _vp, _vp],
    "lzm_ez_lstm_cell": [_i, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp],
    "lzm_ez_lstm_frag_floats": [_i, _i],
    "lzm_ez_lstm_prepare": [_i, _i, _vp, _vp],
    "lzm_ez_lstm_workspace_bytes": [_i, _i],
    "lzm_error_word": [_vp, _i],
    "lzm_debug_lstm_stamps": [_vp],
    "lzm_debug_az_stamps": [_vp],
    "lzm_debug_hold_cus": [_i, _i, _vp],
    "lzm_ez_lstm_step": [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_search_conv": [_vp, _i, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _i,
                        _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_search_conv_ez": [_vp, _i, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _i, _i, _vp,
                           _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_conv_heads": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp],
    "lzm_conv_heads_prepare": [_vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _f,
                               _vp, _vp, _vp],
    "lzm_set_norm_words": [_vp, _vp],
    "lzm_seed_sequence": [_vp, _i64, _i, _vp, _vp],
    "lzm_get_root_outputs": [_vp, _vp, _vp, _vp],
    "lzm_mlp_prepare": [_i, _i, _i, _i, _i, _vp, _vp, _vp],
    "lzm_search_mlp": [_vp, _i, _i, _i, _i, _vp, _i, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_search_diagnostics": [_vp, _vp, _vp],
    "lzm_debug_root_wait_cycles": [_vp, _vp, _i, _i],
    "lzm_search_set_step": [_vp, _vp, _i64, _i, _vp, _vp, _i, _f],
    "lzm_check_errors": [_vp, _vp, _i, _vp],
    "lzm_debug_expf": [_vp, _vp, _i64, _vp],
    "lzm_debug_glibc_rand": [_u32, _i, _vp, _vp],
    "lzm_debug_philox": [_vp, _vp, _i, _vp],
    "lzm_debug_xor": [_vp, _vp, _vp],
    "lzm_debug_az_rules": [_i, _vp, _vp, _vp, _vp],
    "lzm_shutdown": [],
    "lzm_debug_phase_cycles": [_vp, _vp, _i],
    "lzm_cartpole_reset": [_i, _vp, _vp, _vp, _u32, _vp],
    "lzm_cartpole_collect_step": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _vp, _vp, _vp, _vp,
                                  _vp, _vp, _vp, _vp, _vp, _i, _u32, _vp, _vp],
    "lzm_atari_reset": [_i, _vp, _vp, _vp, _vp, _u32, _vp],
    "lzm_atari_collect_step": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp, _vp, _vp, _i, _u32, _vp, _vp],
    "lzm_pong_reset": [_i, _vp, _vp, _vp, _vp, _u32, _vp],
    "lzm_pong_collect_step": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _vp, _vp, _vp, _vp,
                              _vp, _vp, _vp, _vp, _vp, _i, _u32, _vp, _vp],
    "lzm_episodes_scan": [_i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_bias_add_relu": [_vp, _vp, _vp, _i, _i, _i, _i, _vp],
    "lzm_conv_resnet8_p": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_repr_floats": [],
    "lzm_repr_prepare": [_i, _vp, _vp],
    "lzm_repr_workspace_floats": [_i],
    "lzm_repr_downsample": [_i, _i, _vp, _vp, _vp, _vp, _vp],
    "lzm_episodes_pack": [_i, _i, _i, _i, _i, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                          _vp, _vp, _vp],
    "lzm_az_workspace_bytes": [_i, _i, ctypes.POINTER(_i64)],
    "lzm_az_noise_table": [_d, _i, _vp],
    "lzm_az_set_constants": [_i, _i, _vp, _d, _d, _d, _vp],
    "lzm_az_begin": [_i, _i, _vp, _vp, _vp, _vp, _vp],
    "lzm_az_step": [_i, _i, _vp, _i, _vp, _i, _vp, _i, _i, _d, _vp, _vp],
    "lzm_az_finish": [_i, _i, _vp, _d, _i, _u32, _vp, _vp, _vp, _vp, _vp],
    "lzm_az_export_tree": [_i, _i, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_az_net_floats": [_i],
    "lzm_az_net_prepare": [_i, _vp, _vp],
    "lzm_az_net_eval": [_i, _vp, _vp, _i, _vp, _vp, _vp],
    "lzm_az_search_fused": [_i, _i, _vp, _i, _vp, _vp, _vp, _i, _d, _d, _i, _u32, _vp, _vp, _vp, _vp, _i, _vp],
    "lzm_conv_trunk_floats": [_i, _i],
    "lzm_conv_trunk_prepare": [_i, _i, _i, _i, _vp, _vp],
    "lzm_conv_trunk": [_i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_conv_trunk_floats_p": [_i, _i, _i],
    "lzm_conv_trunk_prepare_p": [_i, _i, _i, _i, _i, _vp, _vp],
    "lzm_conv_trunk_actmap_bound": [_i, _i, _f, _vp],
    "lzm_conv_trunk_p": [_i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "lzm_conv_trunk_xin_p": [_i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _i, _vp, _vp, _vp,
                             _vp],
}
_RESTYPE = {"lzm_last_error": ctypes.c_char_p, "lzm_mlp_packed_floats": ctypes.c_int64,
            "lzm_mlp_kernel_floats": ctypes.c_int64, "lzm_az_net_floats": ctypes.c_int64,
            "lzm_conv_trunk_floats": ctypes.c_int64, "lzm_conv_trunk_floats_p": ctypes.c_int64,
            "lzm_ez_lstm_frag_floats": ctypes.c_int64, "lzm_ez_lstm_workspace_bytes": ctypes.c_int64,
            "lzm_error_word": ctypes.c_void_p, "lzm_repr_floats": ctypes.c_int64,
            "lzm_repr_workspace_floats": ctypes.c_int64}

_lib = None


class LzmError(RuntimeError):
    pass


class ResidencyError(LzmError):
    """A launch that needs its whole grid co-resident was refused (LZM_ERR_RESIDENCY); nothing ran."""


class SplitRangeError(LzmError):
    """Split-fp16 network values were non-finite or beyond the power-of-two scales' range (LZM_ERR_RANGE): the
    search's network outputs are not f32-exact. Run the conv network with precision='f32'
    (LZM_CONV_PRECISION=f32)."""


# objects owning device memory allocated by the library (tree handles, ...): closed by the exit hook
_owners = weakref.WeakSet()


def register_owner(obj):
    """obj.close() releases its library resources; called at process exit before the runtime's teardown"""
    _owners.add(obj)


def _teardown():
    """atexit (runs before the interpreter finalises and before any C-level exit handler): close the live
    handles, wait for the device and free the library's static buffers, so nothing of the library is left
    for the HIP runtime's (or a profiler's) exit-time teardown to release (profiles/r05/README.md)."""
    if _lib is None:
        return
    for o in list(_owners):
        try:
            o.close()
        except Exception:
            pass
    try:
        if torch.cuda.is_initialized():
            _lib.lzm_shutdown()
    except Exception:
        pass


def load(path=LIB_PATH):
    """Load the library without touching the GPU (symbol table only)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise LzmError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    _lib = L
    atexit.register(_teardown)
    return L


def require_gpu():
    if not torch.cuda.is_available():
        raise LzmError("lightzero_amd needs a ROCm GPU (MI355X / gfx950); no CPU fallback exists")


def check(rc, what):
    if rc == LZM_OK:
        return rc
    msg = (_lib.lzm_last_error() or b"").decode(errors="replace")
    if rc == LZM_ERR_ARG:
        raise ValueError(f"{what}: {msg}")
    if rc == LZM_ERR_RESIDENCY:
        raise ResidencyError(f"{what}: {msg}")
    if rc == LZM_ERR_RANGE:
        raise SplitRangeError(f"{what}: {msg}")
    raise LzmError(f"{what} failed ({rc}): {msg}")


def call(name, *args):
    L = load()
    return check(getattr(L, name)(*args), name)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
