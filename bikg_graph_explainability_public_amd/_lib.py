"""ctypes binding of libxpgnn.so (include/xpgnn.h).

The product path has no CPU fallback: if the HIP library is missing or fails to load, every
engine entry point raises `NativeLibraryError`.  Build it with `__graft_entry__.build()` (or
`python -m bikg_graph_explainability_public_amd.build`).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libxpgnn.so")
ABI_VERSION = 21
MAX_TERMS = 8

ACT = {None: 0, "identity": 0, "relu": 1, "sigmoid": 2, "tanh": 3, "leaky_relu": 4, "elu": 5}
TERM = {"gcn": 0, "mean": 1, "root": 2}

c_i32, c_i64, c_f32, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p


class NativeLibraryError(RuntimeError):
    pass


class FitExchangeError(RuntimeError):
    """The multi-workgroup surrogate fit's cross-workgroup exchange timed out (its workgroups
    were not all resident on the GPU at once): the fit's outputs are invalid."""


class TermDesc(ctypes.Structure):
    _fields_ = [("kind", c_i32), ("rel", c_i32), ("table", c_vp), ("dst_type", c_i32)]


class LayerDesc(ctypes.Structure):
    _fields_ = [("n_terms", c_i32), ("act", c_i32), ("f_in_pad", c_i32), ("f_out", c_i32),
                ("f_out_pad", c_i32), ("n_tgt", c_i32), ("n_edges", c_i32), ("tgt_prev", c_vp),
                ("tgt_f0", c_vp),
                ("agg_ptr", c_vp), ("agg_src", c_vp), ("agg_f0", c_vp), ("self_mult", c_vp),
                ("terms", TermDesc * MAX_TERMS), ("weight", c_vp), ("bias", c_vp),
                ("tgt_type", c_vp), ("n_types", c_i32),
                ("agg_eid", c_vp), ("self_ptr", c_vp), ("self_eid", c_vp)]


class HeadDesc(ctypes.Structure):
    _fields_ = [("k_pad", c_i32), ("n_real", c_i32), ("n_pad", c_i32), ("act", c_i32),
                ("weight", c_vp), ("bias", c_vp)]


class ForwardPlanDesc(ctypes.Structure):
    _fields_ = [("cols", c_i64), ("n_rel", c_i32), ("n0", c_i32), ("f0_node", c_vp),
                ("deg_ptr", c_vp), ("deg_src", c_vp), ("n_deg_edges", c_i64), ("n_layers", c_i32),
                ("layers", ctypes.POINTER(LayerDesc)), ("n_head", c_i32),
                ("head", ctypes.POINTER(HeadDesc)), ("out_col", c_i32),
                ("edge_masks", c_i32), ("deg_eid", c_vp), ("edge_dot", c_i32), ("dot_a", c_i32),
                ("dot_b", c_i32), ("dot_act", c_i32)]


class WlmParams(ctypes.Structure):
    _fields_ = [("lr", c_f32), ("l1_lambda", c_f32), ("beta1", c_f32), ("beta2", c_f32),
                ("eps", c_f32), ("weight_decay", c_f32)]


_SIGS = {
    "xpg_abi_version": ([], c_i32),
    "xpg_last_error": ([], ctypes.c_char_p),
    "xpg_pack_masks": ([c_vp, c_i64, c_i64, c_vp, c_vp], c_i32),
    "xpg_unpack_masks": ([c_vp, c_i64, c_i64, c_vp, c_vp], c_i32),
    "xpg_sample_shapley": ([ctypes.c_uint64, c_i64, c_i64, c_i64, c_vp, c_vp], c_i32),
    "xpg_sample_shapley_counts": ([ctypes.c_uint64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp], c_i32),
    "xpg_sample_shapley_dev": ([c_vp, c_i64, c_i64, c_i64, c_vp, c_vp], c_i32),
    "xpg_sample_shapley_sets": ([c_vp, c_i32, c_i64, c_i64, c_vp, c_vp], c_i32),
    "xpg_plan_arrays_build": ([c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp], c_i32),
    "xpg_plan_arrays_take": ([c_vp, c_vp], c_i32),
    "xpg_plan_arrays_free": ([c_vp], c_i32),
    "xpg_mt19937_mask_bits": ([c_vp, c_vp, c_vp, c_i64, c_i64, c_vp], c_i32),
    "xpg_mt19937_repeat_draws": ([c_vp, c_vp, c_vp, c_i32, c_i64, ctypes.c_float, ctypes.c_float, c_i32, c_vp,
                                  c_vp], c_i32),
    "xpg_mt19937_community_bits": ([c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_i64,
                                    c_vp], c_i32),
    "xpg_sample_communities": ([ctypes.c_uint64, c_i64, c_i64, c_i32, c_vp, c_i32, c_i64, c_i32, c_vp, c_vp,
                                c_vp, c_vp, c_vp], c_i32),
    "xpg_sample_communities_rows": ([ctypes.c_uint64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i32, c_i64, c_i32, c_vp, c_vp,
                                c_vp, c_vp, c_vp], c_i32),
    "xpg_edge_keep": ([c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp], c_i32),
    "xpg_rows_no_edge": ([c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp], c_i32),
    "xpg_popcount_rows": ([c_vp, c_i64, c_i64, c_vp, c_vp], c_i32),
    "xpg_shap_kernel": ([c_vp, c_i64, c_i64, c_vp, c_vp], c_i32),
    "xpg_dense": ([c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, ctypes.c_int,
                   c_vp, c_i64, c_vp], c_i32),
    "xpg_forward_workspace": ([ctypes.POINTER(ForwardPlanDesc), c_i64,
                               ctypes.POINTER(ctypes.c_size_t)], c_i32),
    "xpg_masked_forward": ([ctypes.POINTER(ForwardPlanDesc), c_vp, c_i64, c_vp, c_vp,
                            ctypes.c_size_t, c_vp], c_i32),
    "xpg_profile_enable": ([ctypes.c_int], c_i32),
    "xpg_profile_read": ([c_vp, c_vp, c_i32], c_i32),
    "xpg_wlm_workspace": ([c_i64, c_i64, c_i64, c_i64, ctypes.POINTER(ctypes.c_size_t)], c_i32),
    "xpg_wlm_plan": ([c_i64, c_i64, c_i64, c_i64, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)], c_i32),
    "xpg_wlm_fit": ([c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, ctypes.POINTER(WlmParams), c_i64,
                     c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp], c_i32),
    "xpg_wlm_fit_from": ([c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, ctypes.POINTER(WlmParams), c_vp,
                          c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp], c_i32),
    "xpg_wlm_prepare": ([c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, ctypes.POINTER(WlmParams), c_vp,
                         c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp], c_i32),
    "xpg_wlm_fit_prepared": ([c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, ctypes.POINTER(WlmParams), c_vp,
                              c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp], c_i32),
    "xpg_wlm_fit_steps": ([c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, ctypes.POINTER(WlmParams), c_vp, c_vp,
                           c_vp, c_vp, ctypes.c_size_t, c_vp], c_i32),
    "xpg_wlm_fit_losses": ([c_i64, c_i64, c_i64, c_i64, c_vp, ctypes.POINTER(WlmParams), c_vp, c_vp, c_vp,
                            c_vp, ctypes.c_size_t, c_vp], c_i32),
    "xpg_khop_workspace": ([c_i64, c_i64, ctypes.POINTER(ctypes.c_size_t)], c_i32),
    "xpg_khop_subgraph": ([c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                           ctypes.c_size_t, c_vp], c_i32),
}

EXPORTED = tuple(_SIGS.keys())
_lib = None


def load(path=None):
    """Load (once) and type the native library; raise NativeLibraryError if unavailable.
    XPG_LIB overrides the path (diagnostic builds, e.g. tools/build_stamps.sh)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("XPG_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"{path} not found: the HIP engine is not built (run __graft_entry__.build()); "
            "there is no CPU fallback")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover
        raise NativeLibraryError(f"failed to load {path}: {e}") from e
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.xpg_abi_version() != ABI_VERSION:
        raise NativeLibraryError("libxpgnn ABI version mismatch")
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        msg = _lib.xpg_last_error().decode() if _lib is not None else "?"
        raise RuntimeError(f"xpgnn error {rc}: {msg}")


def call(name, *args):
    lib = load()
    check(getattr(lib, name)(*args))


def require_device(t, name="tensor"):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise NativeLibraryError(f"{name} must be a CUDA/HIP device tensor (no CPU fallback)")
    return t


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(device=None):
    """The current HIP stream of `device` (a torch.device, or None = the current device) as a
    handle.  Read as torch's raw stream pointer: building a torch.cuda.Stream object per native
    call cost ~9 us of host time each."""
    if _raw_stream is not None:
        idx = device.index if isinstance(device, torch.device) else None
        return ctypes.c_void_p(_raw_stream(torch.cuda.current_device() if idx is None else idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
