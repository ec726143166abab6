"""ctypes binding of libcista_hip.so (C ABI: include/cista_lstc.h).

The library is the product: there is NO Python / CPU fallback.  If the shared object is
missing or fails to load, every entry point raises -- loudly -- instead of computing anything.

torch is imported first on purpose: torch-ROCm ships its own ``libamdhip64.so.7``; loading
it before ``libcista_hip.so`` makes the dynamic linker resolve our NEEDED entry to the SAME HIP
runtime instance, so torch's device pointers and streams are valid inside the library.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must precede the dlopen below, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CISTA_HIP_LIB", os.path.join(_HERE, "libcista_hip.so"))
INCLUDE_DIR = os.path.join(os.path.dirname(_HERE), "include")
HEADER_PATH = os.path.join(INCLUDE_DIR, "cista_lstc.h")

c_int, c_size_t, c_void_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p

PARAM_FIELDS = [
    "We_w", "We_b", "Wi_w", "Wi_b", "W0_w", "W0_b", "gates_w", "gates_b", "out_gates_w",
    "out_gates_b", "P0_w", "P0_b", "lambda_", "D_w", "D_b", "P_w", "P_b", "Dg_w", "Dg_b",
    "lstm_w", "lstm_b", "up_w", "up_b", "final_w", "final_b",
]


class CistaConfig(ctypes.Structure):
    _fields_ = [("base_channels", c_int), ("depth", c_int), ("num_bins", c_int)]


class CistaParams(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in PARAM_FIELDS]


class CistaFrameIO(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in (
        "events", "prev_image", "c_lstc_prev", "z_prev", "h_prev", "c_prev",
        "rec", "c_lstc", "z", "h", "c")]


LAYERS = ["input", "W0", "P0", "gates", "out_gates", "ista_D", "ista_P", "Dg", "lstm",
          "upsample", "final"]          # CISTA_LAYER_* ids, in frame order

class CistaGradIO(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in (
        "g_rec", "g_c_lstc", "g_z", "g_h", "g_c",
        "g_prev_image", "g_c_lstc_prev", "g_z_prev", "g_h_prev", "g_c_prev", "g_events")]


class CistaParamGrads(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in PARAM_FIELDS]


STATUS = {0: "ok", 1: "invalid argument", 2: "unsupported configuration", 3: "HIP runtime error",
          4: "workspace too small", 5: "output aliases input"}


class CistaError(RuntimeError):
    pass


_lib = None
_load_error = None


def _declare(lib):
    P = ctypes.POINTER
    sig = {
        "cista_abi_version": (c_int, []),
        "cista_status_string": (ctypes.c_char_p, [c_int]),
        "cista_packed_bytes": (c_size_t, [P(CistaConfig)]),
        "cista_pack_params": (c_int, [P(CistaConfig), P(CistaParams), c_void_p, c_void_p]),
        "cista_workspace_bytes": (c_size_t, [P(CistaConfig), c_int, c_int, c_int]),
        "cista_forward": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, P(CistaFrameIO),
                                  c_void_p, c_size_t, c_void_p]),
        "cista_stage_input": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
        "cista_stage_lstc": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, c_void_p,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                     c_void_p]),
        "cista_stage_ista": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, c_void_p,
                                     c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
        "cista_stage_decoder": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_size_t, c_void_p]),
        "cista_stage_output": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
        "cista_layer_macs": (ctypes.c_double, [P(CistaConfig), c_int, c_int, c_int, c_int]),
        "cista_layer_fused": (c_int, [P(CistaConfig), c_int]),
        "cista_tile_plan": (c_int, [c_int, c_int, c_int, c_int, P(c_int)]),
        "cista_saved_bytes": (c_size_t, [P(CistaConfig), c_int, c_int, c_int]),
        "cista_train_workspace_bytes": (c_size_t, [P(CistaConfig), c_int, c_int, c_int]),
        "cista_forward_train": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, P(CistaFrameIO),
                                        c_void_p, c_size_t, c_void_p, c_size_t, c_void_p]),
        "cista_backward": (c_int, [P(CistaConfig), c_void_p, P(CistaParams), c_int, c_int, c_int,
                                   P(CistaFrameIO), c_void_p, c_size_t, P(CistaGradIO), c_size_t,
                                   P(CistaParamGrads), c_void_p, c_size_t, c_void_p]),
        "cista_wgrad_ista_p": (c_int, [P(CistaConfig), c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_size_t, c_void_p]),
        "cista_wgrad_w0": (c_int, [P(CistaConfig), c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_size_t, c_void_p]),
        "cista_launch_layer": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, c_int,
                                       P(CistaFrameIO), c_void_p, c_size_t, c_void_p]),
        "cista_sequence_capture": (c_int, [P(CistaConfig), c_void_p, c_int, c_int, c_int, P(CistaFrameIO), c_int,
                                           c_void_p, c_size_t, P(c_void_p), c_void_p]),
        "cista_sequence_launch": (c_int, [c_void_p, c_void_p]),
        "cista_sequence_destroy": (None, [c_void_p]),
        # include/cista_voxel.h
        "cista_voxel_workspace_bytes": (c_size_t, [c_int, ctypes.c_longlong, c_int, c_int, c_int]),
        "cista_voxelize": (c_int, [c_void_p, c_void_p, c_int, ctypes.c_longlong, c_int, c_int, c_int, c_int,
                                   ctypes.c_float, c_void_p, c_void_p, c_size_t, c_void_p]),
        "cista_voxelize_checked": (c_int, [c_void_p, c_void_p, c_int, ctypes.c_longlong, c_int, c_int, c_int, c_int,
                                   ctypes.c_float, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
        "cista_voxel_preprocess": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, ctypes.c_float,
                                           c_void_p, c_size_t, c_void_p]),
        # include/cista_loss.h (config struct passed as a pointer; see losses.CistaSsimConfig)
        "cista_ssim_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
        "cista_ssim_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                       c_void_p, c_void_p, c_size_t, c_void_p]),
        "cista_ssim_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                        c_void_p, c_void_p, c_size_t, c_void_p]),
        # include/cista_v2e.h (config / host-state structs: v2e2v_amd/v2e.py)
        "cista_v2e_state_bytes": (c_size_t, [c_int, c_int, c_int]),
        "cista_v2e_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
        "cista_v2e_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                      c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
        "cista_v2e_raw_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
        "cista_v2e_forward_raw": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                          c_int, c_int, c_void_p, ctypes.c_ulonglong, c_void_p, c_void_p, c_void_p,
                                          c_size_t, c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    """Load (once) and return the ctypes handle; raise if the HIP library is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise CistaError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"libcista_hip.so not found at {LIB_PATH}; build it first "
                       "(`make` or `python -c 'import __graft_entry__ as g; g.build()'`)")
        raise CistaError(_load_error)
    try:
        _lib = _declare(ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL))
    except OSError as e:  # pragma: no cover - environment dependent
        _load_error = f"failed to load {LIB_PATH}: {e}"
        raise CistaError(_load_error) from e
    return _lib


def header_functions(path: str | None = None):
    """Names of every function declared in include/*.h (or in one header `path`)."""
    paths = [path] if path else sorted(
        os.path.join(INCLUDE_DIR, f) for f in os.listdir(INCLUDE_DIR) if f.endswith(".h"))
    names = set()
    for p in paths:
        src = re.sub(r"/\*.*?\*/", "", open(p).read(), flags=re.S)
        names |= set(re.findall(r"\b(cista_[a-z_]+)\s*\(", src))
    return sorted(names)


def check(status: int, what: str):
    if status != 0:
        msg = lib().cista_status_string(status).decode()
        raise CistaError(f"{what} failed: {msg} (status {status})")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream
