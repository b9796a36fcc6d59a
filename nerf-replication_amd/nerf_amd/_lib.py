"""ctypes binding of libnerf_amd.so (the gfx950 C-ABI declared in include/nerf_amd.h).

The library is built in-tree (``__graft_entry__.build()`` / ``make -C csrc``) and loaded
*after* ``import torch`` so that its ``libamdhip64.so.7`` dependency resolves to the HIP
runtime torch already loaded (one runtime, torch's streams are valid handles).  There is
no fallback: if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnerf_amd.so")

_p = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_f32 = ctypes.c_float
_f64 = ctypes.c_double

# name -> (restype, argtypes); mirrors include/nerf_amd.h
SIGNATURES = {
    "nerf_last_error": (ctypes.c_char_p, []),
    "nerf_abi_version": (_i32, []),
    "nerf_raygen": (_i32, [_p, _i32, _i32, _i32, _f32, _p, _i64, _u64, _u64, _p, _p, _p, _p, _p]),
    "nerf_sample_stratified": (_i32, [_p, _i64, _i32, _p, _p, _p, _i32, _p, _u64, _u64, _p, _p, _p, _p]),
    "nerf_searchsorted": (_i32, [_p, _p, _i64, _i32, _i32, _p, _p]),
    "nerf_sample_pdf": (_i32, [_p, _p, _i64, _i32, _i32, _i32, _p, _p, _u64, _u64, _p, _p, _p, _p, _p, _p, _p]),
    "nerf_sample_pdf_bins": (_i32, [_p, _p, _i64, _i32, _i32, _i32, _p, _p, _u64, _u64, _p, _p, _p, _p]),
    "nerf_composite_fwd": (_i32, [_p, _p, _p, _i32, _i64, _i32, _i32, _p, _p, _p, _p, _p]),
    "nerf_composite_bwd": (_i32, [_p, _p, _p, _i32, _i64, _i32, _i32, _p, _p, _p, _p, _p]),
    "nerf_composite_pdf": (_i32, [_p, _p, _p, _i32, _i64, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _p, _p, _u64, _u64,
                                  _p, _p, _p, _p]),
    "nerf_composite_pdf_fragile": (_i32, [_p, _p, _p, _i32, _i64, _i32, _i32, _p, _p, _p, _i32, _p, _p, _p, _p, _f32,
                                          _f32, _f32, _f32, _p, _p]),
    "nerf_mse2_fwd": (_i32, [_p, _p, _p, _i64, _p, _p]),
    "nerf_mse2_bwd": (_i32, [_p, _p, _p, _i64, _p, _p, _p, _p, _p, _p]),
    "nerf_mlp_net_params": (_i64, []),
    "nerf_mlp_param_offset": (_i64, [_i32]),
    "nerf_mlp_packed_bytes": (_i64, [_i32, _i32]),
    "nerf_mlp_padded_samples": (_i64, [_i64]),
    "nerf_mlp_act_bytes": (_i64, [_i32, _i64]),
    "nerf_mlp_dz_bytes": (_i64, [_i32, _i64]),
    "nerf_mlp_mask_bytes": (_i64, [_i64]),
    "nerf_mlp_dw_items": (_i64, [_i32, _i64]),
    "nerf_mlp_pack": (_i32, [_p, _i32, _p, _p, _p]),
    "nerf_mlp_fwd": (_i32, [_p, _i32, _p, _p, _i32, _p, _i64, _i32, _p, _p, _p, _p]),
    "nerf_mlp_fwd_count": (_i32, [_p, _i32, _p, _p, _i32, _p, _p, _i64, _p, _p]),
    "nerf_mlp_bwd": (_i32, [_p, _i32, _p, _i64, _p, _p, _p, _p, _p]),
    "nerf_mlp_bwd_dx": (_i32, [_p, _i32, _p, _i64, _p, _p, _p]),
    "nerf_mlp_bwd_dw": (_i32, [_i32, _i64, _p, _p, _p, _p]),
    "nerf_mlp_dw_workspace_bytes": (_i64, [_i32, _i64]),
    "nerf_mlp_bwd_dw_ws": (_i32, [_i32, _i64, _p, _p, _p, _p, _p]),
    "nerf_grid_index": (_i32, [_p, _i64, _p, _i32, _p, _p, _p, _p]),
    "nerf_bake_num_points": (_i64, [_i32, _i32]),
    "nerf_bake_points": (_i32, [_i32, _p, _i32, _p, _p]),
    "nerf_bake_reduce": (_i32, [_p, _i32, _i32, _f32, _p, _p]),
    "nerf_bake_num_points_slab": (_i64, [_i32, _i32, _i32, _i32]),
    "nerf_bake_points_slab": (_i32, [_i32, _p, _i32, _i32, _i32, _p, _p]),
    "nerf_bake_reduce_slab": (_i32, [_p, _i32, _i32, _i32, _i32, _f32, _p, _p]),
    "nerf_march_init": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "nerf_march_macro_bytes": (_i64, [_i32]),
    "nerf_march_macro": (_i32, [_p, _i32, _p, _p]),
    "nerf_march_gather": (_i32, [_p, _i64, _p, _i32, _p, _i32, _p, _p, _i32, _i32, _f32, _p, _p, _p, _p, _p, _p, _p,
                                 _p, _p, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "nerf_march_composite": (_i32, [_p, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _f32, _f32, _p, _p]),
    "nerf_march_finish": (_i32, [_p, _p, _i64, _i32, _p]),
    "nerf_metrics_workspace_bytes": (_i64, [_i32, _i32]),
    "nerf_image_metrics": (_i32, [_p, _p, _i32, _i32, _p, _p, _p]),
    "nerf_adam_step": (_i32, [_p, _p, _p, _p, _i64, _f64, _f64, _f64, _f64, _i64, _f64, _p]),
}

_LIB = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the library; raises if it is not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()' or make -C nerf-replication_amd/csrc)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
    return _LIB


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().nerf_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed with status {status}: {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    return None if t is None else t.data_ptr()


def stream_of(t: torch.Tensor) -> int:
    if not t.is_cuda:
        raise RuntimeError("nerf_amd kernels run on the GPU only (got a CPU tensor); there is no CPU fallback")
    return torch.cuda.current_stream(t.device).cuda_stream
