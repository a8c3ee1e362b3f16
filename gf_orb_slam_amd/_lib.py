"""ctypes binding of libgfslam.so (the C-ABI declared in include/gfslam/abi.h).

The product path always goes through this library: if libgfslam.so is missing
or no HIP device is present, every operator raises instead of falling back to
any CPU implementation.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# GF_LIB: a diagnostic build of the same sources (e.g. the phase-stamp build
# `make stamp`); the product build otherwise
LIB_PATH = os.environ.get("GF_LIB") or os.path.join(_HERE, "libgfslam.so")
ABI_HEADER = os.path.join(os.path.dirname(_HERE), "include", "gfslam", "abi.h")

GF_OK = 0
ERRORS = {-1: "GF_ERR_ARG", -2: "GF_ERR_HIP", -3: "GF_ERR_CAP", -4: "GF_ERR_UNSUPPORTED", -5: "GF_ERR_NODEV"}


class GFError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class KeyPoint(ctypes.Structure):
    """cv::KeyPoint layout (28 bytes)."""

    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("size", ctypes.c_float),
                ("angle", ctypes.c_float), ("response", ctypes.c_float),
                ("octave", ctypes.c_int32), ("class_id", ctypes.c_int32)]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
        # torch bundles its own libamdhip64.so.7; load it first so that this
        # process has exactly one HIP runtime (libgfslam binds to the loaded
        # soname) and torch device buffers / streams can be handed to the ABI.
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is optional plumbing
            pass
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.gf_last_error.restype = ctypes.c_char_p
        _declare(_lib)
    return _lib


_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_D = ctypes.c_double
_S = ctypes.c_size_t
_PROTOS = {
    "gf_device_count": [_P],
    "gf_ctx_create": [_I, _P],
    "gf_ctx_destroy": [_P],
    "gf_ctx_stream": [_P, _P],
    "gf_ctx_sync": [_P],
    "gf_prof_enable": [_P, _I],
    "gf_prof_reset": [_P],
    "gf_prof_report": [_P, _I, _P, _I, _P, _P],
    "gf_extractor_create": [_P, _I, _F, _I, _I, _I, _I, _I, _I, _P],
    "gf_extractor_destroy": [_P],
    "gf_extractor_info": [_P, _P, _P, _P],
    "gf_extractor_capacity": [_P, _P],
    "gf_orb_extract": [_P, _P, _I, _P, _P, _I, _P],
    "gf_orb_extract_batch_dev": [_P, _I, _P, _S, _I, _P, _P, _P, _I, _P],
    "gf_extractor_debug_level": [_P, _I, _I, _I, _P, _P, _P],
    "gf_frustum": [_P, _P, _P, _P, _I, _F, _P, _P],
    "gf_match_project": [_P, _P, _P, _P, _I, _P, _P, _I, _F, _F, _P, _P, _P],
    "gf_match_lastframe": [_P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _F, _I, _P, _P, _P],
    "gf_descriptor_distance": [_P, _P, _P, _I, _P],
    "gf_frustum_dev": [_P, _P, _I, _P, _P, _P, _I, _F, _P, _P, _P],
    "gf_match_project_dev": [_P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _I, _F, _F, _P, _P, _P, _P],
    "gf_rng_seed": [_P, ctypes.c_uint32],
    "gf_rng_next": [_P, _P, _I],
    "gf_obs_update": [_D, _P, _D, _P, _P],
    "gf_obs_predict": [_P, _D, _I, _P],
    "gf_obs_build_info": [_P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P],
    "gf_logdet": [_P, _P, _I, _P],
    "gf_obs_active_match": [_P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _I, _F, _F, _P, _P, _P, _P, _P,
                            _P],
    "gf_maxvol_select": [_P, _P, _P, _I, _I, _D, _I, _P, _P, _P],
    "gf_obs_build_info_dev": [_P, _P, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P],
    "gf_obs_accumulate_dev": [_P, _I, _P, _P, _P, _I, _D, _P, _P],
    "gf_obs_active_match_dev": [_P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _F, _F, _P,
                                _P, _P, _P, _P, _P, _P, _P],
    "gf_maxvol_select_dev": [_P, _I, _P, _P, _P, _I, _I, _D, _I, _P, _P, _P, _P],
    "gf_match_lastframe_dev": [_P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _F, _I, _P, _P, _P,
                               _P, _P],
    "gf_obs_update_dev": [_P, _I, _P, _P, _P, _P, _P, _P, _P],
    "gf_obs_frame_info_dev": [_P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _I, _P, _I, _P, _P, _P, _P],
    "gf_obs_map_info_dev": [_P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _I, _P, _P, _P, _P, _P],
    "gf_obs_accumulate_matched_dev": [_P, _I, _P, _P, _I, _P, _P, _P, _I, _I, _D, _P, _P],
    "gf_motion_predict_dev": [_P, _I, _P, _P, _P, _P],
    "gf_discard_outliers_dev": [_P, _I, _P, _P, _P, _I, _I, _P, _P, _P],
    "gf_matched_gather_dev": [_P, _I, _P, _P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P],
    "gf_views_exclude_matched_dev": [_P, _I, _P, _P, _I, _P, _P, _I, _P],
    "gf_pose_opt": [_P, _P, _P, _I, _F, _F, _F, _F, _P, _P, _P, _P],
    "gf_pose_opt_batch_dev": [_P, _I, _P, _P, _P, _I, _F, _F, _F, _F, _P, _P, _P, _P],
    "gf_pose_opt_frames_dev": [_P, _I, _P, _P, _P, _I, _P, _P, _I, _P, _I, _F, _F, _F, _F, _P, _P, _P, _P, _P],
    "gf_vocab_read": [_P, _P],
    "gf_vocab_save_binary": [_P, _P],
    "gf_undistort_keypoints": [_P, _P, _P, _P, _I, _P],
    "gf_undistort_keypoints_dev": [_P, _I, _P, _P, _P, _P, _I, _P, _P],
    "gf_distinctive_descriptors": [_P, _I, _P, _P, _P, _P],
    "gf_distinctive_descriptors_dev": [_P, _I, _P, _P, _P, _P, _I, _P],
    "gf_fuse": [_P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _F, _P, _P],
    "gf_fuse_dev": [_P, _P, _I, _P, _P],
    "gf_search_for_triangulation": [_P, _I, _P, _P, _P, _P, _I, _P, _P],
    "gf_search_for_triangulation_dev": [_P, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P],
    "gf_vocab_create": [_P, _P, _P],
    "gf_vocab_load": [_P, _P, _P],
    "gf_vocab_info": [_P, _P, _P, _P, _P],
    "gf_vocab_destroy": [_P],
    "gf_bow_transform": [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "gf_bow_transform_dev": [_P, _I, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P],
    "gf_match_bow": [_P, _I, _F, _I, _P, _P, _P, _P],
    "gf_match_bow_dev": [_P, _I, _F, _I, _I, _P, _P, _P, _P, _P],
    "gf_pnp_init": [_I, _P, _P],
    "gf_pnp_iterate": [_P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P],
    "gf_pnp_iterate_dev": [_P, _I, _P, _P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P],
    "gf_local_ba": [_P, _P, _P],
    "gf_ba_plan_create": [_P, _I, _P, _P],
    "gf_ba_plan_solve": [_P, _P, _P],
    "gf_ba_plan_results": [_P, _P],
    "gf_ba_plan_destroy": [_P],
    "gf_ba_plan_solve_stop": [_P, _P, _P, _P],
    "gf_local_ba_stop": [_P, _P, _P, _P],
    "gf_orb_extract_ptrs_dev": [_P, _I, _P, _I, _P, _P, _P, _I, _P],
    "gf_frustum_list_dev": [_P, _P, _I, _P, _P, _I, _P, _P, _F, _P, _P, _P],
    "gf_match_project_list_dev": [_P, _P, _I, _P, _P, _P, _I, _P, _P, _I, _P, _P, _F, _F, _P, _P, _P, _P],
    "gf_frontend_create": [_P, _P, _P],
    "gf_frontend_destroy": [_P],
    "gf_frontend_capacity": [_P, _P],
    "gf_frontend_set_source": [_P, _P, _P, _I, _S],
    "gf_frontend_set_map": [_P, _I, _P, _P, _I],
    "gf_frontend_set_rng": [_P, _I, ctypes.c_uint32],
    "gf_frontend_set_covis": [_P, _I, _P],
    "gf_kfdb_create": [_P, _P, _P],
    "gf_kfdb_destroy": [_P],
    "gf_frontend_set_kfdb": [_P, _I, _P],
    "gf_frontend_set_vocab": [_P, _P],
    "gf_window_search": [_P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _F, _I, _P, _P],
    "gf_search_frames": [_P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _F, _P, _P, _P],
    "gf_search_kf_projection": [_P, _P, _P, _P, _I, _P, _P, _P, _I, _P, _P, _I, _P, _F, _I, _I, _P, _P, _P],
    "gf_reloc_candidates": [_P, _P, _P, _I, _P, _P, _P, _P, ctypes.c_uint32, _P, _P, _P],
    "gf_frontend_bootstrap": [_P, _P, _P, _D],
    "gf_frontend_step": [_P],
    "gf_frontend_step_extract": [_P],
    "gf_frontend_step_track": [_P],
    "gf_update_reference": [_P, _P, _P, _I, _P, _P, _I, _P, _P, _I, _P],
    "gf_update_reference_dev": [_P, _P, _I, _P, _P, _I, _P, _P, _I, _P, _P, _I, _P, _P],
    "gf_frontend_set_gate": [_P, _P, _P],
    "gf_frontend_set_gate_stage": [_P, ctypes.c_int],
    "gf_frontend_set_track_priority": [_P, ctypes.c_int],
    "gf_event_create": [_P, _P],
    "gf_event_destroy": [_P],
    "gf_frontend_bootstrap_host": [_P, _P, _P, _P, _D],
    "gf_frontend_step_host": [_P, _P],
    "gf_frontend_capture": [_P],
    "gf_frontend_sync": [_P],
    "gf_frontend_read": [_P, _I, _P, _S],
    "gf_frontend_write": [_P, _I, _P, _S],
    "gf_frontend_field": [_P, _I, _P, _P],
    "gf_set_budgets": [_P, _D, _D],
    "gf_frontend_set_test_clock": [_P, _P],
    "gf_frontend_set_time_log": [_P, _I],
    "gf_frontend_read_time_log": [_P, _P, _P, _P],
    "gf_dist_unique_id": [_P],
    "gf_dist_init": [_P, _I, _I, _P, _P],
    "gf_dist_destroy": [_P],
    "gf_dist_info": [_P, _P, _P],
    "gf_dist_channel_create": [_I, _P],
    "gf_dist_channel_destroy": [_P],
    "gf_dist_init_loopback": [_P, _I, _P, _P],
    "gf_dist_init_host": [_P, _I, _I, _P, _P, _P],
    "gf_dist_transport": [_P, _P],
    "gf_dist_bcast": [_P, _P, _S, _I],
    "gf_dist_allreduce": [_P, _P, _S, _I],
    "gf_dist_bcast_vocab": [_P, _P, _I],
    "gf_dist_bcast_map": [_P, _P, _I],
    "gf_vocab_download": [_P, _P, _P, _P, _P],
    "gf_select_map_points": [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P],
    "gf_select_pool": [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P],
    "gf_initialize": [_P, _P, _F, _I, _I, _P, _I, _P, _I, _P, _P, _P, _P, _P],
    "gf_initialize_dev": [_P, _P, _F, _I, _I, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P],
    "gf_initialize_batch_dev": [_P, _I, _P, _F, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P],
}


def _declare(l) -> None:
    for name, args in _PROTOS.items():
        fn = getattr(l, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int


def check(rc: int) -> None:
    if rc != GF_OK:
        raise GFError(rc, lib().gf_last_error().decode(errors="replace"))


def declared_symbols() -> list[str]:
    """Every function the ABI header declares (for the export test)."""
    src = open(ABI_HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gf_[a-z0-9_]+)\s*\(", src)))


def ptr(a):
    """Host numpy array or torch tensor -> c_void_p."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return ctypes.c_void_p(a.ctypes.data)
