"""gf_orb_slam_amd — MI355X-native GF-ORB-SLAM front-end hot path.

ORB extraction, Hamming matching, good-feature selection and pose
optimisation as hand-written gfx950 HIP kernels behind the C-ABI in
include/gfslam/abi.h (libgfslam.so). This package is the host-side mirror of
the reference operators (ORBextractor / ORBmatcher / Observability /
Optimizer) over that ABI.
"""
from ._lib import GFError, lib  # noqa: F401
from .orb import KEYPOINT_DTYPE, Context, ORBextractor, default_context  # noqa: F401

__all__ = ["GFError", "lib", "KEYPOINT_DTYPE", "Context", "ORBextractor", "default_context"]
