"""Host-side mirror of ORB_SLAM::ORBextractor (include/ORBextractor.h:51-70).

Same constructor arguments and call semantics as the reference operator
(`extractor(image, mask, keypoints, descriptors)` becomes
`keypoints, descriptors = extractor(image)`); all compute runs in
libgfslam.so on the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import KeyPoint, check, lib, ptr

# numpy view of the 28-byte cv::KeyPoint layout
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == ctypes.sizeof(KeyPoint) == 28

HARRIS_SCORE, FAST_SCORE = 0, 1


class Context:
    """One HIP stream on one device (gf_ctx)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check(lib().gf_ctx_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().gf_ctx_stream(self._h, ctypes.byref(s)))
        return s.value or 0

    def sync(self) -> None:
        check(lib().gf_ctx_sync(self._h))

    def close(self) -> None:
        if self._h:
            lib().gf_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


class ORBextractor:
    """ORB_SLAM::ORBextractor(nfeatures, scaleFactor, nlevels, scoreType, fastTh).

    The frame geometry is bound at the first call (or given explicitly), as the
    pyramid/cell plan depends on it.
    """

    HARRIS_SCORE = HARRIS_SCORE
    FAST_SCORE = FAST_SCORE

    def __init__(self, nfeatures: int = 1000, scaleFactor: float = 1.2, nlevels: int = 8,
                 scoreType: int = FAST_SCORE, fastTh: int = 20, *, width: int | None = None,
                 height: int | None = None, max_batch: int = 1, ctx: Context | None = None):
        self.nfeatures, self.scaleFactor, self.nlevels = nfeatures, float(scaleFactor), nlevels
        self.scoreType, self.fastTh, self.max_batch = scoreType, fastTh, max_batch
        self.ctx = ctx or default_context()
        self._h = None
        self._wh = None
        if width is not None and height is not None:
            self._bind(width, height)

    def _bind(self, width: int, height: int) -> None:
        if self._wh == (width, height):
            return
        self._free()
        h = ctypes.c_void_p()
        check(lib().gf_extractor_create(self.ctx.handle, int(self.nfeatures), ctypes.c_float(self.scaleFactor),
                                        int(self.nlevels), int(self.scoreType), int(self.fastTh), int(width),
                                        int(height), int(self.max_batch), ctypes.byref(h)))
        self._h, self._wh = h, (width, height)
        cap = ctypes.c_int()
        check(lib().gf_extractor_capacity(self._h, ctypes.byref(cap)))
        self.capacity = cap.value

    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactor(self) -> float:
        return float(np.float32(self.scaleFactor))

    def features_per_level(self) -> list[int]:
        if self._h is None:
            raise RuntimeError("extractor not bound to a frame size yet")
        arr = (ctypes.c_int * self.nlevels)()
        check(lib().gf_extractor_info(self._h, None, None, arr))
        return list(arr)

    def __call__(self, image: np.ndarray, mask=None):
        """Returns (keypoints: KEYPOINT_DTYPE[N], descriptors: uint8[N, 32])."""
        # The reference takes a CV_8UC1 mask (ORBextractor.cc:775-778) and builds
        # mvMaskPyramid from it (:929-993), but the per-cell FAST call never
        # receives cellMask (:614-621): a mask does not change the outputs. It
        # is accepted and checked the same way, then not used.
        if mask is not None and getattr(mask, "size", 0):
            m = np.asarray(mask)
            if m.dtype != np.uint8 or m.ndim != 2:
                raise ValueError("mask must be an 8-bit single-channel image (CV_8UC1)")
        if image is None or image.size == 0:
            return np.zeros(0, KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8)
        image = np.ascontiguousarray(image, dtype=np.uint8)
        hgt, wid = image.shape
        self._bind(wid, hgt)
        kps = np.zeros(self.capacity, KEYPOINT_DTYPE)
        desc = np.zeros((self.capacity, 32), np.uint8)
        n = ctypes.c_int()
        check(lib().gf_orb_extract(self._h, ptr(image), int(image.strides[0]), ptr(kps), ptr(desc),
                                   int(self.capacity), ctypes.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def extract_batch_dev(self, imgs, kps, desc, counts, stream: int | None = None) -> None:
        """Device family: imgs uint8 [F, H, W] (torch, on GPU), kps int8-viewable
        [F, cap, 28] bytes, desc uint8 [F, cap, 32], counts int32 [F]."""
        f, hgt, wid = imgs.shape
        if imgs.stride(2) != 1:
            raise ValueError("image rows must be contiguous (stride(2) == 1)")
        self._bind(wid, hgt)
        check(lib().gf_orb_extract_batch_dev(self._h, int(f), ptr(imgs), ctypes.c_size_t(int(imgs.stride(0))),
                                             int(imgs.stride(1)), ptr(kps), ptr(desc), ptr(counts),
                                             int(kps.shape[1]), ctypes.c_void_p(stream or self.ctx.stream)))

    def debug_level(self, level: int, which: int = 0, frame: int = 0) -> np.ndarray:
        w, h = ctypes.c_int(), ctypes.c_int()
        check(lib().gf_extractor_debug_level(self._h, frame, level, which, None, ctypes.byref(w), ctypes.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        check(lib().gf_extractor_debug_level(self._h, frame, level, which, ptr(out), ctypes.byref(w),
                                             ctypes.byref(h)))
        return out

    def _free(self):
        if self._h is not None:
            lib().gf_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass
