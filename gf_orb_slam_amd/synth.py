"""Seeded synthetic inputs. No datasets are reachable from the
build or the GPU box, so every benchmark and parity case runs on these.

Frames: 2-octave value noise + ~400 uniform rectangles/discs, Gaussian
sigma 0.8 pre-smoothing, uniform noise +-3, clipped to u8. Seeds follow
0x6F52420 + stream*1000 + frame.
"""
from __future__ import annotations

import numpy as np

CAMERAS = {
    # name: (width, height, fx, fy, cx, cy)
    "euroc": (752, 480, 457.3, 457.3, 367.215, 248.375),
    "tum": (640, 480, 525.0, 525.0, 319.5, 239.5),
}


def frame_seed(stream: int, frame: int) -> int:
    return 0x6F52420 + stream * 1000 + frame


def _value_noise(rng, h, w, cell):
    gh, gw = h // cell + 2, w // cell + 2
    g = rng.uniform(0, 1, (gh, gw)).astype(np.float32)
    ys = np.arange(h, dtype=np.float32) / cell
    xs = np.arange(w, dtype=np.float32) / cell
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    c = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    return a * (1 - fx) * (1 - fy) + b * fx * (1 - fy) + c * (1 - fx) * fy + d * fx * fy


def _gauss1d(sigma):
    r = int(np.ceil(3 * sigma))
    x = np.arange(-r, r + 1, dtype=np.float32)
    k = np.exp(-0.5 * (x / sigma) ** 2)
    return k / k.sum()


def synth_frame(width: int, height: int, seed: int, n_shapes: int = 400) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = 60 * _value_noise(rng, height, width, 48) + 40 * _value_noise(rng, height, width, 12) + 70
    yy, xx = np.mgrid[0:height, 0:width]
    for _ in range(n_shapes):
        val = rng.uniform(0, 255)
        if rng.uniform() < 0.5:
            x0, y0 = rng.integers(0, width), rng.integers(0, height)
            w, h = rng.integers(4, 60), rng.integers(4, 60)
            img[y0:y0 + h, x0:x0 + w] = val
        else:
            cx, cy, r = rng.uniform(0, width), rng.uniform(0, height), rng.uniform(3, 30)
            x0, x1 = max(int(cx - r), 0), min(int(cx + r) + 1, width)
            y0, y1 = max(int(cy - r), 0), min(int(cy + r) + 1, height)
            if x0 >= x1 or y0 >= y1:
                continue
            sub = (xx[y0:y1, x0:x1] - cx) ** 2 + (yy[y0:y1, x0:x1] - cy) ** 2 <= r * r
            img[y0:y1, x0:x1][sub] = val
    k = _gauss1d(0.8)
    img = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, img)
    img = np.apply_along_axis(lambda c: np.convolve(c, k, mode="same"), 0, img)
    img += rng.uniform(-3, 3, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def synth_sequence(camera: str, nframes: int, stream: int = 0) -> np.ndarray:
    w, h = CAMERAS[camera][:2]
    return np.stack([synth_frame(w, h, frame_seed(stream, f)) for f in range(nframes)])
