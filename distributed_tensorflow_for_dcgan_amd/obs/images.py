"""Sample-grid images (reference ``save_images`` / ``merge`` / ``inverse_transform``,
``image_train.py:197-219``) and a dependency-free PNG encoder.

Fixes vs the reference: works for any channel count (c_dim = 1 MNIST grids), uses PIL when
available instead of the removed ``scipy.misc.imsave``, no debug print per image, honours
``--sample_dir``.
"""
from __future__ import annotations

import struct
import zlib
from typing import Sequence, Tuple

import numpy as np


def inverse_transform(images: np.ndarray) -> np.ndarray:
    """[-1, 1] -> [0, 1]"""
    return (np.asarray(images) + 1.0) / 2.0


def merge(images: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """Tile N HxWxC images into an (size[0]*H) x (size[1]*W) x C grid, row-major."""
    images = np.asarray(images)
    n, h, w = images.shape[:3]
    c = images.shape[3] if images.ndim == 4 else 1
    img = np.zeros((h * size[0], w * size[1], c), dtype=np.float32)
    for idx in range(min(n, size[0] * size[1])):
        i, j = idx % size[1], idx // size[1]
        img[j * h:(j + 1) * h, i * w:(i + 1) * w, :] = images[idx].reshape(h, w, c)
    return img


def encode_png(arr: np.ndarray) -> bytes:
    """uint8 HxW or HxWxC (C in 1,3,4) -> PNG bytes (zlib, filter 0)."""
    a = np.asarray(arr)
    if a.dtype != np.uint8:
        a = (np.clip(a, 0, 1) * 255 + 0.5).astype(np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    h, w, c = a.shape
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[c]
    raw = b"".join(b"\x00" + a[y].tobytes() for y in range(h))

    def chunk(t: bytes, d: bytes) -> bytes:
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


def imsave(path: str, img: np.ndarray) -> None:
    a = np.asarray(img)
    if a.dtype != np.uint8:
        a = (np.clip(a, 0, 1) * 255 + 0.5).astype(np.uint8)
    if a.ndim == 3 and a.shape[2] == 1:
        a = a[:, :, 0]
    try:
        from PIL import Image
        Image.fromarray(a).save(path)
    except ImportError:  # pragma: no cover
        with open(path, "wb") as f:
            f.write(encode_png(a))


def save_images(images: np.ndarray, size: Tuple[int, int], path: str) -> None:
    imsave(path, merge(inverse_transform(images), size))


def grid_size(n: int) -> Tuple[int, int]:
    """[8, 8] for the reference's 64 samples; near-square otherwise."""
    r = int(np.floor(np.sqrt(n)))
    while n % r:
        r -= 1
    return (r, n // r) if r > 1 else (int(np.ceil(np.sqrt(n))), int(np.ceil(np.sqrt(n))))
