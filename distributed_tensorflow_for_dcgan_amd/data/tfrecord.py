"""TFRecord files of ``tf.train.Example`` images (reference format, ``image_input.py:40-51``).

Each record: ``uint64 len | uint32 masked_crc32c(len) | data | uint32 masked_crc32c(data)``;
data = Example with one bytes feature ``image_raw`` holding raw little-endian pixels
(float64 in the reference; float32 and uint8 are accepted too). The reference repo ships no
writer -- :func:`write_image_records` creates such files (for tests, fixtures and for
converting image folders).
"""
from __future__ import annotations

import os
import struct
from typing import Iterable, Iterator, List, Optional

import numpy as np

from ..utils import wire


def write_records(path: str, records: Iterable[bytes]) -> int:
    n = 0
    with open(path + ".tmp", "wb") as f:
        for rec in records:
            hdr = struct.pack("<Q", len(rec))
            f.write(hdr)
            f.write(struct.pack("<I", wire.masked_crc32c(hdr)))
            f.write(rec)
            f.write(struct.pack("<I", wire.masked_crc32c(rec)))
            n += 1
    os.replace(path + ".tmp", path)
    return n


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if not hdr:
                return
            if len(hdr) != 12:
                raise IOError("truncated TFRecord header in %s" % path)
            (ln,) = struct.unpack("<Q", hdr[:8])
            (lcrc,) = struct.unpack("<I", hdr[8:])
            if verify and wire.masked_crc32c(hdr[:8]) != lcrc:
                raise IOError("TFRecord length CRC mismatch in %s" % path)
            data = f.read(ln)
            foot = f.read(4)
            if len(data) != ln or len(foot) != 4:
                raise IOError("truncated TFRecord in %s" % path)
            if verify and wire.masked_crc32c(data) != struct.unpack("<I", foot)[0]:
                raise IOError("TFRecord data CRC mismatch in %s" % path)
            yield data


def encode_image_example(img: np.ndarray, dtype: str = "float64", feature: str = "image_raw") -> bytes:
    arr = np.ascontiguousarray(img, dtype={"float64": "<f8", "float32": "<f4", "uint8": "u1"}[dtype])
    return wire.encode_example({feature: arr.tobytes()})


def decode_image_example(rec: bytes, shape, feature: str = "image_raw") -> np.ndarray:
    raw = wire.decode_example(rec)[feature]
    n = int(np.prod(shape))
    if len(raw) == 8 * n:
        a = np.frombuffer(raw, "<f8")
    elif len(raw) == 4 * n:
        a = np.frombuffer(raw, "<f4")
    elif len(raw) == n:
        a = np.frombuffer(raw, "u1").astype(np.float32) / 127.5 - 1.0
    else:
        raise ValueError("image_raw has %d bytes for shape %s" % (len(raw), tuple(shape)))
    return a.astype(np.float32).reshape(shape)


def write_image_records(path: str, images: np.ndarray, dtype: str = "float64") -> int:
    """images: [N,H,W,C] in the model range [-1, 1] (float) or [0,255] uint8."""
    return write_records(path, (encode_image_example(im, dtype) for im in images))


def list_record_files(data_dir: str) -> List[str]:
    """All files of ``data_dir`` (the reference reads every file, ``image_input.py:107-113``)."""
    if not os.path.isdir(data_dir):
        raise FileNotFoundError("data directory not found: %s" % data_dir)
    files = sorted(os.path.join(data_dir, f) for f in os.listdir(data_dir)
                   if not f.startswith(".") and os.path.isfile(os.path.join(data_dir, f)))
    if not files:
        raise FileNotFoundError("no input files in %s" % data_dir)
    return files


def count_records(files: List[str]) -> int:
    try:
        from . import native
        return sum(int(native.ext().count_records(f)) for f in files)
    except Exception:
        return sum(1 for f in files for _ in read_records(f, verify=False))
