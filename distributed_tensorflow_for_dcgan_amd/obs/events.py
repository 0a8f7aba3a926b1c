"""TensorBoard event-file writer (no TensorFlow / tensorboard dependency).

Writes ``events.out.tfevents.<time>.<host>`` files: TFRecord-framed ``Event`` protos, first a
``file_version: "brain.Event:2"`` record, then ``Summary`` values -- scalars, histograms (TF's
default exponential bucket limits) and PNG images -- the same kinds of summaries the reference
emits through ``tf.scalar_summary`` / ``tf.histogram_summary`` / ``tf.image_summary``
(``image_train.py:86-101,114-118``, ``distriubted_model.py:75-80``).
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Iterable, List, Optional, Sequence

import numpy as np

from ..utils import wire
from .images import encode_png


def _default_buckets() -> List[float]:
    """TF histogram bucket limits: +-1e-12 * 1.1^k up to 1e20, +-DBL_MAX, and 0."""
    pos = []
    v = 1e-12
    while v < 1e20:
        pos.append(v)
        v *= 1.1
    pos.append(1.7976931348623157e308)
    return [-x for x in reversed(pos)] + [0.0] + pos


BUCKET_EDGES = _default_buckets()
_BUCKETS = np.array(BUCKET_EDGES)


def histogram_proto(values: np.ndarray) -> bytes:
    v = np.asarray(values, dtype=np.float64).ravel()
    if v.size == 0:
        v = np.zeros(1)
    idx = np.searchsorted(_BUCKETS, v, side="left")
    counts = np.bincount(idx, minlength=len(_BUCKETS)).astype(np.float64)
    nz = np.nonzero(counts)[0]
    # TF emits only the non-empty range (with the limits of the kept buckets)
    lo, hi = (nz[0], nz[-1] + 1) if nz.size else (0, 1)
    limits = _BUCKETS[lo:hi].tolist()
    buckets = counts[lo:hi].tolist()
    return (wire.f_double(1, float(v.min())) + wire.f_double(2, float(v.max())) + wire.f_double(3, float(v.size)) +
            wire.f_double(4, float(v.sum())) + wire.f_double(5, float((v * v).sum())) +
            wire.f_packed_doubles(6, limits) + wire.f_packed_doubles(7, buckets))


def histogram_proto_from_stats(row: Sequence[float]) -> bytes:
    """HistogramProto from a device statistics row (summary.hip: [min, max, n, sum, sumsq,
    zeros, counts over BUCKET_EDGES...]) -- the same proto histogram_proto builds on the host."""
    row = np.asarray(row, dtype=np.float64)
    E = len(_BUCKETS)
    counts = row[6:6 + E].copy()
    if row.size > 6 + E:
        counts[-1] += row[6 + E:].sum()  # values above the last edge (inf): the last bucket
    nz = np.nonzero(counts)[0]
    lo, hi = (nz[0], nz[-1] + 1) if nz.size else (0, 1)
    return (wire.f_double(1, float(row[0])) + wire.f_double(2, float(row[1])) + wire.f_double(3, float(row[2])) +
            wire.f_double(4, float(row[3])) + wire.f_double(5, float(row[4])) +
            wire.f_packed_doubles(6, _BUCKETS[lo:hi].tolist()) + wire.f_packed_doubles(7, counts[lo:hi].tolist()))


class SummaryWriter:
    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.%d.%s%s" % (int(time.time()), socket.gethostname(), filename_suffix)
        self.path = os.path.join(logdir, name)
        self.f = open(self.path, "ab")
        self._write_event(wire.f_double(1, time.time()) + wire.f_bytes(3, "brain.Event:2"))

    def _write_event(self, ev: bytes) -> None:
        hdr = struct.pack("<Q", len(ev))
        self.f.write(hdr + struct.pack("<I", wire.masked_crc32c(hdr)) + ev +
                     struct.pack("<I", wire.masked_crc32c(ev)))

    def add_summary_values(self, values: Sequence[bytes], step: int, wall_time: Optional[float] = None) -> None:
        ev = (wire.f_double(1, wall_time or time.time()) + wire.f_varint(2, int(step)) +
              wire.f_bytes(5, b"".join(values)))
        self._write_event(ev)

    # value builders ---------------------------------------------------
    @staticmethod
    def scalar(tag: str, x: float) -> bytes:
        return wire.f_bytes(1, wire.f_bytes(1, tag) + wire.f_float(2, float(x)))

    @staticmethod
    def histogram(tag: str, values: np.ndarray) -> bytes:
        return wire.f_bytes(1, wire.f_bytes(1, tag) + wire.f_bytes(5, histogram_proto(values)))

    @staticmethod
    def histogram_from_stats(tag: str, row: Sequence[float]) -> bytes:
        return wire.f_bytes(1, wire.f_bytes(1, tag) + wire.f_bytes(5, histogram_proto_from_stats(row)))

    @staticmethod
    def image(tag: str, img: np.ndarray) -> bytes:
        """img: HxWxC float in [0,1] or uint8."""
        a = np.asarray(img)
        if a.dtype != np.uint8:
            a = (np.clip(a, 0, 1) * 255 + 0.5).astype(np.uint8)
        if a.ndim == 2:
            a = a[:, :, None]
        h, w, c = a.shape
        im = (wire.f_varint(1, h) + wire.f_varint(2, w) + wire.f_varint(3, c) + wire.f_bytes(4, encode_png(a)))
        return wire.f_bytes(1, wire.f_bytes(1, tag) + wire.f_bytes(4, im))

    def add_scalars(self, scalars: dict, step: int) -> None:
        self.add_summary_values([self.scalar(k, v) for k, v in scalars.items()], step)

    def flush(self) -> None:
        self.f.flush()

    def close(self) -> None:
        self.f.close()


def read_events(path: str) -> List[dict]:
    """Decode an event file (for tests / tooling): list of {wall_time, step, values}."""
    from ..data.tfrecord import read_records
    out = []
    for rec in read_records(path):
        d = {"values": []}
        for f, wt, v in wire.parse_fields(rec):
            if f == 1:
                d["wall_time"] = struct.unpack("<d", v)[0]
            elif f == 2:
                d["step"] = v
            elif f == 3:
                d["file_version"] = v.decode()
            elif f == 5:
                for f2, _, val in wire.parse_fields(v):
                    if f2 != 1:
                        continue
                    item = {}
                    for f3, wt3, x in wire.parse_fields(val):
                        if f3 == 1:
                            item["tag"] = x.decode()
                        elif f3 == 2:
                            item["simple_value"] = struct.unpack("<f", x)[0]
                        elif f3 == 4:
                            item["image"] = wire.fields_dict(x)
                        elif f3 == 5:
                            item["histo"] = wire.fields_dict(x)
                    d["values"].append(item)
        out.append(d)
    return out
