"""TensorFlow V2 tensor-bundle checkpoints, written and read without TensorFlow.

A checkpoint prefix ``model.ckpt-N`` is two files (the layout ``tf.train.Saver`` produces for
TF >= 0.12):

* ``model.ckpt-N.index`` -- an SSTable (LevelDB table format: prefix-compressed data blocks
  with restart points, a metaindex block, an index block, a 48-byte footer with the magic
  0xdb4775248b80fb57; every block followed by a type byte and a masked CRC32C). Key ``""``
  holds a ``BundleHeaderProto``; every other key is a variable name mapping to a
  ``BundleEntryProto`` {dtype, shape, shard_id, offset, size, crc32c}.
* ``model.ckpt-N.data-00000-of-00001`` -- the raw little-endian tensor bytes.

The writer emits uncompressed blocks (valid for TF readers). The reader also understands
Snappy-compressed blocks (what TF's own writer may produce), so checkpoints written by the
reference can be imported. (Parity with a real TF reader is "unpinned": TensorFlow is not
installed here.)
"""
from __future__ import annotations

import os
import struct
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np

from ..utils import wire

MAGIC = 0xDB4775248B80FB57
DT = {np.dtype("float32"): 1, np.dtype("float64"): 2, np.dtype("int32"): 3, np.dtype("uint8"): 4,
      np.dtype("int16"): 5, np.dtype("int8"): 6, np.dtype("int64"): 9, np.dtype("bool"): 10,
      np.dtype("uint16"): 17}
DT_INV = {v: k for k, v in DT.items()}
DT_BFLOAT16 = 14


# ---------------------------------------------------------------- table writer
class _BlockBuilder:
    def __init__(self, restart_interval: int = 16):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last_key = b""
        self.interval = restart_interval
        self.n = 0

    def add(self, key: bytes, value: bytes) -> None:
        shared = 0
        if self.counter < self.interval:
            m = min(len(self.last_key), len(key))
            while shared < m and self.last_key[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        non_shared = len(key) - shared
        self.buf += wire.varint(shared) + wire.varint(non_shared) + wire.varint(len(value))
        self.buf += key[shared:] + value
        self.last_key = key
        self.counter += 1
        self.n += 1

    def finish(self) -> bytes:
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts)
        return out + struct.pack("<I", len(self.restarts))

    def size_estimate(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4


def _handle(offset: int, size: int) -> bytes:
    return wire.varint(offset) + wire.varint(size)


class TableWriter:
    def __init__(self, path: str, block_size: int = 262144):
        self.f = open(path, "wb")
        self.offset = 0
        self.block = _BlockBuilder()
        self.index = _BlockBuilder(restart_interval=1)
        self.block_size = block_size
        self.last_key = None

    def _write_block(self, contents: bytes) -> Tuple[int, int]:
        trailer_type = b"\x00"
        crc = wire.mask_crc(wire.crc32c(contents + trailer_type))
        off = self.offset
        self.f.write(contents + trailer_type + struct.pack("<I", crc))
        self.offset += len(contents) + 5
        return off, len(contents)

    def _flush(self) -> None:
        if self.block.n == 0:
            return
        off, size = self._write_block(self.block.finish())
        self.index.add(self.block.last_key, _handle(off, size))
        self.block = _BlockBuilder()

    def add(self, key: bytes, value: bytes) -> None:
        if self.last_key is not None and key <= self.last_key:
            raise ValueError("keys must be added in strictly increasing order")
        self.last_key = key
        self.block.add(key, value)
        if self.block.size_estimate() >= self.block_size:
            self._flush()

    def close(self) -> None:
        self._flush()
        meta_off, meta_size = self._write_block(_BlockBuilder().finish())
        idx_off, idx_size = self._write_block(self.index.finish())
        footer = _handle(meta_off, meta_size) + _handle(idx_off, idx_size)
        footer += b"\x00" * (40 - len(footer))
        footer += struct.pack("<Q", MAGIC)
        self.f.write(footer)
        self.f.close()


# ---------------------------------------------------------------- table reader
def _snappy_decompress(src: bytes) -> bytes:
    n, pos = wire.read_varint(src, 0)
    out = bytearray()
    while pos < len(src):
        tag = src[pos]
        pos += 1
        t = tag & 3
        if t == 0:  # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(src[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += src[pos:pos + ln]
            pos += ln
            continue
        if t == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | src[pos]
            pos += 1
        elif t == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 4], "little")
            pos += 4
        start = len(out) - off
        for i in range(ln):  # may overlap
            out.append(out[start + i])
    if len(out) != n:
        raise ValueError("snappy: bad length")
    return bytes(out)


def _read_block(data: bytes, off: int, size: int, verify: bool = True) -> bytes:
    contents = data[off:off + size]
    typ = data[off + size]
    if verify:
        (crc,) = struct.unpack("<I", data[off + size + 1:off + size + 5])
        if wire.mask_crc(wire.crc32c(contents + bytes([typ]))) != crc:
            raise IOError("SSTable block CRC mismatch")
    if typ == 1:
        contents = _snappy_decompress(contents)
    elif typ != 0:
        raise IOError("unsupported block compression %d" % typ)
    return contents


def _block_entries(block: bytes) -> List[Tuple[bytes, bytes]]:
    (nres,) = struct.unpack("<I", block[-4:])
    end = len(block) - 4 - 4 * nres
    pos, key, out = 0, b"", []
    while pos < end:
        shared, pos = wire.read_varint(block, pos)
        non_shared, pos = wire.read_varint(block, pos)
        vlen, pos = wire.read_varint(block, pos)
        key = key[:shared] + block[pos:pos + non_shared]
        pos += non_shared
        out.append((key, block[pos:pos + vlen]))
        pos += vlen
    return out


def read_table(path: str, verify: bool = True) -> "OrderedDict[bytes, bytes]":
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 48 or struct.unpack("<Q", data[-8:])[0] != MAGIC:
        raise IOError("not an SSTable: %s" % path)
    footer = data[-48:-8]
    _, p = wire.read_varint(footer, 0)
    _, p = wire.read_varint(footer, p)
    idx_off, p = wire.read_varint(footer, p)
    idx_size, p = wire.read_varint(footer, p)
    out: "OrderedDict[bytes, bytes]" = OrderedDict()
    for _, handle in _block_entries(_read_block(data, idx_off, idx_size, verify)):
        off, q = wire.read_varint(handle, 0)
        size, _ = wire.read_varint(handle, q)
        for k, v in _block_entries(_read_block(data, off, size, verify)):
            out[k] = v
    return out


# ---------------------------------------------------------------- bundle
def _shape_proto(shape) -> bytes:
    return b"".join(wire.f_bytes(2, wire.f_varint(1, int(d))) for d in shape)


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """Atomically write ``prefix.index`` + ``prefix.data-00000-of-00001``."""
    data_path = prefix + ".data-00000-of-00001"
    index_path = prefix + ".index"
    entries = []
    off = 0
    with open(data_path + ".tmp", "wb") as df:
        for name in sorted(tensors):
            a = np.require(np.asarray(tensors[name]), requirements="C")  # keeps 0-d scalars 0-d
            if a.dtype not in DT:
                raise TypeError("unsupported dtype %s for %s" % (a.dtype, name))
            raw = a.astype(a.dtype.newbyteorder("<")).tobytes()
            df.write(raw)
            crc = wire.mask_crc(wire.crc32c(raw))
            ent = (wire.f_varint(1, DT[a.dtype]) + wire.f_bytes(2, _shape_proto(a.shape)) +
                   (wire.f_varint(4, off) if off else b"") + wire.f_varint(5, len(raw)) + wire.f_fixed32(6, crc))
            entries.append((name.encode(), ent))
            off += len(raw)
    header = wire.f_varint(1, 1) + wire.f_bytes(3, wire.f_varint(1, 1))
    tw = TableWriter(index_path + ".tmp")
    tw.add(b"", header)
    for k, v in entries:
        tw.add(k, v)
    tw.close()
    os.replace(data_path + ".tmp", data_path)
    os.replace(index_path + ".tmp", index_path)


def read_bundle(prefix: str, verify: bool = True) -> "OrderedDict[str, np.ndarray]":
    table = read_table(prefix + ".index", verify)
    header = wire.fields_dict(table.get(b"", b""))
    num_shards = header.get(1, [1])[0]
    shards = {}
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, val in table.items():
        if key == b"":
            continue
        f = wire.fields_dict(val)
        dtype = f.get(1, [0])[0]
        shape = []
        for sp in f.get(2, []):
            for dim in wire.fields_dict(sp).get(2, []):
                shape.append(wire.fields_dict(dim).get(1, [0])[0])
        shard = f.get(3, [0])[0]
        off = f.get(4, [0])[0]
        size = f.get(5, [0])[0]
        crc = struct.unpack("<I", f[6][0])[0] if 6 in f else None
        if shard not in shards:
            with open("%s.data-%05d-of-%05d" % (prefix, shard, num_shards), "rb") as df:
                shards[shard] = df.read()
        raw = shards[shard][off:off + size]
        if verify and crc is not None and wire.mask_crc(wire.crc32c(raw)) != crc:
            raise IOError("tensor %s: CRC mismatch" % key.decode())
        if dtype == DT_BFLOAT16:
            u = np.frombuffer(raw, "<u2").astype(np.uint32) << 16
            arr = u.view(np.float32)
        else:
            arr = np.frombuffer(raw, DT_INV[dtype].newbyteorder("<"))
        out[key.decode()] = arr.reshape(shape).copy()
    return out
