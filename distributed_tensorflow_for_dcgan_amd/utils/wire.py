"""Minimal protobuf wire format + CRC32C, enough for TFRecord / tf.train.Example /
TensorBoard Event / TF tensor-bundle files without TensorFlow or generated _pb2 modules.

The C++ host runtime (``csrc/host``) implements the hot paths (record framing, CRC32C,
Example parsing); this module is the reference implementation used by writers, tests and
the pure-Python fallback reader.
"""
from __future__ import annotations

import struct
from typing import Dict, Iterator, List, Tuple, Union

# ---------------------------------------------------------------- CRC32C (Castagnoli)
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes, crc: int = 0) -> int:
    try:  # fast path through the native extension when it is built
        from ..data import native
        return native.crc32c(data, crc)
    except Exception:
        pass
    crc ^= 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def crc32c_py(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def mask_crc(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def unmask_crc(m: int) -> int:
    rot = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------- varints / fields
def varint(n: int) -> bytes:
    if n < 0:
        n += 1 << 64
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = 0
    result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 70:
            raise ValueError("varint too long")


def f_varint(field: int, n: int) -> bytes:
    return varint(field << 3) + varint(n)


def f_bytes(field: int, data: Union[bytes, str]) -> bytes:
    if isinstance(data, str):
        data = data.encode()
    return varint((field << 3) | 2) + varint(len(data)) + data


def f_double(field: int, x: float) -> bytes:
    return varint((field << 3) | 1) + struct.pack("<d", x)


def f_float(field: int, x: float) -> bytes:
    return varint((field << 3) | 5) + struct.pack("<f", x)


def f_fixed32(field: int, x: int) -> bytes:
    return varint((field << 3) | 5) + struct.pack("<I", x & 0xFFFFFFFF)


def f_packed_doubles(field: int, xs) -> bytes:
    return f_bytes(field, struct.pack("<%dd" % len(xs), *xs))


def parse_fields(buf: bytes) -> Iterator[Tuple[int, int, Union[int, bytes]]]:
    """Yield (field_number, wire_type, value) for each field of a message."""
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = read_varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = read_varint(buf, pos)
        elif wt == 1:
            v = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = read_varint(buf, pos)
            v = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError("unsupported wire type %d" % wt)
        yield field, wt, v


def fields_dict(buf: bytes) -> Dict[int, List]:
    d: Dict[int, List] = {}
    for f, _, v in parse_fields(buf):
        d.setdefault(f, []).append(v)
    return d


# ---------------------------------------------------------------- tf.train.Example
def encode_example(features: Dict[str, Union[bytes, List[float], List[int]]]) -> bytes:
    """features: name -> bytes (BytesList), list of float (FloatList) or list of int (Int64List)."""
    entries = b""
    for name in sorted(features):
        val = features[name]
        if isinstance(val, (bytes, bytearray)):
            feat = f_bytes(1, f_bytes(1, bytes(val)))
        elif val and isinstance(val[0], float):
            feat = f_bytes(2, f_bytes(1, struct.pack("<%df" % len(val), *val)))
        else:
            feat = f_bytes(3, f_bytes(1, b"".join(varint(int(v)) for v in val)))
        entries += f_bytes(1, f_bytes(1, name) + f_bytes(2, feat))
    return f_bytes(1, entries)


def decode_example(buf: bytes) -> Dict[str, Union[bytes, List[float], List[int]]]:
    out: Dict[str, Union[bytes, List[float], List[int]]] = {}
    for f, _, features in parse_fields(buf):
        if f != 1:
            continue
        for f2, _, entry in parse_fields(features):
            if f2 != 1:
                continue
            key, feat = b"", b""
            for f3, _, v in parse_fields(entry):
                if f3 == 1:
                    key = v
                elif f3 == 2:
                    feat = v
            for kind, _, lst in parse_fields(feat):
                vals = [v for ff, _, v in parse_fields(lst) if ff == 1]
                if kind == 1:
                    out[key.decode()] = vals[0] if len(vals) == 1 else b"".join(vals)
                elif kind == 2:
                    fl: List[float] = []
                    for v in vals:
                        if isinstance(v, bytes):
                            fl += list(struct.unpack("<%df" % (len(v) // 4), v))
                    out[key.decode()] = fl
                elif kind == 3:
                    il: List[int] = []
                    for v in vals:
                        if isinstance(v, bytes):
                            p = 0
                            while p < len(v):
                                x, p = read_varint(v, p)
                                il.append(x)
                        else:
                            il.append(v)
                    out[key.decode()] = il
    return out
