"""Dependency-free TensorBoard scalar writer.

The reference logs `Train/Samples/*` scalars through tensorboardX.SummaryWriter
(engine.py:1057-1068,1223-1275).  Neither tensorboard nor tensorboardX is part of this stack,
so this writes the event-file format directly: TFRecord framing (length, masked CRC32C of the
length, payload, masked CRC32C of the payload) around hand-encoded `Event{wall_time, step,
file_version | summary{value{tag, simple_value}}}` protobufs.  Files are readable by any
TensorBoard.  A `scalars.csv` sidecar is written next to them for quick inspection.
"""

from __future__ import annotations

import os
import socket
import struct
import time

_CRC_TABLE = None


def _crc32c(data: bytes) -> int:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        tbl = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            tbl.append(c)
        _CRC_TABLE = tbl
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = _crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _len_delimited(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int = 0, file_version: str = None, scalars=None) -> bytes:
    ev = _field(1, 1) + struct.pack("<d", wall_time)
    ev += _field(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _len_delimited(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, val in scalars:
            v = _len_delimited(1, tag.encode()) + _field(2, 5) + struct.pack("<f", float(val))
            summ += _len_delimited(1, v)
        ev += _len_delimited(5, summ)
    return ev


def frame(payload: bytes) -> bytes:
    hdr = struct.pack("<Q", len(payload))
    return hdr + struct.pack("<I", masked_crc32c(hdr)) + payload + struct.pack("<I", masked_crc32c(payload))


class EventFileWriter:
    """Minimal SummaryWriter: add_scalar / add_scalars / flush / close."""

    def __init__(self, log_dir: str, filename_suffix: str = ""):
        os.makedirs(log_dir, exist_ok=True)
        self.log_dir = log_dir
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{filename_suffix}"
        self.path = os.path.join(log_dir, name)
        self._f = open(self.path, "ab")
        self._csv = open(os.path.join(log_dir, "scalars.csv"), "a")
        self._f.write(frame(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalar(self, tag, scalar_value, global_step=None, walltime=None):
        if hasattr(scalar_value, "item"):
            scalar_value = scalar_value.item()
        wt = walltime or time.time()
        self._f.write(frame(encode_event(wt, global_step or 0, scalars=[(tag, scalar_value)])))
        self._csv.write(f"{wt:.3f},{global_step or 0},{tag},{float(scalar_value)}\n")

    def add_scalars(self, main_tag, tag_scalar_dict, global_step=None, walltime=None):
        for k, v in tag_scalar_dict.items():
            self.add_scalar(f"{main_tag}/{k}", v, global_step, walltime)

    def flush(self):
        self._f.flush()
        self._csv.flush()

    def close(self):
        self.flush()
        self._f.close()
        self._csv.close()


def read_events(path):
    """Decode an event file written above -> list of (step, tag, value) (tests/tools)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        (n,) = struct.unpack_from("<Q", data, pos)
        assert struct.unpack_from("<I", data, pos + 8)[0] == masked_crc32c(data[pos:pos + 8])
        payload = data[pos + 12: pos + 12 + n]
        assert struct.unpack_from("<I", data, pos + 12 + n)[0] == masked_crc32c(payload)
        pos += 16 + n
        out += _decode_event(payload)
    return out


def _read_varint(b, i):
    shift = v = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << shift
        shift += 7
        if not x & 0x80:
            return v, i


def _decode_event(b):
    i, step, res = 0, 0, []
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wire = key >> 3, key & 7
        if wire == 1:
            i += 8
        elif wire == 0:
            val, i = _read_varint(b, i)
            if num == 2:
                step = val
        elif wire == 2:
            ln, i = _read_varint(b, i)
            chunk = b[i:i + ln]
            i += ln
            if num == 5:
                res += [(tag, val) for tag, val in _decode_summary(chunk)]
    return [(step, t, v) for t, v in res]


def _decode_summary(b):
    i, out = 0, []
    while i < len(b):
        key, i = _read_varint(b, i)
        ln, i = _read_varint(b, i)
        v = b[i:i + ln]
        i += ln
        j, tag, val = 0, None, None
        while j < len(v):
            k, j = _read_varint(v, j)
            if k >> 3 == 1:
                l2, j = _read_varint(v, j)
                tag = v[j:j + l2].decode()
                j += l2
            elif k >> 3 == 2:
                val = struct.unpack_from("<f", v, j)[0]
                j += 4
        out.append((tag, val))
    return out
