"""Dependency-free TensorBoard event writer.

The reference logs through ``torch.utils.tensorboard.SummaryWriter``
(``train.py:56-61``, ``utils/tools.py:82-107``); the ``tensorboard`` package is
not installed on the target image, so this module writes the TFRecord event
format directly (length + masked CRC32C framing, hand-encoded ``Event`` /
``Summary`` protobufs).  Tags are kept identical (``Loss/total_loss``,
``Weight/learning_rate`` ...) so existing dashboards work.  Scalars go to
TensorBoard events *and* a ``scalars.jsonl`` side file; audio is written as
WAV files next to the events, figures as PNG.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _bytes_field(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def _event(wall: float, step: int, summary: bytes = b"", file_version: str = "") -> bytes:
    out = _field(1, 1) + struct.pack("<d", wall)
    out += _field(2, 0) + _varint(int(step))
    if file_version:
        out += _bytes_field(3, file_version.encode())
    if summary:
        out += _bytes_field(5, summary)
    return out


def _scalar_summary(tag: str, value: float) -> bytes:
    val = _bytes_field(1, tag.encode()) + _field(2, 5) + struct.pack("<f", float(value))
    return _bytes_field(1, val)


class SummaryWriter:
    def __init__(self, log_dir: str):
        os.makedirs(log_dir, exist_ok=True)
        self.log_dir = log_dir
        name = "events.out.tfevents.%d.%s.ssamd" % (int(time.time()), socket.gethostname())
        self._f = open(os.path.join(log_dir, name), "ab")
        self._json = open(os.path.join(log_dir, "scalars.jsonl"), "a")
        self._write(_event(time.time(), 0, file_version="brain.Event:2"))

    def _write(self, rec: bytes):
        header = struct.pack("<Q", len(rec))
        self._f.write(header + struct.pack("<I", _masked_crc(header)) + rec + struct.pack("<I", _masked_crc(rec)))
        self._f.flush()

    def add_scalar(self, tag, value, step=0):
        self._write(_event(time.time(), step or 0, _scalar_summary(tag, value)))
        self._json.write(json.dumps({"tag": tag, "value": float(value), "step": int(step or 0)}) + "\n")
        self._json.flush()

    def add_figure(self, tag, fig, step=0):
        safe = tag.replace("/", "_")
        fig.savefig(os.path.join(self.log_dir, f"{safe}.png"))

    def add_audio(self, tag, audio, step=0, sample_rate=22050):
        from ..audio.io import write_wav

        safe = tag.replace("/", "_")
        write_wav(os.path.join(self.log_dir, f"{safe}.wav"), sample_rate, audio)

    def close(self):
        self._f.close()
        self._json.close()


def read_scalars(path: str):
    """Parse an event file back into [(step, tag, value)] (used by tests)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        (n,) = struct.unpack_from("<Q", data, pos)
        rec = data[pos + 12: pos + 12 + n]
        pos += 12 + n + 4
        # minimal decode: find step (field 2) and scalar summaries (field 5)
        i, step, tags = 0, 0, []
        while i < len(rec):
            key, i = _read_varint(rec, i)
            num, wire = key >> 3, key & 7
            if wire == 0:
                v, i = _read_varint(rec, i)
                if num == 2:
                    step = v
            elif wire == 1:
                i += 8
            elif wire == 5:
                i += 4
            elif wire == 2:
                ln, i = _read_varint(rec, i)
                payload = rec[i:i + ln]
                i += ln
                if num == 5:
                    tags += _decode_summary(payload)
        out += [(step, t, v) for t, v in tags]
    return out


def _read_varint(b, i):
    shift = res = 0
    while True:
        x = b[i]
        i += 1
        res |= (x & 0x7F) << shift
        if not x & 0x80:
            return res, i
        shift += 7


def _decode_summary(payload):
    vals = []
    i = 0
    while i < len(payload):
        key, i = _read_varint(payload, i)
        ln, i = _read_varint(payload, i)
        val = payload[i:i + ln]
        i += ln
        j, tag, sv = 0, "", None
        while j < len(val):
            k, j = _read_varint(val, j)
            if k >> 3 == 1:
                l2, j = _read_varint(val, j)
                tag = val[j:j + l2].decode()
                j += l2
            elif k & 7 == 5:
                sv = struct.unpack_from("<f", val, j)[0]
                j += 4
            else:
                break
        vals.append((tag, sv))
    return vals
