"""TFRecord / tf.Event encoding without TensorFlow."""
import os
import socket
import struct
import time
from typing import Iterator, List, Optional, Tuple


def _make_table() -> List[int]:
    poly = 0x82F63B78
    table = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        table.append(c)
    return table


_TABLE = _make_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


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


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: Optional[float] = None) -> bytes:
    val = _ld(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(value))
    summary = _ld(1, val)
    return (_varint((1 << 3) | 1) + struct.pack("<d", wall_time if wall_time is not None else time.time())
            + _varint((2 << 3) | 0) + _varint(int(step)) + _ld(5, summary))


def encode_file_version_event(wall_time: Optional[float] = None) -> bytes:
    return (_varint((1 << 3) | 1) + struct.pack("<d", wall_time if wall_time is not None else time.time())
            + _ld(3, b"brain.Event:2"))


def frame(record: bytes) -> bytes:
    header = struct.pack("<Q", len(record))
    return header + struct.pack("<I", masked_crc32c(header)) + record + struct.pack("<I", masked_crc32c(record))


class EventFileWriter:
    def __init__(self, logdir: str, suffix: str = "") -> None:
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{suffix}"
        self.path = os.path.join(logdir, name)
        self.f = open(self.path, "ab")
        self.f.write(frame(encode_file_version_event()))
        self.f.flush()

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self.f.write(frame(encode_scalar_event(tag, value, step)))

    def flush(self) -> None:
        self.f.flush()

    def close(self) -> None:
        self.f.close()


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = n = 0
    while True:
        x = b[i]
        i += 1
        n |= (x & 0x7F) << shift
        if not x & 0x80:
            return n, i
        shift += 7


def read_events(path: str) -> Iterator[Tuple[int, str, float]]:
    """(step, tag, value) of every scalar in an event file; verifies both CRCs."""
    for _, step, tag, value in read_scalars(path):
        yield step, tag, value


def read_scalars(path: str) -> Iterator[Tuple[float, int, str, float]]:
    """(wall_time, step, tag, value) of every scalar in an event file; verifies both CRCs."""
    data = open(path, "rb").read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        (hcrc,) = struct.unpack_from("<I", data, i + 8)
        if hcrc != masked_crc32c(data[i:i + 8]):
            raise ValueError("bad header crc")
        rec = data[i + 12:i + 12 + n]
        (dcrc,) = struct.unpack_from("<I", data, i + 12 + n)
        if dcrc != masked_crc32c(rec):
            raise ValueError("bad data crc")
        i += 16 + n
        step, j = 0, 0
        wall = 0.0
        summary = None
        while j < len(rec):
            key, j = _read_varint(rec, j)
            f, wt = key >> 3, key & 7
            if wt == 1:
                if f == 1:
                    (wall,) = struct.unpack_from("<d", rec, j)
                j += 8
            elif wt == 0:
                v, j = _read_varint(rec, j)
                if f == 2:
                    step = v
            elif wt == 2:
                ln, j = _read_varint(rec, j)
                if f == 5:
                    summary = rec[j:j + ln]
                j += ln
            elif wt == 5:
                j += 4
        if summary is None:
            continue
        k = 0
        while k < len(summary):
            key, k = _read_varint(summary, k)
            ln, k = _read_varint(summary, k)
            val = summary[k:k + ln]
            k += ln
            tag, value, m = "", 0.0, 0
            while m < len(val):
                vk, m = _read_varint(val, m)
                if vk >> 3 == 1:
                    ln2, m = _read_varint(val, m)
                    tag = val[m:m + ln2].decode()
                    m += ln2
                elif vk >> 3 == 2:
                    (value,) = struct.unpack_from("<f", val, m)
                    m += 4
                else:
                    break
            yield wall, step, tag, value
