"""TFRecord datasets of the reference without TensorFlow.

create_tfrecords.py writes one tf.train.Example per image with features 'img' (raw float32
bytes of the [1, H, W, D] image), 'height' / 'width' / 'depth' (int64) and 'label' (raw float32
bytes of the one-hot row) (`create_tfrecords.py:150-238`); conv_cINN_base_functions.py:26-65
(`_parse_example`) reads them back. This module restates both sides over the two published wire
formats involved — TFRecord framing (little-endian uint64 length, masked CRC-32C of the length,
payload, masked CRC-32C of the payload) and the protobuf encoding of Example / Features /
Feature / BytesList / Int64List / FloatList — so reference datasets load into numpy (then onto
the GPU) and files written here load in TensorFlow.
"""
from __future__ import annotations

import struct
from typing import Dict, Iterator, List, Tuple

import numpy as np

# ---------------------------------------------------------------------------------------------
# CRC-32C (Castagnoli, reflected polynomial 0x82F63B78) and TFRecord's masking
# ---------------------------------------------------------------------------------------------
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        crc = tab[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------------------------------------
# protobuf wire format (varints, length-delimited fields, packed repeated scalars)
# ---------------------------------------------------------------------------------------------
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = res = 0
    while True:
        b = buf[i]
        i += 1
        res |= (b & 0x7F) << shift
        if not b & 0x80:
            return res, i
        shift += 7


def _field(num: int, payload: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(payload)) + payload


def _fields(buf: bytes):
    """yield (field number, wire type, value) of a message; value = int or bytes."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            n, i = _read_varint(buf, i)
            v = buf[i:i + n]
            i += n
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        else:
            raise ValueError(f'unsupported protobuf wire type {wt}')
        yield num, wt, v


def encode_example(features: Dict[str, object]) -> bytes:
    """tf.train.Example(features=Features(feature={name: Feature})) serialised. Values: bytes ->
    BytesList, int / list of int -> Int64List (packed), float / float ndarray -> FloatList (packed)."""
    entries = b''
    for name in features:   # insertion order, like the reference's dict
        v = features[name]
        if isinstance(v, (bytes, bytearray)):
            feat = _field(1, _field(1, bytes(v)))
        elif isinstance(v, (int, np.integer)) or (isinstance(v, (list, tuple)) and all(
                isinstance(t, (int, np.integer)) for t in v)):
            vals = [v] if isinstance(v, (int, np.integer)) else list(v)
            feat = _field(3, _field(1, b''.join(_varint(int(t)) for t in vals)))
        else:
            arr = np.asarray(v, dtype='<f4').reshape(-1)
            feat = _field(2, _field(1, arr.tobytes()))
        entries += _field(1, _field(1, name.encode()) + _field(2, feat))
    return _field(1, entries)


def decode_example(buf: bytes) -> Dict[str, object]:
    """Inverse of encode_example: {name: bytes | list[int] | float32 ndarray}."""
    out: Dict[str, object] = {}
    for num, _, feats in _fields(buf):
        if num != 1:
            continue
        for fnum, _, entry in _fields(feats):
            if fnum != 1:
                continue
            key, val = None, b''
            for enum_, _, ev in _fields(entry):
                if enum_ == 1:
                    key = bytes(ev).decode()
                elif enum_ == 2:
                    val = ev
            for knd, _, lst in _fields(val):
                if knd == 1:       # BytesList
                    vals = [bytes(x) for n, _, x in _fields(lst) if n == 1]
                    out[key] = vals[0] if len(vals) == 1 else vals
                elif knd == 3:     # Int64List (packed or not)
                    ints: List[int] = []
                    for n, wt, x in _fields(lst):
                        if n != 1:
                            continue
                        if wt == 0:
                            ints.append(x)
                        else:
                            j = 0
                            while j < len(x):
                                v, j = _read_varint(x, j)
                                ints.append(v)
                    out[key] = [v - (1 << 64) if v >= 1 << 63 else v for v in ints]
                elif knd == 2:     # FloatList
                    fl = b''.join(x if wt == 2 else x for n, wt, x in _fields(lst) if n == 1)
                    out[key] = np.frombuffer(fl, dtype='<f4').copy()
    return out


# ---------------------------------------------------------------------------------------------
# TFRecord files
# ---------------------------------------------------------------------------------------------
def write_records(path: str, records) -> None:
    with open(path, 'wb') as f:
        for rec in records:
            ln = struct.pack('<Q', len(rec))
            f.write(ln + struct.pack('<I', masked_crc(ln)) + rec + struct.pack('<I', masked_crc(rec)))


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, 'rb') as f:
        while True:
            hdr = f.read(12)
            if not hdr:
                return
            if len(hdr) < 12:
                raise ValueError('truncated TFRecord header')
            (n,) = struct.unpack('<Q', hdr[:8])
            if verify and struct.unpack('<I', hdr[8:])[0] != masked_crc(hdr[:8]):
                raise ValueError('TFRecord length CRC mismatch')
            rec = f.read(n)
            tail = f.read(4)
            if len(rec) < n or len(tail) < 4:
                raise ValueError('truncated TFRecord payload')
            if verify and struct.unpack('<I', tail)[0] != masked_crc(rec):
                raise ValueError('TFRecord payload CRC mismatch')
            yield rec


def make_tfrecord(x: np.ndarray, y: np.ndarray, output_file: str) -> None:
    """create_tfrecords._make_TFRecord (:206-238): x [N, H, W, D] images, y [N, classes] one-hot;
    both serialised as their raw bytes (float32 here, as the training pipeline decodes float32)."""
    x = np.asarray(x, dtype=np.float32)
    y = np.asarray(y, dtype=np.float32)

    def gen():
        for i in range(x.shape[0]):
            img = x[i:i + 1]
            yield encode_example({'img': img.tobytes(), 'height': int(img.shape[1]), 'width': int(img.shape[2]),
                                  'depth': int(img.shape[3]), 'label': y[i:i + 1].tobytes()})
    write_records(output_file, gen())


def parse_example(serialized: bytes) -> Tuple[np.ndarray, np.ndarray]:
    """conv_cINN_base_functions._parse_example (:26-65): (img [H, W, D] float32, label float32)."""
    f = decode_example(serialized)
    h, w, d = (int(f[k][0]) for k in ('height', 'width', 'depth'))
    img = np.frombuffer(f['img'], dtype='<f4').reshape(h, w, d).copy()
    label = np.frombuffer(f['label'], dtype='<f4').copy()
    return img, label


def load_tfrecord(path: str, verify: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """All examples of a file as (images [N, H, W, D], labels [N, classes])."""
    imgs, labels = [], []
    for rec in read_records(path, verify):
        i, l = parse_example(rec)
        imgs.append(i)
        labels.append(l)
    return np.stack(imgs), np.stack(labels)
