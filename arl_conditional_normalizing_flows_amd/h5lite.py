"""Minimal HDF5 reader / writer for Keras weight files, without h5py.

The reference saves and restores its flows with Keras `model.save_weights(... .h5)` /
`model.load_weights(...)` (conv_cINN.py:579,641; conv_pre_training_cINN_on_noise.py:138,147),
which go through h5py / libhdf5. Neither h5py nor TensorFlow is importable by this package's
interpreter, so this module reads and writes the subset of the HDF5 file format such files use:

* superblock version 0 (h5py's default, `libver='earliest'`), 8-byte offsets and lengths;
* object headers version 1 and 2 (with continuation blocks);
* groups as symbol tables (v1 B-tree of type 0 + local heap + symbol table nodes) and as
  compact link messages (hard links);
* datasets with contiguous or compact layout (Keras never chunks or filters weights);
* attributes (message versions 1-3) of fixed-point, IEEE float, fixed-length and
  variable-length strings (the latter through the global heap).

Files are read from bytes with explicit little-endian parsing: nothing in a file is executed.
The writer emits superblock 0, v1 object headers and symbol-table groups, which libhdf5 of
every version reads. Format compatibility with the real library is pinned by
tests/test_h5weights.py against a fixture written by h5py 3.3 / libhdf5 (tests/golden/
make_h5_golden.py) and, when that interpreter is present, by h5py reading this writer's files.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Tuple, Union

import numpy as np

_SIG = b'\x89HDF\r\n\x1a\n'
_UNDEF = 0xFFFFFFFFFFFFFFFF


class H5Error(ValueError):
    pass


# ----------------------------------------------------------------------------------------------
# reader
# ----------------------------------------------------------------------------------------------

class _Dtype:
    """A decoded datatype message: numpy dtype, or ('vlen_str',) for variable-length strings."""

    def __init__(self, np_dtype=None, vlen_str=False):
        self.np = np_dtype
        self.vlen_str = vlen_str


class Dataset:
    def __init__(self, f: 'File', shape, dtype: _Dtype, layout, attrs):
        self._f, self.shape, self._dt, self._layout, self.attrs = f, shape, dtype, layout, attrs

    @property
    def dtype(self):
        return self._dt.np

    def read(self) -> np.ndarray:
        n = int(np.prod(self.shape)) if self.shape else 1
        kind, a, b = self._layout
        if self._dt.vlen_str:
            raw = self._f._raw_layout(kind, a, b, 16 * n)
            return np.array(self._f._vlen_strings(raw, n), dtype=object).reshape(self.shape)
        nbytes = n * self._dt.np.itemsize
        if kind == 'contiguous' and a == _UNDEF:   # never written: the fill value (0)
            return np.zeros(self.shape, self._dt.np)
        raw = self._f._raw_layout(kind, a, b, nbytes)
        return np.frombuffer(raw, dtype=self._dt.np, count=n).reshape(self.shape).copy()

    def __getitem__(self, key):
        return self.read()[key]


class Group:
    def __init__(self, f: 'File', links: Dict[str, int], attrs):
        self._f, self._links, self.attrs = f, links, attrs

    def keys(self) -> List[str]:
        return sorted(self._links)

    def __contains__(self, path):
        try:
            self[path]
            return True
        except KeyError:
            return False

    def __getitem__(self, path: str) -> Union['Group', Dataset]:
        node: Union[Group, Dataset] = self
        for part in [p for p in path.split('/') if p]:
            if not isinstance(node, Group) or part not in node._links:
                raise KeyError(path)
            node = node._f._object(node._links[part])
        return node

    def visit_datasets(self, prefix='') -> List[Tuple[str, Dataset]]:
        out = []
        for k in self.keys():
            obj = self[k]
            name = f'{prefix}{k}'
            if isinstance(obj, Group):
                out.extend(obj.visit_datasets(name + '/'))
            else:
                out.append((name, obj))
        return out


class File(Group):
    """Read-only view of an HDF5 file held in memory."""

    def __init__(self, path_or_bytes):
        if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
            self.buf = bytes(path_or_bytes)
        else:
            with open(path_or_bytes, 'rb') as fh:
                self.buf = fh.read()
        self._cache: Dict[int, Union[Group, Dataset]] = {}
        root = self._superblock()
        g = self._object(root)
        if not isinstance(g, Group):
            raise H5Error('root object is not a group')
        super().__init__(self, g._links, g.attrs)

    # -- primitives
    def _u(self, off, n):
        if off + n > len(self.buf):
            raise H5Error(f'read past end of file at {off}')
        return int.from_bytes(self.buf[off:off + n], 'little')

    def _sig(self, off, sig):
        if self.buf[off:off + len(sig)] != sig:
            raise H5Error(f'expected {sig!r} at {off}')

    def _superblock(self) -> int:
        base = None
        for off in [0] + [512 << i for i in range(20)]:   # user block: 0, 512, 1024, ...
            if off + 8 <= len(self.buf) and self.buf[off:off + 8] == _SIG:
                base = off
                break
        if base is None:
            raise H5Error('not an HDF5 file')
        ver = self.buf[base + 8]
        if ver in (0, 1):
            so, sl = self.buf[base + 13], self.buf[base + 14]
            if so != 8 or sl != 8:
                raise H5Error('only 8-byte offsets / lengths are supported')
            p = base + 24 + (4 if ver == 1 else 0)
            self.base = self._u(p, 8)
            p += 32   # base, free-space, EOF, driver
            return self.base + self._u(p + 8, 8)   # root symbol table entry: object header address
        if ver in (2, 3):
            so, sl = self.buf[base + 9], self.buf[base + 10]
            if so != 8 or sl != 8:
                raise H5Error('only 8-byte offsets / lengths are supported')
            self.base = self._u(base + 12, 8)
            return self.base + self._u(base + 12 + 24, 8)
        raise H5Error(f'superblock version {ver} unsupported')

    def _addr(self, off):
        a = self._u(off, 8)
        return a if a == _UNDEF else self.base + a

    # -- object headers
    def _messages(self, addr) -> List[Tuple[int, bytes]]:
        msgs: List[Tuple[int, bytes]] = []
        if self.buf[addr:addr + 4] == b'OHDR':
            flags = self.buf[addr + 5]
            p = addr + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            sz_len = 1 << (flags & 3)
            size = self._u(p, sz_len)
            p += sz_len
            blocks = [(p, size)]
            while blocks:
                start, size = blocks.pop(0)
                q, end = start, start + size - 4   # trailing checksum
                while q + 4 <= end:
                    mtype, msize, mflags = self.buf[q], self._u(q + 1, 2), self.buf[q + 3]
                    q += 4 + (2 if flags & 0x04 else 0)
                    data = self.buf[q:q + msize]
                    q += msize
                    if mtype == 0x10:
                        ca = self.base + int.from_bytes(data[0:8], 'little')
                        cl = int.from_bytes(data[8:16], 'little')
                        self._sig(ca, b'OCHK')
                        blocks.append((ca + 4, cl - 4))
                    elif mtype:
                        msgs.append((mtype, data))
            return msgs
        if self.buf[addr] != 1:
            raise H5Error(f'object header version {self.buf[addr]} at {addr} unsupported')
        nmsg = self._u(addr + 2, 2)
        blocks = [(addr + 16, self._u(addr + 8, 4))]
        while blocks and len(msgs) < nmsg + 64:
            start, size = blocks.pop(0)
            q, end = start, start + size
            while q + 8 <= end:
                mtype, msize = self._u(q, 2), self._u(q + 2, 2)
                data = self.buf[q + 8:q + 8 + msize]
                q += 8 + msize
                if mtype == 0x10:
                    blocks.append((self.base + int.from_bytes(data[0:8], 'little'), int.from_bytes(data[8:16], 'little')))
                elif mtype:
                    msgs.append((mtype, data))
        return msgs

    def _object(self, addr) -> Union[Group, Dataset]:
        if addr in self._cache:
            return self._cache[addr]
        msgs = self._messages(addr)
        attrs: Dict[str, object] = {}
        links: Dict[str, int] = {}
        shape = dtype = layout = None
        is_group = False
        for mtype, data in msgs:
            if mtype == 0x01:
                shape = self._dataspace(data)[0]
            elif mtype == 0x03:
                dtype = self._datatype(data)[0]
            elif mtype == 0x08:
                layout = self._layout_msg(data)
            elif mtype == 0x0C:
                k, v = self._attribute(data)
                attrs[k] = v
            elif mtype == 0x11:
                is_group = True
                links.update(self._symbol_table(self.base + int.from_bytes(data[0:8], 'little'),
                                                self.base + int.from_bytes(data[8:16], 'little')))
            elif mtype == 0x06:
                is_group = True
                k, v = self._link(data)
                if v is not None:
                    links[k] = v
            elif mtype == 0x02:
                is_group = True   # link info: compact storage assumed (dense storage unsupported)
                fheap = int.from_bytes(data[2 + (8 if data[1] & 1 else 0):][:8], 'little')
                if fheap != _UNDEF:
                    raise H5Error('dense (fractal heap) link storage unsupported')
        if is_group:
            obj: Union[Group, Dataset] = Group(self, links, attrs)
        elif shape is not None and dtype is not None and layout is not None:
            obj = Dataset(self, shape, dtype, layout, attrs)
        else:
            raise H5Error(f'object at {addr}: neither group nor dataset')
        self._cache[addr] = obj
        return obj

    # -- groups
    def _symbol_table(self, btree, heap) -> Dict[str, int]:
        self._sig(heap, b'HEAP')
        data_addr = self._addr(heap + 24)

        def name_at(off):
            s = data_addr + off
            e = self.buf.index(b'\0', s)
            return self.buf[s:e].decode('utf-8')

        links: Dict[str, int] = {}

        def walk(node):
            self._sig(node, b'TREE')
            if self.buf[node + 4] != 0:
                raise H5Error('expected a group B-tree')
            level, used = self.buf[node + 5], self._u(node + 6, 2)
            p = node + 24
            for i in range(used):
                child = self._addr(p + 8)
                p += 16
                if level > 0:
                    walk(child)
                else:
                    self._sig(child, b'SNOD')
                    nsym = self._u(child + 6, 2)
                    for j in range(nsym):
                        e = child + 8 + 40 * j
                        links[name_at(self._u(e, 8))] = self._addr(e + 8)

        walk(btree)
        return links

    def _link(self, d: bytes):
        if d[0] != 1:
            raise H5Error('link message version')
        flags = d[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = d[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        nlen_sz = 1 << (flags & 3)
        nlen = int.from_bytes(d[p:p + nlen_sz], 'little')
        p += nlen_sz
        name = d[p:p + nlen].decode('utf-8')
        p += nlen
        if ltype != 0:
            return name, None   # soft / external links are not followed
        return name, self.base + int.from_bytes(d[p:p + 8], 'little')

    # -- dataspace / datatype / layout / attributes
    def _dataspace(self, d: bytes):
        ver, rank, flags = d[0], d[1], d[2]
        if ver == 1:
            p = 8
            stype = 1 if rank > 0 else 0
        elif ver == 2:
            stype = d[3]
            p = 4
        else:
            raise H5Error(f'dataspace version {ver}')
        dims = tuple(int.from_bytes(d[p + 8 * i:p + 8 * i + 8], 'little') for i in range(rank))
        p += 8 * rank * (2 if flags & 1 else 1)
        if stype == 2:
            return None, p   # null dataspace
        return dims, p

    def _datatype(self, d: bytes):
        cls, ver = d[0] & 0x0F, d[0] >> 4
        b0, b1 = d[1], d[2]
        size = int.from_bytes(d[4:8], 'little')
        if cls == 0:
            order = '>' if b0 & 1 else '<'
            kind = 'i' if b0 & 8 else 'u'
            return _Dtype(np.dtype(f'{order}{kind}{size}')), 8 + 4
        if cls == 1:
            order = '>' if b0 & 1 else '<'
            if size not in (2, 4, 8):
                raise H5Error(f'float size {size}')
            return _Dtype(np.dtype(f'{order}f{size}')), 8 + 12
        if cls == 3:
            return _Dtype(np.dtype(f'S{size}')), 8
        if cls == 9:
            vtype = b0 & 0x0F
            base_dt, n = self._datatype(d[8:])
            if vtype == 1:
                return _Dtype(vlen_str=True), 8 + n
            raise H5Error('variable-length sequences unsupported')
        raise H5Error(f'datatype class {cls} unsupported')

    def _layout_msg(self, d: bytes):
        ver = d[0]
        if ver != 3:
            raise H5Error(f'layout message version {ver} unsupported')
        cls = d[1]
        if cls == 0:
            n = int.from_bytes(d[2:4], 'little')
            return ('compact', d[4:4 + n], n)
        if cls == 1:
            a = int.from_bytes(d[2:10], 'little')
            return ('contiguous', a if a == _UNDEF else self.base + a, int.from_bytes(d[10:18], 'little'))
        raise H5Error('chunked datasets unsupported (Keras weights are contiguous)')

    def _raw_layout(self, kind, a, b, nbytes):
        if kind == 'compact':
            return a[:nbytes]
        if nbytes > b:
            raise H5Error('dataset storage shorter than its dataspace')
        return self.buf[a:a + nbytes]

    def _vlen_strings(self, raw: bytes, n: int) -> List[str]:
        out = []
        for i in range(n):
            length = int.from_bytes(raw[16 * i:16 * i + 4], 'little')
            coll = self.base + int.from_bytes(raw[16 * i + 4:16 * i + 12], 'little')
            idx = int.from_bytes(raw[16 * i + 12:16 * i + 16], 'little')
            out.append(self._gheap(coll, idx)[:length].decode('utf-8'))
        return out

    def _gheap(self, coll, idx) -> bytes:
        self._sig(coll, b'GCOL')
        size = self._u(coll + 8, 8)
        p, end = coll + 16, coll + size
        while p + 16 <= end:
            oi, osz = self._u(p, 2), self._u(p + 8, 8)
            if oi == idx:
                return self.buf[p + 16:p + 16 + osz]
            if oi == 0:
                break
            p += 16 + ((osz + 7) & ~7)
        raise H5Error('global heap object not found')

    def _attribute(self, d: bytes):
        ver = d[0]
        nsz, tsz, ssz = (int.from_bytes(d[i:i + 2], 'little') for i in (2, 4, 6))
        p = 8 if ver != 3 else 9
        pad = (lambda n: (n + 7) & ~7) if ver == 1 else (lambda n: n)
        name = d[p:p + nsz].split(b'\0', 1)[0].decode('utf-8')
        p += pad(nsz)
        dt = self._datatype(d[p:p + tsz])[0]
        p += pad(tsz)
        shape = self._dataspace(d[p:p + ssz])[0]
        p += pad(ssz)
        n = int(np.prod(shape)) if shape else 1
        raw = d[p:]
        if shape is None:
            return name, None
        if dt.vlen_str:
            vals = self._vlen_strings(raw, n)
            return name, (vals[0] if shape == () else np.array(vals, dtype=object).reshape(shape))
        arr = np.frombuffer(raw, dtype=dt.np, count=n).reshape(shape).copy()
        return name, (arr[()] if shape == () else arr)


# ----------------------------------------------------------------------------------------------
# writer
# ----------------------------------------------------------------------------------------------

_LEAF_K, _NODE_K = 4, 16   # symbol table node holds 2*4 entries; B-tree node 2*16 children


def _pad8(b: bytes) -> bytes:
    return b + b'\0' * ((-len(b)) % 8)


def _dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.byteorder == '>':
        raise H5Error('big-endian data: convert to little-endian first')
    if dt.kind == 'f':
        n = dt.itemsize
        if n == 4:
            props = struct.pack('<HHBBBBI', 0, 32, 23, 8, 0, 23, 127)
            bits = bytes([0x20, 31, 0])
        elif n == 8:
            props = struct.pack('<HHBBBBI', 0, 64, 52, 11, 0, 52, 1023)
            bits = bytes([0x20, 63, 0])
        else:
            raise H5Error(f'float{8 * n} unsupported')
        return bytes([0x11]) + bits + struct.pack('<I', n) + props
    if dt.kind in 'iu':
        return bytes([0x10, 0x08 if dt.kind == 'i' else 0, 0, 0]) + struct.pack('<I', dt.itemsize) + \
            struct.pack('<HH', 0, 8 * dt.itemsize)
    if dt.kind == 'S':
        return bytes([0x13, 0x01, 0, 0]) + struct.pack('<I', max(1, dt.itemsize))   # NULLPAD, ASCII
    raise H5Error(f'dtype {dt} unsupported')


def _space_msg(shape) -> bytes:
    return struct.pack('<BBBB4x', 1, len(shape), 0, 0) + b''.join(struct.pack('<Q', int(s)) for s in shape)


def _to_array(value) -> np.ndarray:
    if isinstance(value, str):
        value = value.encode('utf-8')
    if isinstance(value, bytes):
        return np.array(value)
    a = np.asarray(value)
    if a.dtype.kind == 'U':
        a = np.char.encode(a, 'utf-8')
    if a.dtype.kind == 'O':
        a = np.array([x.encode('utf-8') if isinstance(x, str) else x for x in a.reshape(-1)]).reshape(a.shape)
    return a


class _Node:
    def __init__(self):
        self.attrs: Dict[str, np.ndarray] = {}


class WGroup(_Node):
    def __init__(self):
        super().__init__()
        self.children: Dict[str, _Node] = {}

    def create_group(self, path: str) -> 'WGroup':
        g: WGroup = self
        for part in [p for p in path.split('/') if p]:
            nxt = g.children.get(part)
            if nxt is None:
                nxt = g.children[part] = WGroup()
            if not isinstance(nxt, WGroup):
                raise H5Error(f'{part} is a dataset')
            g = nxt
        return g

    def create_dataset(self, path: str, data) -> 'WDataset':
        parts = [p for p in path.split('/') if p]
        g = self.create_group('/'.join(parts[:-1])) if len(parts) > 1 else self
        if parts[-1] in g.children:
            raise H5Error(f'{path} exists')
        d = g.children[parts[-1]] = WDataset(data)
        return d


class WDataset(_Node):
    def __init__(self, data):
        super().__init__()
        self.data = np.array(_to_array(data), order='C', copy=True)   # keeps 0-d scalars 0-d


class Writer(WGroup):
    """Build a tree of groups / datasets / attributes in memory, then `save(path)`."""

    def save(self, path: Optional[str] = None) -> bytes:
        out = bytearray(96)   # superblock v0, filled in last

        def alloc(b: bytes) -> int:
            a = len(out)
            out.extend(_pad8(b))
            return a

        # byte-string attributes are stored as variable-length strings in one global heap
        # collection, as h5py 3 stores Python bytes (what Keras's save_weights writes)
        vstr: Dict[bytes, int] = {}

        def collect(node: _Node):
            for val in node.attrs.values():
                a = _to_array(val)
                if a.dtype.kind == 'S':
                    for x in a.reshape(-1):
                        vstr.setdefault(bytes(x), len(vstr) + 1)
            for ch in getattr(node, 'children', {}).values():
                collect(ch)

        collect(self)
        gcol = 0
        if vstr:
            objs = b''.join(struct.pack('<HH4xQ', i, 1, len(x)) + _pad8(x) for x, i in vstr.items())
            size = max(4096, 16 + len(objs) + 16)
            free = size - 16 - len(objs)
            gcol = alloc(b'GCOL' + bytes([1, 0, 0, 0]) + struct.pack('<Q', size) + objs +
                         struct.pack('<HH4xQ', 0, 0, free) + b'\0' * (free - 16))

        def obj_header(msgs: List[Tuple[int, bytes]]) -> int:
            body = b''.join(struct.pack('<HHB3x', t, len(_pad8(m)), 0) + _pad8(m) for t, m in msgs)
            return alloc(struct.pack('<BBHII', 1, 0, len(msgs), 1, len(body)) + b'\0' * 4 + body)

        def attr_msgs(node: _Node):
            msgs = []
            for name, val in node.attrs.items():
                a = _to_array(val)
                nb = name.encode('utf-8') + b'\0'
                sp = _space_msg(a.shape)
                if a.dtype.kind == 'S':   # vlen string of uint8, null-terminated, ASCII (h5py's encoding)
                    dt = bytes([0x19, 0x01, 0, 0]) + struct.pack('<I', 16) + bytes([0x10, 0, 0, 0]) + \
                        struct.pack('<IHH', 1, 0, 8)
                    raw = b''.join(struct.pack('<IQI', len(bytes(x)), gcol, vstr[bytes(x)]) for x in a.reshape(-1))
                else:
                    dt, raw = _dtype_msg(a.dtype), a.tobytes()
                msgs.append((0x0C, struct.pack('<BBHHH', 1, 0, len(nb), len(dt), len(sp)) + _pad8(nb) + _pad8(dt) +
                             _pad8(sp) + raw))
            return msgs

        def write(node: _Node) -> Tuple[int, int, int]:
            """-> (object header address, B-tree, heap) (B-tree/heap 0 for datasets)."""
            if isinstance(node, WDataset):
                a = node.data
                data_addr = alloc(a.tobytes()) if a.nbytes else _UNDEF
                layout = struct.pack('<BBQQ', 3, 1, data_addr, a.nbytes)
                msgs = [(0x01, _space_msg(a.shape)), (0x03, _dtype_msg(a.dtype)), (0x08, layout)] + attr_msgs(node)
                return obj_header(msgs), 0, 0
            assert isinstance(node, WGroup)
            names = sorted(node.children, key=lambda s: s.encode('utf-8'))
            kids = {n: write(node.children[n]) for n in names}
            # local heap: "" at 0, then every name (8-byte padded)
            heap_data = bytearray(8)
            name_off = {}
            for n in names:
                name_off[n] = len(heap_data)
                heap_data.extend(_pad8(n.encode('utf-8') + b'\0'))
            heap_data.extend(b'\0' * 16)   # one free block at the end (libhdf5's own layout)
            free_off = len(heap_data) - 16
            struct.pack_into('<QQ', heap_data, free_off, 1, 16)   # next free (1 = none), size
            heap_data_addr = alloc(bytes(heap_data))
            heap = alloc(b'HEAP' + bytes([0, 0, 0, 0]) + struct.pack('<QQQ', len(heap_data), free_off, heap_data_addr))
            # symbol table nodes of up to 2K entries, then a B-tree over them
            snods = []
            per = 2 * _LEAF_K
            for s in range(0, max(len(names), 1), per):
                chunk = names[s:s + per]
                ent = b''
                for n in chunk:
                    oh, bt, hp = kids[n]
                    if bt:
                        ent += struct.pack('<QQII', name_off[n], oh, 1, 0) + struct.pack('<QQ', bt, hp)
                    else:
                        ent += struct.pack('<QQII', name_off[n], oh, 0, 0) + b'\0' * 16
                ent += b'\0' * (40 * per - len(ent))
                snods.append((alloc(b'SNOD' + bytes([1, 0]) + struct.pack('<H', len(chunk)) + ent),
                              name_off[chunk[-1]] if chunk else 0))
            if not names:
                snods = []

            def tree(level, children):   # children: [(address, largest-name key)]
                cap = 2 * _NODE_K
                nodes = []
                for s in range(0, max(len(children), 1), cap):
                    ch = children[s:s + cap]
                    body = struct.pack('<Q', 0)
                    for addr, key in ch:
                        body += struct.pack('<QQ', addr, key)
                    body += b'\0' * ((8 + 16 * cap) - len(body))
                    hdr = b'TREE' + bytes([0, level]) + struct.pack('<HQQ', len(ch), _UNDEF, _UNDEF)
                    nodes.append((hdr + body, ch[-1][1] if ch else 0))
                # siblings: patch left/right pointers once addresses are known
                addrs = []
                for raw, key in nodes:
                    addrs.append((alloc(raw), key))
                for i, (a, _) in enumerate(addrs):
                    if i > 0:
                        struct.pack_into('<Q', out, a + 8, addrs[i - 1][0])
                    if i + 1 < len(addrs):
                        struct.pack_into('<Q', out, a + 16, addrs[i + 1][0])
                return addrs

            level, layer = 0, tree(0, snods)
            while len(layer) > 1:
                level += 1
                layer = tree(level, layer)
            bt = layer[0][0]
            oh = obj_header([(0x11, struct.pack('<QQ', bt, heap))] + attr_msgs(node))
            return oh, bt, heap

        root_oh, root_bt, root_hp = write(self)
        sb = _SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack('<HHI', _LEAF_K, _NODE_K, 0)
        sb += struct.pack('<QQQQ', 0, _UNDEF, len(out), _UNDEF)
        sb += struct.pack('<QQII', 0, root_oh, 1, 0) + struct.pack('<QQ', root_bt, root_hp)
        assert len(sb) == 96
        out[0:96] = sb
        data = bytes(out)
        if path is not None:
            with open(path, 'wb') as fh:
                fh.write(data)
        return data
