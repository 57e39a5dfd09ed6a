"""Test infrastructure: writes small HDF5 files byte by byte from the HDF5 file format specification
(version 3.0), independently of the reader in gigapath/slide_io.py, so that the reader can be checked
where h5py is absent (this image).  Two styles:

- "earliest" (h5py's default ``libver``): superblock v0, version-1 object headers, a symbol-table root
  group (v1 B-tree + local heap + symbol table node), version-1 dataspace / attribute / filter
  messages, version-3 layouts.
- "latest": superblock v2, version-2 object headers ("OHDR") with link messages in the root group,
  version-2 dataspaces, version-3 attributes, version-2 filter pipelines.

Checksums of v2 structures are written as zeros (the reader does not verify them).  Options cover
what the reader must handle: a user block (base address), object-header continuation blocks,
chunked data over a two-level chunk B-tree, deflate / shuffle / fletcher32 filters, compact layout,
variable-length string attributes in a global heap, and h5py's bool enumeration.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


def _pad8(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


def fletcher32_spec(data: bytes) -> int:
    """Fletcher-32 as the HDF5 spec's reference loop computes it (written independently of the
    reader's vectorised form): big-endian 16-bit words in blocks of 360, both sums folded after each
    block, an odd last byte as a high byte, two final folds."""
    s1 = s2 = 0
    nw = len(data) // 2
    i = 0
    while nw:
        t = min(nw, 360)
        nw -= t
        for _ in range(t):
            s1 += (data[i] << 8) | data[i + 1]
            i += 2
            s2 += s1
        s1 = (s1 & 0xffff) + (s1 >> 16)
        s2 = (s2 & 0xffff) + (s2 >> 16)
    if len(data) % 2:
        s1 += data[i] << 8
        s2 += s1
        s1 = (s1 & 0xffff) + (s1 >> 16)
        s2 = (s2 & 0xffff) + (s2 >> 16)
    s1 = (s1 & 0xffff) + (s1 >> 16)
    s2 = (s2 & 0xffff) + (s2 >> 16)
    return (s2 << 16) | s1


class _File:
    def __init__(self, base: int):
        self.base = base
        self.buf = bytearray(b"\0" * base)          # user block (zeros)

    def alloc(self, data: bytes) -> int:
        """Append 8-aligned; returns the address RELATIVE to the base."""
        while len(self.buf) % 8:
            self.buf.append(0)
        a = len(self.buf) - self.base
        self.buf += data
        return a

    def reserve(self, n: int) -> int:
        return self.alloc(b"\0" * n)

    def put(self, addr: int, data: bytes):
        p = self.base + addr
        self.buf[p:p + len(data)] = data


# ---- datatypes (spec §IV.A.2.d) -----------------------------------------------------------------
def dt_message(arr_dtype) -> bytes:
    dt = np.dtype(arr_dtype)
    be = 1 if dt.byteorder == ">" else 0
    if dt.kind in "iu":
        bits = be | (0x08 if dt.kind == "i" else 0)
        return struct.pack("<B3sI", 0x10 | 0, bytes([bits, 0, 0]), dt.itemsize) + struct.pack("<HH", 0, 8 * dt.itemsize)
    if dt.kind == "f":
        exp = {2: (10, 5, 0, 10, 15), 4: (23, 8, 0, 23, 127), 8: (52, 11, 0, 52, 1023)}[dt.itemsize]
        sign = 8 * dt.itemsize - 1
        bits = bytes([be | 0x20, sign, 0])       # bit 5: mantissa normalisation "implied"; byte 2: sign location
        return (struct.pack("<B3sI", 0x10 | 1, bits, dt.itemsize)
                + struct.pack("<HHBBBBI", 0, 8 * dt.itemsize, exp[0], exp[1], exp[2], exp[3], exp[4]))
    if dt.kind == "S":
        return struct.pack("<B3sI", 0x10 | 3, bytes([0, 0, 0]), dt.itemsize)
    raise ValueError(dt)


def dt_vlen_str() -> bytes:
    base = struct.pack("<B3sI", 0x10 | 0, bytes([0, 0, 0]), 1) + struct.pack("<HH", 0, 8)   # u8 char
    return struct.pack("<B3sI", 0x10 | 9, bytes([0x01, 0x01, 0]), 16) + base               # string, utf-8


def dt_bool_enum() -> bytes:
    base = struct.pack("<B3sI", 0x10 | 0, bytes([0x08, 0, 0]), 1) + struct.pack("<HH", 0, 8)  # int8
    names = _pad8(b"FALSE\0") + _pad8(b"TRUE\0")
    return struct.pack("<B3sI", 0x10 | 8, struct.pack("<H", 2) + b"\0", 1) + base + names + bytes([0, 1])


# ---- dataspace (spec §IV.A.2.b) -----------------------------------------------------------------
def ds_message(shape, version: int, maxshape=None) -> bytes:
    flags = 1 if maxshape is not None else 0
    if version == 1:
        out = struct.pack("<BBBB4x", 1, len(shape), flags, 0)
    else:
        out = struct.pack("<BBBB", 2, len(shape), flags, 0 if len(shape) == 0 else 1)
    out += b"".join(struct.pack("<Q", s) for s in shape)
    if maxshape is not None:
        out += b"".join(struct.pack("<Q", UNDEF if m is None else m) for m in maxshape)
    return out


class Writer:
    """Collects datasets / attributes, then ``save(path)``."""

    def __init__(self, style: str = "earliest", userblock: int = 0, continuation: bool = False):
        assert style in ("earliest", "latest")
        self.style, self.userblock, self.continuation = style, userblock, continuation
        self.items = []

    def dataset(self, name, data, layout="contiguous", chunks=None, filters=(), attrs=None, btree_leaf=64,
                alloc_seed=None):
        """``alloc_seed``: place the chunks in the file in a shuffled order (as a file grown by appends
        and rewrites can have them)."""
        self.items.append((name, np.asarray(data), layout, chunks, tuple(filters), dict(attrs or {}), btree_leaf,
                           alloc_seed))

    # -- header messages --------------------------------------------------------------------------
    def _msgs_v1(self, f: _File, msgs) -> int:
        body = b""
        for t, data in msgs:
            d = _pad8(data)
            body += struct.pack("<HHB3x", t, len(d), 0) + d
        if self.continuation and len(msgs) > 2:
            # first two messages in the header, the rest in a continuation block
            head = b""
            for t, data in msgs[:2]:
                d = _pad8(data)
                head += struct.pack("<HHB3x", t, len(d), 0) + d
            tail = body[len(head):]
            ca = f.alloc(tail)
            head += struct.pack("<HHB3x", 0x10, 16, 0) + struct.pack("<QQ", ca, len(tail))
            return f.alloc(struct.pack("<BBHII4x", 1, 0, len(msgs) + 1, 1, len(head)) + head)
        return f.alloc(struct.pack("<BBHII4x", 1, 0, len(msgs), 1, len(body)) + body)

    def _msgs_v2(self, f: _File, msgs) -> int:
        def enc(ms):
            return b"".join(struct.pack("<BHB", t, len(d), 0) + d for t, d in ms)
        if self.continuation and len(msgs) > 2:
            tail = b"OCHK" + enc(msgs[2:]) + b"\0\0\0\0"
            ca = f.alloc(tail)
            body = enc(msgs[:2] + [(0x10, struct.pack("<QQ", ca, len(tail)))])
        else:
            body = enc(msgs)
        flags = 0x02                                   # chunk-0 size in 4 bytes
        return f.alloc(b"OHDR" + struct.pack("<BBI", 2, flags, len(body)) + body + b"\0\0\0\0")

    def _header(self, f, msgs):
        return self._msgs_v1(f, msgs) if self.style == "earliest" else self._msgs_v2(f, msgs)

    # -- attributes (spec §IV.A.2.m) ----------------------------------------------------------------
    def _attr(self, f: _File, name: str, value) -> bytes:
        nm = name.encode() + b"\0"
        if isinstance(value, str):
            sdata = value.encode()
            col = self._gheap(f, sdata)
            dt, ds = dt_vlen_str(), ds_message((), 1 if self.style == "earliest" else 2)
            raw = struct.pack("<IQI", len(sdata), col, 1)
        elif isinstance(value, (bool, np.bool_)):
            dt, ds = dt_bool_enum(), ds_message((), 1 if self.style == "earliest" else 2)
            raw = bytes([1 if value else 0])
        else:
            a = np.asarray(value)
            dt, ds = dt_message(a.dtype), ds_message(a.shape, 1 if self.style == "earliest" else 2)
            raw = a.tobytes()
        if self.style == "earliest":
            return (struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds)) + _pad8(nm) + _pad8(dt) + _pad8(ds) + raw)
        return struct.pack("<BBHHHB", 3, 0, len(nm), len(dt), len(ds), 0) + nm + dt + ds + raw

    def _gheap(self, f: _File, data: bytes) -> int:
        obj = struct.pack("<HH4xQ", 1, 1, len(data)) + _pad8(data)
        size = max(4096, 16 + len(obj) + 16)
        free = size - 16 - len(obj)
        body = b"GCOL" + struct.pack("<B3xQ", 1, size) + obj + struct.pack("<HH4xQ", 0, 0, free)
        return f.alloc(body + b"\0" * (size - len(body)))

    # -- data layouts ---------------------------------------------------------------------------------
    def _filters_msg(self, filters, esize):
        out = []
        for fl in filters:
            if fl == "deflate":
                out.append((1, b"deflate", [4]))
            elif fl == "shuffle":
                out.append((2, b"shuffle", [esize]))
            elif fl == "fletcher32":
                out.append((3, b"fletcher32", []))
        if self.style == "earliest":
            body = struct.pack("<BB6x", 1, len(out))
            for fid, nm, vals in out:
                nmp = _pad8(nm + b"\0")
                body += struct.pack("<HHHH", fid, len(nmp), 0, len(vals)) + nmp
                body += b"".join(struct.pack("<I", v) for v in vals) + (b"\0" * 4 if len(vals) % 2 else b"")
        else:
            body = struct.pack("<BB", 2, len(out))
            for fid, nm, vals in out:
                body += struct.pack("<HHH", fid, 0, len(vals)) + b"".join(struct.pack("<I", v) for v in vals)
        return body

    @staticmethod
    def _apply(raw: bytes, filters, esize) -> bytes:
        for fl in filters:
            if fl == "shuffle":
                a = np.frombuffer(raw, dtype=np.uint8)
                n = len(a) // esize
                raw = a[:n * esize].reshape(n, esize).T.tobytes() + a[n * esize:].tobytes()
            elif fl == "deflate":
                raw = zlib.compress(raw, 4)
            elif fl == "fletcher32":
                raw = raw + struct.pack("<I", fletcher32_spec(raw))
        return raw

    def _chunked(self, f: _File, data: np.ndarray, chunks, filters, leaf_max, alloc_seed=None):
        nd = data.ndim
        esize = data.dtype.itemsize
        grid = [range(0, s, c) for s, c in zip(data.shape, chunks)]
        all_offs = np.array(np.meshgrid(*grid, indexing="ij")).reshape(nd, -1).T
        alloc_order = (np.random.default_rng(alloc_seed).permutation(len(all_offs)) if alloc_seed is not None
                       else np.arange(len(all_offs)))
        placed = {}
        for k in alloc_order:
            offs = all_offs[k]
            block = np.zeros(chunks, dtype=data.dtype)
            sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, chunks, data.shape))
            part = data[sl]
            block[tuple(slice(0, p) for p in part.shape)] = part
            raw = self._apply(block.tobytes(), filters, esize)
            placed[int(k)] = (tuple(int(o) for o in offs), len(raw), f.alloc(raw))
        entries = [placed[k] for k in range(len(all_offs))]       # B-tree keys stay in offset order

        def key(csize, offs):
            return struct.pack("<II", csize, 0) + b"".join(struct.pack("<Q", o) for o in offs) + struct.pack("<Q", 0)

        def node(level, kids):                    # kids: [(first offs, size, addr)], plus an end key
            body = b"TREE" + struct.pack("<BBHQQ", 1, level, len(kids), UNDEF, UNDEF)
            for offs, csize, addr in kids:
                body += key(csize, offs) + struct.pack("<Q", addr)
            end = tuple(s for s in data.shape)
            return f.alloc(body + key(0, end))

        leaves = [entries[i:i + leaf_max] for i in range(0, len(entries), leaf_max)]
        if len(leaves) == 1:
            return node(0, leaves[0])
        return node(1, [(lv[0][0], 0, node(0, lv)) for lv in leaves])

    def _dataset_header(self, f: _File, item) -> int:
        name, data, layout, chunks, filters, attrs, leaf_max, alloc_seed = item
        esize = data.dtype.itemsize
        ver = 1 if self.style == "earliest" else 2
        msgs = [(0x01, ds_message(data.shape, ver)), (0x03, dt_message(data.dtype))]
        if layout == "contiguous":
            a = f.alloc(data.tobytes())
            msgs.append((0x08, struct.pack("<BBQQ", 3, 1, a, data.nbytes)))
        elif layout == "compact":
            raw = data.tobytes()
            msgs.append((0x08, struct.pack("<BBH", 3, 0, len(raw)) + raw))
        else:
            if filters:
                msgs.append((0x0B, self._filters_msg(filters, esize)))
            bt = self._chunked(f, data, chunks, filters, leaf_max, alloc_seed)
            msgs.append((0x08, struct.pack("<BBBQ", 3, 2, data.ndim + 1, bt)
                         + b"".join(struct.pack("<I", c) for c in chunks) + struct.pack("<I", esize)))
        for k, v in attrs.items():
            msgs.append((0x0C, self._attr(f, k, v)))
        return self._header(f, msgs)

    # -- file -----------------------------------------------------------------------------------------
    def save(self, path: str):
        f = _File(self.userblock)
        sb_size = 96 if self.style == "earliest" else 48
        sb = f.reserve(sb_size)
        assert sb == 0
        ds_addr = [(it[0], self._dataset_header(f, it)) for it in self.items]
        if self.style == "earliest":
            # local heap holding the names (offset 0 = empty string), then the B-tree leaf + SNOD
            names = b"\0" * 8
            offs = []
            for nm, _ in ds_addr:
                offs.append(len(names))
                names += _pad8(nm.encode() + b"\0")
            hdata = f.alloc(names)
            heap = f.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(names), UNDEF, hdata))
            order = sorted(range(len(ds_addr)), key=lambda i: ds_addr[i][0])
            ents = b"".join(struct.pack("<QQI4x16x", offs[i], ds_addr[i][1], 0) for i in order)
            snod = f.alloc(b"SNOD" + struct.pack("<BBH", 1, 0, len(order)) + ents)
            last = offs[order[-1]] if order else 0
            bt = f.alloc(b"TREE" + struct.pack("<BBHQQ", 0, 0, 1, UNDEF, UNDEF) + struct.pack("<QQQ", 0, snod, last))
            root = self._msgs_v1(f, [(0x11, struct.pack("<QQ", bt, heap))])
            eof = len(f.buf) - f.base
            f.put(0, SIG + struct.pack("<BBBBBBBBHHI", 0, 0, 0, 0, 0, 8, 8, 0, 4, 16, 0)
                  + struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
                  + struct.pack("<QQI4x", 0, root, 1) + struct.pack("<QQ", bt, heap))
        else:
            links = []
            for nm, a in ds_addr:
                n = nm.encode()
                links.append((0x06, struct.pack("<BBB", 1, 0x00, len(n)) + n + struct.pack("<Q", a)))
            linfo = (0x02, struct.pack("<BBQQ", 0, 0, UNDEF, UNDEF))
            root = self._msgs_v2(f, [linfo] + links)
            eof = len(f.buf) - f.base
            f.put(0, SIG + struct.pack("<BBBB", 2, 8, 8, 0) + struct.pack("<QQQQ", 0, UNDEF, eof, root) + b"\0" * 4)
        # base address: the superblock's own position (user block before it)
        if self.userblock:
            base_off = self.userblock + (24 if self.style == "earliest" else 12)
            f.buf[base_off:base_off + 8] = struct.pack("<Q", self.userblock)
        with open(path, "wb") as fh:
            fh.write(bytes(f.buf))
