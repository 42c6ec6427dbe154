"""A minimal HDF5 / netCDF-4 writer for the reader tests (TEST INFRASTRUCTURE).

No HDF5 library (h5py, netCDF4, libhdf5) is importable in this image, so the
netCDF-4 reader of gsky_amd/csrc/hdf5.cpp is checked against files written
here from the HDF5 file format specification 3.0 -- parity unpinned.  The
files have the layout netCDF-C 4.x gives them: every dimension a dimension
scale dataset (CLASS / NAME / _Netcdf4Dimid), every variable a dataset whose
DIMENSION_LIST attribute holds object references to its dimensions' scales
(a variable-length sequence in the global heap), global attributes on the
root group.

Structures written: superblock 0 (symbol-table root group: v1 B-tree, SNOD,
local heap; v1 object headers) or 2 (v2 object headers with lookup3
checksums, link messages, Group Info), compact or dense attributes and links
(fractal heap with a root direct block + v2 B-tree name index, one leaf or
one internal level), contiguous / compact / chunked datasets (v1 B-tree chunk
index, one or two levels) with deflate, shuffle and fletcher32 filters,
either byte order, fixed-length and variable-length strings.

    write_nc4(path, dims=[("lat", 4), ("lon", 5)],
              variables=[Var("lat", ("lat",), lat), Var("v", ("lat", "lon"), data, atts={...}, chunks=(2, 3))],
              gatts={"Conventions": "CF-1.6"}, superblock=0)
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
SIG = b"\x89HDF\r\n\x1a\n"


# ---------------------------------------------------------------- lookup3 (Bob Jenkins' hashlittle)
def _rot(x, k):
    return ((x << k) | (x >> (32 - k))) & 0xFFFFFFFF


def lookup3(data: bytes, initval: int = 0) -> int:
    """H5_checksum_lookup3: hashlittle() over the bytes, little-endian words."""
    n = len(data)
    a = b = c = (0xDEADBEEF + n + initval) & 0xFFFFFFFF
    i = 0
    M = 0xFFFFFFFF
    while n - i > 12:
        a = (a + int.from_bytes(data[i:i + 4], "little")) & M
        b = (b + int.from_bytes(data[i + 4:i + 8], "little")) & M
        c = (c + int.from_bytes(data[i + 8:i + 12], "little")) & M
        a = (a - c) & M; a ^= _rot(c, 4); c = (c + b) & M
        b = (b - a) & M; b ^= _rot(a, 6); a = (a + c) & M
        c = (c - b) & M; c ^= _rot(b, 8); b = (b + a) & M
        a = (a - c) & M; a ^= _rot(c, 16); c = (c + b) & M
        b = (b - a) & M; b ^= _rot(a, 19); a = (a + c) & M
        c = (c - b) & M; c ^= _rot(b, 4); b = (b + a) & M
        i += 12
    rest = data[i:] + bytes(12 - (n - i))
    if n - i == 0:
        return c
    a = (a + int.from_bytes(rest[0:4], "little")) & M
    b = (b + int.from_bytes(rest[4:8], "little")) & M
    c = (c + int.from_bytes(rest[8:12], "little")) & M
    c ^= b; c = (c - _rot(b, 14)) & M
    a ^= c; a = (a - _rot(c, 11)) & M
    b ^= a; b = (b - _rot(a, 25)) & M
    c ^= b; c = (c - _rot(b, 16)) & M
    a ^= c; a = (a - _rot(c, 4)) & M
    b ^= a; b = (b - _rot(a, 14)) & M
    c ^= b; c = (c - _rot(b, 24)) & M
    return c


# ---------------------------------------------------------------- datatypes / dataspaces
def _pad8(b: bytes) -> bytes:
    return b + bytes((-len(b)) % 8)


def dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    be = 1 if dt.byteorder == ">" else 0
    if dt.kind in "iu":
        bf = be | (8 if dt.kind == "i" else 0)
        return bytes([0x10, bf, 0, 0]) + struct.pack("<IHH", dt.itemsize, 0, 8 * dt.itemsize)
    if dt.kind == "f":
        if dt.itemsize == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            sign = 31
        else:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            sign = 63
        return bytes([0x11, 0x20 | be, sign, 0]) + struct.pack("<I", dt.itemsize) + props
    raise ValueError(dt)


def str_dtype(n: int) -> bytes:
    return bytes([0x13, 0x00, 0, 0]) + struct.pack("<I", max(1, n))   # null-terminated ASCII


def vlen_str_dtype() -> bytes:
    base = bytes([0x10, 0, 0, 0]) + struct.pack("<IHH", 1, 0, 8)     # unsigned char
    return bytes([0x19, 0x01, 0x00, 0]) + struct.pack("<I", 16) + base


def vlen_ref_dtype() -> bytes:
    base = bytes([0x17, 0x00, 0, 0]) + struct.pack("<I", 8)           # object reference
    return bytes([0x19, 0x00, 0x00, 0]) + struct.pack("<I", 16) + base


def dspace_msg(dims: Sequence[int], version: int = 1) -> bytes:
    if version == 1:
        return bytes([1, len(dims), 0, 0, 0, 0, 0, 0]) + b"".join(struct.pack("<Q", d) for d in dims)
    typ = 0 if len(dims) == 0 else 1
    return bytes([2, len(dims), 0, typ]) + b"".join(struct.pack("<Q", d) for d in dims)


# ---------------------------------------------------------------- the file image
class Img:
    def __init__(self):
        self.b = bytearray()

    def alloc(self, data: bytes, align: int = 8) -> int:
        pad = (-len(self.b)) % align
        self.b += bytes(pad)
        at = len(self.b)
        self.b += data
        return at

    def reserve(self, n: int) -> int:
        return self.alloc(bytes(n))

    def put(self, at: int, data: bytes):
        self.b[at:at + len(data)] = data


@dataclass
class Var:
    name: str
    dims: Tuple[str, ...]
    data: np.ndarray
    atts: Dict[str, object] = field(default_factory=dict)
    chunks: Optional[Tuple[int, ...]] = None        # None: contiguous
    filters: Tuple[str, ...] = ("shuffle", "deflate")
    compact: bool = False
    skip_chunks: Tuple[int, ...] = ()               # linear chunk indices never written (read as the fill value)
    fill_msg: bool = True                           # the fill-value message (0x05), as netCDF-C always writes it


def nc_fill_default(dt: np.dtype):
    """netCDF-C's NC_FILL_* default of a numpy type (netcdf.h)."""
    return {"i1": -127, "u1": 255, "i2": -32767, "u2": 65535, "i4": -2147483647, "u4": 4294967295,
            "i8": -9223372036854775806, "u8": 18446744073709551614, "f4": 9.9692099683868690e+36,
            "f8": 9.9692099683868690e+36}[np.dtype(dt).str[1:]]


class _Heap:
    """The global heap collection of the file's variable-length data."""

    def __init__(self):
        self.objs: List[bytes] = []
        self.addr = None

    def add(self, data: bytes) -> int:
        self.objs.append(data)
        return len(self.objs)            # object index (1-based)

    def image(self, size: int) -> bytes:
        body = b""
        for i, d in enumerate(self.objs, 1):
            body += struct.pack("<HHIQ", i, 1, 0, len(d)) + _pad8(d)
        assert 16 + len(body) + 16 <= size
        free = size - 16 - len(body)
        body += struct.pack("<HHIQ", 0, 0, 0, free)
        return b"GCOL" + bytes([1, 0, 0, 0]) + struct.pack("<Q", size) + body + bytes(size - 16 - len(body))


class Writer:
    def __init__(self, superblock: int, dense_atts: bool, dense_links: bool, crt_order: bool):
        self.sb = superblock
        self.dense_atts = dense_atts
        self.dense_links = dense_links
        self.crt = crt_order and superblock >= 2
        self.img = Img()
        self.heap = _Heap()
        self.heap_addr = 0              # the global heap collection (reserved before any object)

    # ------------------------------------------------------------ attributes
    def att_msg(self, name: str, value, version: int) -> bytes:
        nb = name.encode() + b"\0"
        refs = None
        if isinstance(value, tuple) and value and value[0] == "__refs__":
            refs = value[1]
            dt, ds, data = vlen_ref_dtype(), dspace_msg([len(refs)], 1 if version == 1 else 2), b""
            for r in refs:
                idx = self.heap.add(struct.pack("<Q", r))
                data += struct.pack("<I", 1) + struct.pack("<Q", self.heap_addr) + struct.pack("<I", idx)
        elif isinstance(value, tuple) and value and value[0] == "__vstr__":
            s = value[1].encode()
            idx = self.heap.add(s)
            dt, ds = vlen_str_dtype(), dspace_msg([], 1 if version == 1 else 2)
            data = struct.pack("<I", len(s)) + struct.pack("<Q", self.heap_addr) + struct.pack("<I", idx)
        elif isinstance(value, str):
            s = value.encode()
            dt, ds, data = str_dtype(len(s)), dspace_msg([], 1 if version == 1 else 2), s if s else b"\0"
        else:
            arr = np.atleast_1d(np.asarray(value))
            dt = dtype_msg(arr.dtype)
            ds = dspace_msg([arr.size] if np.ndim(value) else [], 1 if version == 1 else 2)
            data = arr.tobytes()
        if version == 1:
            body = (bytes([1, 0]) + struct.pack("<HHH", len(nb), len(dt), len(ds)) + _pad8(nb) + _pad8(dt) +
                    _pad8(ds))
        else:
            body = bytes([version, 0]) + struct.pack("<HHH", len(nb), len(dt), len(ds))
            if version == 3:
                body += b"\0"
            body += nb + dt + ds
        return body + data

    # ------------------------------------------------------------ object headers
    def ohdr(self, msgs: List[Tuple[int, bytes]]) -> int:
        """Writes an object header with the messages; returns its address.
        Heap-address fields inside message bytes are patched in finish()."""
        if self.sb < 2:
            body = b""
            for t, d in msgs:
                d = _pad8(d)
                body += struct.pack("<HHB3x", t, len(d), 0) + d
            hdr = struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + bytes(4)
            return self.img.alloc(hdr + body)
        body = b""
        for k, (t, d) in enumerate(msgs):
            body += struct.pack("<BHB", t, len(d), 0)
            if self.crt:
                body += struct.pack("<H", k)
            body += d
        flags = 0x02 | (0x04 if self.crt else 0)
        pre = b"OHDR" + bytes([2, flags]) + struct.pack("<I", len(body))
        img = pre + body
        return self.img.alloc(img + struct.pack("<I", lookup3(img)))

    # ------------------------------------------------------------ dense storage
    def fheap(self, objs: List[bytes], id_len: int) -> Tuple[int, List[bytes]]:
        """A fractal heap whose root is one direct block holding objs; returns
        (header address, heap IDs)."""
        hdr_size = 4 + 1 + 8 + 4
        need = hdr_size + sum(len(o) for o in objs)
        block = 512
        while block < need:
            block *= 2
        assert block <= 65536
        ids, off = [], hdr_size
        for o in objs:
            ids.append(bytes([0]) + struct.pack("<I", off) + struct.pack("<H", len(o)) + bytes(id_len - 7))
            off += len(o)
        hdr_at = self.img.reserve(256)
        dblock = b"FHDB" + bytes([0]) + struct.pack("<Q", hdr_at) + struct.pack("<I", 0) + b"".join(objs)
        dblock += bytes(block - len(dblock))
        db_at = self.img.alloc(dblock)
        L = lambda v: struct.pack("<Q", v)
        h = b"FRHP" + bytes([0]) + struct.pack("<HH", id_len, 0) + bytes([0]) + struct.pack("<I", 4096)
        h += L(0) + L(UNDEF) + L(block - off) + L(UNDEF) + L(block) + L(block) + L(off) + L(len(objs))
        h += L(0) + L(0) + L(0) + L(0)
        h += struct.pack("<H", 4) + L(block) + L(65536) + struct.pack("<HH", 32, 1) + L(db_at) + struct.pack("<H", 0)
        h += struct.pack("<I", lookup3(h))
        self.img.put(hdr_at, h)
        return hdr_at, ids

    def btree2(self, btype: int, records: List[bytes]) -> int:
        """A v2 B-tree of the records (sorted by the caller): one leaf, or one
        internal level when they do not fit one 512-byte node."""
        node = 512
        rsize = len(records[0]) if records else (11 if btype == 5 else 17)
        leaf_max = (node - 10) // rsize

        def leaf(recs):
            img = b"BTLF" + bytes([0, btype]) + b"".join(recs)
            img += struct.pack("<I", lookup3(img))
            return self.img.alloc(img + bytes(node - len(img)))

        if len(records) <= leaf_max:
            root, depth, nroot = leaf(records), 0, len(records)
        else:
            # leaves of leaf_max // 2 records separated by one record each
            per = max(1, leaf_max // 2)
            children, seps, i = [], [], 0
            while i < len(records):
                chunk = records[i:i + per]
                children.append((leaf(chunk), len(chunk)))
                i += per
                if i < len(records):
                    seps.append(records[i])
                    i += 1
            nsz = (leaf_max.bit_length() - 1) // 8 + 1
            img = b"BTIN" + bytes([0, btype]) + b"".join(seps)
            for addr, n in children:
                img += struct.pack("<Q", addr) + n.to_bytes(nsz, "little")
            img += struct.pack("<I", lookup3(img))
            root, depth, nroot = self.img.alloc(img + bytes(node - len(img))), 1, len(seps)
        h = b"BTHD" + bytes([0, btype]) + struct.pack("<IHHBB", node, rsize, depth, 100, 40)
        h += struct.pack("<QHQ", root, nroot, len(records))
        h += struct.pack("<I", lookup3(h))
        return self.img.alloc(h)

    def attribute_msgs(self, atts: Dict[str, object]) -> List[Tuple[int, bytes]]:
        version = 1 if self.sb < 2 else 3
        bodies = [(n, self.att_msg(n, v, version)) for n, v in atts.items()]
        if not (self.dense_atts and self.sb >= 2) or not bodies:
            return [(0x0C, b) for _, b in bodies]
        # dense: the messages in a fractal heap, a v2 B-tree of (heap ID, flags, order, name hash)
        objs = [b for _, b in bodies]
        heap_at, ids = self.fheap(objs, 8)
        recs = sorted(((lookup3(n.encode()), ids[k] + bytes([0]) + struct.pack("<II", k, lookup3(n.encode())))
                       for k, (n, _) in enumerate(bodies)), key=lambda r: r[0])
        bt = self.btree2(8, [r for _, r in recs])
        return [(0x15, bytes([0, 0]) + struct.pack("<QQ", heap_at, bt))]

    # ------------------------------------------------------------ datasets
    def dataset(self, v: Var, dim_refs: List[int], extra_atts: Dict[str, object]) -> int:
        arr = np.ascontiguousarray(v.data)
        es = arr.dtype.itemsize
        msgs = [(0x01, dspace_msg(arr.shape, 1 if self.sb < 2 else 2)), (0x03, dtype_msg(arr.dtype))]
        if v.fill_msg:
            # netCDF-C sets the dataset's fill value to _FillValue, else to the
            # type's NC_FILL_* default; version 2 for superblocks 0 / 1, else 3
            fv = v.atts.get("_FillValue")
            fv = np.asarray(fv if fv is not None else nc_fill_default(arr.dtype), arr.dtype.newbyteorder("="))
            raw = fv.astype(arr.dtype).tobytes()
            if self.sb < 2:
                msgs.append((0x05, bytes([2, 2, 2, 1]) + struct.pack("<I", len(raw)) + raw))
            else:
                msgs.append((0x05, bytes([3, 2 | (2 << 2) | 0x20]) + struct.pack("<I", len(raw)) + raw))
        if v.compact:
            raw = arr.tobytes()
            msgs.append((0x08, bytes([3, 0]) + struct.pack("<H", len(raw)) + raw))
        elif v.chunks is None:
            at = self.img.alloc(arr.tobytes())
            msgs.append((0x08, bytes([3, 1]) + struct.pack("<QQ", at, arr.nbytes)))
        else:
            ch = tuple(v.chunks)
            grid = [(s + c - 1) // c for s, c in zip(arr.shape, ch)]
            entries = []
            lin = 0
            for idx in np.ndindex(*grid):
                off = [i * c for i, c in zip(idx, ch)]
                block = np.zeros(ch, dtype=arr.dtype)
                sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(off, ch, arr.shape))
                part = arr[sl]
                block[tuple(slice(0, p) for p in part.shape)] = part
                raw = block.tobytes()
                for f in v.filters:
                    if f == "shuffle":
                        raw = np.frombuffer(raw, np.uint8).reshape(-1, es).T.tobytes()
                    elif f == "deflate":
                        raw = zlib.compress(raw, 4)
                    elif f == "fletcher32":
                        raw = raw + struct.pack("<I", 0x12345678)   # the reader strips it (no verification)
                if lin not in v.skip_chunks:
                    entries.append((off, self.img.alloc(raw), len(raw)))
                lin += 1
            rank = arr.ndim

            def key(off, size):
                return struct.pack("<II", size, 0) + b"".join(struct.pack("<Q", o) for o in off) + struct.pack("<Q", 0)

            def node(level, items):   # items: (key bytes, child address); final key after the last child
                body = b"TREE" + bytes([1, level]) + struct.pack("<H", len(items)) + struct.pack("<QQ", UNDEF, UNDEF)
                for k, c in items:
                    body += k + struct.pack("<Q", c)
                body += key(list(arr.shape), 0)
                full = 8 + 16 + 64 * (len(key([0] * rank, 0)) + 8) + len(key([0] * rank, 0))
                return self.img.alloc(body + bytes(max(0, full - len(body))))

            leaves = [entries[i:i + 64] for i in range(0, len(entries), 64)] or [[]]
            leaf_at = [node(0, [(key(o, s), a) for o, a, s in lv]) for lv in leaves]
            if len(leaves) == 1:
                root = leaf_at[0]
            else:
                root = node(1, [(key(lv[0][0], 0), la) for lv, la in zip(leaves, leaf_at)])
            msgs.append((0x08, bytes([3, 2, rank + 1]) + struct.pack("<Q", root) +
                         b"".join(struct.pack("<I", c) for c in ch) + struct.pack("<I", es)))
            if v.filters:
                fl = b""
                for f in v.filters:
                    if f == "shuffle":
                        fl += struct.pack("<HHHH", 2, 0, 1, 1) + struct.pack("<I", es) + bytes(4)
                    elif f == "deflate":
                        fl += struct.pack("<HHHH", 1, 0, 1, 1) + struct.pack("<I", 4) + bytes(4)
                    elif f == "fletcher32":
                        fl += struct.pack("<HHHH", 3, 0, 1, 0)
                msgs.append((0x0B, bytes([1, len(v.filters)]) + bytes(6) + fl))
        atts = dict(extra_atts)
        if dim_refs:
            atts["DIMENSION_LIST"] = ("__refs__", dim_refs)
        atts.update(v.atts)
        msgs += self.attribute_msgs(atts)
        return self.ohdr(msgs)

    # ------------------------------------------------------------ groups
    def root_group(self, links: List[Tuple[str, int]], gatts: Dict[str, object]) -> Tuple[int, int, int]:
        """Returns (root object header address, B-tree address, local heap
        address) -- the last two UNDEF for new-style groups."""
        if self.sb < 2:
            data = b"\0" * 8
            offs = []
            for n, _ in links:
                offs.append(len(data))
                data += _pad8(n.encode() + b"\0")
            data_at = self.img.alloc(data + bytes(64))
            heap = self.img.alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(data) + 64, len(data),
                                                                                   data_at))
            ents = sorted(zip([n for n, _ in links], offs, [a for _, a in links]))
            snods, per = [], 8
            for i in range(0, max(1, len(ents)), per):
                grp = ents[i:i + per]
                body = b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(grp))
                for _, off, addr in grp:
                    body += struct.pack("<QQII", off, addr, 0, 0) + bytes(16)
                body += bytes(8 + per * 40 - len(body))
                snods.append((self.img.alloc(body), grp[-1][1] if grp else 0))
            body = b"TREE" + bytes([0, 0]) + struct.pack("<H", len(snods)) + struct.pack("<QQ", UNDEF, UNDEF)
            body += struct.pack("<Q", 0)
            for addr, last in snods:
                body += struct.pack("<Q", addr) + struct.pack("<Q", last)
            btree = self.img.alloc(body + bytes(max(0, 24 + 32 * 16 + 8 - len(body))))
            msgs = [(0x11, struct.pack("<QQ", btree, heap))] + self.attribute_msgs(gatts)
            return self.ohdr(msgs), btree, heap
        lmsgs = []
        for k, (n, addr) in enumerate(links):
            nb = n.encode()
            flags = 0x04 if self.crt else 0
            m = bytes([1, flags]) + (struct.pack("<Q", k) if self.crt else b"") + bytes([len(nb)]) + nb
            lmsgs.append(m + struct.pack("<Q", addr))
        gi = bytes([0, 0])
        if self.dense_links and lmsgs:
            heap_at, ids = self.fheap(lmsgs, 7)
            recs = sorted(((lookup3(n.encode()), struct.pack("<I", lookup3(n.encode())) + ids[k][:7])
                           for k, (n, _) in enumerate(links)), key=lambda r: r[0])
            bt = self.btree2(5, [r for _, r in recs])
            li = bytes([0, 0]) + struct.pack("<QQ", heap_at, bt)
            msgs = [(0x02, li), (0x0A, gi)]
        else:
            li = bytes([0, 0]) + struct.pack("<QQ", UNDEF, UNDEF)
            msgs = [(0x02, li), (0x0A, gi)] + [(0x06, m) for m in lmsgs]
        msgs += self.attribute_msgs(gatts)
        return self.ohdr(msgs), UNDEF, UNDEF


def write_nc4(path: str, dims: Sequence[Tuple[str, int]], variables: Sequence[Var], gatts: Dict[str, object] = None,
              superblock: int = 0, dense_atts: bool = False, dense_links: bool = False, crt_order: bool = True,
              dimids: bool = True) -> None:
    gatts = dict(gatts or {})
    w = Writer(superblock, dense_atts, dense_links, crt_order)
    img = w.img
    sb_size = 96 if superblock < 2 else 48
    img.alloc(bytes(sb_size))
    # the global heap collection (64 KiB, objects added as attributes are built), written last
    heap_size = 65536
    w.heap_addr = heap_slot = img.reserve(heap_size)
    scale_addr, links = {}, []
    by_name = {v.name: v for v in variables}
    for k, (dn, dl) in enumerate(dims):
        extra = {"CLASS": "DIMENSION_SCALE"}
        if dimids:
            extra["_Netcdf4Dimid"] = np.int32(k)
        if dn in by_name:
            v = by_name[dn]
            extra["NAME"] = dn
        else:
            v = Var(dn, (dn,), np.zeros(dl, np.float32), chunks=None, filters=())
            extra["NAME"] = "This is a netCDF dimension but not a netCDF variable.%10d" % dl
        a = w.dataset(v, [], extra)
        scale_addr[dn] = a
        links.append((dn, a))
    for v in variables:
        if v.name in scale_addr:
            continue
        refs = [scale_addr[d] for d in v.dims]
        links.append((v.name, w.dataset(v, refs, {})))
    root, _, _ = w.root_group(links, gatts)
    img.put(heap_slot, w.heap.image(heap_size))
    eof = len(img.b)
    if superblock < 2:
        sb = SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", 4, 16, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, root, 0, 0) + bytes(16)
    else:
        sb = SIG + bytes([superblock, 8, 8, 0]) + struct.pack("<QQQQ", 0, UNDEF, eof, root)
        sb += struct.pack("<I", lookup3(sb))
    img.put(0, sb)
    with open(path, "wb") as f:
        f.write(bytes(img.b))
