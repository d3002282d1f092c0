"""Minimal, dependency-free HDF5 reader and writer (the subset Keras weight files use).

The reference persists every model with ``model.save(...keras)`` (``cnn_baseline_train.py:230``,
``train_deep_ensemble_cnns.py:170``); a Keras v3 ``.keras`` archive stores its weights in an
HDF5 file (``model.weights.h5``), and the legacy ``.h5`` format is HDF5 throughout.  h5py is not
installed in this image, so this module implements the file format directly (HDF5 File Format
Specification v3) -- only as much of it as h5py/libhdf5 emit for Keras weight files:

reader
  * superblock v0/v1 (h5py's default ``libver='earliest'``) and v2/v3;
  * object headers v1 and v2 (with continuation blocks);
  * "old-style" groups (symbol-table message -> v1 B-tree of SNOD nodes + local heap) and
    "new-style" compact groups (link messages).  Dense link storage (fractal heap) is rejected;
  * datasets: contiguous, compact and unfiltered chunked layouts; fixed-point, IEEE float and
    fixed-length string element types;
  * attributes (message versions 1-3), including variable-length strings in the global heap
    (how h5py stores ``str`` attributes such as the legacy ``model_config``).
  Filtered (compressed) datasets and shared/committed datatypes raise ``NotImplementedError``.

writer
  superblock v0 + v1 object headers + symbol-table groups + contiguous little-endian numeric
  datasets + fixed-length string attributes: the oldest, most widely readable flavour of the
  format (what libhdf5 itself writes with ``libver='earliest'``).

Nothing here executes data from a file: values are decoded with ``numpy.frombuffer`` only.
The byte layout was written from the specification; no libhdf5-produced file is available in
this environment to pin it against ("parity unpinned", see ``tests/test_keras_io_cpu.py``).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Tuple, Union

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class HDF5Error(ValueError):
    pass


# ============================================================================ reader
class Dataset:
    def __init__(self, f: "File", name: str, addr: int, msgs):
        self.file, self.name, self.obj_addr, self._msgs = f, name, addr, msgs
        self.attrs = f._attrs(msgs)

    @property
    def shape(self) -> Tuple[int, ...]:
        return self.file._dataspace(self._msgs)

    @property
    def dtype(self) -> np.dtype:
        return self.file._dtype(self._msgs)[0]

    def read(self) -> np.ndarray:
        return self.file._read_dataset(self._msgs)

    def __array__(self, dtype=None):
        a = self.read()
        return a if dtype is None else a.astype(dtype)


class Group:
    def __init__(self, f: "File", name: str, addr: int, msgs):
        self.file, self.name, self.obj_addr, self._msgs = f, name, addr, msgs
        self.attrs = f._attrs(msgs)
        self._links: Optional[Dict[str, int]] = None

    def links(self) -> Dict[str, int]:
        if self._links is None:
            self._links = self.file._group_links(self._msgs)
        return self._links

    def keys(self) -> List[str]:
        return list(self.links().keys())

    def __contains__(self, key: str) -> bool:
        try:
            self[key]
            return True
        except KeyError:
            return False

    def __getitem__(self, path: str) -> Union["Group", Dataset]:
        node: Union[Group, Dataset] = self
        for part in [p for p in path.split("/") if p]:
            if not isinstance(node, Group) or part not in node.links():
                raise KeyError(f"{path!r} not found in {self.name!r}")
            node = self.file._open(node.name.rstrip("/") + "/" + part, node.links()[part])
        return node

    def visit(self, fn, prefix: str = ""):
        """Depth-first walk calling ``fn(path, node)`` for every member (paths relative to self)."""
        for k in self.keys():
            node = self[k]
            p = f"{prefix}{k}"
            fn(p, node)
            if isinstance(node, Group):
                node.visit(fn, p + "/")


class File(Group):
    """Read-only HDF5 file held in memory (Keras weight files are a few MB)."""

    def __init__(self, source: Union[str, bytes]):
        if isinstance(source, (bytes, bytearray, memoryview)):
            self.buf = bytes(source)
        else:
            with open(source, "rb") as fh:
                self.buf = fh.read()
        self.base = self.buf.find(SIGNATURE)
        if self.base < 0 or self.base % 512 != 0:
            raise HDF5Error("not an HDF5 file (signature missing)")
        root = self._superblock()
        self.file = self
        super().__init__(self, "/", root, self._header(root))

    # ------------------------------------------------------------------ primitives
    def _u(self, off: int, n: int) -> int:
        return int.from_bytes(self.buf[off:off + n], "little")

    def _addr(self, off: int) -> int:
        return self._u(off, self.so)

    def _len(self, off: int) -> int:
        return self._u(off, self.sl)

    def _abs(self, addr: int) -> int:
        return self.base_addr + addr

    # ------------------------------------------------------------------ superblock
    def _superblock(self) -> int:
        p = self.base + 8
        ver = self.buf[p]
        if ver in (0, 1):
            self.so, self.sl = self.buf[p + 5], self.buf[p + 6]
            q = p + 16 + (4 if ver == 1 else 0)
            self.base_addr = self._addr(q)
            q += 4 * self.so  # base, free-space, EOF, driver info
            # root group symbol table entry: link name offset, object header address, ...
            return self._addr(q + self.so)
        if ver in (2, 3):
            self.so, self.sl = self.buf[p + 1], self.buf[p + 2]
            q = p + 4
            self.base_addr = self._addr(q)
            return self._addr(q + 3 * self.so)
        raise NotImplementedError(f"HDF5 superblock version {ver}")

    # ------------------------------------------------------------------ object headers
    def _header(self, addr: int) -> List[Tuple[int, int, bytes]]:
        """All messages (type, flags, payload) of the object header at ``addr``."""
        off = self._abs(addr)
        msgs: List[Tuple[int, int, bytes]] = []
        if self.buf[off:off + 4] == b"OHDR":
            ver, flags = self.buf[off + 4], self.buf[off + 5]
            if ver != 2:
                raise NotImplementedError(f"object header v{ver}")
            q = off + 6 + (16 if flags & 0x20 else 0) + (4 if flags & 0x10 else 0)
            nsz = 1 << (flags & 3)
            size = self._u(q, nsz)
            q += nsz
            blocks = [(q, q + size)]
            while blocks:
                start, end = blocks.pop(0)
                p = start
                while p + 4 <= end:
                    mtype, msize, mflags = self.buf[p], self._u(p + 1, 2), self.buf[p + 3]
                    p += 4 + (2 if flags & 0x04 else 0)
                    data = self.buf[p:p + msize]
                    p += msize
                    if mtype == 0x10:  # continuation -> "OCHK" block (signature + messages + checksum)
                        c = self._abs(int.from_bytes(data[:self.so], "little"))
                        ln = int.from_bytes(data[self.so:self.so + self.sl], "little")
                        blocks.append((c + 4, c + ln - 4))
                    else:
                        msgs.append((mtype, mflags, data))
            return msgs
        ver = self.buf[off]
        if ver != 1:
            raise HDF5Error(f"bad object header at {addr:#x} (version byte {ver})")
        nmsg, size = self._u(off + 2, 2), self._u(off + 8, 4)
        blocks = [(off + 16, off + 16 + size)]
        while blocks and len(msgs) < nmsg + 64:
            start, end = blocks.pop(0)
            p = start
            while p + 8 <= end:
                mtype, msize, mflags = self._u(p, 2), self._u(p + 2, 2), self.buf[p + 4]
                data = self.buf[p + 8:p + 8 + msize]
                p += 8 + msize
                if mtype == 0x10:
                    c = self._abs(int.from_bytes(data[:self.so], "little"))
                    ln = int.from_bytes(data[self.so:self.so + self.sl], "little")
                    blocks.append((c, c + ln))
                elif mtype != 0:
                    msgs.append((mtype, mflags, data))
        return msgs

    def _open(self, name: str, addr: int) -> Union[Group, Dataset]:
        msgs = self._header(addr)
        types = {t for t, _, _ in msgs}
        if 0x08 in types:
            return Dataset(self, name, addr, msgs)
        return Group(self, name, addr, msgs)

    # ------------------------------------------------------------------ groups
    def _group_links(self, msgs) -> Dict[str, int]:
        links: Dict[str, int] = {}
        for t, _, d in msgs:
            if t == 0x11:  # symbol table: v1 B-tree + local heap
                btree = int.from_bytes(d[:self.so], "little")
                heap = int.from_bytes(d[self.so:2 * self.so], "little")
                self._walk_group_btree(btree, self._local_heap(heap), links)
            elif t == 0x06:
                name, addr = self._link_message(d)
                if addr is not None:
                    links[name] = addr
            elif t == 0x02:
                fheap = int.from_bytes(d[2 + (8 if d[1] & 1 else 0):][:self.so], "little")
                if fheap != UNDEF and fheap != (1 << (8 * self.so)) - 1:
                    raise NotImplementedError("dense (fractal-heap) link storage")
        return links

    def _local_heap(self, addr: int) -> bytes:
        off = self._abs(addr)
        if self.buf[off:off + 4] != b"HEAP":
            raise HDF5Error("bad local heap signature")
        size = self._len(off + 8)
        data = self._abs(self._addr(off + 8 + 2 * self.sl))
        return self.buf[data:data + size]

    @staticmethod
    def _cstr(heap: bytes, off: int) -> str:
        end = heap.index(b"\x00", off)
        return heap[off:end].decode("utf-8")

    def _walk_group_btree(self, addr: int, heap: bytes, links: Dict[str, int]) -> None:
        off = self._abs(addr)
        sig = self.buf[off:off + 4]
        if sig == b"SNOD":
            n = self._u(off + 6, 2)
            e = off + 8
            esz = 2 * self.so + 24
            for i in range(n):
                q = e + i * esz
                links[self._cstr(heap, self._addr(q))] = self._addr(q + self.so)
            return
        if sig != b"TREE" or self.buf[off + 4] != 0:
            raise HDF5Error("bad group B-tree node")
        used = self._u(off + 6, 2)
        q = off + 8 + 2 * self.so + self.sl  # skip siblings and key 0
        for _ in range(used):
            self._walk_group_btree(self._addr(q), heap, links)
            q += self.so + self.sl

    def _link_message(self, d: bytes) -> Tuple[str, Optional[int]]:
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
        nsz = 1 << (flags & 3)
        nlen = int.from_bytes(d[p:p + nsz], "little")
        p += nsz
        name = d[p:p + nlen].decode("utf-8")
        p += nlen
        if ltype != 0:  # soft / external links are not followed
            return name, None
        return name, int.from_bytes(d[p:p + self.so], "little")

    # ------------------------------------------------------------------ datatypes / dataspaces
    def _parse_dtype(self, d: bytes) -> Tuple[np.dtype, int, dict]:
        cls, size = d[0] & 0x0F, self._u_b(d, 4, 4)
        bits = d[1:4]
        if cls == 0:  # fixed point
            order = ">" if bits[0] & 1 else "<"
            kind = "i" if bits[0] & 0x08 else "u"
            return np.dtype(f"{order}{kind}{size}"), size, {}
        if cls == 1:  # IEEE float
            order = ">" if bits[0] & 1 else "<"
            if size not in (2, 4, 8):
                raise NotImplementedError(f"float of {size} bytes")
            return np.dtype(f"{order}f{size}"), size, {}
        if cls == 3:  # fixed-length string
            return np.dtype(f"S{size}"), size, {}
        if cls == 9:  # variable length
            vtype = bits[0] & 0x0F
            return np.dtype(object), size, {"vlen_string": vtype == 1, "base": d[8:]}
        raise NotImplementedError(f"HDF5 datatype class {cls}")

    @staticmethod
    def _u_b(d: bytes, off: int, n: int) -> int:
        return int.from_bytes(d[off:off + n], "little")

    def _parse_space(self, d: bytes) -> Tuple[int, ...]:
        ver, ndim, flags = d[0], d[1], d[2]
        if ver == 1:
            p = 8
        elif ver == 2:
            if d[3] == 0:
                return ()
            if d[3] == 2:
                return (0,)
            p = 4
        else:
            raise NotImplementedError(f"dataspace v{ver}")
        return tuple(self._u_b(d, p + i * self.sl, self.sl) for i in range(ndim))

    def _dtype(self, msgs):
        for t, fl, d in msgs:
            if t == 0x03:
                if fl & 0x02:
                    raise NotImplementedError("shared (committed) datatype")
                return self._parse_dtype(d)
        raise HDF5Error("dataset without datatype message")

    def _dataspace(self, msgs) -> Tuple[int, ...]:
        for t, _, d in msgs:
            if t == 0x01:
                return self._parse_space(d)
        raise HDF5Error("dataset without dataspace message")

    # ------------------------------------------------------------------ dataset data
    def _read_dataset(self, msgs) -> np.ndarray:
        for t, _, d in msgs:
            if t == 0x0B and len(d) > 2 and d[1] > 0:
                raise NotImplementedError("filtered (compressed) HDF5 dataset")
        dt, esz, extra = self._dtype(msgs)
        shape = self._dataspace(msgs)
        n = int(np.prod(shape)) if shape else 1
        layout = next(d for t, _, d in msgs if t == 0x08)
        raw = self._layout_bytes(layout, n * esz, shape, esz)
        if extra:
            return self._decode_vlen(raw, n, extra).reshape(shape)
        return np.frombuffer(raw, dtype=dt, count=n).reshape(shape).copy()

    def _layout_bytes(self, d: bytes, nbytes: int, shape, esz: int) -> bytes:
        ver = d[0]
        if ver in (1, 2):
            ndim, cls = d[1], d[2]
            p = 8
            if cls == 0:  # compact
                p += 4 * ndim
                size = self._u_b(d, p, 4)
                return d[p + 4:p + 4 + size][:nbytes]
            addr = self._u_b(d, p, self.so)
            if cls == 1:
                off = self._abs(addr)
                return self.buf[off:off + nbytes]
            dims = [self._u_b(d, p + self.so + 4 * i, 4) for i in range(ndim)]
            return self._read_chunked(addr, dims, shape, esz)
        if ver == 3:
            cls = d[1]
            if cls == 0:
                size = self._u_b(d, 2, 2)
                return d[4:4 + size][:nbytes]
            if cls == 1:
                addr = self._u_b(d, 2, self.so)
                if addr == UNDEF:
                    return bytes(nbytes)  # never written: fill value 0
                off = self._abs(addr)
                return self.buf[off:off + nbytes]
            if cls == 2:
                ndim = d[2]
                addr = self._u_b(d, 3, self.so)
                dims = [self._u_b(d, 3 + self.so + 4 * i, 4) for i in range(ndim)]
                return self._read_chunked(addr, dims, shape, esz)
        raise NotImplementedError(f"data layout message v{ver}")

    def _read_chunked(self, addr: int, cdims, shape, esz: int) -> bytes:
        """Unfiltered chunked storage: v1 B-tree (type 1) of chunks, copied into a dense array."""
        rank = len(shape)
        cshape = tuple(cdims[:rank])
        out = np.zeros(tuple(shape) + (esz,), dtype=np.uint8)
        if addr == UNDEF:
            return out.tobytes()

        def walk(a: int):
            off = self._abs(a)
            if self.buf[off:off + 4] != b"TREE" or self.buf[off + 4] != 1:
                raise HDF5Error("bad chunk B-tree node")
            level, used = self.buf[off + 5], self._u(off + 6, 2)
            ksz = 8 + 8 * (rank + 1)
            q = off + 8 + 2 * self.so
            for _ in range(used):
                csize, fmask = self._u(q, 4), self._u(q + 4, 4)
                origin = [self._u(q + 8 + 8 * i, 8) for i in range(rank)]
                child = self._addr(q + ksz)
                if level > 0:
                    walk(child)
                else:
                    if fmask:
                        raise NotImplementedError("filtered chunk")
                    c = self._abs(child)
                    blk = np.frombuffer(self.buf[c:c + int(np.prod(cshape)) * esz], dtype=np.uint8)
                    blk = blk.reshape(cshape + (esz,))
                    sl = tuple(slice(o, min(o + cs, s)) for o, cs, s in zip(origin, cshape, shape))
                    out[sl] = blk[tuple(slice(0, x.stop - x.start) for x in sl)]
                q += ksz + self.so

        walk(addr)
        return out.tobytes()

    def _decode_vlen(self, raw: bytes, n: int, extra: dict) -> np.ndarray:
        out = np.empty(n, dtype=object)
        step = 4 + self.so + 4
        for i in range(n):
            q = i * step
            length = self._u_b(raw, q, 4)
            coll = self._u_b(raw, q + 4, self.so)
            idx = self._u_b(raw, q + 4 + self.so, 4)
            data = self._global_heap_object(coll, idx)[:length] if length else b""
            out[i] = data.decode("utf-8") if extra.get("vlen_string") else data
        return out

    def _global_heap_object(self, coll: int, idx: int) -> bytes:
        off = self._abs(coll)
        if self.buf[off:off + 4] != b"GCOL":
            raise HDF5Error("bad global heap collection")
        size = self._len(off + 8)
        p, end = off + 8 + self.sl, off + size
        while p + 8 + self.sl <= end:
            oid, osz = self._u(p, 2), self._len(p + 8)
            if oid == 0:
                break
            if oid == idx:
                return self.buf[p + 8 + self.sl:p + 8 + self.sl + osz]
            p += 8 + self.sl + ((osz + 7) & ~7)
        raise HDF5Error(f"global heap object {idx} not found")

    # ------------------------------------------------------------------ attributes
    def _attrs(self, msgs) -> Dict[str, np.ndarray]:
        out = {}
        for t, _, d in msgs:
            if t != 0x0C:
                continue
            ver = d[0]
            nsz, tsz, ssz = self._u_b(d, 2, 2), self._u_b(d, 4, 2), self._u_b(d, 6, 2)
            if ver == 1:
                p = 8
                pad = lambda x: (x + 7) & ~7  # noqa: E731
            elif ver in (2, 3):
                p = 8 + (1 if ver == 3 else 0)
                pad = lambda x: x  # noqa: E731
            else:
                raise NotImplementedError(f"attribute message v{ver}")
            name = d[p:p + nsz].split(b"\x00")[0].decode("utf-8")
            p += pad(nsz)
            tdesc = d[p:p + tsz]
            p += pad(tsz)
            shape = self._parse_space(d[p:p + ssz])
            p += pad(ssz)
            dt, esz, extra = self._parse_dtype(tdesc)
            n = int(np.prod(shape)) if shape else 1
            raw = d[p:p + n * (4 + self.so + 4 if extra else esz)]
            if extra:
                val = self._decode_vlen(raw, n, extra)
            else:
                val = np.frombuffer(raw, dtype=dt, count=n).copy()
            out[name] = val.reshape(shape) if shape else val.reshape(())
        return out


def attr_str(v) -> Union[str, List[str]]:
    """Decode a string attribute (scalar or array, fixed- or variable-length) to ``str``."""
    a = np.asarray(v)
    conv = lambda x: x.decode("utf-8") if isinstance(x, (bytes, np.bytes_)) else str(x)  # noqa: E731
    if a.shape == ():
        return conv(a.item())
    return [conv(x) for x in a.reshape(-1)]


# ============================================================================ writer
_GROUP_LEAF_K = 64      # SNOD holds 2K = 128 entries: every Keras group fits one node
_GROUP_INTERNAL_K = 16


class _Node:
    def __init__(self, attrs=None):
        self.attrs: Dict[str, object] = dict(attrs or {})


class _WGroup(_Node):
    def __init__(self, attrs=None):
        super().__init__(attrs)
        self.children: Dict[str, _Node] = {}


class _WData(_Node):
    def __init__(self, arr: np.ndarray, attrs=None):
        super().__init__(attrs)
        a = np.asarray(arr)
        if a.dtype.kind not in "fiu" and a.dtype.kind != "S":
            raise TypeError(f"unsupported dataset dtype {a.dtype}")
        self.arr = np.array(a.astype(a.dtype.newbyteorder("<")) if a.dtype.kind in "fiu" else a, order="C")


class Writer:
    """Build an HDF5 tree in memory, then ``save(path)``.

    >>> w = Writer(); w.create_dataset("layers/dense/vars/0", np.ones((96, 1), np.float32)); w.save(p)
    """

    def __init__(self):
        self.root = _WGroup()

    def _group(self, path: str, create: bool = True) -> _WGroup:
        g = self.root
        for part in [p for p in path.split("/") if p]:
            if part not in g.children:
                if not create:
                    raise KeyError(path)
                g.children[part] = _WGroup()
            g = g.children[part]
            if not isinstance(g, _WGroup):
                raise ValueError(f"{path!r} crosses a dataset")
        return g

    def create_group(self, path: str, attrs=None) -> None:
        self._group(path).attrs.update(attrs or {})

    def set_attr(self, path: str, name: str, value) -> None:
        node = self._group(path) if path.strip("/") == "" else self._lookup(path)
        node.attrs[name] = value

    def _lookup(self, path: str) -> _Node:
        parts = [p for p in path.split("/") if p]
        g = self._group("/".join(parts[:-1]), create=False)
        return g.children[parts[-1]]

    def create_dataset(self, path: str, data, attrs=None) -> None:
        parts = [p for p in path.split("/") if p]
        g = self._group("/".join(parts[:-1]))
        g.children[parts[-1]] = _WData(data, attrs)

    # ------------------------------------------------------------------ serialisation
    def tobytes(self) -> bytes:
        self.out = bytearray()
        sb_size = 8 + 16 + 4 * 8 + 40  # v0 superblock incl. root symbol-table entry
        self.out += bytes(sb_size)
        root_hdr, root_btree, root_heap = self._write_group(self.root)
        eof = len(self.out)
        sb = bytearray(SIGNATURE)
        sb += bytes([0, 0, 0, 0, 0, 8, 8, 0])
        sb += struct.pack("<HHI", _GROUP_LEAF_K, _GROUP_INTERNAL_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, root_hdr, 1, 0) + struct.pack("<QQ", root_btree, root_heap)
        assert len(sb) == sb_size
        self.out[:sb_size] = sb
        return bytes(self.out)

    def save(self, path: str) -> str:
        with open(path, "wb") as fh:
            fh.write(self.tobytes())
        return path

    def _alloc(self, data: bytes, align: int = 8) -> int:
        while len(self.out) % align:
            self.out += b"\x00"
        addr = len(self.out)
        self.out += data
        return addr

    @staticmethod
    def _msg(mtype: int, payload: bytes, flags: int = 0) -> bytes:
        payload = payload + bytes((-len(payload)) % 8)
        return struct.pack("<HHB3x", mtype, len(payload), flags) + payload

    def _header(self, messages: List[bytes]) -> int:
        body = b"".join(messages)
        hdr = struct.pack("<BBHII", 1, 0, len(messages), 1, len(body)) + bytes(4)
        return self._alloc(hdr + body)

    @staticmethod
    def _dtype_msg(a: np.ndarray) -> bytes:
        k, size = a.dtype.kind, a.dtype.itemsize
        if k == "f":
            if size == 4:
                props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
                bits = bytes([0x20, 0x1F, 0])
            elif size == 8:
                props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
                bits = bytes([0x20, 0x3F, 0])
            else:
                raise TypeError(f"float{8 * size}")
            return bytes([0x11]) + bits + struct.pack("<I", size) + props
        if k in "iu":
            bits = bytes([0x08 if k == "i" else 0, 0, 0])
            return bytes([0x10]) + bits + struct.pack("<I", size) + struct.pack("<HH", 0, 8 * size)
        if k == "S":
            return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", size)  # null-padded ASCII (numpy "S")
        raise TypeError(a.dtype)

    @staticmethod
    def _space_msg(shape) -> bytes:
        out = struct.pack("<BBB5x", 1, len(shape), 0)
        for s in shape:
            out += struct.pack("<Q", s)
        return out

    def _global_heap(self, objs: List[bytes]) -> int:
        """One global-heap collection holding ``objs`` (indices 1..n), padded to libhdf5's 4 KiB minimum."""
        body = bytearray()
        for i, o in enumerate(objs, 1):
            body += struct.pack("<HH4xQ", i, 1, len(o)) + o + bytes((-len(o)) % 8)
        size = max(4096, 16 + len(body) + 16)
        free = size - 16 - len(body)
        body += struct.pack("<HH4xQ", 0, 0, free) + bytes(free - 16)
        return self._alloc(b"GCOL" + bytes([1, 0, 0, 0]) + struct.pack("<Q", size) + bytes(body))

    def _attr_msgs(self, attrs: Dict[str, object]) -> List[bytes]:
        msgs = []
        pad = lambda x: x + bytes((-len(x)) % 8)  # noqa: E731
        for name, v in attrs.items():
            nm = name.encode("utf-8") + b"\x00"
            if isinstance(v, str):  # h5py stores a Python str as a variable-length UTF-8 string
                b = v.encode("utf-8")
                coll = self._global_heap([b])
                base = bytes([0x10, 0, 0, 0]) + struct.pack("<I", 1) + struct.pack("<HH", 0, 8)
                dt = bytes([0x19, 0x01, 0x01, 0x00]) + struct.pack("<I", 16) + base
                sp = struct.pack("<BBB5x", 1, 0, 0)
                data = struct.pack("<IQI", len(b), coll, 1)
                payload = struct.pack("<BxHHH", 1, len(nm), len(dt), len(sp)) + pad(nm) + pad(dt) + pad(sp) + data
                msgs.append(self._msg(0x0C, payload))
                continue
            if isinstance(v, bytes):
                a = np.array(v, dtype=f"S{max(len(v), 1)}")
            elif isinstance(v, (list, tuple)) and v and all(isinstance(x, (str, bytes)) for x in v):
                bs = [x.encode("utf-8") if isinstance(x, str) else x for x in v]
                a = np.array(bs, dtype=f"S{max(max(len(x) for x in bs), 1)}")
            else:
                a = np.asarray(v)
                if a.dtype.kind in "fiu":
                    a = a.astype(a.dtype.newbyteorder("<"))
            dt = self._dtype_msg(a)
            sp = self._space_msg(a.shape) if a.shape else struct.pack("<BBB5x", 1, 0, 0)
            payload = struct.pack("<BxHHH", 1, len(nm), len(dt), len(sp)) + pad(nm) + pad(dt) + pad(sp) + a.tobytes()
            msgs.append(self._msg(0x0C, payload))
        return msgs

    def _write_dataset(self, d: _WData) -> int:
        a = d.arr
        data_addr = self._alloc(a.tobytes()) if a.nbytes else UNDEF
        fill = struct.pack("<BBBB", 2, 1, 2, 0)  # v2: early allocation, fill if set, none defined
        layout = struct.pack("<BBQQ", 3, 1, data_addr, a.nbytes)
        msgs = [self._msg(0x01, self._space_msg(a.shape) if a.shape else struct.pack("<BBB5x", 1, 0, 0)),
                self._msg(0x03, self._dtype_msg(a)),
                self._msg(0x05, fill),
                self._msg(0x08, layout)] + self._attr_msgs(d.attrs)
        return self._header(msgs)

    def _write_group(self, g: _WGroup) -> Tuple[int, int, int]:
        names = sorted(g.children)  # symbol-table nodes are kept in name order
        if len(names) > 2 * _GROUP_LEAF_K:
            raise NotImplementedError(f"group with more than {2 * _GROUP_LEAF_K} members")
        child_addrs = []
        for n in names:
            c = g.children[n]
            child_addrs.append(self._write_group(c)[0] if isinstance(c, _WGroup) else self._write_dataset(c))
        # local heap: offset 0 = "" (B-tree key 0), then the member names
        heap = bytearray(b"\x00" * 8)
        offs = []
        for n in names:
            offs.append(len(heap))
            heap += n.encode("utf-8") + b"\x00"
            heap += bytes((-len(heap)) % 8)
        heap += bytes(max(8, (-len(heap)) % 8))
        heap_data = self._alloc(bytes(heap))
        heap_addr = self._alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap), 1, heap_data))
        # one symbol-table node (allocated at full capacity, as libhdf5 does)
        snod = bytearray(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(names)))
        for off, addr in zip(offs, child_addrs):
            snod += struct.pack("<QQII", off, addr, 0, 0) + bytes(16)
        snod += bytes(8 + 2 * _GROUP_LEAF_K * 40 - len(snod))
        snod_addr = self._alloc(bytes(snod))
        # v1 B-tree (type 0, leaf level) with one child: keys = heap offsets of "" and the last name
        tree = bytearray(b"TREE" + bytes([0, 0]) + struct.pack("<H", 1 if names else 0))
        tree += struct.pack("<QQ", UNDEF, UNDEF)
        if names:
            tree += struct.pack("<QQQ", 0, snod_addr, offs[-1])
        else:
            tree += struct.pack("<Q", 0)
        tree += bytes(8 + 2 * 8 + (2 * _GROUP_INTERNAL_K + 1) * 8 + 2 * _GROUP_INTERNAL_K * 8 - len(tree))
        btree_addr = self._alloc(bytes(tree))
        stab = struct.pack("<QQ", btree_addr, heap_addr)
        hdr = self._header([self._msg(0x11, stab)] + self._attr_msgs(g.attrs))
        return hdr, btree_addr, heap_addr
