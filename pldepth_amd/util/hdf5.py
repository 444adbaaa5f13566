"""A minimal HDF5 reader/writer for Keras weight files (h5py / libhdf5 are not in this image).

Replaces what the reference gets from h5py under Keras: ``model.load_weights(path)``
(pldepth/PLDepth.py:136-137), ``model.save(... .h5)`` (:181) and ``ModelCheckpoint(filepath=
'...h5')`` (pldepth/util/tracking_utils.py:21-30). Only the subset of the HDF5 file format
(HDF Group, "HDF5 File Format Specification Version 3.0") those files use is implemented:

writer — the layout libhdf5 produces with its default ("earliest") format, which is what h5py
  writes for Keras: superblock version 0, version-1 object headers, old-style groups (symbol
  table message -> version-1 B-tree of symbol-table nodes + local heap of names), contiguous
  datasets, attributes in the object header (fixed-length strings, ints, floats; scalar or 1-D);
reader — the same plus what newer libraries write for such files: superblock versions 0-3,
  object header versions 1 and 2 with continuation blocks, compact (link-message) groups,
  attribute messages versions 1-3, dataspace versions 1-2, contiguous and compact layouts
  (layout message versions 1-4), fixed-point / floating-point / fixed-length string datatypes,
  and variable-length strings (datatype class 9, the elements in global-heap collections): what
  h5py stores for a Python ``str`` attribute (h5py 2.10 under Keras writes e.g. the root
  ``keras_version`` / ``backend`` that way when handed str). The writer emits them for
  ``VLenStr`` values (so tests can build such files). Dense (fractal-heap) link or attribute
  storage and chunked or filtered datasets raise NotImplementedError (Keras' HDF5 weight files
  use none of them); an attribute of an unsupported datatype is skipped with a warning instead
  of failing the whole load.

In memory a file is a tree of ``Group`` (``attrs`` + ordered members) and ``Dataset``
(``data`` numpy array + ``attrs``). Paths with '/' create / look up nested groups like h5py.
Parity with h5py-written files is unpinned: no HDF5 library exists here to produce or check one.
"""
import struct
import warnings

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF
GROUP_INTERNAL_K = 16
LOCAL_HEAP_FREE_NULL = 1  # libhdf5's end-of-free-list marker for local heaps
GLOBAL_HEAP_MIN = 4096  # libhdf5's smallest global-heap collection (H5HG_MINSIZE)


class VLenStr(str):
    """A str attribute value written as an HDF5 variable-length UTF-8 string (h5py's encoding of
    a Python str) instead of a fixed-length one."""


class _VLen(object):
    """Decoded class-9 datatype: a variable-length string (or sequence of `base`)."""

    def __init__(self, is_str, base, size):
        self.is_str, self.base, self.itemsize = is_str, base, size


class Dataset(object):
    def __init__(self, data, attrs=None):
        self.data = np.asarray(data)
        self.attrs = dict(attrs or {})

    @property
    def shape(self):
        return self.data.shape

    def __array__(self, dtype=None):
        return self.data if dtype is None else self.data.astype(dtype)


class Group(object):
    def __init__(self, attrs=None):
        self.attrs = dict(attrs or {})
        self.members = {}

    def _walk(self, path, create):
        parts = [p for p in path.split("/") if p]
        g = self
        for p in parts[:-1]:
            if p not in g.members:
                if not create:
                    raise KeyError(path)
                g.members[p] = Group()
            g = g.members[p]
            if not isinstance(g, Group):
                raise KeyError(f"{path}: {p} is not a group")
        return g, parts[-1]

    def create_group(self, path):
        g, last = self._walk(path, True)
        if last in g.members:
            raise ValueError(f"{path} already exists")
        g.members[last] = Group()
        return g.members[last]

    def require_group(self, path):
        g, last = self._walk(path, True)
        if last not in g.members:
            g.members[last] = Group()
        return g.members[last]

    def create_dataset(self, path, data):
        g, last = self._walk(path, True)
        if last in g.members:
            raise ValueError(f"{path} already exists")
        g.members[last] = Dataset(data)
        return g.members[last]

    def __getitem__(self, path):
        g, last = self._walk(path, False)
        return g.members[last]

    def __contains__(self, path):
        try:
            self[path]
            return True
        except KeyError:
            return False

    def keys(self):
        return list(self.members)


# ----------------------------------------------------------------------------- encoding
def _pad8(b):
    return b + b"\0" * (-len(b) % 8)


def _dtype_message(dt):
    """Datatype message body (version 1) for a numpy dtype."""
    dt = np.dtype(dt)
    if dt.kind == "f":
        n = dt.itemsize
        sign, eloc, esz, msz, bias = {4: (31, 23, 8, 23, 127), 8: (63, 52, 11, 52, 1023),
                                      2: (15, 10, 5, 10, 15)}[n]
        head = struct.pack("<BBBBI", (1 << 4) | 1, 0x20, sign, 0, n)
        return head + struct.pack("<HHBBBBI", 0, 8 * n, eloc, esz, 0, msz, bias)
    if dt.kind in "iu":
        n = dt.itemsize
        return struct.pack("<BBBBI", (1 << 4) | 0, 0x08 if dt.kind == "i" else 0, 0, 0, n) + \
            struct.pack("<HH", 0, 8 * n)
    if dt.kind == "b":
        return _dtype_message(np.uint8)
    if dt.kind == "S":
        return struct.pack("<BBBBI", (1 << 4) | 3, 0x01, 0, 0, max(dt.itemsize, 1))  # nullpad
    raise NotImplementedError(f"HDF5 writer: dtype {dt}")


def _dataspace_message(shape):
    """Dataspace message version 1 (rank 0 = scalar)."""
    return struct.pack("<BBBB4x", 1, len(shape), 0, 0) + b"".join(
        struct.pack("<Q", int(d)) for d in shape)


def _as_storable(v):
    """Attribute / dataset values as numpy arrays of a storable dtype (str -> fixed bytes)."""
    if isinstance(v, str):
        v = v.encode("utf8")
    if isinstance(v, bytes):
        return np.array(v, dtype=f"S{max(len(v), 1)}")
    a = np.asarray(v)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "utf8")
    if a.dtype.kind == "O":
        a = np.array([x.encode("utf8") if isinstance(x, str) else x for x in a.reshape(-1)]
                     ).reshape(a.shape)
    if a.dtype.kind == "b":
        a = a.astype(np.uint8)
    if a.dtype.byteorder == ">":
        a = a.astype(a.dtype.newbyteorder("<"))
    return a


def _message(mtype, body, flags=0):
    body = _pad8(body)
    return struct.pack("<HHB3x", mtype, len(body), flags) + body


def _vlen_str_dtype_message():
    """Class 9 (variable-length) version 1: type 1 = string, padding 0 = null-terminated,
    character set 1 = UTF-8; element size 16 (u32 length + global heap id: u64 collection
    address + u32 object index); base type: 1-byte unsigned fixed-point (libhdf5's parent type
    of a variable-length string)."""
    return struct.pack("<BBBBI", (1 << 4) | 9, 0x01, 0x01, 0, 16) + \
        struct.pack("<BBBBI", (1 << 4) | 0, 0, 0, 0, 1) + struct.pack("<HH", 0, 8)


def _global_heap_collection(objects):
    """A global heap collection ("GCOL", version 1) holding `objects` (bytes) at indices
    1..n, then the free-space object (index 0) covering the rest of the >= 4 KiB collection."""
    body = b""
    for i, data in enumerate(objects, 1):
        body += struct.pack("<HH4xQ", i, 1, len(data)) + _pad8(data)
    size = 16 + len(body) + 16
    size = max(size, GLOBAL_HEAP_MIN)
    size += -size % 8
    free = size - 16 - len(body)
    body += struct.pack("<HH4xQ", 0, 0, free) + b"\0" * (free - 16)
    return b"GCOL" + struct.pack("<B3xQ", 1, size) + body


def _attribute_message(name, value, writer=None):
    nm = name.encode("utf8") + b"\0"
    if isinstance(value, VLenStr):
        if writer is None:
            raise ValueError("variable-length strings need the file writer (global heap)")
        data = value.encode("utf8")
        coll = writer.alloc(_global_heap_collection([data]))
        dtm, dsm = _vlen_str_dtype_message(), _dataspace_message(())
        raw = struct.pack("<IQI", len(data), coll, 1)
    else:
        a = _as_storable(value)
        dtm, dsm = _dtype_message(a.dtype), _dataspace_message(a.shape)
        raw = np.ascontiguousarray(a).tobytes()
    body = struct.pack("<BBHHH", 1, 0, len(nm), len(dtm), len(dsm))
    body += _pad8(nm) + _pad8(dtm) + _pad8(dsm) + raw
    return _message(0x000C, body)


class _Writer(object):
    def __init__(self):
        self.buf = bytearray(96)  # superblock, written last

    def alloc(self, data):
        while len(self.buf) % 8:
            self.buf += b"\0"
        off = len(self.buf)
        self.buf += data
        return off

    def object_header(self, messages):
        body = b"".join(messages)
        if not messages:
            body = _message(0x0000, b"")  # a NIL message: headers are never empty
            messages = [body]
        pfx = struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(body))
        return self.alloc(pfx + body)

    def dataset(self, ds):
        a = _as_storable(ds.data)
        raw = np.ascontiguousarray(a).tobytes()
        addr = self.alloc(raw) if raw else UNDEF
        msgs = [_message(0x0001, _dataspace_message(a.shape)),
                _message(0x0003, _dtype_message(a.dtype), flags=1),  # constant
                _message(0x0005, struct.pack("<BBBB", 2, 1, 2, 0)),   # fill value: undefined
                _message(0x0008, struct.pack("<BBQQ", 3, 1, addr, len(raw)))]
        msgs += [_attribute_message(k, v, self) for k, v in ds.attrs.items()]
        return self.object_header(msgs)

    def group(self, g, leaf_k):
        """Children first (post-order): returns (object header, B-tree, local heap) addresses."""
        entries = []
        for name, m in g.members.items():
            if isinstance(m, Group):
                oh, bt, hp = self.group(m, leaf_k)
                entries.append((name.encode("utf8"), oh, (bt, hp)))
            else:
                entries.append((name.encode("utf8"), self.dataset(m), None))
        entries.sort(key=lambda e: e[0])
        # local heap: "" at 0, then the names (8-aligned), then one free block
        heap, offs = bytearray(b"\0" * 8), []
        for name, _, _ in entries:
            offs.append(len(heap))
            heap += _pad8(name + b"\0")
        free_off = len(heap)
        heap += struct.pack("<QQ", LOCAL_HEAP_FREE_NULL, 16)
        heap_data = self.alloc(bytes(heap))
        heap_addr = self.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), free_off,
                                                     heap_data))
        # symbol-table nodes of <= 2K entries each, under one level-0 B-tree node
        cap = 2 * leaf_k
        chunks = [list(range(i, min(i + cap, len(entries)))) for i in
                  range(0, max(len(entries), 1), cap)] if entries else [[]]
        if len(chunks) > 2 * GROUP_INTERNAL_K:
            raise NotImplementedError("group too large for one B-tree node")
        snods, keys = [], [0]
        for ch in chunks:
            body = b"SNOD" + struct.pack("<BxH", 1, len(ch))
            for i in ch:
                name, oh, cache = entries[i]
                if cache is None:
                    body += struct.pack("<QQII16x", offs[i], oh, 0, 0)
                else:
                    body += struct.pack("<QQIIQQ", offs[i], oh, 1, 0, cache[0], cache[1])
            body += b"\0" * (40 * (cap - len(ch)))
            snods.append(self.alloc(body))
            keys.append(offs[ch[-1]] if ch else 0)
        nchild = len(snods) if entries else 0
        bt = b"TREE" + struct.pack("<BBHQQ", 0, 0, nchild, UNDEF, UNDEF)
        for i in range(2 * GROUP_INTERNAL_K):
            bt += struct.pack("<Q", keys[i] if i < len(keys) else 0)
            bt += struct.pack("<Q", snods[i] if (i < nchild) else 0)
        bt += struct.pack("<Q", keys[nchild] if nchild < len(keys) else 0)
        bt_addr = self.alloc(bt)
        msgs = [_message(0x0011, struct.pack("<QQ", bt_addr, heap_addr))]
        msgs += [_attribute_message(k, v, self) for k, v in g.attrs.items()]
        return self.object_header(msgs), bt_addr, heap_addr


def _max_members(g):
    n = len(g.members)
    for m in g.members.values():
        if isinstance(m, Group):
            n = max(n, _max_members(m))
    return n


def save(path, root):
    """Write a Group tree as an HDF5 file (libhdf5 'earliest' layout, see module docstring)."""
    leaf_k = max(4, -(-_max_members(root) // (4 * GROUP_INTERNAL_K)))
    w = _Writer()
    oh, bt, hp = w.group(root, leaf_k)
    eof = len(w.buf)
    sb = SIGNATURE + struct.pack("<BBBBBBBBHHI", 0, 0, 0, 0, 0, 8, 8, 0, leaf_k,
                                 GROUP_INTERNAL_K, 0)
    sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
    sb += struct.pack("<QQIIQQ", 0, oh, 1, 0, bt, hp)
    assert len(sb) == 96
    w.buf[0:96] = sb
    with open(path, "wb") as f:
        f.write(w.buf)


# ----------------------------------------------------------------------------- decoding
class _Reader(object):
    def __init__(self, raw):
        self.b = raw
        if raw[:8] != SIGNATURE:
            raise ValueError("not an HDF5 file (no superblock at offset 0)")
        ver = raw[8]
        if ver in (0, 1):
            self.so, self.sl = raw[13], raw[14]
            if (self.so, self.sl) != (8, 8):
                raise NotImplementedError("HDF5 reader: 8-byte offsets/lengths only")
            p = 24 + (4 if ver == 1 else 0)
            self.base = self.u64(p)
            p += 32
            self.root = self.u64(p + 8)  # root symbol-table entry: name off, header addr
        elif ver in (2, 3):
            self.so, self.sl = raw[9], raw[10]
            if (self.so, self.sl) != (8, 8):
                raise NotImplementedError("HDF5 reader: 8-byte offsets/lengths only")
            self.base = self.u64(12)
            self.root = self.u64(12 + 24)
        else:
            raise NotImplementedError(f"HDF5 superblock version {ver}")

    def u64(self, p):
        return struct.unpack_from("<Q", self.b, p)[0]

    # -- object headers
    def messages(self, addr):
        b = self.b
        out = []
        if b[addr:addr + 4] == b"OHDR":
            flags = b[addr + 5]
            p = addr + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            szb = 1 << (flags & 3)
            size = int.from_bytes(b[p:p + szb], "little")
            p += szb
            blocks = [(p, p + size)]  # chunk 0's messages (its checksum follows)
            while blocks:
                s, e = blocks.pop(0)
                q = s
                while q + 4 <= e:
                    mt, ms, mf = b[q], struct.unpack_from("<H", b, q + 1)[0], b[q + 3]
                    q += 4 + (2 if flags & 0x04 else 0)
                    body = bytes(b[q:q + ms])
                    q += ms
                    if mt == 0x10:
                        ca, cl = struct.unpack_from("<QQ", body)
                        blocks.append((ca + 4, ca + cl - 4))  # "OCHK" ... checksum
                    elif mt != 0:
                        out.append((mt, body, mf))
            return out
        ver = b[addr]
        if ver != 1:
            raise NotImplementedError(f"object header version {ver}")
        nmsg, _, size = struct.unpack_from("<HII", b, addr + 2)
        blocks = [(addr + 16, addr + 16 + size)]
        seen = 0
        while blocks and seen < nmsg:
            s, e = blocks.pop(0)
            q = s
            while q + 8 <= e and seen < nmsg:
                mt, ms, mf = struct.unpack_from("<HHB", b, q)
                body = bytes(b[q + 8:q + 8 + ms])
                q += 8 + ms
                seen += 1
                if mt == 0x10:
                    ca, cl = struct.unpack_from("<QQ", body)
                    blocks.append((ca, ca + cl))
                elif mt != 0:
                    out.append((mt, body, mf))
        return out

    # -- message bodies
    def dtype(self, m):
        cls, ver = m[0] & 0x0F, m[0] >> 4
        bf0 = m[1]
        size = struct.unpack_from("<I", m, 4)[0]
        if cls == 0:
            bo = ">" if bf0 & 1 else "<"
            return np.dtype(f"{bo}{'i' if bf0 & 0x08 else 'u'}{size}"), 8 + 4
        if cls == 1:
            bo = ">" if bf0 & 1 else "<"
            return np.dtype(f"{bo}f{size}"), 8 + 12
        if cls == 3:
            return np.dtype(f"S{size}"), 8
        if cls == 9:
            base, blen = self.dtype(m[8:])
            return _VLen((bf0 & 0x0F) == 1, base, size), 8 + blen
        raise NotImplementedError(f"HDF5 datatype class {cls} (version {ver})")

    def global_heap_object(self, coll, index):
        b, p = self.b, self.base + coll
        if b[p:p + 4] != b"GCOL":
            raise ValueError("bad global heap collection")
        size = struct.unpack_from("<Q", b, p + 8)[0]
        q, end = p + 16, p + size
        while q + 16 <= end:
            idx, _, osz = struct.unpack_from("<HH4xQ", b, q)
            if idx == index:
                return bytes(b[q + 16:q + 16 + osz])
            if idx == 0:
                break
            q += 16 + osz + (-osz % 8)
        raise ValueError(f"global heap object {index} not found in collection at {coll}")

    def decode_vlen(self, vt, raw, shape):
        """Elements of a class-9 datatype: 16-byte (length, collection, index) records."""
        n = int(np.prod(shape)) if shape else 1
        vals = []
        for i in range(n):
            ln, coll, idx = struct.unpack_from("<IQI", raw, 16 * i)
            if coll in (0, UNDEF) or ln == 0:
                data = b""
            else:
                data = self.global_heap_object(coll, idx)
            if vt.is_str:
                vals.append(data[:ln].split(b"\0")[0].decode("utf8", errors="replace"))
            else:
                vals.append(np.frombuffer(data, vt.base, ln).copy())
        if not shape:
            return vals[0]
        out = np.empty(n, dtype=object)
        out[:] = vals
        return out.reshape(shape)

    @staticmethod
    def dataspace(m):
        ver, rank, flags = m[0], m[1], m[2]
        if ver == 1:
            p = 8
        elif ver == 2:
            p = 4
            if m[3] == 2:  # null dataspace
                return None, 4
        else:
            raise NotImplementedError(f"dataspace version {ver}")
        dims = struct.unpack_from(f"<{rank}Q", m, p)
        p += 8 * rank * (2 if flags & 1 else 1)
        return tuple(int(d) for d in dims), p

    def attribute(self, m):
        ver = m[0]
        if ver == 1:
            nsz, tsz, ssz = struct.unpack_from("<HHH", m, 2)
            p = 8
            name = m[p:p + nsz].split(b"\0")[0].decode()
            p += nsz + (-nsz % 8)
            dt, _ = self.dtype(m[p:p + tsz])
            p += tsz + (-tsz % 8)
            shape, _ = self.dataspace(m[p:p + ssz])
            p += ssz + (-ssz % 8)
        elif ver in (2, 3):
            nsz, tsz, ssz = struct.unpack_from("<HHH", m, 2)
            p = 8 + (1 if ver == 3 else 0)
            name = m[p:p + nsz].split(b"\0")[0].decode()
            p += nsz
            if m[1] & 0x01:
                raise NotImplementedError("shared attribute datatype")
            dt, _ = self.dtype(m[p:p + tsz])
            p += tsz
            shape, _ = self.dataspace(m[p:p + ssz])
            p += ssz
        else:
            raise NotImplementedError(f"attribute message version {ver}")
        if shape is None:
            return name, None
        n = int(np.prod(shape)) if shape else 1
        if isinstance(dt, _VLen):
            return name, self.decode_vlen(dt, m[p:p + 16 * n], shape)
        val = np.frombuffer(m, dt, n, p).reshape(shape).copy()
        return name, val

    def read_data(self, dt, shape, layout):
        if isinstance(dt, _VLen):
            raw = self.read_data(np.dtype("V16"), shape, layout)
            return self.decode_vlen(dt, np.ascontiguousarray(raw).tobytes(), shape)
        n = int(np.prod(shape)) if shape else 1
        ver = layout[0]
        if ver in (1, 2):
            rank, cls = layout[1], layout[2]
            p = 8
            if cls == 0:
                p += 4 * rank
                size = struct.unpack_from("<I", layout, p)[0]
                return np.frombuffer(layout, dt, n, p + 4).reshape(shape).copy()
            if cls != 1:
                raise NotImplementedError("chunked HDF5 dataset")
            addr = struct.unpack_from("<Q", layout, p)[0]
        elif ver in (3, 4):
            cls = layout[1]
            if cls == 0:
                size = struct.unpack_from("<H", layout, 2)[0]
                return np.frombuffer(layout, dt, n, 4).reshape(shape).copy()
            if cls != 1:
                raise NotImplementedError("chunked / virtual HDF5 dataset")
            addr = struct.unpack_from("<Q", layout, 2)[0]
        else:
            raise NotImplementedError(f"layout message version {ver}")
        if addr == UNDEF:
            return np.zeros(shape, dt)
        return np.frombuffer(self.b, dt, n, self.base + addr).reshape(shape).copy()

    # -- objects
    def obj(self, addr):
        msgs = self.messages(addr)
        attrs = {}
        for mt, body, _ in msgs:
            if mt == 0x000C:
                try:
                    k, v = self.attribute(body)
                except NotImplementedError as e:  # keep loading: callers look attrs up by name
                    warnings.warn(f"HDF5 attribute skipped: {e}")
                    continue
                attrs[k] = v
            elif mt == 0x0015 and struct.unpack_from("<Q", body, 2 + (2 if body[1] & 1 else 0))[0] \
                    != UNDEF:
                raise NotImplementedError("dense attribute storage")
        types = {mt for mt, _, _ in msgs}
        if 0x0011 in types or 0x0006 in types or 0x0002 in types:
            g = Group(attrs)
            for mt, body, _ in msgs:
                if mt == 0x0011:
                    bt, hp = struct.unpack_from("<QQ", body)
                    for name, a in self.symbol_table(bt, hp):
                        g.members[name] = self.obj(a)
                elif mt == 0x0006:
                    name, a = self.link(body)
                    if a is not None:
                        g.members[name] = self.obj(a)
                elif mt == 0x0002:
                    fh = struct.unpack_from("<Q", body, 2 + (8 if body[1] & 1 else 0))[0]
                    if fh != UNDEF:
                        raise NotImplementedError("dense link storage (fractal heap)")
            return g
        dt = shape = layout = None
        for mt, body, _ in msgs:
            if mt == 0x0001:
                shape, _ = self.dataspace(body)
            elif mt == 0x0003:
                dt, _ = self.dtype(body)
            elif mt == 0x0008:
                layout = body
            elif mt == 0x000B:
                raise NotImplementedError("filtered (compressed) HDF5 dataset")
        if dt is None or layout is None:
            raise NotImplementedError("HDF5 object is neither a group nor a dataset")
        return Dataset(self.read_data(dt, shape or (), layout), attrs)

    def symbol_table(self, bt, hp):
        b = self.b
        if b[hp:hp + 4] != b"HEAP":
            raise ValueError("bad local heap")
        heap_data = struct.unpack_from("<Q", b, hp + 24)[0]

        def name_at(off):
            s = heap_data + off
            return bytes(b[s:b.index(b"\0", s)]).decode("utf8")

        out = []

        def walk(node):
            if b[node:node + 4] != b"TREE":
                raise ValueError("bad B-tree node")
            ntype, level, used = b[node + 4], b[node + 5], struct.unpack_from("<H", b, node + 6)[0]
            if ntype != 0:
                raise ValueError("not a group B-tree")
            p = node + 24
            for i in range(used):
                child = struct.unpack_from("<Q", b, p + 8 + 16 * i)[0]
                if level > 0:
                    walk(child)
                else:
                    if b[child:child + 4] != b"SNOD":
                        raise ValueError("bad symbol-table node")
                    nsym = struct.unpack_from("<H", b, child + 6)[0]
                    for j in range(nsym):
                        no, oh = struct.unpack_from("<QQ", b, child + 8 + 40 * j)
                        out.append((name_at(no), oh))

        walk(bt)
        return out

    @staticmethod
    def link(m):
        flags = m[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = m[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        nb = 1 << (flags & 3)
        n = int.from_bytes(m[p:p + nb], "little")
        p += nb
        name = m[p:p + n].decode("utf8")
        p += n
        if ltype != 0:
            return name, None  # soft / external links: not followed
        return name, struct.unpack_from("<Q", m, p)[0]


def load(path):
    """Read an HDF5 file into a Group tree (module docstring lists the supported subset)."""
    with open(path, "rb") as f:
        raw = f.read()
    r = _Reader(raw)
    return r.obj(r.root)


def is_hdf5(path):
    try:
        with open(path, "rb") as f:
            return f.read(8) == SIGNATURE
    except OSError:
        return False
