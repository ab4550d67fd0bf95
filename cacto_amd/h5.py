"""Keras-2.11 `.h5` weight checkpoints, read and written natively (no h5py) — SURVEY §8f.3.

The reference saves and restores its three networks with Keras `save_weights` / `load_weights`
on `.h5` files (RL.py:191-195 `RL_save_weights`, main.py:154-158 / RL.py:52-62 recover_training).
This module reads those files and writes files Keras can load, so runs can resume from the
reference's checkpoints and hand weights back to it.

Keras layout (`save_weights` to HDF5): root attributes `layer_names` (fixed-length byte strings),
`backend`, `keras_version`; one group per layer with attribute `weight_names` (e.g.
b"dense/kernel:0"); each weight a float32 dataset at `<layer>/<weight_name>`, kernels [in, out].
`load_weights` matches layers that have weights in topological order (names need not agree).

HDF5 subset (File Format Specification, the structures h5py writes with libver="earliest"):
superblock v0/v1 (v2/v3 read too); object headers v1 and v2 with continuation blocks; old-style
groups (symbol-table message -> v1 B-tree of group nodes -> symbol-table nodes, names in a local
heap) and compact new-style groups (link messages); simple dataspaces; IEEE-float, integer and
fixed-length string datatypes; contiguous and compact layouts; attribute messages v1-v3. Chunked
or filtered datasets and dense link storage are rejected with an error (Keras does not write them).
Writing produces the same v0-superblock / v1-header / symbol-table structure.
"""
import struct

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF

MSG_DATASPACE, MSG_LINK_INFO, MSG_DATATYPE, MSG_FILL_OLD, MSG_FILL = 0x01, 0x02, 0x03, 0x04, 0x05
MSG_LINK, MSG_LAYOUT, MSG_GROUP_INFO, MSG_FILTERS, MSG_ATTRIBUTE = 0x06, 0x08, 0x0A, 0x0B, 0x0C
MSG_CONTINUATION, MSG_SYMBOL_TABLE = 0x10, 0x11


class H5Error(ValueError):
    pass


def _pad8(n):
    return (n + 7) & ~7


# ---------------------------------------------------------------------------------------- reading
class _Object:
    def __init__(self, messages):
        self.messages = messages        # [(type, bytes)]

    def first(self, mtype):
        for t, d in self.messages:
            if t == mtype:
                return d
        return None

    def all(self, mtype):
        return [d for t, d in self.messages if t == mtype]


class H5File:
    """Read-only view of an HDF5 file held in memory."""

    def __init__(self, data):
        self.d = bytes(data)
        base = None
        for off in [0] + [512 << k for k in range(20)]:
            if off + 8 <= len(self.d) and self.d[off:off + 8] == SIGNATURE:
                base = off
                break
        if base is None:
            raise H5Error("not an HDF5 file (no signature)")
        d = self.d
        ver = d[base + 8]
        if ver in (0, 1):
            self.O, self.L = d[base + 13], d[base + 14]
            p = base + 24 + (4 if ver == 1 else 0)
            self.base = self._u(p, self.O)
            p += 4 * self.O                                # base, free space, EOF, driver info
            self.root = self._u(p + self.O, self.O)        # root symbol-table entry: header address
        elif ver in (2, 3):
            self.O, self.L = d[base + 9], d[base + 10]
            p = base + 12
            self.base = self._u(p, self.O)
            self.root = self._u(p + 3 * self.O, self.O)
        else:
            raise H5Error("unsupported superblock version %d" % ver)
        if self.O != 8 or self.L != 8:
            raise H5Error("only 8-byte offsets and lengths are supported")

    # -- primitives
    def _u(self, p, n):
        return int.from_bytes(self.d[p:p + n], "little")

    def _addr(self, a):
        return self.base + a

    # -- object headers
    def object(self, addr):
        p = self._addr(addr)
        d = self.d
        msgs = []
        if d[p:p + 4] == b"OHDR":
            flags = d[p + 5]
            q = p + 6 + (16 if flags & 0x20 else 0) + (4 if flags & 0x10 else 0)
            sz = 1 << (flags & 3)
            n = self._u(q, sz)
            q += sz
            chunks = [(q, n)]
            while chunks:
                s, n = chunks.pop(0)
                end = s + n
                while s + 4 <= end - 4:                       # 4-byte checksum closes each chunk
                    t, size, mflags = d[s], self._u(s + 1, 2), d[s + 3]
                    s += 4 + (2 if flags & 0x04 else 0)
                    body = d[s:s + size]
                    s += size
                    if t == MSG_CONTINUATION:
                        a, ln = self._u(s - size, 8), self._u(s - size + 8, 8)
                        chunks.append((self._addr(a) + 4, ln - 4))   # skip "OCHK"
                    elif t:
                        msgs.append((t, body))
            return _Object(msgs)
        if d[p] != 1:
            raise H5Error("unsupported object header version %d" % d[p])
        nmsg, hsize = self._u(p + 2, 2), self._u(p + 8, 4)
        chunks = [(p + 16, hsize)]
        while chunks and len(msgs) < nmsg:
            s, n = chunks.pop(0)
            end = s + n
            while s + 8 <= end:
                t, size = self._u(s, 2), self._u(s + 2, 2)
                body = d[s + 8:s + 8 + size]
                s += 8 + size
                if t == MSG_CONTINUATION:
                    chunks.append((self._addr(self._u(s - size, 8)), self._u(s - size + 8, 8)))
                elif t:
                    msgs.append((t, body))
        return _Object(msgs)

    # -- groups
    def _local_heap(self, addr):
        p = self._addr(addr)
        if self.d[p:p + 4] != b"HEAP":
            raise H5Error("bad local heap")
        return self._addr(self._u(p + 24, 8))              # data segment address

    def _heap_str(self, seg, off):
        e = self.d.index(b"\0", seg + off)
        return self.d[seg + off:e].decode()

    def _btree_group(self, addr, heap, out):
        p = self._addr(addr)
        d = self.d
        if d[p:p + 4] != b"TREE" or d[p + 4] != 0:
            raise H5Error("bad group B-tree node")
        level, used = d[p + 5], self._u(p + 6, 2)
        q = p + 24
        for i in range(used):
            child = self._u(q + 8, 8)
            q += 16
            if level > 0:
                self._btree_group(child, heap, out)
                continue
            s = self._addr(child)
            if d[s:s + 4] != b"SNOD":
                raise H5Error("bad symbol-table node")
            for k in range(self._u(s + 6, 2)):
                e = s + 8 + 40 * k
                out[self._heap_str(heap, self._u(e, 8))] = self._u(e + 8, 8)

    def links(self, obj):
        """name -> object header address of a group's members."""
        out = {}
        st = obj.first(MSG_SYMBOL_TABLE)
        if st is not None:
            self._btree_group(self._u_b(st, 0, 8), self._local_heap(self._u_b(st, 8, 8)), out)
            return out
        li = obj.first(MSG_LINK_INFO)
        if li is not None:
            fh = self._u_b(li, 2 + (8 if li[1] & 1 else 0), 8)
            if fh != UNDEF:
                raise H5Error("dense link storage (fractal heap) is not supported")
        for m in obj.all(MSG_LINK):
            flags = m[1]
            q = 2
            ltype = 0
            if flags & 0x08:
                ltype = m[q]
                q += 1
            if flags & 0x04:
                q += 8
            if flags & 0x10:
                q += 1
            ls = 1 << (flags & 3)
            n = int.from_bytes(m[q:q + ls], "little")
            q += ls
            name = m[q:q + n].decode()
            q += n
            if ltype == 0:
                out[name] = int.from_bytes(m[q:q + 8], "little")
        return out

    @staticmethod
    def _u_b(b, p, n):
        return int.from_bytes(b[p:p + n], "little")

    # -- datatypes / dataspaces / data
    @staticmethod
    def dtype(dt):
        cls, size = dt[0] & 0x0F, int.from_bytes(dt[4:8], "little")
        order = ">" if dt[1] & 1 else "<"
        if cls == 1:
            return np.dtype(order + "f%d" % size)
        if cls == 0:
            return np.dtype(order + ("i%d" if dt[1] & 0x08 else "u%d") % size)
        if cls == 3:
            return np.dtype("S%d" % size)
        if cls == 9 and (dt[1] & 0x0F) == 1:
            return "vlen-str"                               # h5py's str attributes
        raise H5Error("unsupported datatype class %d" % cls)

    def _global_heap_object(self, addr, index):
        p = self._addr(addr)
        if self.d[p:p + 4] != b"GCOL":
            raise H5Error("bad global heap collection")
        end = p + self._u(p + 8, 8)
        q = p + 16
        while q + 16 <= end:
            k, size = self._u(q, 2), self._u(q + 8, 8)
            if k == 0:
                break
            if k == index:
                return self.d[q + 16:q + 16 + size]
            q += 16 + _pad8(size)
        raise H5Error("global heap object %d not found" % index)

    @staticmethod
    def shape(ds):
        ver, rank = ds[0], ds[1]
        if ver == 2 and ds[3] == 2:
            return None                                     # null dataspace
        q = 8 if ver == 1 else 4
        return tuple(int.from_bytes(ds[q + 8 * i:q + 8 * i + 8], "little") for i in range(rank))

    def attributes(self, obj):
        out = {}
        for a in obj.all(MSG_ATTRIBUTE):
            ver = a[0]
            nsz, dsz, ssz = (int.from_bytes(a[k:k + 2], "little") for k in (2, 4, 6))
            if ver == 1:
                q = 8
                name = a[q:q + nsz].rstrip(b"\0").decode()
                q += _pad8(nsz)
                dt = a[q:q + dsz]
                q += _pad8(dsz)
                ds = a[q:q + ssz]
                q += _pad8(ssz)
            else:
                q = 8 + (1 if ver == 3 else 0)
                name = a[q:q + nsz].rstrip(b"\0").decode()
                q += nsz
                dt = a[q:q + dsz]
                q += dsz
                ds = a[q:q + ssz]
                q += ssz
            dtype = self.dtype(dt)
            shp = self.shape(ds)
            n = int(np.prod(shp)) if shp else 1
            if isinstance(dtype, str):                      # variable-length strings in the global heap
                vals = [self._global_heap_object(self._u_b(a, q + 16 * i + 4, 8), self._u_b(a, q + 16 * i + 12, 4))
                        for i in range(0 if shp is None else n)]
                out[name] = vals[0] if shp == () else np.array(vals, dtype=object).reshape(shp or (0,))
                continue
            if shp is None:
                out[name] = np.zeros(0, dtype=dtype)
                continue
            out[name] = np.frombuffer(a[q:q + n * dtype.itemsize], dtype=dtype).reshape(shp).copy()
        return out

    def dataset(self, obj):
        if obj.first(MSG_FILTERS) is not None:
            raise H5Error("filtered datasets are not supported")
        dtype = self.dtype(obj.first(MSG_DATATYPE))
        shp = self.shape(obj.first(MSG_DATASPACE))
        lay = obj.first(MSG_LAYOUT)
        n = int(np.prod(shp)) if shp else 1
        nbytes = n * dtype.itemsize
        if lay[0] == 3:
            cls = lay[1]
            if cls == 0:
                raw = lay[4:4 + nbytes]
            elif cls == 1:
                a = self._u_b(lay, 2, 8)
                raw = b"" if a == UNDEF else self.d[self._addr(a):self._addr(a) + nbytes]
            else:
                raise H5Error("chunked datasets are not supported")
        elif lay[0] in (1, 2) and lay[2] == 1:
            a = self._u_b(lay, 8, 8)
            raw = self.d[self._addr(a):self._addr(a) + nbytes]
        else:
            raise H5Error("unsupported data layout")
        if len(raw) < nbytes:                               # never written: fill value 0
            raw = bytes(nbytes)
        return np.frombuffer(raw, dtype=dtype).reshape(shp).copy()

    def get(self, path):
        obj = self.object(self.root)
        for part in [p for p in path.split("/") if p]:
            ln = self.links(obj)
            if part not in ln:
                raise KeyError(path)
            obj = self.object(ln[part])
        return obj


def _strings(a):
    return [x.decode() if isinstance(x, bytes) else str(x) for x in np.asarray(a).reshape(-1)]


def read_keras_weights(path):
    """Weights of a Keras `save_weights` .h5 file in `model.get_weights()` order (layers with
    weights in `layer_names` order, each layer's `weight_names` order): a list of numpy arrays."""
    with open(path, "rb") as f:
        h = H5File(f.read())
    root = h.object(h.root)
    attrs = h.attributes(root)
    if "layer_names" not in attrs:
        raise H5Error("%s: no Keras layer_names attribute" % path)
    out = []
    for lname in _strings(attrs["layer_names"]):
        g = h.get(lname)
        wn = h.attributes(g).get("weight_names")
        if wn is None or len(wn) == 0:
            continue
        for w in _strings(wn):
            out.append(h.dataset(h.get(lname + "/" + w)))
    return out


# ---------------------------------------------------------------------------------------- writing
LEAF_K, INTERNAL_K = 16, 16


class _Writer:
    def __init__(self):
        self.buf = bytearray(96)                            # superblock v0, filled last

    def alloc(self, data):
        a = len(self.buf)
        self.buf += data
        self.buf += bytes(_pad8(len(data)) - len(data))
        return a

    @staticmethod
    def message(mtype, body):
        body = body + bytes(_pad8(len(body)) - len(body))
        return struct.pack("<HHB3x", mtype, len(body), 0) + body

    def header(self, messages):
        body = b"".join(messages)
        return self.alloc(struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(body)) + body)

    @staticmethod
    def dataspace(shape):
        return struct.pack("<BBBB4x", 1, len(shape), 0, 0) + b"".join(struct.pack("<Q", n) for n in shape)

    @staticmethod
    def datatype(dtype):
        dtype = np.dtype(dtype)
        if dtype.kind == "f":
            if dtype.itemsize == 4:
                props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            else:
                props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            sign = 8 * dtype.itemsize - 1
            return struct.pack("<BBBBI", 0x11, 0x20, sign, 0, dtype.itemsize) + props
        if dtype.kind == "S":
            return struct.pack("<BBBBI", 0x13, 0x01, 0, 0, dtype.itemsize)    # null-padded ASCII
        raise H5Error("cannot write dtype %s" % dtype)

    def attribute(self, name, value):
        value = np.asarray(value)
        if value.dtype.kind == "U":
            value = value.astype("S")
        nm = name.encode() + b"\0"
        dt = self.datatype(value.dtype)
        ds = self.dataspace(value.shape)
        body = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds))
        for part in (nm, dt, ds):
            body += part + bytes(_pad8(len(part)) - len(part))
        body += np.ascontiguousarray(value).tobytes()
        return self.message(MSG_ATTRIBUTE, body)

    def dataset(self, array, attrs=()):
        array = np.ascontiguousarray(array)
        data_addr = self.alloc(array.tobytes())
        layout = struct.pack("<BBQQ", 3, 1, data_addr, array.nbytes)
        fill = struct.pack("<BBBB", 2, 2, 2, 0)             # late allocation, write if set, undefined
        msgs = [self.message(MSG_DATASPACE, self.dataspace(array.shape)),
                self.message(MSG_DATATYPE, self.datatype(array.dtype)),
                self.message(MSG_FILL, fill), self.message(MSG_LAYOUT, layout)]
        msgs += [self.attribute(k, v) for k, v in attrs]
        return self.header(msgs)

    def group(self, members, attrs=()):
        """members: {name: object header address}. One symbol-table node under a one-entry B-tree."""
        names = sorted(members, key=lambda s: s.encode())
        if len(names) > 2 * LEAF_K:
            raise H5Error("too many members in one group (%d)" % len(names))
        heap = bytearray(8)                                  # offset 0: the empty string
        offs = {}
        for n in names:
            offs[n] = len(heap)
            b = n.encode() + b"\0"
            heap += b + bytes(_pad8(len(b)) - len(b))
        heap_data = self.alloc(bytes(heap))
        # free-list head 1 = "no free block" (offsets are 8-aligned, so 1 is never one)
        heap_hdr = self.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), 1, heap_data))
        snod = bytearray(b"SNOD" + struct.pack("<BBH", 1, 0, len(names)))
        for n in names:
            snod += struct.pack("<QQII16x", offs[n], members[n], 0, 0)
        snod += bytes(8 + 40 * 2 * LEAF_K - len(snod))
        snod_addr = self.alloc(bytes(snod))
        tree = bytearray(b"TREE" + struct.pack("<BBHQQ", 0, 0, 1 if names else 0, UNDEF, UNDEF))
        if names:
            tree += struct.pack("<QQQ", 0, snod_addr, offs[names[-1]])
        tree += bytes(24 + (2 * INTERNAL_K + 1) * 8 + 2 * INTERNAL_K * 8 - len(tree))
        tree_addr = self.alloc(bytes(tree))
        msgs = [self.message(MSG_SYMBOL_TABLE, struct.pack("<QQ", tree_addr, heap_hdr))]
        msgs += [self.attribute(k, v) for k, v in attrs]
        return self.header(msgs), tree_addr, heap_hdr

    def finish(self, root, tree, heap):
        sb = SIGNATURE + struct.pack("<BBBBBBBBHHI", 0, 0, 0, 0, 0, 8, 8, 0, LEAF_K, INTERNAL_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, len(self.buf), UNDEF)
        sb += struct.pack("<QQII", 0, root, 1, 0) + struct.pack("<QQ", tree, heap)
        assert len(sb) == 96
        self.buf[:96] = sb
        return bytes(self.buf)


def write_keras_weights(path, layers, keras_version="2.11.0", backend="tensorflow"):
    """Write a Keras `save_weights`-layout .h5 file. layers: [(layer_name, [(weight_name,
    array)])], e.g. ("dense", [("dense/kernel:0", W), ("dense/bias:0", b)])."""
    w = _Writer()
    top = {}
    for lname, weights in layers:
        sub = {}
        for wname, arr in weights:
            parts = wname.split("/")
            if len(parts) != 2 or parts[0] != lname:
                raise H5Error("weight name %r must be '<layer>/<name>'" % wname)
            sub[parts[1]] = w.dataset(np.asarray(arr))
        inner = w.group(sub)[0]
        top[lname] = w.group({lname: inner},
                             attrs=[("weight_names", np.array([n.encode() for n, _ in weights]))])[0]
    root, tree, heap = w.group(top, attrs=[("backend", np.array(backend.encode())),
                                           ("keras_version", np.array(keras_version.encode())),
                                           ("layer_names", np.array([n.encode() for n, _ in layers]))])
    with open(path, "wb") as f:
        f.write(w.finish(root, tree, heap))
