"""Key/value stores with the reference's range-read contract (host byte sources).

Mirrors M/store/Store.java:9-41, StoreHandle.java:20-70, FilesystemStore.java:40-102 and
MemoryStore.java:17-56: `get(keys)` whole value or None; `get(keys, start)` from start
(negative start = suffix); `get(keys, start, end)` = [start, end) with a negative start
counted from the end.
"""
import os
import threading


class Store:
    def exists(self, keys):
        raise NotImplementedError

    def get(self, keys, start=None, end=None):
        raise NotImplementedError

    def set(self, keys, data):
        raise NotImplementedError

    def size(self, keys):
        """Byte length of the key's value, or None when unknown / missing."""
        return None

    def get_into(self, keys, view, start, end):
        """get(keys, start, end) written into `view` (a writable memoryview of end - start
        bytes); returns the bytes written, or None for a missing key.  Stores override it to
        skip the intermediate buffer."""
        b = self.get(keys, start, end)
        if b is None:
            return None
        view[:len(b)] = b
        return len(b)

    def delete(self, keys):
        raise NotImplementedError

    def resolve(self, *keys):
        return StoreHandle(self, *keys)


class FilesystemStore(Store):
    """FilesystemStore.java: one file per key under a root directory."""

    def __init__(self, path):
        self.path = os.path.abspath(str(path))

    def _p(self, keys):
        return os.path.join(self.path, *keys)

    def exists(self, keys):
        return os.path.isfile(self._p(keys))

    def get(self, keys, start=None, end=None):
        p = self._p(keys)
        try:
            with open(p, "rb") as f:
                if start is None:
                    return f.read()
                size = os.fstat(f.fileno()).st_size
                s = start if start >= 0 else size + start
                e = size if end is None else end
                f.seek(s)
                return f.read(e - s)
        except FileNotFoundError:
            return None

    def size(self, keys):
        try:
            return os.stat(self._p(keys)).st_size
        except FileNotFoundError:
            return None

    def get_into(self, keys, view, start, end):
        try:
            with open(self._p(keys), "rb", buffering=0) as f:
                f.seek(start)
                got = 0
                while got < len(view):
                    r = f.readinto(view[got:])
                    if not r:
                        break
                    got += r
                return got
        except FileNotFoundError:
            return None

    def set(self, keys, data):
        p = self._p(keys)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".tmp%d" % threading.get_ident()
        with open(tmp, "wb") as f:
            f.write(bytes(data))
        os.replace(tmp, p)

    def delete(self, keys):
        try:
            os.remove(self._p(keys))
        except FileNotFoundError:
            pass

    def __repr__(self):
        return f"file://{self.path}"


class MemoryStore(Store):
    """MemoryStore.java: a dict of key tuples → bytes.  Unlike the reference (Q8) a
    negative start is served as a suffix read."""

    def __init__(self):
        self.map = {}
        self.lock = threading.Lock()

    def exists(self, keys):
        return tuple(keys) in self.map

    def get(self, keys, start=None, end=None):
        b = self.map.get(tuple(keys))
        if b is None:
            return None
        if start is None:
            return b
        s = start if start >= 0 else len(b) + start
        e = len(b) if end is None else end
        return b[s:e]

    def set(self, keys, data):
        with self.lock:
            self.map[tuple(keys)] = bytes(data)

    def delete(self, keys):
        with self.lock:
            self.map.pop(tuple(keys), None)


class StoreHandle:
    """StoreHandle.java: a store plus a key path."""

    def __init__(self, store, *keys):
        self.store = store
        self.keys = tuple(str(k) for k in keys)

    def resolve(self, *keys):
        return StoreHandle(self.store, *(self.keys + tuple(str(k) for k in keys)))

    def read(self, start=None, end=None):
        return self.store.get(self.keys, start, end)

    def read_into(self, view, start, end):
        return self.store.get_into(self.keys, view, start, end)

    def size(self):
        return self.store.size(self.keys)

    def exists(self):
        return self.store.exists(self.keys)

    def set(self, data):
        self.store.set(self.keys, data)

    def delete(self):
        self.store.delete(self.keys)

    def __repr__(self):
        return f"{self.store!r}/{'/'.join(self.keys)}"
