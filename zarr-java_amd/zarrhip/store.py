"""Key/value stores with the reference's range-read contract (host byte sources).

Mirrors M/store/Store.java:9-41, StoreHandle.java:20-70, FilesystemStore.java:40-102,
MemoryStore.java:17-56 and HttpStore.java:13-232: `get(keys)` whole value or None;
`get(keys, start)` from start (negative start = suffix); `get(keys, start, end)` = [start, end)
with a negative start counted from the end (HttpStore: rejected, as in the reference).
"""
import os
import threading
import time
import urllib.error
import urllib.parse
import urllib.request


class StoreException(RuntimeError):
    """M/store/StoreException.java:17-43: `readFailed` / `writeFailed` / `deleteFailed` wrap the
    cause's message with the store and the '/'-joined key (the library's zh_array_read_files /
    zh_array_write_files raise the same text)."""

    @staticmethod
    def read_failed(store_path, keys, cause):
        return StoreException("Failed to read from store '%s' at key '%s': %s"
                              % (store_path, "/".join(keys), cause))

    @staticmethod
    def write_failed(store_path, keys, cause):
        return StoreException("Failed to write to store '%s' at key '%s': %s"
                              % (store_path, "/".join(keys), cause))

    @staticmethod
    def delete_failed(store_path, keys, cause):
        return StoreException("Failed to delete from store '%s' at key '%s': %s"
                              % (store_path, "/".join(keys), cause))


def _io_cause(path, e):
    """IOException.getMessage() of a failed file operation as the JDK words it (UnixException:
    AccessDeniedException carries just the file; other errors "file: reason")."""
    import errno
    if e.errno in (errno.EACCES, errno.EPERM):
        return path
    return "%s: %s" % (path, e.strerror or e)


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
        """get(keys) / get(keys, start) / get(keys, start, end) (FilesystemStore.java:47-102):
        a negative start counts from the end (a resolved start below 0 raises, as the
        channel's position(< 0) does); a [start, end) read returns end - start bytes, zeros
        past the end of the file (the reference allocates the buffer and reads what the file
        has)."""
        p = self._p(keys)
        try:
            with open(p, "rb") as f:
                if start is None:
                    return f.read()
                size = os.fstat(f.fileno()).st_size
                s = start if start >= 0 else size + start
                if s < 0:
                    raise ValueError("newPosition < 0: (%d < 0)" % s)
                e = size if end is None else end
                f.seek(s)
                b = f.read(max(0, e - s))
                return b + bytes(max(0, e - s - len(b))) if end is not None else b
        except FileNotFoundError:
            return None
        except IsADirectoryError as err:  # exists() is false for it: read as a failed read
            raise StoreException.read_failed(repr(self), keys, _io_cause(p, err)) from None
        except PermissionError as err:
            raise StoreException.read_failed(repr(self), keys, _io_cause(p, err)) from None

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
                    if not r:  # the end of the file: the rest of [start, end) reads as zeros
                        view[got:] = bytes(len(view) - got)
                        break
                    got += r
                return len(view)
        except FileNotFoundError:
            return None
        except PermissionError as err:
            raise StoreException.read_failed(repr(self), keys,
                                             _io_cause(self._p(keys), err)) from None

    def set(self, keys, data):
        """FilesystemStore.set (:105-128): the parent directories, then the bytes — through a
        temporary file renamed into place, as the library writes."""
        p = self._p(keys)
        parent = os.path.dirname(p)
        try:
            os.makedirs(parent, exist_ok=True)
        except OSError:
            raise StoreException.write_failed(
                repr(self), keys, "Failed to create parent directories for path: " + parent) \
                from None
        tmp = p + ".tmp%d" % threading.get_ident()
        b = bytes(data)
        try:
            with open(tmp, "wb") as f:
                f.write(b)
            os.replace(tmp, p)
        except OSError:
            try:
                os.remove(tmp)
            except OSError:
                pass
            raise StoreException.write_failed(
                repr(self), keys, "Failed to write %d bytes to file: %s" % (len(b), p)) from None

    def delete(self, keys):
        p = self._p(keys)
        try:
            os.remove(p)
        except FileNotFoundError:
            pass
        except OSError:
            raise StoreException.delete_failed(repr(self), keys,
                                               "Failed to delete file: " + p) from None

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


class HttpStore(Store):
    """HttpStore.java: read-only HTTP(S) store.  Keys are appended as path segments
    (`resolveKeys`, :34-45); ranges go out as `Range` headers (:79-98: `bytes=s-`,
    `bytes=-n` suffix, `bytes=s-(e-1)`); 404 → None, other failures raise StoreException
    (`readFailed`); 502/503/504-style 5xx responses and I/O errors are retried
    `max_retries` times `retry_delay_ms` apart (RetryInterceptor, :200-231); `size` is a
    HEAD Content-Length with identity encoding (:166-196, -1 → None here)."""

    def __init__(self, uri, timeout_seconds=60, max_retries=3, retry_delay_ms=1000):
        if not urllib.parse.urlparse(uri).scheme.startswith("http"):
            raise ValueError("Invalid base URI: " + uri)
        self.uri = uri
        self.timeout = timeout_seconds
        self.max_retries = max_retries
        self.delay = retry_delay_ms / 1000.0

    def _url(self, keys):
        segs = [urllib.parse.quote(seg, safe="") for k in keys for seg in str(k).split("/")]
        return self.uri.rstrip("/") + "/" + "/".join(segs)

    def _open(self, req):
        """RetryInterceptor: the response, or None for 404; raises HTTPError / OSError."""
        last = None
        for i in range(self.max_retries + 1):
            if i:
                time.sleep(self.delay)
            try:
                return urllib.request.urlopen(req, timeout=self.timeout)
            except urllib.error.HTTPError as e:
                if e.code == 404:
                    return None
                if e.code < 500 or i == self.max_retries:
                    raise
                last = e
            except OSError as e:
                last = e
                if i == self.max_retries:
                    raise
        raise last if last else OSError("Request failed after retries")

    def _get(self, keys, headers):
        req = urllib.request.Request(self._url(keys), headers=headers)
        try:
            r = self._open(req)
            if r is None:
                return None
            with r:
                return r.read()
        except urllib.error.HTTPError as e:
            raise StoreException.read_failed(
                self.uri, keys, "HTTP request failed with status code: %d %s" % (e.code, e.reason)) from None
        except OSError as e:
            raise StoreException.read_failed(self.uri, keys, e) from None

    def exists(self, keys):
        try:
            r = self._open(urllib.request.Request(self._url(keys), method="HEAD"))
        except OSError:
            return False
        if r is None:
            return False
        with r:
            return 200 <= r.status < 300

    def get(self, keys, start=None, end=None):
        if start is None:
            return self._get(keys, {})
        if end is None:
            rng = "bytes=%d" % start if start < 0 else "bytes=%d-" % start
            return self._get(keys, {"Range": rng})
        if start < 0:
            raise ValueError("Argument 'start' needs to be non-negative.")
        return self._get(keys, {"Range": "bytes=%d-%d" % (start, end - 1)})

    def size(self, keys):
        req = urllib.request.Request(self._url(keys), method="HEAD",
                                     headers={"Accept-Encoding": "identity"})
        try:
            r = self._open(req)
        except urllib.error.HTTPError:
            return None
        except OSError as e:
            raise StoreException.read_failed(
                self.uri, keys, "Failed to get content length from HTTP HEAD request to: "
                + self._url(keys) + " (%s)" % e) from None
        if r is None:
            return None
        with r:
            n = r.headers.get("Content-Length")
        if n is None:
            return None
        try:
            return int(n)
        except ValueError:
            raise StoreException.read_failed(
                self.uri, keys, "Invalid Content-Length header value from: " + self._url(keys)) from None

    def set(self, keys, data):
        raise NotImplementedError("Not implemented")

    def delete(self, keys):
        raise NotImplementedError("Not implemented")

    def __repr__(self):
        return self.uri


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
