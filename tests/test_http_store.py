"""HttpStore (M/store/HttpStore.java) against a loopback HTTP server with Range support:
the StoreTest range semantics (StoreTest.java:83-107), 404 → None, retries on 5xx
(RetryInterceptor), the readFailed message, and a sub-shard read staged over HTTP ranges
(StoreHandleDataProvider, ShardingIndexedCodec.java:333-357) decoding to the oracle's bytes."""
import http.server
import os
import re
import threading

import numpy as np
import pytest

import zarrhip as z


class _Handler(http.server.BaseHTTPRequestHandler):
    root = None
    flaky = {}        # path → number of 503 answers still to give
    requests = []     # (method, path, Range header)

    def log_message(self, *a):
        pass

    def _file(self):
        p = os.path.join(self.root, *self.path.lstrip("/").split("/"))
        return p if os.path.isfile(p) else None

    def _fail_first(self):
        n = self.flaky.get(self.path, 0)
        if n:
            self.flaky[self.path] = n - 1 if n > 0 else n
            self.send_response(503)
            self.send_header("Content-Length", "0")
            self.end_headers()
            return True
        return False

    def do_HEAD(self):
        self.requests.append(("HEAD", self.path, None))
        p = self._file()
        if p is None:
            self.send_response(404)
            self.send_header("Content-Length", "0")
            self.end_headers()
            return
        self.send_response(200)
        self.send_header("Content-Length", str(os.path.getsize(p)))
        self.end_headers()

    def do_GET(self):
        rng = self.headers.get("Range")
        self.requests.append(("GET", self.path, rng))
        if self._fail_first():
            return
        p = self._file()
        if p is None:
            self.send_response(404)
            self.send_header("Content-Length", "0")
            self.end_headers()
            return
        data = open(p, "rb").read()
        code = 200
        if rng:
            m = re.fullmatch(r"bytes=(\d*)-(\d*)", rng)
            s, e = m.group(1), m.group(2)
            if s == "":                      # suffix: bytes=-n
                s, e = max(0, len(data) - int(e)), len(data) - 1
            else:
                s, e = int(s), (int(e) if e else len(data) - 1)
            data = data[s:e + 1]
            code = 206
        self.send_response(code)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)


@pytest.fixture
def server(tmp_path):
    _Handler.root = str(tmp_path)
    _Handler.flaky = {}
    _Handler.requests = []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield tmp_path, f"http://127.0.0.1:{srv.server_address[1]}/"
    srv.shutdown()
    srv.server_close()


def test_http_store_range_reads(server):
    root, url = server
    data = bytes(range(100))
    z.FilesystemStore(root).resolve("a", "b").set(data)
    h = z.HttpStore(url, retry_delay_ms=1).resolve("a", "b")
    assert h.exists() and h.read() == data
    assert h.read(5, 15) == data[5:15]
    assert h.read(len(data) - 10) == data[-10:]
    assert h.read(-10) == data[-10:]
    assert h.size() == 100
    ranges = [r for m, p, r in _Handler.requests if m == "GET"]
    assert ranges == [None, "bytes=5-14", "bytes=90-", "bytes=-10"]
    missing = z.HttpStore(url).resolve("a", "nope")
    assert missing.read() is None and not missing.exists() and missing.size() is None
    with pytest.raises(ValueError, match="Argument 'start' needs to be non-negative."):
        h.read(-10, 5)
    with pytest.raises(NotImplementedError):
        h.set(b"x")
    with pytest.raises(NotImplementedError):
        h.delete()
    with pytest.raises(ValueError, match="Invalid base URI"):
        z.HttpStore("not a url")


def test_http_store_retries_then_fails(server):
    root, url = server
    z.FilesystemStore(root).resolve("k").set(b"payload")
    _Handler.flaky["/k"] = 2                     # two 503s, then the data
    assert z.HttpStore(url, max_retries=3, retry_delay_ms=1).resolve("k").read() == b"payload"
    _Handler.flaky["/k"] = -1                    # 503 forever
    with pytest.raises(z.StoreException) as e:
        z.HttpStore(url, max_retries=2, retry_delay_ms=1).resolve("k").read()
    assert str(e.value) == (f"Failed to read from store '{url}' at key 'k': "
                            "HTTP request failed with status code: 503 Service Unavailable")
    assert sum(1 for m, p, _ in _Handler.requests if p == "/k" and m == "GET") == 3 + 3


@pytest.mark.parametrize("loc", ["start", "end"])
def test_http_partial_staging(server, loc):
    """A sub-shard part read over HTTP stages the index (one suffix/prefix range) and the
    referenced inner-chunk runs (range reads) only, and decodes (oracle) to the region."""
    import oracle as O
    from helpers import encode_oracle, shard_from_pieces
    root, url = server
    m = (z.ArrayMetadataBuilder().withShape(32, 32, 16).withDataType(z.DataType.UINT32)
         .withChunkShape(32, 32, 16)
         .withCodecs(lambda c: c.withSharding([4, 4, 4], lambda i: i.withBytes("BIG"), loc))
         .build())
    a = z.Array.create(z.FilesystemStore(root).resolve("p"), m)
    data = np.random.default_rng(7).integers(0, 2 ** 32, (32, 32, 16), dtype=np.uint32)
    data[:8, :8, :8] = 0
    shard = encode_oracle(a.zmeta, data)[0]
    a._handle((0, 0, 0)).set(shard)
    b = z.Array.open(z.HttpStore(url).resolve("p"))
    lo, hi = [3, 5, 2], [13, 11, 9]
    _Handler.requests.clear()
    b.staged_bytes = 0
    lease = []
    ss, keep = b._stage_shard(b._handle((0, 0, 0)), lo, hi, lease)
    compact = shard_from_pieces(b.zmeta, ss)
    assert b.staged_bytes < len(shard) / 4
    gets = [r for mth, p, r in _Handler.requests if mth == "GET"]
    assert all(r is not None for r in gets)     # ranges only, never the whole shard
    off, shp = lo, [h - l for l, h in zip(lo, hi)]
    got = np.frombuffer(O.array_read(b.zmeta, [compact], off, shp), np.uint32).reshape(shp)
    np.testing.assert_array_equal(got, data[3:13, 5:11, 2:9])


@pytest.mark.gpu
def test_http_array_read_on_device(server):
    """Array.read through HttpStore on the device: whole-shard reads (parallel range pieces
    when the size is known) and sub-shard parts (index + referenced ranges), both orders."""
    root, url = server
    m = (z.ArrayMetadataBuilder().withShape(40, 48, 64).withDataType(z.DataType.UINT32)
         .withChunkShape(16, 16, 32)
         .withCodecs(lambda c: c.withSharding(
             [8, 8, 16], lambda i: i.withTranspose([2, 1, 0]).withBytes("BIG")))
         .build())
    a = z.Array.create(z.FilesystemStore(root).resolve("q"), m)
    data = np.random.default_rng(9).integers(0, 2 ** 32, (40, 48, 64), dtype=np.uint32)
    a.write([0, 0, 0], data)
    b = z.Array.open(z.HttpStore(url).resolve("q"))
    np.testing.assert_array_equal(b.read(), data)
    np.testing.assert_array_equal(b.read([3, 5, 7], [30, 20, 40]), data[3:33, 5:25, 7:47])
