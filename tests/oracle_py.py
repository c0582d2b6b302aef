"""ctypes access to the C oracle (oracle/ii_oracle.c) — TEST INFRASTRUCTURE ONLY.
The oracle is the parity checker; it is never part of the product path."""
import ctypes
import os

_ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "build",
                       "libii_oracle.so")
_lib = None


def _bytes_at(addr, n):
    # (not ctypes.string_at: it passes the size as a C int, so texts past 2 GiB came back cut)
    return bytes((ctypes.c_char * n).from_address(addr)) if n else b""


def _load():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(_ORACLE)
        _lib.ii_oracle_index.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                         ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
        _lib.ii_oracle_index_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
        _lib.ii_oracle_free.argtypes = [ctypes.c_void_p]
        _lib.ii_oracle_partials.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.c_void_p]
    return _lib


def oracle_index(text, file_off, file_id0, threads=1):
    """-> {letter: bytes} exactly as the reference would write a.txt..z.txt.
    threads > 1: the multithreaded restatement (ii_oracle_index_mt)."""
    import numpy as np
    L = _load()
    if hasattr(text, "ctypes"):
        tb = np.ascontiguousarray(text, dtype=np.uint8)
    else:
        tb = np.frombuffer(bytes(text), dtype=np.uint8)
    off = np.ascontiguousarray(np.asarray(file_off, dtype=np.uint64))
    ids = np.ascontiguousarray(np.asarray(file_id0, dtype=np.uint32))
    out = ctypes.c_void_p()
    loff = (ctypes.c_uint64 * 27)()
    if threads > 1:
        rc = L.ii_oracle_index_mt(tb.ctypes.data if tb.size else None, off.ctypes.data, ids.ctypes.data, len(ids),
                                  threads, ctypes.byref(out), loff)
    else:
        rc = L.ii_oracle_index(tb.ctypes.data if tb.size else None, off.ctypes.data, ids.ctypes.data, len(ids),
                               ctypes.byref(out), loff)
    assert rc == 0
    res = {chr(97 + l): _bytes_at(out.value + loff[l], loff[l + 1] - loff[l]) for l in range(26)}
    L.ii_oracle_free(out)
    return res


def oracle_partials(text, file_off, file_id0, order):
    """-> {letter: bytes} of partial_<letter>.txt when one mapper reads the
    files `order` (indices) one after another (main.c:93-124)."""
    import numpy as np
    L = _load()
    if hasattr(text, "ctypes"):
        tb = np.ascontiguousarray(text, dtype=np.uint8)
    else:
        tb = np.frombuffer(bytes(text), dtype=np.uint8)
    off = np.ascontiguousarray(np.asarray(file_off, dtype=np.uint64))
    ids = np.ascontiguousarray(np.asarray(file_id0, dtype=np.uint32))
    od = np.ascontiguousarray(np.asarray(list(order), dtype=np.uint32))
    out = ctypes.c_void_p()
    loff = (ctypes.c_uint64 * 27)()
    rc = L.ii_oracle_partials(tb.ctypes.data if tb.size else None, off.ctypes.data, ids.ctypes.data, len(ids),
                              od.ctypes.data if od.size else None, len(od), ctypes.byref(out), loff)
    assert rc == 0
    res = {chr(97 + l): _bytes_at(out.value + loff[l], loff[l + 1] - loff[l]) for l in range(26)}
    L.ii_oracle_free(out)
    return res


class OracleStream:
    """The streaming, letter-range oracle (ii_oracle_stream_*): batches of
    files in ascending id order, only words whose first letter is in [lo, hi)
    kept — for corpora too large for one in-memory call (configs[4])."""

    def __init__(self, lo, hi):
        L = _load()
        L.ii_oracle_stream_open.restype = ctypes.c_void_p
        L.ii_oracle_stream_open.argtypes = [ctypes.c_int, ctypes.c_int]
        L.ii_oracle_stream_add.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_int]
        L.ii_oracle_stream_letter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.ii_oracle_stream_close.argtypes = [ctypes.c_void_p]
        self.L, self.lo, self.hi = L, lo, hi
        self.h = L.ii_oracle_stream_open(lo, hi)
        assert self.h

    def add(self, text, file_off, file_id0, threads=8):
        import numpy as np
        tb = np.ascontiguousarray(text, dtype=np.uint8) if hasattr(text, "ctypes") else \
            np.frombuffer(bytes(text), dtype=np.uint8)
        off = np.ascontiguousarray(np.asarray(file_off, dtype=np.uint64))
        ids = np.ascontiguousarray(np.asarray(file_id0, dtype=np.uint32))
        rc = self.L.ii_oracle_stream_add(self.h, tb.ctypes.data if tb.size else None, off.ctypes.data,
                                         ids.ctypes.data if ids.size else None, len(ids), threads)
        assert rc == 0, "ids must ascend across batches"

    def letter(self, l, consume):
        """Order + format letter l; consume(memoryview of its text) is called
        on the text in place; returns (bytes, lines)."""
        out = ctypes.c_void_p()
        n = ctypes.c_uint64()
        words = ctypes.c_uint64()
        assert self.L.ii_oracle_stream_letter(self.h, l, ctypes.byref(out), ctypes.byref(n), ctypes.byref(words)) == 0
        try:
            if n.value:
                consume(memoryview((ctypes.c_char * n.value).from_address(out.value)).cast("B"))
            else:
                consume(memoryview(b""))
        finally:
            self.L.ii_oracle_free(out)
        return n.value, words.value

    def close(self):
        if self.h:
            self.L.ii_oracle_stream_close(self.h)
            self.h = None
