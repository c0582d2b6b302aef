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
