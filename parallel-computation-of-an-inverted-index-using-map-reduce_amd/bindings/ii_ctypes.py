"""ctypes binding of libii.so (include/ii.h) and libiigen.so.

This is the Python-side caller of the C ABI — the same binding a maintainer
of the reference would add to drive the MI355X path from a script (see
INTEGRATION.md).  It loads the in-tree libraries and raises if they are
missing: there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALPHABET = 26

II_OK = 0
ERRORS = {
    -1: "II_ERR_ARG", -2: "II_ERR_HIP", -3: "II_ERR_NOMEM", -4: "II_ERR_IO", -5: "II_ERR_STATE",
    -6: "II_ERR_LAYOUT", -7: "II_ERR_INTERNAL", -8: "II_ERR_NODEV",
}


class IIError(RuntimeError):
    def __init__(self, code, what):
        super().__init__("%s failed: %s (%d)" % (what, ERRORS.get(code, "?"), code))
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [
        ("bytes", ctypes.c_uint64), ("tokens", ctypes.c_uint64), ("pairs", ctypes.c_uint64),
        ("words", ctypes.c_uint64), ("long_tokens", ctypes.c_uint64), ("out_bytes", ctypes.c_uint64),
        ("table_cap", ctypes.c_uint64), ("retries", ctypes.c_uint32), ("sort_passes", ctypes.c_uint32),
        ("letter_tokens", ctypes.c_uint64 * ALPHABET),
        ("ms_map", ctypes.c_double), ("ms_dict", ctypes.c_double), ("ms_sort", ctypes.c_double),
        ("ms_reduce", ctypes.c_double), ("ms_order", ctypes.c_double), ("ms_format", ctypes.c_double),
        ("ms_total", ctypes.c_double), ("scatter_ms_avg", ctypes.c_double), ("scatter_bytes", ctypes.c_uint64),
        ("scatter_launches", ctypes.c_uint32), ("sorted_records", ctypes.c_uint64),
        ("emit_ms", ctypes.c_double), ("emit_bytes", ctypes.c_uint64), ("resolve_ms", ctypes.c_double),
        ("resolved_tokens", ctypes.c_uint64),
        ("sort0_ms", ctypes.c_double), ("sort0_bytes", ctypes.c_uint64),
        ("io_ms", ctypes.c_double), ("io_bytes", ctypes.c_uint64),
        ("sort_bytes", ctypes.c_uint64), ("sort_packed", ctypes.c_uint32),
        ("sort_key_bits", ctypes.c_uint32), ("sort_id_bits", ctypes.c_uint32),
        ("pair_bytes", ctypes.c_uint32), ("deep_probe", ctypes.c_uint32),
    ]

    def as_dict(self):
        d = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            d[name] = list(v) if name == "letter_tokens" else v
        return d


class IIFile(ctypes.Structure):
    _fields_ = [("path", ctypes.c_char_p), ("size", ctypes.c_uint64), ("id0", ctypes.c_uint32),
                ("mapper", ctypes.c_int32)]


_lib = None


def _init_torch_first():
    """torch ships its own libamdhip64; whichever HIP runtime initialises first
    owns the device in this process.  When torch is importable, let it
    initialise first so libii.so binds to the same runtime (same soname)."""
    try:
        import torch
        torch.cuda.is_available()
    except Exception:
        pass


def lib():
    global _lib
    if _lib is None:
        _init_torch_first()
        # II_LIB_VARIANT=x loads libii_x.so (A/B builds of kernel variants, tools/gpu_ab.sh)
        var = os.environ.get("II_LIB_VARIANT")
        path = os.path.join(PKG_DIR, "libii_%s.so" % var if var else "libii.so")
        if not os.path.exists(path):
            raise FileNotFoundError("libii.so not built (make -C %s)" % PKG_DIR)
        L = ctypes.CDLL(path)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.ii_open.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
        L.ii_close.argtypes = [ctypes.c_void_p]
        L.ii_close.restype = None
        L.ii_strerror.argtypes = [ctypes.c_int]
        L.ii_strerror.restype = ctypes.c_char_p
        L.ii_map_files.argtypes = [ctypes.c_void_p, ctypes.POINTER(IIFile), ctypes.c_uint32, ctypes.c_int, u64p]
        L.ii_map_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u64p, u32p, ctypes.c_uint32, u64p]
        L.ii_map_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, u64p, u32p, ctypes.c_uint32,
                                    u64p]
        L.ii_reduce.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ii_letter_text.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.ii_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(Stats)]
        L.ii_device_text.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), u64p]
        L.ii_reducer_letters.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_int)]
        L.ii_partition.argtypes = [u64p, ctypes.c_uint32, ctypes.c_int, u32p, u32p, u32p]
        L.ii_reduce_local.argtypes = [ctypes.c_void_p]
        L.ii_export_plan.argtypes = [ctypes.c_void_p, ctypes.c_int, u64p]
        L.ii_export.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, u64p]
        L.ii_import.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, u64p, ctypes.c_uint32]
        i32p = ctypes.POINTER(ctypes.c_int)
        L.ii_letter_load.argtypes = [ctypes.c_void_p, u64p]
        L.ii_balanced_letters.argtypes = [u64p, ctypes.c_int, i32p, i32p]
        L.ii_export_plan_ranges.argtypes = [ctypes.c_void_p, ctypes.c_int, i32p, i32p, u64p]
        L.ii_partials.argtypes = [ctypes.c_void_p, u32p, ctypes.c_uint32]
        L.ii_partial_text.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                      ctypes.POINTER(ctypes.c_size_t)]
        _lib = L
    return _lib


def bytes_at(addr, n):
    """The n bytes at addr.  (ctypes.string_at passes its size as a C int: a
    letter text of 4.37 GB came back as its first 79 MB.)"""
    return bytes((ctypes.c_char * n).from_address(addr)) if n else b""


def _check(rc, what):
    if rc != II_OK:
        raise IIError(rc, what)


def _array(seq, ctype, dtype):
    """A C array of seq: a contiguous numpy array of the right dtype is passed
    in place (no per-call copy: a 10^5-entry file table took milliseconds to
    marshal element by element), anything else is copied into a ctypes array."""
    if isinstance(seq, np.ndarray) and seq.dtype == dtype and seq.flags.c_contiguous and len(seq):
        return seq.ctypes.data_as(ctypes.POINTER(ctype))  # keeps a reference to seq
    return (ctype * max(1, len(seq)))(*seq)


def _u64(seq):
    return _array(seq, ctypes.c_uint64, np.uint64)


def _u32(seq):
    return _array(seq, ctypes.c_uint32, np.uint32)


class Index:
    """One context on one GPU (ii_open .. ii_close)."""

    def __init__(self, device=0):
        self.h = ctypes.c_void_p()
        _check(lib().ii_open(ctypes.byref(self.h), device), "ii_open")

    def close(self):
        if self.h:
            lib().ii_close(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def map_host(self, text, file_off, file_id0):
        """text: bytes/bytearray/numpy u8; file f = text[file_off[f]:file_off[f+1]]."""
        n = len(file_id0)
        hist = (ctypes.c_uint64 * ALPHABET)()
        if hasattr(text, "ctypes"):
            ptr = text.ctypes.data
        else:
            buf = (ctypes.c_uint8 * max(1, len(text))).from_buffer_copy(bytes(text) or b"\0")
            ptr = ctypes.addressof(buf)
        _check(lib().ii_map_host(self.h, ptr, _u64(file_off), _u32(file_id0), n, hist), "ii_map_host")
        return list(hist)

    def map_device(self, d_text_ptr, nbytes, file_start, file_id0):
        hist = (ctypes.c_uint64 * ALPHABET)()
        _check(lib().ii_map_device(self.h, ctypes.c_void_p(d_text_ptr), nbytes, _u64(file_start), _u32(file_id0),
                                   len(file_id0), hist), "ii_map_device")
        return list(hist)

    def map_files(self, paths, nthreads=4, id0=None, sizes=None, mappers=None):
        """ii_map_files; `sizes` overrides the stat sizes (tests of the
        reader's short-file padding and grown-file fallback); `mappers` the
        mapper id printed for a missing file (main.c:98)."""
        files = (IIFile * max(1, len(paths)))()
        keep = []
        for i, p in enumerate(paths):
            b = os.fsencode(p)
            keep.append(b)
            size = os.path.getsize(p) if os.path.exists(p) else 0
            if sizes is not None:
                size = sizes[i]
            files[i] = IIFile(b, size, i if id0 is None else id0[i], 0 if mappers is None else mappers[i])
        hist = (ctypes.c_uint64 * ALPHABET)()
        _check(lib().ii_map_files(self.h, files, len(paths), nthreads, hist), "ii_map_files")
        return list(hist)

    def reduce(self, copy_text=True):
        _check(lib().ii_reduce(self.h, 1 if copy_text else 0), "ii_reduce")

    def reduce_local(self):
        _check(lib().ii_reduce_local(self.h), "ii_reduce_local")

    def export_plan(self, nparts):
        out = (ctypes.c_uint64 * nparts)()
        _check(lib().ii_export_plan(self.h, nparts, out), "ii_export_plan")
        return list(out)

    def export_plan_ranges(self, letter_lo, letter_hi):
        n = len(letter_lo)
        out = (ctypes.c_uint64 * n)()
        _check(lib().ii_export_plan_ranges(self.h, n, (ctypes.c_int * n)(*letter_lo), (ctypes.c_int * n)(*letter_hi),
                                           out), "ii_export_plan_ranges")
        return list(out)

    def letter_load(self):
        out = (ctypes.c_uint64 * ALPHABET)()
        _check(lib().ii_letter_load(self.h, out), "ii_letter_load")
        return list(out)

    def export(self, nparts, d_send_ptr, send_off):
        _check(lib().ii_export(self.h, nparts, ctypes.c_void_p(d_send_ptr), _u64(send_off)), "ii_export")

    def import_(self, nparts, d_recv_ptr, recv_off, id_bound):
        _check(lib().ii_import(self.h, nparts, ctypes.c_void_p(d_recv_ptr), _u64(recv_off), id_bound), "ii_import")

    def letter_text(self, letter):
        buf = ctypes.c_char_p()
        n = ctypes.c_size_t()
        _check(lib().ii_letter_text(self.h, letter, ctypes.byref(buf), ctypes.byref(n)), "ii_letter_text")
        return bytes_at(ctypes.cast(buf, ctypes.c_void_p).value, n.value)

    def letters(self):
        return {chr(97 + l): self.letter_text(l) for l in range(ALPHABET)}

    def partials(self, order):
        """Text of the 26 partial_<letter>.txt files (ii_partials): `order`
        lists indices of the mapped files in emission order."""
        order = list(order)
        _check(lib().ii_partials(self.h, _u32(order) if order else None, len(order)), "ii_partials")
        out = {}
        for l in range(ALPHABET):
            buf = ctypes.c_char_p()
            n = ctypes.c_size_t()
            _check(lib().ii_partial_text(self.h, l, ctypes.byref(buf), ctypes.byref(n)), "ii_partial_text")
            out[chr(97 + l)] = bytes_at(ctypes.cast(buf, ctypes.c_void_p).value, n.value)
        return out

    def stats(self):
        s = Stats()
        _check(lib().ii_get_stats(self.h, ctypes.byref(s)), "ii_get_stats")
        return s

    def device_text(self):
        p = ctypes.c_void_p()
        off = (ctypes.c_uint64 * (ALPHABET + 1))()
        _check(lib().ii_device_text(self.h, ctypes.byref(p), off), "ii_device_text")
        return p.value, list(off)


def reducer_letters(r, R):
    lo, hi = ctypes.c_int(), ctypes.c_int()
    _check(lib().ii_reducer_letters(r, R, ctypes.byref(lo), ctypes.byref(hi)), "ii_reducer_letters")
    return lo.value, hi.value


def balanced_letters(weights, parts):
    """-> (letter_lo, letter_hi) lists, ii_balanced_letters."""
    lo = (ctypes.c_int * parts)()
    hi = (ctypes.c_int * parts)()
    _check(lib().ii_balanced_letters(_u64(list(weights)), parts, lo, hi), "ii_balanced_letters")
    return list(lo), list(hi)


def partition(sizes, M):
    n = len(sizes)
    order = (ctypes.c_uint32 * max(1, n))()
    sb = (ctypes.c_uint32 * M)()
    se = (ctypes.c_uint32 * M)()
    _check(lib().ii_partition(_u64(sizes), n, M, order, sb, se), "ii_partition")
    return list(order)[:n], list(sb), list(se)


# ---------------------------------------------------------------- generator
class GenParams(ctypes.Structure):
    _fields_ = [("total_bytes", ctypes.c_uint64), ("nfiles", ctypes.c_uint32), ("vocab", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("size_sigma", ctypes.c_double)]


_gen = None


def genlib():
    global _gen
    if _gen is None:
        path = os.path.join(PKG_DIR, "libiigen.so")
        if not os.path.exists(path):
            raise FileNotFoundError("libiigen.so not built (make -C %s)" % PKG_DIR)
        _gen = ctypes.CDLL(path)
    return _gen


def zipf_corpus(total_bytes, nfiles, vocab, seed, threads=8, out=None):
    """Returns (numpy u8 text, numpy u64 file offsets[nfiles+1])."""
    import numpy as np
    p = GenParams(total_bytes, nfiles, vocab, seed, 1.0)
    off = np.zeros(nfiles + 1, dtype=np.uint64)
    if out is None:
        out = np.empty(total_bytes + 16, dtype=np.uint8)
    g = genlib()
    if g.iigen_layout(ctypes.byref(p), ctypes.c_void_p(off.ctypes.data)) != 0:
        raise RuntimeError("iigen_layout failed")
    if g.iigen_fill(ctypes.byref(p), ctypes.c_void_p(off.ctypes.data), ctypes.c_void_p(out.ctypes.data), threads) != 0:
        raise RuntimeError("iigen_fill failed")
    return out[:total_bytes], off


def zipf_layout(total_bytes, nfiles, seed):
    """File offsets (numpy u64[nfiles+1]) of the corpus zipf_corpus would make,
    without making it (the sizes ii_partition shards by)."""
    import numpy as np
    p = GenParams(total_bytes, nfiles, 1, seed, 1.0)
    off = np.zeros(nfiles + 1, dtype=np.uint64)
    if genlib().iigen_layout(ctypes.byref(p), ctypes.c_void_p(off.ctypes.data)) != 0:
        raise RuntimeError("iigen_layout failed")
    return off


def zipf_shard(total_bytes, nfiles, vocab, seed, files, threads=8, pad=16):
    """Only the files `files` (indices, any order) of zipf_corpus(total_bytes,
    nfiles, vocab, seed), back to back in that order — one GPU's shard.
    Returns (numpy u8 text, numpy u64 offsets[len(files)+1]); the bytes of every
    file equal its slice of the whole corpus."""
    import numpy as np
    p = GenParams(total_bytes, nfiles, vocab, seed, 1.0)
    full = zipf_layout(total_bytes, nfiles, seed)
    sel = np.ascontiguousarray(np.asarray(list(files), dtype=np.uint32))
    sizes = (full[1:] - full[:-1])[sel.astype(np.int64)] if len(sel) else np.zeros(0, dtype=np.uint64)
    n = int(sizes.sum())
    out = np.empty(n + pad, dtype=np.uint8)
    off = np.zeros(len(sel) + 1, dtype=np.uint64)
    g = genlib()
    if g.iigen_fill_files(ctypes.byref(p), ctypes.c_void_p(full.ctypes.data),
                          ctypes.c_void_p(sel.ctypes.data if len(sel) else None), ctypes.c_uint32(len(sel)),
                          ctypes.c_void_p(off.ctypes.data), ctypes.c_void_p(out.ctypes.data), threads) != 0:
        raise RuntimeError("iigen_fill_files failed")
    return out[:n], off
