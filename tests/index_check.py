"""ctypes wrapper of oracle/ii_check.c (test infrastructure): the properties
every <letter>.txt the reference writes has (main.c:55-64, 215-234), checked
in C over a whole letter text — for corpora no oracle output exists for."""
import ctypes
import os

from conftest import ORACLE

KINDS = {-1: "word length", -2: "first letter", -3: "line syntax", -4: "id syntax", -5: "id out of range",
         -6: "ids not strictly ascending", -7: "lines out of order", -8: "no final line end", -9: "argument"}
_lib = None


def _L():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(os.path.join(ORACLE, "build", "libii_check.so"))
        _lib.ii_check_letter.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_uint64)]
    return _lib


def check_letter(text, letter, id_max, nthreads=8):
    """-> (rc, lines, sum_df, max_df, first_bad_offset); rc 0 = every property holds."""
    out = (ctypes.c_uint64 * 4)()
    rc = _L().ii_check_letter(text, len(text), letter, id_max, nthreads, out)
    return rc, out[0], out[1], out[2], out[3]
