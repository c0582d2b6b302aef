"""CPU: the letter-file property checker (oracle/ii_check.c) that the full-size
configs[4] GPU test relies on — it must accept every reference golden (the
real binary's output) with the right line and pair counts, and reject each
kind of defect."""
import pytest

from conftest import CASES, load_case
from index_check import check_letter

LETTERS = "abcdefghijklmnopqrstuvwxyz"


@pytest.mark.parametrize("case", CASES)
def test_goldens_pass(case):
    list_text, _, expected = load_case(case)
    n = int(list_text.split()[0])
    for l, ch in enumerate(LETTERS):
        t = expected[ch]
        for th in (1, 3, 16):
            rc, lines, sdf, mdf, bad = check_letter(t, l, n, th)
            assert rc == 0, (case, ch, th, rc, bad, t[max(0, bad - 40):bad + 40] if bad < len(t) else b"")
            assert lines == t.count(b"\n")
            assert sdf == t.count(b" ") + t.count(b"\n")


def _config2_s():
    return load_case("config2")[2]["s"]


@pytest.mark.parametrize("mut,kind", [
    (lambda t: t.replace(b"\n", b"", 1)[:0] + t[:-1], -8),                       # no final line end
    (lambda t: b"x" + t, -2),                                                    # other first letter
    (lambda t: t.replace(b":[", b":[0", 1), -4),                                 # leading zero
    (lambda t: t.replace(b"]\n", b" 356]\n", 1), -5),                            # id > id_max
    (lambda t: t.replace(b"]\n", b"]]\n", 1), -3),                               # syntax
    (lambda t: t.replace(b"s", b"S", 1), -1),                                    # not a lowercase word
])
def test_defects_rejected(mut, kind):
    t = mut(_config2_s())
    rc, *_ = check_letter(t, 18, 355, 4)
    assert rc == kind


def test_order_and_ascending_ids_rejected():
    t = _config2_s()
    lines = t.split(b"\n")[:-1]
    # two lines swapped (df desc / word asc order broken), in the middle of a piece
    sw = lines[:]
    k = len(sw) // 2
    sw[k], sw[k + 1] = sw[k + 1], sw[k]
    for th in (1, 7):
        assert check_letter(b"\n".join(sw) + b"\n", 18, 355, th)[0] == -7
    # a repeated id inside a line
    i = next(i for i, x in enumerate(lines) if x.count(b" ") >= 2)
    w, ids = lines[i].split(b":[")
    v = ids[:-1].split(b" ")
    v[1] = v[0]
    dup = lines[:i] + [w + b":[" + b" ".join(v) + b"]"] + lines[i + 1:]
    assert check_letter(b"\n".join(dup) + b"\n", 18, 355, 4)[0] == -6
