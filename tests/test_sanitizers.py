"""CPU: the C host CLI (host/ii_index.c) and the oracle's CLI built with
AddressSanitizer + UndefinedBehaviorSanitizer, run over the
list-parsing and partitioning cases where the reference itself has undefined
behaviour: more than 360 files (files[MAX_FILES] overflow,
main.c:8, 270, 274), more mappers than realised shards (uninitialised
file_start / file_end, main.c:307-309), M = 0 (SIGFPE, main.c:307), list
errors (main.c:257-285) and over-long names.  The new host defines each case;
the sanitizers must stay silent and the exit codes follow the reference's
(255 for list errors).  Without a GPU the CLI stops at ii_open (exit 1) after
parsing, sharding and printing the mapper ranges — the code under test here.
"""
import os
import subprocess
import tempfile

import pytest

from conftest import GOLDEN, ORACLE, PKG, materialize

SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
LETTERS = "abcdefghijklmnopqrstuvwxyz"


@pytest.fixture(scope="module")
def cli():
    subprocess.run(["make", "-C", PKG, "ii_index_san"], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(PKG, "ii_index_san")


@pytest.fixture(scope="module")
def oracle_cli():
    subprocess.run(["make", "-C", ORACLE, "build/ii_oracle_san"], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(ORACLE, "build", "ii_oracle_san")


def run(binary, args, cwd):
    r = subprocess.run([binary] + args, cwd=cwd, capture_output=True, env=SAN_ENV, timeout=120)
    err = r.stderr.decode(errors="replace")
    for marker in ("AddressSanitizer", "LeakSanitizer", "runtime error:", "UndefinedBehaviorSanitizer"):
        assert marker not in err, err[-3000:]
    assert r.returncode not in (98, 99), err[-3000:]
    return r.returncode, r.stdout.decode(), err


def write_list(td, names, count=None):
    with open(os.path.join(td, "list.txt"), "w") as f:
        f.write("%d\n%s\n" % (len(names) if count is None else count, "\n".join(names)))


def make_files(td, n, size=lambda i: 10 + i % 7):
    names = []
    for i in range(n):
        p = "f%04d.txt" % i
        with open(os.path.join(td, p), "w") as f:
            f.write(("w%s " % chr(97 + i % 26)) * size(i))
        names.append(p)
    return names


def test_cli_usage_and_list_errors(cli):
    with tempfile.TemporaryDirectory() as td:
        rc, _, err = run(cli, ["1", "1"], td)  # main.c:248-250
        assert rc == 255 and "Usage" in err
        rc, _, err = run(cli, ["1", "1", "absent.txt"], td)
        assert rc == 255 and "Error opening input file list" in err
        with open(os.path.join(td, "bad.txt"), "w") as f:
            f.write("many\nx\n")
        rc, _, err = run(cli, ["1", "1", "bad.txt"], td)
        assert rc == 255 and "number of files" in err
        names = make_files(td, 3)
        write_list(td, names, count=5)  # fewer names than the count (main.c:277-284)
        rc, _, err = run(cli, ["2", "2", "list.txt"], td)
        assert rc == 255 and "Error reading file name from input file list" in err
        write_list(td, names, count=-4)  # a negative count: no files
        rc, out, _ = run(cli, ["2", "2", "list.txt"], td)
        assert rc in (0, 1) and "Mapper 0: Files 0 to 0" in out


def test_cli_beyond_360_files(cli):
    # the reference overflows files[MAX_FILES] past 360 (main.c:8, 270); here any count
    with tempfile.TemporaryDirectory() as td:
        names = make_files(td, 400)
        write_list(td, names)
        rc, out, _ = run(cli, ["8", "4", "list.txt"], td)
        assert rc in (0, 1)
        lines = [l for l in out.splitlines() if l.startswith("Mapper ")]
        assert len(lines) == 8 and lines[-1].endswith("to 400")


def test_cli_more_mappers_than_shards_and_zero_mappers(cli):
    with tempfile.TemporaryDirectory() as td:
        names = make_files(td, 3, size=lambda i: 100)
        write_list(td, names)
        rc, out, _ = run(cli, ["8", "2", "list.txt"], td)  # main.c:307-309: empty shards here
        assert rc in (0, 1)
        lines = [l for l in out.splitlines() if l.startswith("Mapper ")]
        assert len(lines) == 8 and lines[-1] == "Mapper 7: Files 3 to 3"
        rc, out, _ = run(cli, ["0", "1", "list.txt"], td)  # main.c:307 SIGFPE in the reference: M = 1 here
        assert rc in (0, 1) and out.count("Mapper ") == 1


def test_cli_long_and_missing_names(cli):
    with tempfile.TemporaryDirectory() as td:
        names = make_files(td, 2) + ["missing_%s.txt" % ("x" * 5000), "y" * 4095]
        write_list(td, names)
        rc, _, err = run(cli, ["2", "3", "list.txt"], td)
        assert rc in (0, 1, 255) and "Error getting size of file" in err


def test_oracle_cli_on_goldens(oracle_cli):
    for case, args in [("edge", ["1", "5"]), ("config1", ["2", "2"]), ("tiny360", ["4", "26"])]:
        with tempfile.TemporaryDirectory() as td:
            _, _, expected = materialize(case, td)
            rc, _, _ = run(oracle_cli, args + ["list.txt"], td)
            assert rc == 0
            for l in LETTERS:
                assert open(os.path.join(td, l + ".txt"), "rb").read() == expected[l], (case, l)


def test_oracle_cli_beyond_360_files_and_list_errors(oracle_cli):
    with tempfile.TemporaryDirectory() as td:
        names = make_files(td, 400)
        write_list(td, names)
        rc, _, _ = run(oracle_cli, ["3", "7", "list.txt"], td)
        assert rc == 0
        assert b"wa:[" in open(os.path.join(td, "w.txt"), "rb").read()
        write_list(td, names[:2], count=4)
        rc, _, err = run(oracle_cli, ["3", "7", "list.txt"], td)
        assert rc == 255 and "Error reading file name" in err


@pytest.mark.parametrize("binary", ["plain", "san"])
def test_cli_failed_context_exits_promptly(cli, binary):
    """A context that fails while others are stuck (II_TEST_FAIL=map:g: context
    g returns II_ERR_INTERNAL, every other context of the phase blocks, as
    behind a faulted device — round 3's hang) must end the CLI at once with a
    non-zero exit and the error on stderr, without waiting for the others."""
    import time
    exe = cli if binary == "san" else os.path.join(PKG, "ii_index")
    with tempfile.TemporaryDirectory() as td:
        write_list(td, make_files(td, 12))
        env = dict(SAN_ENV, II_GPUS="5", II_TEST_FAIL="map:3")
        t0 = time.time()
        r = subprocess.run([exe, "3", "4", "list.txt"], cwd=td, capture_output=True, env=env, timeout=60)
        dt = time.time() - t0
        err = r.stderr.decode(errors="replace")
    assert r.returncode == 1, err
    assert "internal consistency check failed" in err, err
    assert dt < 15.0, dt
    for marker in ("AddressSanitizer", "runtime error:", "UndefinedBehaviorSanitizer"):
        assert marker not in err, err


@pytest.mark.parametrize("knob", ["map:9", "map:-1", "map:", "map:2x", "merge:5"])
def test_cli_stray_test_knob_is_ignored(cli, knob):
    """II_TEST_FAIL naming no context of the phase (index outside
    0 .. G-1, or not a number) must not block the CLI or skip its checks: here
    (no GPU) it fails at once with the no-device error, as without the knob."""
    with tempfile.TemporaryDirectory() as td:
        write_list(td, make_files(td, 6))
        env = dict(SAN_ENV, II_GPUS="5", II_TEST_FAIL=knob)
        r = subprocess.run([cli, "2", "3", "list.txt"], cwd=td, capture_output=True, env=env, timeout=60)
        err = r.stderr.decode(errors="replace")
    assert r.returncode == 1, err
    assert "no HIP device" in err, err


@pytest.fixture(scope="module")
def reader():
    subprocess.run(["make", "-C", PKG, "reader_san"], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(PKG, "reader_san")


@pytest.mark.parametrize("win,threads", [(7, 1), (64, 4), (1 << 20, 3)])
def test_reader_windows_under_sanitizers(reader, win, threads):
    """ii_map_files' pread reader (csrc/ii_reader.h io_fill) on
    the host under ASan + UBSan: windows that cut files anywhere, several
    threads, an empty file, a missing file (reported once, main.c:98, read as
    spaces), a file shorter than its stat size (padded with spaces) and one
    longer (the 'grown' verdict that makes ii_map_files re-read whole files)."""
    with tempfile.TemporaryDirectory() as td:
        specs = []  # (path, stat size given, bytes on disk or None)
        rnd = __import__("random").Random(win)
        for i in range(9):
            body = bytes(rnd.choice(b"abc xyz\nQ!") for _ in range(rnd.randrange(1, 300)))
            specs.append(("f%d.txt" % i, len(body), body))
        specs.append(("empty.txt", 0, b""))
        specs.append(("missing.txt", 40, None))
        specs.append(("short.txt", 50, b"only twenty bytes ok"))
        specs.append(("long.txt", 10, b"twenty-five bytes in here"))
        for p, _, body in specs:
            if body is not None:
                with open(os.path.join(td, p), "wb") as f:
                    f.write(body)
        args = [str(win), str(threads)]
        for p, size, _ in specs:
            args += [str(size), p]
        r = subprocess.run([reader] + args, cwd=td, capture_output=True, env=SAN_ENV, timeout=60)
    err = r.stderr.decode(errors="replace")
    for marker in ("AddressSanitizer", "LeakSanitizer", "runtime error:", "ThreadSanitizer"):
        assert marker not in err, err[-3000:]
    assert r.returncode == 0, err
    head, _, img = r.stdout.partition(b"\n")
    assert head == b"grown=1"
    want = b""
    for p, size, body in specs:
        data = (body or b"")[:size]
        want += data + b" " * (size - len(data)) + b"\n"
    assert img == want
    assert err.count("Error opening file missing.txt") == 1, err
    assert "Mapper 1: Error opening file missing.txt" in err, err
