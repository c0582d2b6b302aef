#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
binary itself (oracle/_ref/tema1, compiled by oracle/Makefile from
/root/reference/main.c) on every input set.

Run in the build container (needs /root/reference and oracle/_ref/tema1):

    python tests/golden/make_golden.py

Each case becomes tests/golden/<case>.tar.xz holding
    list.txt            the reference's list-file format (count, then paths)
    in/...              the input files (data only)
    expected/a.txt..z.txt   the reference's outputs
and tests/golden/golden.json records M, R, per-letter sha256 and totals.

Cases:
  config1   test_small.txt + test_in_small/ (BASELINE.json configs[0]), M/R 2/2
  config2   test.txt + test_in/ (configs[1]), M/R 4/4
  edge      hand-built corpus exercising every tokenizer rule of SURVEY.md §9
  rand_*    seeded byte-soup corpora (all delimiter / NUL / high-byte classes)
  tiny360   360 tiny files (the reference's MAX_FILES), many files per 64 KiB
  zipf_small  a small corpus from the repo's Zipf generator (iigen)
All raw tokens stay < 300 bytes, where the reference is well defined.
"""
import hashlib
import io
import json
import os
import random
import shutil
import subprocess
import sys
import tarfile
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF_DIR = "/root/reference"
TEMA1 = os.path.join(REPO, "oracle", "_ref", "tema1")
PKG = os.path.join(REPO, "parallel-computation-of-an-inverted-index-using-map-reduce_amd")


def run_reference(workdir, M, R, listname="list.txt"):
    subprocess.run([TEMA1, str(M), str(R), listname], cwd=workdir, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    out = {}
    for l in "abcdefghijklmnopqrstuvwxyz":
        with open(os.path.join(workdir, l + ".txt"), "rb") as f:
            out[l] = f.read()
    return out


def write_case(name, files, M, R, extra_list_entries=None, list_text=None):
    """files: list of (relative path, bytes); the list enumerates them in order
    (plus extra_list_entries, e.g. a missing path, spliced in at given index)."""
    with tempfile.TemporaryDirectory() as td:
        for rel, data in files:
            p = os.path.join(td, rel)
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "wb") as f:
                f.write(data)
        if list_text is None:
            paths = [rel for rel, _ in files]
            for idx, entry in (extra_list_entries or []):
                paths.insert(idx, entry)
            list_text = "%d\n%s\n" % (len(paths), "\n".join(paths))
        with open(os.path.join(td, "list.txt"), "w") as f:
            f.write(list_text)
        out = run_reference(td, M, R)
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w:xz") as tar:
            tar.add(os.path.join(td, "list.txt"), arcname="list.txt")
            seen = set()
            for rel, _ in files:
                if rel in seen:
                    continue
                seen.add(rel)
                tar.add(os.path.join(td, rel), arcname=rel)
            for l, data in out.items():
                ti = tarfile.TarInfo("expected/%s.txt" % l)
                ti.size = len(data)
                tar.addfile(ti, io.BytesIO(data))
        with open(os.path.join(HERE, name + ".tar.xz"), "wb") as f:
            f.write(buf.getvalue())
    allb = b"".join(out[l] for l in "abcdefghijklmnopqrstuvwxyz")
    return {
        "M": M, "R": R,
        "nfiles": int(list_text.split()[0]),
        "input_bytes": sum(len(d) for _, d in files),
        "out_bytes": len(allb),
        "lines": allb.count(b"\n"),
        "sha256": hashlib.sha256(allb).hexdigest(),
        "letters": {l: {"bytes": len(out[l]), "lines": out[l].count(b"\n"),
                        "sha256": hashlib.sha256(out[l]).hexdigest()} for l in out},
    }


def ref_files(listname):
    with open(os.path.join(REF_DIR, listname)) as f:
        toks = f.read().split()
    n = int(toks[0])
    files = []
    for rel in toks[1:1 + n]:
        with open(os.path.join(REF_DIR, rel), "rb") as f:
            files.append(("in/" + rel, f.read()))
    return files


def edge_files():
    long299 = b"x" * 299
    long150 = b"Q" * 150
    f1 = (b"ABCdef caf\xc3\xa9 don't end. ff\x0cff? tab\there vt\x0bvt na\xc3\xafve "
          b"wel-l_known 12345 ---- internationalization internationalize internationally "
          b"abcdefghijklmnopqrstuvwxyzab abcdefghijklmnopqrstuvwxyzaa abcdefghijkl abcdefghijklm "
          b"zz9top \r\nfinal")
    f2 = (b"a ab abc " + long150 + b" " + long299 + b"\nA AB aBc\x00zzz \x00hidden "
          b"mid\x00dle ab\x00cd zZ " + b"prefixsharedxxxxxxxxxxxxA prefixsharedxxxxxxxxxxxxB "
          b"prefixsharedxxxxxxxxxxxx prefixsharedxxxxxxxxxxxxAB\n")
    f3 = b""                      # empty file
    f5 = b"b\tb\nB\x0bdont\x0ca\r"   # all six C-locale spaces
    f6 = f1                         # same bytes as file 1 (distinct ID)
    f7 = b"sep\x1cword\x1d\x1e\x1fnbsp\x85\xa0x \xff\xfe\x80 \x01\x02"
    files = [("in/f1.txt", f1), ("in/f2.txt", f2), ("in/f3.txt", f3),
             ("in/f5.txt", f5), ("in/f6.txt", f6), ("in/f7.txt", f7)]
    # ID 4 is a missing file: keeps its ID, contributes nothing (main.c:294, 98)
    return files, [(3, "in/missing.txt")]


def rand_files(seed, nfiles, max_bytes):
    rng = random.Random(seed)
    letters = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
    junk = b"0123456789.,;:!?'\"-_()[]{}<>/\\@#$%^&*+=~`|"
    high = bytes(range(0x80, 0x100))
    ctrl = bytes([1, 2, 3, 0x1c, 0x1d, 0x1e, 0x1f, 0x7f])
    spaces = b" \t\n\x0b\x0c\r"
    vocab = []
    for _ in range(400):
        L = rng.choice([1, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 16, 20, 25])
        vocab.append(bytes(rng.choice(letters) for _ in range(L)))
    files = []
    for fi in range(nfiles):
        if rng.random() < 0.08:
            files.append(("in/r%03d.txt" % fi, b""))
            continue
        out = bytearray()
        target = rng.randint(0, max_bytes)
        while len(out) < target:
            r = rng.random()
            if r < 0.70:
                tok = bytearray(rng.choice(vocab))
            elif r < 0.80:
                tok = bytearray(rng.choice(letters) for _ in range(rng.randint(1, 40)))
            else:
                tok = bytearray()
            # decorations, keeping raw tokens < 300 bytes
            for _ in range(rng.choice([0, 0, 0, 1, 2])):
                pool = rng.choice([junk, high, ctrl, b"\x00", letters])
                tok.insert(rng.randint(0, len(tok)), rng.choice(pool))
            if rng.random() < 0.01:
                tok = bytearray(rng.choice(letters) for _ in range(rng.randint(200, 299)))
            if not tok:
                tok = bytearray(rng.choice(junk) for _ in range(rng.randint(1, 3)))
            out += tok[:299]
            out += bytes(rng.choice(spaces) for _ in range(rng.choice([1, 1, 1, 2, 3])))
        if rng.random() < 0.3 and out:
            out = out.rstrip(spaces) or out   # file not ending in whitespace
        files.append(("in/r%03d.txt" % fi, bytes(out)))
    return files


def tiny360_files(seed):
    rng = random.Random(seed)
    words = [b"alpha", b"Beta", b"gamma", b"delta", b"eps", b"zeta", b"eta", b"theta", b"iota", b"kappa"]
    files = []
    for fi in range(360):
        n = rng.randint(0, 6)
        data = b" ".join(rng.choice(words) + rng.choice([b"", b"s", b"ed", b"!"]) for _ in range(n))
        files.append(("in/t%03d.txt" % fi, data))
    return files


def zipf_files():
    import ctypes
    lib = ctypes.CDLL(os.path.join(PKG, "libiigen.so"))

    class P(ctypes.Structure):
        _fields_ = [("total_bytes", ctypes.c_uint64), ("nfiles", ctypes.c_uint32), ("vocab", ctypes.c_uint32),
                    ("seed", ctypes.c_uint64), ("size_sigma", ctypes.c_double)]
    p = P(2_000_000, 60, 20000, 11, 1.0)
    off = (ctypes.c_uint64 * 61)()
    buf = (ctypes.c_uint8 * (p.total_bytes + 1))()
    assert lib.iigen_layout(ctypes.byref(p), off) == 0
    assert lib.iigen_fill(ctypes.byref(p), off, buf, 4) == 0
    raw = bytes(buf)[:p.total_bytes]
    files = [("in/z%02d.txt" % f, raw[off[f]:off[f + 1]]) for f in range(60)]
    return files, hashlib.sha256(raw).hexdigest()


def main():
    if not os.path.exists(TEMA1):
        sys.exit("build the reference first: make -C oracle")
    meta = {"generator": "tests/golden/make_golden.py", "reference_binary": "oracle/_ref/tema1 (gcc -O2 main.c)",
            "cases": {}}
    meta["cases"]["config1"] = write_case("config1", ref_files("test_small.txt"), 2, 2)
    meta["cases"]["config2"] = write_case("config2", ref_files("test.txt"), 4, 4)
    ef, extra = edge_files()
    meta["cases"]["edge"] = write_case("edge", ef, 1, 5, extra_list_entries=extra)
    for i, (seed, nf, mb) in enumerate([(101, 23, 4000), (202, 64, 20000), (303, 7, 120000)]):
        meta["cases"]["rand_%d" % i] = write_case("rand_%d" % i, rand_files(seed, nf, mb), 3, 7)
    meta["cases"]["tiny360"] = write_case("tiny360", tiny360_files(7), 8, 26)
    zf, zsha = zipf_files()
    meta["cases"]["zipf_small"] = write_case("zipf_small", zf, 4, 26)
    meta["cases"]["zipf_small"]["iigen"] = {"total_bytes": 2_000_000, "nfiles": 60, "vocab": 20000, "seed": 11,
                                            "corpus_sha256": zsha}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    for k, v in meta["cases"].items():
        print("%-10s files=%-4d in=%-8d out=%-8d lines=%-6d %s" % (k, v["nfiles"], v["input_bytes"], v["out_bytes"],
                                                                   v["lines"], v["sha256"][:16]))


if __name__ == "__main__":
    main()
