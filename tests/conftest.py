"""Shared test setup.

Markers: `gpu` = needs an MI355X (runs on the GPU box).  Everything else runs
on a CPU-only container.  Built artefacts are made in-tree (make) if absent.
"""
import io
import os
import subprocess
import sys
import tarfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "parallel-computation-of-an-inverted-index-using-map-reduce_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE = os.path.join(REPO, "oracle")
sys.path.insert(0, os.path.join(PKG, "bindings"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU")


def _ensure_built():
    need_pkg = [os.path.join(PKG, f) for f in ("libii.so", "ii_index", "libiigen.so")]
    if not all(os.path.exists(p) for p in need_pkg):
        subprocess.run(["make", "-C", PKG, "-j4"], check=True, stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ORACLE, "build", "libii_oracle.so")):
        subprocess.run(["make", "-C", ORACLE, "restatement"], check=True, stdout=subprocess.DEVNULL)


_ensure_built()


def load_case(name):
    """-> (list_text, {relpath: bytes}, {letter: expected bytes})"""
    with tarfile.open(os.path.join(GOLDEN, name + ".tar.xz"), "r:xz") as tar:
        files, expected, list_text = {}, {}, None
        for m in tar.getmembers():
            if not m.isfile():
                continue
            data = tar.extractfile(m).read()
            if m.name == "list.txt":
                list_text = data.decode()
            elif m.name.startswith("expected/"):
                expected[m.name[len("expected/")][0]] = data
            else:
                files[m.name] = data
    return list_text, files, expected


def materialize(name, dest):
    list_text, files, expected = load_case(name)
    for rel, data in files.items():
        p = os.path.join(dest, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(data)
    with open(os.path.join(dest, "list.txt"), "w") as f:
        f.write(list_text)
    return list_text, files, expected


def case_arrays(name):
    """Concatenated text + offsets + ids in list order (missing files empty)."""
    list_text, files, expected = load_case(name)
    toks = list_text.split()
    n = int(toks[0])
    paths = toks[1:1 + n]
    text = bytearray()
    off = [0]
    for p in paths:
        text += files.get(p, b"")
        off.append(len(text))
    return bytes(text), off, list(range(n)), expected


CASES = ["config1", "config2", "edge", "rand_0", "rand_1", "rand_2", "tiny360", "zipf_small"]


def partials_meta():
    """tests/golden/partials.json: the reference's partial files, M = 1."""
    import json
    return json.load(open(os.path.join(GOLDEN, "partials.json")))["cases"]


def size_order(case):
    """Files in the reference's one-mapper read order (main.c:300: size
    descending; glibc's qsort is a stable merge sort, so ties keep list order;
    a missing file has size 0, main.c:294)."""
    list_text, files, _ = load_case(case)
    toks = list_text.split()
    paths = toks[1:1 + int(toks[0])]
    sizes = [len(files[p]) if p in files else 0 for p in paths]
    return sorted(range(len(paths)), key=lambda i: (-sizes[i], i))
