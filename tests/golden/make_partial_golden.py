#!/usr/bin/env python3
"""Record the REFERENCE binary's partial files for every
golden case: oracle/_ref/tema1 (built from /root/reference/main.c by
oracle/Makefile) is run with ONE mapper and one reducer on each case's inputs,
and the sha256 / size / line count of each partial_<letter>.txt it leaves in
its working directory (main.c:332-341, lines written at main.c:116) goes into
tests/golden/partials.json.

With one mapper the reference's line order is deterministic: files in size
order (qsort main.c:300, glibc's stable merge sort: ties keep list order),
tokens in text order.  Run in the build container:

    python tests/golden/make_partial_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tarfile
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
TEMA1 = os.path.join(REPO, "oracle", "_ref", "tema1")
CASES = ["config1", "config2", "edge", "rand_0", "rand_1", "rand_2", "tiny360", "zipf_small"]


def main():
    if not os.path.exists(TEMA1):
        sys.exit("build the reference first: make -C oracle reference")
    res = {"generator": "tests/golden/make_partial_golden.py", "M": 1, "R": 1, "cases": {}}
    for case in CASES:
        with tempfile.TemporaryDirectory() as td:
            with tarfile.open(os.path.join(HERE, case + ".tar.xz"), "r:xz") as tar:
                for m in tar.getmembers():
                    if m.isfile() and not m.name.startswith("expected/"):
                        data = tar.extractfile(m).read()
                        p = os.path.join(td, m.name)
                        os.makedirs(os.path.dirname(p), exist_ok=True)
                        with open(p, "wb") as f:
                            f.write(data)
            subprocess.run([TEMA1, "1", "1", "list.txt"], cwd=td, check=True, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
            letters = {}
            for l in "abcdefghijklmnopqrstuvwxyz":
                with open(os.path.join(td, "partial_%s.txt" % l), "rb") as f:
                    d = f.read()
                letters[l] = {"bytes": len(d), "lines": d.count(b"\n"), "sha256": hashlib.sha256(d).hexdigest()}
            res["cases"][case] = letters
    with open(os.path.join(HERE, "partials.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote partials.json for %d cases" % len(CASES))


if __name__ == "__main__":
    main()
