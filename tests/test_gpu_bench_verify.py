"""GPU: the benchmark corpora at FULL size against the oracle — every letter
of the index of BASELINE configs[2] (10 GB, 10^4 files, vocab 10^6, seed 3)
and of configs[4]'s per-GPU share (12.5 GB, 1.25*10^5 files, vocab 10^7,
seed 5) hashed and compared with tests/golden/bench_hashes.json (made by the
oracle in the build container, tests/golden/make_bench_hashes.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

import ii_ctypes
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DB = json.load(open(os.path.join(GOLDEN, "bench_hashes.json")))["workloads"]


@pytest.mark.parametrize("name", ["config3", "config5share"])
def test_full_size_index_matches_oracle(name):
    import torch
    if name not in DB:
        pytest.skip("no oracle hashes for %s" % name)
    w = DB[name]
    p = w["iigen"]
    text, off = ii_ctypes.zipf_corpus(p["total_bytes"], p["nfiles"], p["vocab"], p["seed"], threads=16)
    n = int(off[-1])
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    d[:n].copy_(torch.from_numpy(text))
    torch.cuda.synchronize()
    del text
    with ii_ctypes.Index(0) as ix:
        ix.map_device(d.data_ptr(), n, off[:-1].tolist(), list(range(p["nfiles"])))
        ix.reduce(copy_text=True)
        st = ix.stats()
        assert st.words == w["words"] and st.out_bytes == w["out_bytes"]
        bad = [l for l in w["letters"] if hashlib.sha256(ix.letter_text(ord(l) - 97)).hexdigest()
               != w["letters"][l]["sha256"]]
    assert not bad, "letters differ from the oracle: %s" % bad
