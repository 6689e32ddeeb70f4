"""CPU checks of crdts_gpu.gset's row views (contains / read; gset.rs:83-85, :103-105) on bitmap
rows built from the oracle's GSet — the views only index the rows, so they run on host tensors."""
import numpy as np
import torch

import oracle as O
import crdts_gpu as cg


def _rows(sets, U):
    W = (U + 63) // 64
    r = np.zeros((len(sets), W), np.uint64)
    for i, s in enumerate(sets):
        for e in s.value:
            r[i, e // 64] |= np.uint64(1) << np.uint64(e % 64)
    return torch.from_numpy(r.view(np.int64))


def test_contains_and_read_match_oracle():
    rng = np.random.default_rng(3)
    U = 150
    sets = [O.GSet(rng.integers(0, U, rng.integers(0, 40)).tolist()) for _ in range(60)]
    sets.append(O.GSet([63, 64, 127, 128, 149]))  # word edges, incl. the sign bit of a word
    st = _rows(sets, U)
    assert cg.gset.read(st) == [sorted(s.value) for s in sets]
    d = torch.arange(U, dtype=torch.int64) * 11
    assert cg.gset.read(st, d) == [[11 * e for e in sorted(s.value)] for s in sets]
    for probe in (rng.integers(-3, U + 80, len(sets)), np.array([63] * len(sets)), np.array([64] * len(sets))):
        got = cg.gset.contains(st, torch.from_numpy(probe)).tolist()
        assert got == [s.contains(int(p)) for s, p in zip(sets, probe)]


def test_empty_rows():
    st = torch.zeros((3, 2), dtype=torch.int64)
    assert cg.gset.read(st) == [[], [], []]
    assert cg.gset.contains(st, torch.tensor([0, 127, 128])).tolist() == [False, False, False]
