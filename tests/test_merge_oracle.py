"""Oracle for the compaction merge (iter.MergeSort, internal/iter/merge.go:12-111): the C
restatement (oracle/slate_oracle.c or_merge_sort) against merge_test.go's known answers and an
independent heapq restatement on random iterators with duplicates, empty keys and shared prefixes."""
import random

import numpy as np
import pytest

from oracle import binding as ob
from tests import mergegen as mg


@pytest.mark.parametrize("case", range(len(mg.REFERENCE_CASES)))
def test_reference_cases(case):
    sources, want_keys, want_iter = mg.REFERENCE_CASES[case]
    flat = [k for s in sources for k in s]
    starts = np.cumsum([0] + [len(s) for s in sources])
    got = ob.merge_sort(sources)
    assert [flat[i] for i in got] == want_keys
    assert [int(np.searchsorted(starts, i, side="right") - 1) for i in got] == want_iter
    assert list(got) == mg.py_merge(sources)


def test_empty_keys_never_returned():
    # lastKey starts nil and bytes.Equal([]byte{}, nil) is true (merge.go:67)
    assert list(ob.merge_sort([[b"", b"a"], [b"", b"b"]])) == [1, 3]
    assert list(ob.merge_sort([[b""], []])) == []
    assert list(ob.merge_sort([[], []])) == []


@pytest.mark.parametrize("seed", range(40))
def test_random_vs_heapq(seed):
    rng = random.Random(seed)
    long = b"p" * rng.choice([0, 0, 15, 16, 17, 30])
    sources = mg.random_sources(rng, rng.randint(1, 9), 40, long_prefix=long)
    assert list(ob.merge_sort(sources)) == mg.py_merge(sources)


def test_compaction_runs_shape():
    keys, off, ss = mg.compaction_runs(4, 5000, 0.3)
    got = ob.merge_arrays(keys, off, ss)
    k = keys.reshape(-1, 16)
    merged = k[got]
    # strictly ascending (duplicates dropped) and every distinct input key present
    as_bytes = [bytes(r) for r in merged]
    assert all(a < b for a, b in zip(as_bytes, as_bytes[1:]))
    assert len(set(bytes(r) for r in k)) == len(as_bytes)
    # the heapq restatement agrees on a slice of the same shape
    keys, off, ss = mg.compaction_runs(3, 700, 0.5, seed=3)
    k = keys.reshape(-1, 16)
    sources = [[bytes(r) for r in k[int(ss[j]):int(ss[j + 1])]] for j in range(3)]
    assert list(ob.merge_arrays(keys, off, ss)) == mg.py_merge(sources)
