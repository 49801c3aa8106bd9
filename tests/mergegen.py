"""Merge-input generators shared by the oracle and GPU merge tests: k sorted iterators of keys,
concatenated (keys arena, key_off, src_start), as executeCompaction hands its decoded sorted runs
to iter.MergeSort (compaction/executor.go:92-151, internal/iter/merge.go:12-111)."""
import heapq
import random

import numpy as np

# Known answers from internal/iter/merge_test.go: (iterators, expected returned keys, expected
# winning iterator per returned key).  Values there only name the winner, so the iterator index
# stands in for them.
REFERENCE_CASES = [
    # TestMergeUniqueIteratorPrecedence (merge_test.go:13-37)
    ([[b"aaaa", b"cccc"], [b"cccc", b"xxxx"], [b"bbbb", b"cccc", b"xxxx"]],
     [b"aaaa", b"bbbb", b"cccc", b"xxxx"], [0, 2, 0, 1]),
    # TestMergeUnique (merge_test.go:39-70)
    ([[b"aaaa", b"cccc", b"zzzz"], [b"bbbb", b"xxxx", b"yyyy"], [b"dddd", b"eeee", b"gggg"]],
     [b"aaaa", b"bbbb", b"cccc", b"dddd", b"eeee", b"gggg", b"xxxx", b"yyyy", b"zzzz"], [0, 1, 0, 2, 2, 2, 1, 1, 0]),
    # TestMergeSortTwoIterators (merge_test.go:72-92)
    ([[b"aaaa", b"cccc", b"zzzz"], [b"bbbb", b"xxxx", b"yyyy"]],
     [b"aaaa", b"bbbb", b"cccc", b"xxxx", b"yyyy", b"zzzz"], [0, 1, 0, 1, 1, 0]),
    # TestMergeSortTwoIteratorsPrecedence (merge_test.go:94-110)
    ([[b"aaaa", b"cccc"], [b"cccc", b"xxxx"]], [b"aaaa", b"cccc", b"xxxx"], [0, 0, 1]),
]


def py_merge(sources: list[list[bytes]]) -> list[int]:
    """Pure-Python restatement of MergeSort.Next (merge.go:54-76) with heapq: returns flat indices."""
    starts = [0]
    for s in sources:
        starts.append(starts[-1] + len(s))
    h = [(s[0], i, 0) for i, s in enumerate(sources) if s]
    heapq.heapify(h)
    last = None  # lastKey == nil
    out = []
    while h:
        key, i, p = heapq.heappop(h)
        if p + 1 < len(sources[i]):
            heapq.heappush(h, (sources[i][p + 1], i, p + 1))
        equal = (len(key) == 0) if last is None else key == last
        if not equal:
            last = key
            out.append(starts[i] + p)
    return out


def random_sources(rng: random.Random, k: int, n_max: int, alphabet: bytes = b"ab\x00", kmax: int = 4,
                   long_prefix: bytes = b"") -> list[list[bytes]]:
    """k sorted iterators of short keys over a tiny alphabet (many duplicates across and inside
    iterators, empty keys, keys that are prefixes of each other, NUL bytes); long_prefix pushes
    keys past the 16-byte head so the tail comparison runs."""
    out = []
    for _ in range(k):
        n = rng.randint(0, n_max)
        keys = [long_prefix + bytes(rng.choice(alphabet) for _ in range(rng.randint(0, kmax))) for _ in range(n)]
        out.append(sorted(keys))
    return out


def arrays(sources: list[list[bytes]]):
    flat = [k for s in sources for k in s]
    off = np.zeros(len(flat) + 1, np.uint64)
    if flat:
        off[1:] = np.cumsum([len(x) for x in flat])
    keys = np.frombuffer(b"".join(flat) or b"\0", np.uint8).copy()
    ss = np.zeros(len(sources) + 1, np.uint64)
    ss[1:] = np.cumsum([len(s) for s in sources])
    return keys, off, ss


def compaction_runs(k: int, n_per: int, overlap: float, seed: int = 7):
    """k sorted runs of b"k%015d" keys (SURVEY 8d key shape) drawn from a shared key space so that
    about `overlap` of each run's keys also appear in other runs: the L0 -> sorted-run compaction
    shape.  Returns (keys arena, key_off, src_start) without building Python lists."""
    rng = np.random.default_rng(seed)
    space = int(n_per * k * (1.0 - overlap) + n_per)
    runs = [np.sort(rng.choice(space, size=n_per, replace=False)) for _ in range(k)]
    ids = np.concatenate(runs)
    digits = np.zeros((len(ids), 16), np.uint8)
    digits[:, 0] = ord("k")
    v = ids.copy()
    for c in range(15, 0, -1):
        digits[:, c] = ord("0") + (v % 10)
        v //= 10
    key_off = np.arange(len(ids) + 1, dtype=np.uint64) * 16
    ss = np.arange(k + 1, dtype=np.uint64) * n_per
    return digits.reshape(-1), key_off, ss
