"""GPU parity for the compaction merge (iter.MergeSort, internal/iter/merge.go:12-111) through the
C ABI (slate_merge_sorted / slate_merge_sorted_device): merge_test.go's known answers, random
iterators with heavy duplication, empty keys, empty iterators, keys past the 16-byte head, the
unsorted-input error, and compaction-shaped runs up to 4 x 1 M keys, bit-exact (returned element
indices) against the oracle's heap restatement."""
import random

import numpy as np
import pytest

from oracle import binding as ob
from tests import mergegen as mg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    # torch's HIP runtime is initialised before the library's context (the device-path test
    # shares device memory with torch; bench.py uses the same order)
    import torch
    torch.cuda.init()
    torch.cuda.set_device(0)
    import slatecodec as sc
    return sc.Context(0)


@pytest.mark.parametrize("case", range(len(mg.REFERENCE_CASES)))
def test_reference_cases(ctx, case):
    sources, want_keys, _ = mg.REFERENCE_CASES[case]
    flat = [k for s in sources for k in s]
    got = ctx.merge_sort(sources)
    assert [flat[i] for i in got] == want_keys
    assert np.array_equal(got, ob.merge_sort(sources))


def test_edges(ctx):
    for sources in ([[b"", b"a"], [b"", b"b"]], [[b""], []], [[], []], [[]], [[b"x"]],
                    [[b"a", b"a", b"a"]], [[b"a"], [b"a"], [b"a"]], [[b"ab"], [b"ab\x00"], [b"a"]]):
        assert np.array_equal(ctx.merge_sort(sources), ob.merge_sort(sources)), sources


@pytest.mark.parametrize("seed", range(30))
def test_random(ctx, seed):
    rng = random.Random(1000 + seed)
    long = b"q" * rng.choice([0, 0, 8, 15, 16, 17, 40])
    sources = mg.random_sources(rng, rng.randint(1, 12), 300, kmax=rng.choice([2, 4, 24]), long_prefix=long)
    assert np.array_equal(ctx.merge_sort(sources), ob.merge_sort(sources))


def test_unsorted_iterator(ctx):
    import slatecodec as sc
    with pytest.raises(sc.SlateError) as ei:
        ctx.merge_sort([[b"a", b"c"], [b"d", b"b"]])
    assert ei.value.status == sc.E_MERGE_UNSORTED


@pytest.mark.parametrize("k,n_per,overlap", [(2, 100_000, 0.5), (4, 1_000_000, 0.3), (8, 200_000, 0.9)])
def test_compaction_runs(ctx, k, n_per, overlap):
    keys, off, ss = mg.compaction_runs(k, n_per, overlap, seed=k)
    got = ctx.merge_arrays(keys, off, ss)
    assert np.array_equal(got, ob.merge_arrays(keys, off, ss))


def test_device_path(ctx):
    import torch
    keys, off, ss = mg.compaction_runs(4, 50_000, 0.4, seed=11)
    n = int(ss[-1])
    dev = torch.device("cuda:0")
    d_keys = torch.from_numpy(keys).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    d_n = torch.zeros(1, dtype=torch.int64, device=dev)
    d_flags = torch.zeros(1, dtype=torch.int32, device=dev)
    import slatecodec as sc
    scratch = torch.empty(sc.lib().slate_merge_scratch_bytes(n, 4), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ctx.merge_device(d_keys.data_ptr(), d_off.data_ptr(), ss, d_out.data_ptr(), d_n.data_ptr(), d_flags.data_ptr(),
                     scratch.data_ptr())
    ctx.synchronize()
    m = int(d_n.item())
    assert int(d_flags.item()) == 0
    assert np.array_equal(d_out[:m].cpu().numpy().view(np.uint32), ob.merge_arrays(keys, off, ss))
