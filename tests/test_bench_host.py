"""Host logic of bench.py (no GPU): the C5 located leg's record-budget chunking."""
import numpy as np

import bench


def test_record_chunks_cover_and_bound():
    rng = np.random.default_rng(3)
    for budget in (1, 7, 100, 1e4):
        counts = rng.integers(0, 50, size=1000)
        counts[rng.integers(0, 1000, size=5)] = 10_000  # single patterns above the budget
        cuts = bench.record_chunks(counts, budget)
        assert cuts[0] == 0 and cuts[-1] == counts.size and all(b > a for a, b in zip(cuts, cuts[1:]))
        for a, b in zip(cuts, cuts[1:]):
            tot = int(counts[a:b].sum())
            assert tot <= budget or b == a + 1, (a, b, tot)
            if b < counts.size:  # greedy: the next pattern would not have fitted
                assert tot + int(counts[b]) > budget


def test_record_chunks_edge_cases():
    assert bench.record_chunks(np.zeros(0, np.int64), 10) == [0]
    assert bench.record_chunks(np.zeros(5, np.int64), 10) == [0, 5]
    assert bench.record_chunks(np.array([11, 0, 0]), 10) == [0, 1, 3]
