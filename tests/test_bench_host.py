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


def _pats(strs):
    buf = np.frombuffer(b"".join(strs), np.uint8).copy()
    offs = np.zeros(len(strs) + 1, np.int64)
    offs[1:] = np.cumsum([len(s) for s in strs])
    return buf, offs


def test_suffix_order_groups_shared_suffixes():
    """Patterns sharing their last k characters are contiguous in the order (one reversed-trie
    subtree each), shorter ones first, ties in line order (stable)."""
    strs = [b"ACGTTGCA", b"TTTTGCA", b"GGGGGGGA", b"CA", b"AAAAGGGA", b"ACGTTGCA", b"", b"A", b"TTGCA"]
    buf, offs = _pats(strs)
    order = bench.suffix_order(buf, offs, k=3)
    assert sorted(order.tolist()) == list(range(len(strs)))
    keys = [strs[i][::-1][:3] for i in order]
    assert keys == sorted(keys)  # reversed-suffix order (bytes compare: b"" < b"A" < b"AC" ...)
    pos = {i: p for p, i in enumerate(order.tolist())}
    assert pos[0] < pos[5]  # equal keys keep line order
    gca = sorted(pos[i] for i in (0, 1, 5, 8))  # the suffix "GCA": one contiguous run
    assert gca == list(range(gca[0], gca[0] + 4))


def test_suffix_order_random_matches_sorted_reversed_suffixes():
    rng = np.random.default_rng(5)
    strs = [bytes(rng.choice(list(b"ACGT"), size=int(n))) for n in rng.integers(0, 12, size=400)]
    buf, offs = _pats(strs)
    order = bench.suffix_order(buf, offs, k=8).tolist()
    want = sorted(range(len(strs)), key=lambda i: (strs[i][::-1][:8], i))
    assert order == want
