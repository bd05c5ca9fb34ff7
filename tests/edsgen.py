"""Small random EDS / pattern generators and a brute-force EDS matcher (tests only).

The brute-force matcher is independent of any BWT: an occurrence of P is a start
(word, offset) inside a non-empty word from which P can be spelled left to right,
continuing at the start of any word of the next segment, where a segment holding
an empty word may be skipped (README.md:126-141; the link() semantics of
MOVE_EDSBWTSearch.cpp:512-625 seen forwards)."""
from __future__ import annotations

import functools
import random


def random_eds(rng: random.Random, nseg: int, alphabet: str = "ACGT", kmax: int = 4, lmax: int = 5,
               p_empty: float = 0.15) -> list[list[str]]:
    segs = []
    for _ in range(nseg):
        k = rng.randint(1, kmax)
        words = []
        for _ in range(k):
            if k > 1 and rng.random() < p_empty:
                words.append("")
            else:
                words.append("".join(rng.choice(alphabet) for _ in range(rng.randint(1, lmax))))
        if all(w == "" for w in words) and rng.random() < 0.5:
            words[0] = rng.choice(alphabet)
        segs.append(words)
    # a leading all-empty segment would start the EDS with "{,": keep it valid but rare
    return segs


def eds_text(segs: list[list[str]], use_E: bool = False) -> str:
    return "".join("{" + ",".join(("E" if (use_E and w == "") else w) for w in s) + "}" for s in segs)


def planted(rng: random.Random, segs: list[list[str]], m: int, tries: int = 1000) -> str | None:
    for _ in range(tries):
        si = rng.randrange(len(segs))
        w = rng.choice(segs[si])
        if not w:
            continue
        out = w[rng.randrange(len(w)):]
        s = si + 1
        while len(out) < m and s < len(segs):
            out += rng.choice(segs[s])
            s += 1
        if len(out) >= m:
            return out[:m]
    return None


def brute_occurrences(segs: list[list[str]], pat: str) -> set[tuple[int, int, int, int]]:
    """{(word id, 1-based segment, word in segment, offset)}"""
    nseg = len(segs)

    @functools.lru_cache(maxsize=None)
    def from_segment(si: int, p: int) -> bool:
        if p == len(pat):
            return True
        if si >= nseg:
            return False
        for w in segs[si]:
            if w == "":
                if from_segment(si + 1, p):
                    return True
            elif from_word(si, w, 0, p):
                return True
        return False

    def from_word(si: int, w: str, o: int, p: int) -> bool:
        n = min(len(w) - o, len(pat) - p)
        if w[o:o + n] != pat[p:p + n]:
            return False
        if p + n == len(pat):
            return True
        return from_segment(si + 1, p + n)

    res = set()
    wid = 0
    for si, seg in enumerate(segs):
        for wi, w in enumerate(seg):
            for o in range(len(w)):
                if from_word(si, w, o, 0):
                    res.add((wid, si + 1, wi, o))
            wid += 1
    return res
