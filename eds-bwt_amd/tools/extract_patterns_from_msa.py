#!/usr/bin/env python3
"""Pattern sampler over a multiple sequence alignment — the reference's
extract_patterns_from_msa.py:7-71 (used by launch_COVID.sh to draw query k-mers from the
sequences an EDS was built from).

    extract_patterns_from_msa.py <msa> <out> -l LENGTH [-n NUM] [--seed S]

Sequences are the FASTA records of the MSA with '-' gaps removed (:7-27); the population is
every length-L window of every sequence at least L long, in sequence order (:30-42); NUM of
them are drawn without replacement with random.sample (:60) and written one per line with no
newline after the last (:62-68).  The population is never materialised: random.sample picks
indices, so sampling range(#windows) and mapping each index back to (sequence, start) draws
exactly the windows random.sample(list_of_windows, NUM) would for the same random state.
--seed (not in the reference, whose draw is unseeded) makes the draw reproducible.
"""
import argparse
import bisect
import random


def load_sequences(path):
    """FASTA records, gap characters removed, each record's lines joined (:7-27)."""
    seqs, cur = [], []
    with open(path) as f:
        for line in f:
            if line.startswith(">"):
                if cur:
                    seqs.append("".join(cur))
                    cur = []
                continue
            cur.append(line.strip().replace("-", ""))
    if cur:
        seqs.append("".join(cur))
    return seqs


def sample_windows(seqs, length, num, rng=random):
    """`num` distinct length-`length` windows, as random.sample over the window list (:30-42, :60)."""
    starts, total = [], 0          # first window index of each usable sequence
    usable = []
    for s in seqs:
        if len(s) < length:
            continue
        usable.append(s)
        starts.append(total)
        total += len(s) - length + 1
    picks = rng.sample(range(total), num)  # ValueError when num > windows, as the reference
    out = []
    for g in picks:
        q = bisect.bisect_right(starts, g) - 1
        off = g - starts[q]
        out.append(usable[q][off:off + length])
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("-l", "--length", type=int, required=True)
    ap.add_argument("-n", "--num", type=int, default=90)
    ap.add_argument("--seed", type=int, default=None)
    a = ap.parse_args(argv)
    rng = random.Random(a.seed) if a.seed is not None else random
    sel = sample_windows(load_sequences(a.input), a.length, a.num, rng)
    with open(a.output, "w") as f:
        f.write("\n".join(sel))


if __name__ == "__main__":
    main()
