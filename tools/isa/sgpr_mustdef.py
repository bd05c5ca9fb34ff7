"""Must-defined SGPRs: every SGPR use that some path from the kernel entry reaches without a write
to that register (e.g. a spill reload in a block a branch can skip, used after the join)."""
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from cfg import parse
F = sys.argv[1]
ENTRY_DEF = set(range(0, int(sys.argv[2]) if len(sys.argv) > 2 else 16))
blocks, succ, pred, reach = parse(F)
ALL = set(range(0, 112))
IN = [set(ALL) for _ in blocks]; OUT = [set(ALL) for _ in blocks]
changed = True
while changed:
    changed = False
    for i in sorted(reach):
        new_in = set(ENTRY_DEF) if i == 0 else (set.intersection(*[OUT[p] for p in pred[i]]) if pred[i] else set())
        s = set(new_in)
        for (_, _, d, _, _) in blocks[i]["ins"]:
            s |= set(d)
        if new_in != IN[i] or s != OUT[i]:
            IN[i], OUT[i] = new_in, s; changed = True
bad = 0
for i in sorted(reach):
    s = set(IN[i])
    for (n, op, d, u, t) in blocks[i]["ins"]:
        miss = [r for r in u if r not in s]
        if miss:
            bad += 1
            print(f"{n}: [{blocks[i]['label']}] uses s{miss} not written on every path: {t}")
        s |= set(d)
print(f"blocks {len(blocks)}, reachable {len(reach)}, SGPR uses not written on every path: {bad}")
