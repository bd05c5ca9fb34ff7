"""Must-defined VGPRs (exec masks ignored: a write under any mask counts) at each vector memory
access's address operand: an address VGPR some path reaches without any write is an undefined
address (the compiler's implicit-def)."""
import re, sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from cfg import parse, _ops
F = sys.argv[1]
blocks, succ, pred, reach = parse(F)
def vregs(tok):
    tok = tok.strip()
    m = re.fullmatch(r"v(\d+)", tok)
    if m: return [int(m.group(1))]
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m: return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []
NOVDST = ("global_store", "ds_write", "buffer_store", "flat_store", "s_", "v_cmp", "v_writelane", "v_readlane", "v_readfirstlane")
def vdefs(op, t):
    parts = t.split(None, 1)
    ops = _ops(parts[1]) if len(parts) > 1 else []
    if not ops or op.startswith(NOVDST): return []
    if op.startswith("global_atomic") and " sc0" not in t and " glc" not in t: return []
    if op.startswith("v_writelane"): return []
    return vregs(ops[0])
def addr_uses(op, t):
    parts = t.split(None, 1)
    ops = _ops(parts[1]) if len(parts) > 1 else []
    if op.startswith(("global_load", "global_atomic")): return vregs(ops[1]) if len(ops) > 1 else []
    if op.startswith("global_store"): return vregs(ops[0])
    return []
ALL = set(range(512))
IN = [set(ALL) for _ in blocks]; OUT = [set(ALL) for _ in blocks]
entry = {0, 1}  # workitem id
changed = True
while changed:
    changed = False
    for i in sorted(reach):
        new_in = set(entry) if i == 0 else (set.intersection(*[OUT[p] for p in pred[i]]) if pred[i] else set())
        s = set(new_in)
        for (n, op, d, u, t) in blocks[i]["ins"]:
            s |= set(vdefs(op, t))
        if new_in != IN[i] or s != OUT[i]:
            IN[i], OUT[i] = new_in, s; changed = True
bad = 0
for i in sorted(reach):
    s = set(IN[i])
    for (n, op, d, u, t) in blocks[i]["ins"]:
        miss = [r for r in addr_uses(op, t) if r not in s]
        if miss:
            bad += 1; print(f"{n}: [{blocks[i]['label']}] address v{miss} not written on every path: {t}")
        s |= set(vdefs(op, t))
print("undefined-address uses:", bad, file=sys.stderr)
