"""Symbolic value flow of SGPRs through the spill slots (v_writelane / v_readlane) of an AMDGPU
function: each SGPR (and each spill slot vN:lane) carries the set of values it may hold — a kernel
argument dword 'karg+0xOFF' (s_load from the kernarg pointer s[0:1]), or 'op@line' for anything
computed.  A may-analysis over the CFG (union at joins).  Then every memory access whose address
takes an SGPR pair is listed with the values that pair may hold: a pointer that may hold two
different kernel arguments, or a kernel argument and a computed value, is a clobbered address."""
import re, sys
from collections import defaultdict
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from cfg import parse, _regs, _ops

F = sys.argv[1]
blocks, succ, pred, reach = parse(F)
lines = open(F).read().split("\n")

def ins_effect(n, op, t, state):
    """apply one instruction to state {key: frozenset(values)}; returns uses' values for reporting"""
    parts = t.split(None, 1)
    ops = _ops(parts[1]) if len(parts) > 1 else []
    if op.startswith("s_load_dword") and len(ops) >= 3 and ops[1] == "s[0:1]":
        d = _regs(ops[0]); off = int(ops[2], 0)
        for k, r in enumerate(d):
            state[f"s{r}"] = frozenset([f"karg+{off + 4 * k:#x}"])
        return
    if op == "v_writelane_b32":
        src = _regs(ops[1]); lane = ops[2]
        key = f"{ops[0]}:{lane}"
        state[key] = state.get(f"s{src[0]}", frozenset()) if src else frozenset([f"imm@{n}"])
        return
    if op == "v_readlane_b32":
        d = _regs(ops[0]); key = f"{ops[1]}:{ops[2]}"
        state[f"s{d[0]}"] = state.get(key, frozenset())
        return
    if op in ("s_mov_b32", "s_mov_b64") and _regs(ops[1]):
        d = _regs(ops[0]); s_ = _regs(ops[1])
        for a, b in zip(d, s_):
            state[f"s{a}"] = state.get(f"s{b}", frozenset())
        return
    # any other SGPR definition: a computed value
    for b in blocks_by_line.get(n, []):
        pass
    defs = defs_of.get(n, [])
    for r in defs:
        state[f"s{r}"] = frozenset([f"{op}@{n}"])

defs_of = {}
blocks_by_line = {}
for b in blocks:
    for (n, op, d, u, t) in b["ins"]:
        defs_of[n] = d

def run_block(i, s):
    s = dict(s)
    for (n, op, d, u, t) in blocks[i]["ins"]:
        ins_effect(n, op, t, s)
    return s

def join(a, b):
    out = dict(a)
    for k, v in b.items():
        out[k] = out.get(k, frozenset()) | v
    return out

IN = [None] * len(blocks); OUT = [None] * len(blocks)
entry = {f"s{r}": frozenset([f"entry_s{r}"]) for r in range(0, 16)}
order = sorted(reach)
changed = True
it = 0
while changed:
    changed = False; it += 1
    for i in order:
        new_in = dict(entry) if i == 0 else {}
        for p in pred[i]:
            if OUT[p] is not None:
                new_in = join(new_in, OUT[p])
        if new_in == IN[i] and OUT[i] is not None:
            continue
        IN[i] = new_in
        new_out = run_block(i, new_in)
        if new_out != OUT[i]:
            OUT[i] = new_out; changed = True
print(f"fixpoint after {it} passes", file=sys.stderr)
# report address uses
addr_kinds = ("global_load", "global_store", "global_atomic", "v_lshl_add_u64", "v_mov_b64", "v_add_co_u32", "v_addc_co_u32")
bad = 0
summary = defaultdict(set)
for i in order:
    s = dict(IN[i] or {})
    for (n, op, d, u, t) in blocks[i]["ins"]:
        if op.startswith(addr_kinds):
            parts = t.split(None, 1)
            ops = _ops(parts[1]) if len(parts) > 1 else []
            for o in ops:
                m = re.fullmatch(r"s\[(\d+):(\d+)\]", o)
                if not m: continue
                a, b = int(m.group(1)), int(m.group(2))
                if b != a + 1: continue
                lo, hi = s.get(f"s{a}", frozenset(["?"])), s.get(f"s{b}", frozenset(["?"]))
                kargs_lo = {v for v in lo if v.startswith("karg")}
                summary[(n, o)] = (lo, hi)
                mixed = len(lo) != 1 or len(hi) != 1 or (kargs_lo and any(not v.startswith("karg") for v in lo | hi))
                if mixed:
                    bad += 1
                    print(f"{n}: {t}\n    {o}: lo {sorted(lo)} hi {sorted(hi)}")
        ins_effect(n, op, t, s)
print(f"address SGPR pairs checked: {len(summary)}, ambiguous: {bad}", file=sys.stderr)
if len(sys.argv) > 2:
    for (n, o), (lo, hi) in sorted(summary.items()):
        print(n, o, sorted(lo), sorted(hi))
