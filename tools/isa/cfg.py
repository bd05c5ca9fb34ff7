import re
from collections import defaultdict
def _regs(tok):
    tok = tok.strip()
    m = re.fullmatch(r"s(\d+)", tok)
    if m: return [int(m.group(1))]
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m: return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []
def _ops(s):
    s = s.split(";")[0]
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "[": depth += 1
        if ch == "]": depth -= 1
        if ch == "," and depth == 0: out.append(cur); cur = ""
        else: cur += ch
    if cur.strip(): out.append(cur)
    return [o.strip() for o in out]
NODST = ("s_cbranch", "s_branch", "s_waitcnt", "s_nop", "global_store", "ds_write", "buffer_store", "flat_store",
         "s_endpgm", "s_barrier", "s_cmp", "s_bitcmp", "s_sleep", "s_setprio", "s_trap", "scratch_store",
         "s_sendmsg", "s_setpc", "s_wait")
def parse(F):
    lines = open(F).read().split("\n")
    blocks = []
    cur = {"label": "ENTRY", "ins": [], "succ": [], "fall": True}
    blocks.append(cur)
    def nb(label):
        c = {"label": label, "ins": [], "succ": [], "fall": True}
        blocks.append(c)
        return c
    for n, raw in enumerate(lines, 1):
        t = raw.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", t)
        m2 = re.match(r"^; %bb\.(\d+):", t)
        if m or m2:
            lab = m.group(1) if m else f"%bb.{m2.group(1)}"
            if cur["ins"] or cur["label"] != "ENTRY": cur = nb(lab)
            else: cur["label"] = lab
            continue
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"): continue
        parts = t.split(None, 1)
        op = parts[0]
        ops = _ops(parts[1]) if len(parts) > 1 else []
        defs, uses = [], []
        if op.startswith(NODST) or (op.startswith("global_atomic") and " sc0" not in t and " glc" not in t):
            for o in ops: uses += _regs(o)
        elif ops:
            defs += _regs(ops[0])
            rest = ops[1:]
            if op.startswith(("v_add_co", "v_sub_co", "v_addc_co", "v_subb_co", "v_subrev_co", "v_mad_u64_u32", "v_mad_i64_i32", "v_div_scale")) and rest and _regs(rest[0]):
                defs += _regs(rest[0]); rest = rest[1:]
            for o in rest: uses += _regs(o)
        cur["ins"].append((n, op, defs, uses, t))
        if op == "s_branch":
            cur["succ"].append(ops[0]); cur["fall"] = False; cur = nb(f"after{n}")
        elif op.startswith("s_cbranch"):
            cur["succ"].append(ops[0]); cur = nb(f"after{n}")
        elif op in ("s_endpgm", "s_setpc_b64"):
            cur["fall"] = False; cur = nb(f"after{n}")
    idx = {b["label"]: i for i, b in enumerate(blocks)}
    succ = defaultdict(list)
    for i, b in enumerate(blocks):
        for s in b["succ"]:
            if s in idx: succ[i].append(idx[s])
        if b["fall"] and i + 1 < len(blocks): succ[i].append(i + 1)
    reach = {0}; st = [0]
    while st:
        i = st.pop()
        for j in succ[i]:
            if j not in reach: reach.add(j); st.append(j)
    pred = defaultdict(list)
    for i, ss in succ.items():
        if i in reach:
            for j in ss: pred[j].append(i)
    return blocks, succ, pred, reach
