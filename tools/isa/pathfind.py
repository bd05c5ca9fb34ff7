import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from cfg import parse
from collections import deque
F, L, pat = sys.argv[1], int(sys.argv[2]), sys.argv[3]   # pat: substring of a defining instruction, e.g. "v_writelane_b32 v111, s20, 61"
blocks, succ, pred, reach = parse(F)
tgt = next(i for i, b in enumerate(blocks) if any(x[0] == L for x in b["ins"]))
prev = {0: None}; dq = deque([0])
while dq:
    i = dq.popleft()
    if i == tgt: break
    if any(pat in x[4] for x in blocks[i]["ins"]): continue
    for j in succ[i]:
        if j not in prev: prev[j] = i; dq.append(j)
if tgt not in prev: print("no path avoids it"); sys.exit()
path = []; i = tgt
while i is not None:
    b = blocks[i]; path.append(f"{b['label']}@{b['ins'][0][0] if b['ins'] else '-'}-{b['ins'][-1][0] if b['ins'] else '-'}"); i = prev[i]
print(" <- ".join(path))
