"""For each ds_bpermute_b32 in a gfx950 .s file, the nearest earlier VALU write of its data VGPR:
prints a histogram of (instructions between, VALU between, s_nop cycles) for v_pk_* producers.
usage: python isa_pk_bpermute.py <file.s>"""
import re, sys, collections
lines = [l.strip() for l in open(sys.argv[1])]
ins = [l for l in lines if l and not l.startswith((";", ".", "//")) and not l.endswith(":")]
def regs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m: return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    if m: return {int(m.group(1))}
    return set()
dist = collections.Counter()
examples = []
for i, l in enumerate(ins):
    if not l.startswith("ds_bpermute_b32"):
        continue
    ops = [o.strip() for o in l.split(None, 1)[1].split(",")]
    data = regs(ops[2])
    for j in range(i - 1, max(-1, i - 12), -1):
        p = ins[j]
        name = p.split()[0]
        if not p.startswith("v_") and not p.startswith("s_nop"):
            continue
        dst = p.split(None, 1)[1].split(",")[0].strip() if " " in p else ""
        if name.startswith("v_") and regs(dst) & data:
            if name.startswith("v_pk_"):
                # count VALU instrs and nops in between
                between = ins[j + 1:i]
                nops = sum(int(re.search(r"s_nop (\d+)", b).group(1)) + 1 for b in between if b.startswith("s_nop"))
                nv = sum(1 for b in between if b.startswith("v_"))
                dist[(len(between), nv, nops)] += 1
                if len(examples) < 8 and len(between) <= 1:
                    examples.append(ins[j:i + 1])
            break
print(sorted(dist.items()))
for e in examples:
    print("----"); print("\n".join(e))
