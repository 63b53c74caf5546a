"""Instruction mix per basic block of one kernel in a hipcc -S listing.

    python tools/isa_loop.py x6.s <kernel-symbol-substring> [min_mfma]

Prints, for each block with at least min_mfma MFMAs (default 16), its label, whether
a branch jumps back to it (a loop), and the counts of MFMA, other VALU, LDS, global /
buffer, scalar and wait instructions: the VALU-per-MFMA of the main loop without a
counter run.
"""
import re
import sys


def blocks(lines):
    cur, body = "entry", []
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            if re.match(r"^\.LBB\S+:", s):
                pass
            else:
                continue
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            yield cur, body
            cur, body = m.group(1), []
            continue
        body.append(s.split(";")[0].strip())
    yield cur, body


def classify(ins):
    op = ins.split()[0] if ins else ""
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, sym, min_mfma=16):
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*:", l) and sym in l)
    end = next(i for i in range(start + 1, len(text)) if text[i].strip().startswith(".Lfunc_end"))
    body = text[start + 1:end]
    targets = {}
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if m:
            targets.setdefault(m.group(1) or m.group(2), []).append(i)
    pos = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l.strip())
        if m:
            pos[m.group(1)] = i
    tot = {}
    for name, ins in blocks(body):
        c = {}
        for x in ins:
            k = classify(x)
            c[k] = c.get(k, 0) + 1
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        if c.get("mfma", 0) >= min_mfma:
            loop = any(j > pos.get(name, 1 << 30) for j in targets.get(name, []))
            vm = c.get("valu", 0)
            print(f"{name:14s} loop={int(loop)} mfma={c.get('mfma', 0):4d} valu={vm:4d} "
                  f"({vm / c['mfma']:.2f}/mfma) lds={c.get('lds', 0):3d} vmem={c.get('vmem', 0):3d} "
                  f"salu={c.get('salu', 0):3d} wait={c.get('wait', 0):3d} bar={c.get('barrier', 0)}")
    print("kernel total:", tot)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 16)
