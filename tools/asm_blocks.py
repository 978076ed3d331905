"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (for reading hot loops).
    python tools/asm_blocks.py file.s <kernel-symbol-substring> [min_mfma]"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_read", "ds_write", "ds_bpermute", "ds_swizzle")):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    min_mfma = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + sym + r"\w*:", l) or
                 (l.startswith("_Z") and sym in l and l.rstrip().endswith(":") is False and ":" in l and sym in l.split(":")[0]))
    blocks, cur, name = [], Counter(), lines[start].split(":")[0]
    ops = []
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        if re.match(r"^\.LBB\w+:", s):
            blocks.append((name, cur, ops))
            cur, name, ops = Counter(), s.rstrip(":").split()[0], []
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        cur[classify(op)] += 1
        ops.append(op)
    blocks.append((name, cur, ops))
    for name, c, ops in blocks:
        if c["mfma"] >= min_mfma:
            tot = sum(c.values())
            print(f"{name}: total {tot} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
            if "-v" in sys.argv:
                print("   ", Counter(o for o in ops if o.startswith("v_") and not o.startswith("v_mfma")).most_common(30))


if __name__ == "__main__":
    main()
