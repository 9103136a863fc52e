"""Static instruction mix of one kernel in a hipcc -S (gfx950) listing.

  python tools/isa_mix.py FILE.s SUBSTRING

Counts v_*_f64 (FP64 VALU), other v_* (non-FP64 VALU), s_*, ds_*, global/buffer
memory instructions of the first kernel whose symbol contains SUBSTRING, plus
the .vgpr/.sgpr counts.  Static counts (each instruction once, loops not
expanded): a guide to what the unrolled levels issue, not a profile."""
import re
import sys
from collections import Counter


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and ":" in l
                 and sub in l.split(":")[0])
    name = lines[start].split(":")[0]
    c = Counter()
    ops = Counter()
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        ops[op] += 1
        if op.startswith("v_"):
            c["valu_f64" if "_f64" in op else "valu_other"] += 1
        elif op.startswith("s_"):
            c["salu/smem/ctl"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        else:
            c["other"] += 1
    txt = "\n".join(lines)
    m = re.search(r"\.name:\s+%s\n" % re.escape(name), txt)
    print(name)
    for k in ("valu_f64", "valu_other", "salu/smem/ctl", "lds", "vmem", "other"):
        print("  %-14s %6d" % (k, c[k]))
    for k in re.findall(r"^\s*\.(?:vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count):\s+\d+", txt[m.start():m.start() + 3000] if m else "", re.M)[:4]:
        print("  " + k.strip())
    print("  top non-FP64 VALU:", ", ".join("%s %d" % (o, n) for o, n in ops.most_common()
                                            if o.startswith("v_") and "_f64" not in o)[:400])


if __name__ == "__main__":
    main()
