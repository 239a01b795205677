"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (VALU / LDS / SALU / VMEM).

    python tools/asm_blocks.py listing.s kernel_substring [min_instructions]
"""
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and key in l.split(":")[0])
    name = lines[start].split(":")[0]
    blk, cnt, order = name, {}, [name]
    cnt[name] = dict(v=0, ds=0, s=0, g=0, tot=0)
    for l in lines[start + 1:]:
        l = l.strip()
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            blk = m.group(1)
            order.append(blk)
            cnt[blk] = dict(v=0, ds=0, s=0, g=0, tot=0)
            continue
        if not l or l.startswith(";") or l.startswith("."):
            continue
        op = l.split()[0]
        c = cnt[blk]
        c["tot"] += 1
        k = "v" if op.startswith("v_") else "ds" if op.startswith("ds_") else "s" if op.startswith("s_") else \
            "g" if op.startswith(("global_", "buffer_")) else None
        if k:
            c[k] += 1
    print(name)
    tot = dict(v=0, ds=0, s=0, g=0, tot=0)
    for b in order:
        c = cnt[b]
        for k in tot:
            tot[k] += c[k]
        if c["tot"] >= lo:
            print(f"  {b:14s} " + " ".join(f"{k}={c[k]}" for k in ("tot", "v", "ds", "s", "g")))
    print("  total          " + " ".join(f"{k}={tot[k]}" for k in ("tot", "v", "ds", "s", "g")))


if __name__ == "__main__":
    main()
