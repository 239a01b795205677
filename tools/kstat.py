"""VGPR / SGPR / scratch / instruction count of kernels in a hipcc -S listing.

    python tools/kstat.py listing.s [name_substring ...]
"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    keys = sys.argv[2:]
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name = m.group(1)
        if keys and not any(k in name for k in keys):
            continue
        seg = s[m.start():]
        end = seg.find(".Lfunc_end")
        if end < 0:
            continue
        body, meta = seg[:end], seg[end:end + 4000]
        g = lambda k: (re.search(k + r": (\d+)", meta) or [None, "?"])[1]
        print(f"{name[:70]:70s} vgpr {g('NumVgprs'):>4} sgpr {g('NumSgprs'):>4} scratch {g('ScratchSize'):>4} "
              f"occ {g('Occupancy'):>2} instr {body.count(chr(10) + chr(9)):6d} scratch_ops {body.count('scratch_')}")


if __name__ == "__main__":
    main()
