#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (static cost map).

  python tools/isa_blocks.py build/spt_kernel.s render_kernelINS_4TopoILi6
"""
import re
import sys


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_load") or op.startswith("s_buffer") or op == "s_memtime":
        return "smem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return None


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l and ":" in l and not l.startswith("\t"))
    blocks, cur = [], None
    for l in lines[start:]:
        s = l.strip()
        if s == "s_endpgm":
            break
        m = re.match(r"^(\.LBB[^:]+|_Z[^:]+):", s)
        if m:
            cur = {"name": m.group(1), "valu": 0, "salu": 0, "smem": 0, "lds": 0, "vmem": 0,
                   "wait": 0, "ops": []}
            blocks.append(cur)
            continue
        if not s or s.startswith((";", ".")) or cur is None:
            continue
        op = s.split()[0]
        c = classify(op)
        if c:
            cur[c] += 1
            cur["ops"].append(op)
    tot = {k: sum(b[k] for b in blocks) for k in ("valu", "salu", "smem", "lds", "vmem")}
    print("total", tot, "blocks", len(blocks))
    for b in blocks:
        br = [o for o in b["ops"] if o.startswith("s_cbranch") or o == "s_branch"]
        print(f"{b['name']:24s} valu {b['valu']:4d} salu {b['salu']:3d} smem {b['smem']:3d} "
              f"lds {b['lds']:2d} vmem {b['vmem']:2d}  {' '.join(br)}")


if __name__ == "__main__":
    main()
