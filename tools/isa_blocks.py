#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (static cost map).

  python tools/isa_blocks.py build/spt_kernel.s render_kernelINS_4TopoILi6 [--bb] [--min N]

--bb splits at LLVM's '; %bb.N' comments too (fall-through blocks), --min hides blocks with fewer
VALU. `slots` weights each VALU by its issue cost on gfx950 (tools/valu_rates.hip,
profiles/r01_valu_rates.txt): full-rate 1, half-rate 2, transcendental 4.
"""
import re
import sys
from collections import Counter

# Issue cost in VALU slots (one slot = a full-rate wave64 instruction, 2 cycles on a SIMD-32),
# measured by tools/valu_rates.hip (profiles/r01_valu_rates.txt): half-rate ops 2, transcendental 4.
HALF = ("v_mad_u64_u32", "v_mad_i64_i32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24",
        "v_mul_hi_u32_u24", "v_mad_u32_u24", "v_cvt_", "v_perm_b32", "v_bfe_", "v_bfi_b32",
        "v_add3_u32", "v_lshl_add_u32", "v_lshl_or_b32", "v_and_or_b32", "v_or3_b32", "v_med3_",
        "v_xad_u32", "v_pk_", "v_fma_f64", "v_add_f64", "v_mul_f64", "v_lshl_add_u64")
QUARTER = ("v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_", "v_exp_", "v_log_", "v_div_")


def slots(op):
    if op.startswith(QUARTER):
        return 4
    if op.startswith(HALF):
        return 2
    return 1


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


def blocks_of(path, key, bb=False):
    lines = open(path).read().splitlines()
    # mangled kernels by a substring of the name, extern "C" ones by the whole name ("k_philox:")
    start = next(i for i, l in enumerate(lines)
                 if (l.startswith("_Z") and key in l and ":" in l and not l.startswith("\t"))
                 or l.startswith(key))
    blocks, cur = [], None
    for n, l in enumerate(lines[start:]):
        if n == 0 and not l.startswith("_Z"):
            l = "_Z" + l  # an extern "C" entry label starts the first block like a mangled one
        s = l.strip()
        if s == "s_endpgm":
            break
        m = re.match(r"^(\.LBB[^:]+|_Z[^:]+):", s)
        m2 = re.match(r"^; (%bb\.\d+):", s) if bb else None
        if m or m2:
            cur = {"name": (m or m2).group(1)[:24], "valu": 0, "slots": 0, "salu": 0, "smem": 0,
                   "lds": 0, "vmem": 0, "wait": 0, "ops": [], "vops": Counter()}
            blocks.append(cur)
            continue
        if not s or s.startswith((";", ".")) or cur is None:
            continue
        op = s.split()[0]
        c = classify(op)
        if c:
            cur[c] += 1
            cur["ops"].append(op)
            if c == "valu":
                cur["slots"] += slots(op)
                cur["vops"][op] += 1
    return blocks


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path, key = args[0], args[1]
    bb = "--bb" in sys.argv
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 0
    blocks = blocks_of(path, key, bb)
    tot = {k: sum(b[k] for b in blocks) for k in ("valu", "slots", "salu", "smem", "lds", "vmem")}
    print("total", tot, "blocks", len(blocks))
    for b in blocks:
        if b["valu"] < mn:
            continue
        br = [o for o in b["ops"] if o.startswith("s_cbranch") or o == "s_branch"]
        top = ", ".join(f"{k}:{v}" for k, v in b["vops"].most_common(4))
        print(f"{b['name']:24s} valu {b['valu']:4d} slots {b['slots']:4d} salu {b['salu']:3d} "
              f"smem {b['smem']:3d} lds {b['lds']:2d} vmem {b['vmem']:2d}  {' '.join(br)}  [{top}]")


if __name__ == "__main__":
    main()
