"""Issue cost of a kernel's VALU mix (hipcc -S listing), priced with the per-opcode rates measured on
gfx950 by tools/micro/issue_micro.hip (wave64 instructions per SIMD-cycle at 4-8 waves per SIMD;
profiles/r5_issue_micro.txt):
  full rate  ~0.44 : v_add/sub/xor/or/and/not/mov/shifts (VOP2 or e64)           -> 2.27 SIMD-cycles
  half rate  ~0.235: everything else measured -- VOP3 integer ops, v_max/min, mul24, mul_lo/hi,
                     bfe, cmp, cndmask, DPP, SDWA, add3, lshl_or, alignbit, v_mad_i64_i32,
                     v_mad_u64_u32, f64 fma/mul/add                                  -> 4.26
  quarter    ~0.127: ffbh / ffbl / bcnt                                              -> 7.87
(Round 4's cndmask figure, 0.061, read an uninitialised vcc: with an SGPR-pair mask it is 0.23.)

The listing gives the STATIC mix of the kernel; the inner loops are fully unrolled and a frame runs
its straight-line body once, but uniform dispatches (predictor order, candidate kind) instantiate
several copies of which one runs, so this is an estimate of the dynamic mix, not a count of it.

Usage: python tools/valu_rates.py file.s symbol_substring [--json]
  --json: one line {"kernel", "static_valu", "cycles_per_instr", "full_rate_frac"}"""
import json
import re
import sys
from collections import Counter

FULL = re.compile(r"^v_(add|sub|subrev|xor|or|and|lshlrev|lshrrev|ashrrev|mov|not)_(u32|b32|i32|co_u32)(_e32|_e64)?$")
QUARTER = re.compile(r"^v_(ffbh|ffbl|bcnt)")
CYCLES = {1: 1 / 0.44, 2: 1 / 0.235, 4: 1 / 0.127}


def slots(op):
    if "_dpp" in op or "_sdwa" in op:
        return 2
    if FULL.match(op):
        return 1
    if QUARTER.match(op):
        return 4
    return 2


def mix(src, key):
    lines = open(src).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    ops = [l.strip().split()[0] for l in lines[start:end + 1] if l.startswith("\t") and l.strip().startswith("v_")]
    return Counter(ops)


def main():
    src, key = sys.argv[1], sys.argv[2]
    c = mix(src, key)
    tot = sum(c.values())
    cyc = sum(CYCLES[slots(o)] * n for o, n in c.items())
    full = sum(n for o, n in c.items() if slots(o) == 1)
    if "--json" in sys.argv:
        print(json.dumps({"kernel": key, "static_valu": tot, "cycles_per_instr": round(cyc / tot, 4),
                          "full_rate_frac": round(full / tot, 4)}))
        return
    print(f"{key}: {tot} static VALU, {cyc / tot:.2f} SIMD-cycles per instruction, {full / tot:.0%} full rate")
    for o, n in c.most_common(20):
        print(f"  {o:28s} {n:6d}  x{slots(o)}")


if __name__ == "__main__":
    main()
