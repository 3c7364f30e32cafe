"""Issue-slot estimate of a kernel's static VALU mix (hipcc -S listing), using the per-opcode rates
measured on gfx950 by tools/micro/issue_micro.hip (wave64 instructions per SIMD-cycle, 8 waves per
SIMD; profiles/r5_issue_micro.txt): full rate ~0.44 (v_add/sub/xor/or/shifts: 1 slot), half rate
~0.23 (VOP3 integer ops, v_max/min, mul24, mul_lo, bfe, cmp, cndmask, DPP, SDWA, add3, lshl_or,
alignbit, mul_hi, v_mad_i64_i32 / v_mad_u64_u32, f64 fma/mul/add: 2 slots); ffbh ~quarter.
(Round 4's cndmask figure, 0.061, read an uninitialised vcc: with an SGPR-pair mask it is 0.23.)
Usage: python tools/valu_rates.py file.s symbol_substring"""
import re
import sys
from collections import Counter

FULL = re.compile(r"^v_(add|sub|subrev|xor|or|and|lshlrev|lshrrev|ashrrev|mov|not)_(u32|b32|i32|co_u32)(_e32|_e64)?$")
QUARTER = re.compile(r"^v_(ffbh|ffbl|bcnt)")


def slots(op):
    if "_dpp" in op or "_sdwa" in op:
        return 2
    if FULL.match(op):
        return 1
    if QUARTER.match(op):
        return 4
    return 2


def main():
    src, key = sys.argv[1], sys.argv[2]
    lines = open(src).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    ops = [l.strip().split()[0] for l in lines[start:end + 1] if l.startswith("\t") and l.strip().startswith("v_")]
    c = Counter(ops)
    tot = sum(c.values())
    sl = sum(slots(o) * n for o, n in c.items())
    full = sum(n for o, n in c.items() if slots(o) == 1)
    print(f"{key}: {tot} static VALU, {sl} issue slots ({sl / tot:.2f} per instruction), {full / tot:.0%} full rate")
    for o, n in c.most_common(20):
        print(f"  {o:28s} {n:6d}  x{slots(o)}")


if __name__ == "__main__":
    main()
