"""Generate the 2^(k/128) table of the exp restatement in csrc/gp_libm.h (glibc 2.35 sysdeps/ieee754/dbl-64/e_exp.c
with EXP_TABLE_BITS = 7, the ARM optimized-routines algorithm): for k in [0, 128)
    H_k = RN(2^(k/128)),  tail_k = RN(2^(k/128) / H_k - 1),  tab[2k] = bits(tail_k),  tab[2k+1] = bits(H_k) - (k << 45).
Computed here in 60-digit decimal arithmetic; tests/test_libm_cpu.py pins the result against the C library's exp.
"""
import struct
from decimal import Decimal, getcontext

getcontext().prec = 60


def rn(x: Decimal) -> float:
    return float(x)  # Decimal -> nearest double (correctly rounded)


def bits(f: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", f))[0]


def table():
    out = []
    for k in range(128):
        v = Decimal(2) ** (Decimal(k) / Decimal(128))
        h = rn(v)
        tail = rn(v / Decimal(h) - 1)
        out += [bits(tail), (bits(h) - (k << 45)) & (2 ** 64 - 1)]
    return out


if __name__ == "__main__":
    t = table()
    for i in range(0, 256, 4):
        print("    " + ", ".join(f"0x{x:016x}ull" for x in t[i:i + 4]) + ",")
