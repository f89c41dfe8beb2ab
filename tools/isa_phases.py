"""Static instruction mix between the s_memtime stamps of a GP_STAMPS build's fused kernel.

    python tools/isa_phases.py [OK] [QPT] [STG]   (compiles csrc/grid.hip -S with -DGP_STAMPS)
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ok, qpt = (sys.argv[1] if len(sys.argv) > 1 else "0"), (sys.argv[2] if len(sys.argv) > 2 else "2")
stg = sys.argv[3] if len(sys.argv) > 3 else "1"  # 1 = the LDS-staged variant (the headline kernel)
out = "/tmp/grid_stamps.s"
if not os.environ.get("ISA_REUSE"): subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O3", "-DGP_STAMPS", "-I",
                os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                os.path.join(ROOT, "gym-po-taxi_amd", "csrc", "grid.hip"), "-o", out], check=True,
               stderr=subprocess.DEVNULL)
s = open(out).read()
name = f"_ZN12_GLOBAL__N_118grid_rollout_numpyILi{ok}ELi{qpt}ELi4ELb{stg}EEEvNS_7GridDevEiPKiPvPfPhS6_"
i = s.index(name + ":")
j = s.index(".amdhsa_kernel " + name, i)
lines = s[i:j].split("\n")
c = collections.Counter()
seg = 0
def dump(tag):
    v = sum(n for k, n in c.items() if k.startswith("v_"))
    sa = sum(n for k, n in c.items() if k.startswith("s_"))
    lds = sum(n for k, n in c.items() if k.startswith("ds_"))
    gm = sum(n for k, n in c.items() if k.startswith(("global_", "buffer_")))
    top = ", ".join(f"{k}:{n}" for k, n in c.most_common(10))
    print(f"[{tag}] VALU {v} SALU {sa} LDS {lds} GMEM {gm} | {top}")
for ln in lines:
    t = ln.strip()
    if t.startswith(("s_memtime", "s_memrealtime")):
        dump(f"before stamp #{seg}")
        seg += 1
        c = collections.Counter()
        continue
    m = re.match(r"([sv]_[a-z0-9_]+|ds_[a-z0-9_]+|global_[a-z0-9_]+|buffer_[a-z0-9_]+)", t)
    if m:
        c[m.group(1)] += 1
dump("tail")
