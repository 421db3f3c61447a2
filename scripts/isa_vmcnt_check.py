"""Static check of compiled HIP kernels: count `s_waitcnt vmcnt(N)` placed directly before an MFMA.

Such a wait inside a main loop usually means the compiler could not prove that an earlier global load
(e.g. operands loaded before the loop) has retired, and so drains the loop's own prefetch loads before
every MFMA, exposing their latency each iteration. Usage: python scripts/isa_vmcnt_check.py csrc/kernels/x.hip ...
(cross-compiles for gfx950 with --save-temps into a temporary directory; no GPU needed).
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def check(src):
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/csrc/kernels", "-c",
                        os.path.abspath(src), "-o", "k.o", "--save-temps"], cwd=d, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
        s = open(os.path.join(d, asm)).read()
    out = []
    for name in re.findall(r"^(_Z\w+):", s, re.M):
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        lines = [l.strip() for l in s[i:j].split("\n") if l.strip() and not l.strip().startswith(";")]
        hits = sum(1 for k, l in enumerate(lines)
                   if l.startswith("s_waitcnt") and "vmcnt(" in l and "mfma" in " ".join(lines[k + 1:k + 3]))
        nm = sum(1 for l in lines if "mfma" in l)
        if nm:
            out.append((hits, nm, name))
    return out


if __name__ == "__main__":
    for src in sys.argv[1:]:
        for hits, nm, name in check(src):
            print(f"{hits:4d} vmcnt-before-mfma / {nm:5d} mfma  {name[:110]}")
