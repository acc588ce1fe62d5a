#!/usr/bin/env python3
"""Device-asm statistics for the hot kernels (development aid, CPU only).

    python scripts/isa_stats.py [regex]

Compiles escalator_amd/csrc/esc_kernels.hip for gfx950 to assembly and prints, per
kernel matching `regex` (default k_pod_reduce|k_node_reduce), the register/scratch
footprint and the instruction mix of its hottest loop (the largest basic-block cycle
the assembler labels as a loop header)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "escalator_amd", "csrc")


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else "k_pod_reduce|k_node_reduce")
    out = "/tmp/esc_kernels.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-fast-math", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only",
                    "-S", os.path.join(CSRC, "esc_kernels.hip"), "-o", out], check=True)
    s = open(out).read()
    for name in re.findall(r"^(_Z\S+):", s, re.M):
        demangled = subprocess.run(["c++filt", name], capture_output=True,
                                   text=True).stdout.strip()
        if not pat.search(demangled):
            continue
        i = s.index("\n" + name + ":")
        j = s.index(".Lfunc_end", i)
        body = s[i:j]
        meta = s[j:j + 3000]
        regs = {k: re.search(r"; %s:\s+(\d+)" % k, meta) for k in ("NumVgprs", "NumSgprs")}
        scratch = re.search(r"ScratchSize:\s*(\d+)", meta)
        ins = [ln.strip().split()[0] for ln in body.split("\n")
               if ln.startswith("\t") and not ln.strip().startswith((".", ";"))]
        c = collections.Counter(ins)
        cls = collections.Counter()
        for k, v in c.items():
            cls[k.split("_")[0]] += v
        print(f"== {demangled}")
        print("   static instrs", len(ins), dict(cls.most_common()), "scratch", scratch and scratch.group(1),
              {k: (m.group(1) if m else None) for k, m in regs.items()})
        print("   top:", c.most_common(30))


if __name__ == "__main__":
    main()
