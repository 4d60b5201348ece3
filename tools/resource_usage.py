"""Per-kernel register / scratch / LDS use of libspx's device code, from the
compiler's resource-usage remarks (diagnostic; not part of the product).

usage: python tools/resource_usage.py [OUT]   (default: print)
Compiles spx_capi.hip for gfx950 device-only with -Rpass-analysis=kernel-resource-usage
(the build's own flags) and tabulates the window kernels at K = 24 plus the
single-pivot kernels.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "simplex-solver_amd", "csrc", "spx_capi.hip")
KEYS = ["VGPRs", "AGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize",
        "Occupancy", "LDS Size"]


def main():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-ffp-contract=off", "--cuda-device-only", "-c", "-mllvm",
           "-amdgpu-kernarg-preload-count=8", "-Rpass-analysis=kernel-resource-usage", SRC,
           "-o", "/tmp/spx_ru.o"]
    txt = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    rows, cur = {}, None
    for line in txt.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[-Rpass", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = m.group(2)
    demangled = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True,
                               text=True).stdout.splitlines()
    out = ["kernel | " + " | ".join(KEYS)]
    for (mangled, d), name in zip(rows.items(), demangled):
        short = name.split("(")[0].replace("spx::", "")
        if "<24" not in short and "<" in short:
            continue
        out.append(short + " | " + " | ".join(d.get(k, "-") for k in KEYS))
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
