"""Per-kernel register / scratch / occupancy report of the gfx950 build (from the compiler's
assembly comments): python tools/kernel_resources.py [extra hipcc flags...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    flags = sys.argv[1:]
    text = ""
    with tempfile.TemporaryDirectory() as d:
        for src in ("kernels.hip", "bpe.hip", "html.hip"):
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only",
                            "-S", *flags, os.path.join(ROOT, "csrc/hip", src), "-o", os.path.join(d, "k.s")],
                           check=True)
            text += open(os.path.join(d, "k.s")).read()
    cur = None
    info = {}
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            info.setdefault(cur, {})
        m = re.match(r"^; (NumVgprs|NumAgprs|ScratchSize|Occupancy|NumSgprs): (\d+)", line)
        if m and cur:
            info[cur][m.group(1)] = int(m.group(2))
    for name, d in info.items():
        if "NumVgprs" not in d:
            continue
        short = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", name)[:40]
        print(f"{short:<42} vgpr={d.get('NumVgprs'):>4} agpr={d.get('NumAgprs', 0):>3} "
              f"sgpr={d.get('NumSgprs', 0):>3} scratch={d.get('ScratchSize'):>4} occ={d.get('Occupancy', '-')}")


if __name__ == "__main__":
    main()
