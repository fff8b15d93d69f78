#!/usr/bin/env python3
"""Register/spill/LDS metadata of the k_march specialisations for a set of
extra compiler flags (experiment triage before a GPU A/B run).

    python tools/kernel_regs.py [-DFOO=1 ...]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
CSRC = REPO / "vpt-spectral-volume-rendering_amd" / "csrc"


def main():
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "k.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17",
                        "-ffp-contract=off", "-fno-slp-vectorize", "--cuda-device-only", "-S",
                        f"-I{REPO / 'include'}", *sys.argv[1:], str(CSRC / "kernels.hip"), "-o", str(out)],
                       check=True, stderr=subprocess.DEVNULL)
        s = out.read_text()
    for m in re.finditer(r"\.name:\s+(_ZN3vpt7k_march\S+)\n((?:\s+\..*\n)+?)\s+\.wavefront_size", s):
        name, meta = m.group(1), m.group(2)
        f = dict(re.findall(r"\.(\w+):\s+(\d+)", meta))
        tpl = re.search(r"k_marchILj(\d)ELb(\d)ELj(\d)ELb(\d)EE", name).groups()
        print(f"k_march<L={tpl[0]},SPEC={tpl[1]},MODE={tpl[2]},MAJ={tpl[3]}> vgpr={f.get('vgpr_count')} "
              f"sgpr={f.get('sgpr_count')} sgpr_spill={f.get('sgpr_spill_count')} "
              f"vgpr_spill={f.get('vgpr_spill_count')}")


if __name__ == "__main__":
    main()
