"""Register / LDS / scratch / occupancy of every gfx950 kernel in a HIP source,
from hipcc's kernel-resource-usage remarks (no GPU needed).

usage: python tools/kernel_resources.py csrc/arnoldi.hip [name-filter]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "icl-mixed-precision-gmres_amd"


def resources(src: str):
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT / 'include'}", f"-I{PKG / 'csrc'}",
           "--cuda-device-only", "-c", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage", src]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    kernels, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            kernels.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(-?\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return kernels


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in resources(src):
        if filt in k["name"]:
            print(f"{k['name'][:70]:70s} vgpr={k.get('VGPRs', '?'):>4} sgpr={k.get('SGPRs', '?'):>4} "
                  f"scratch={k.get('ScratchSize [bytes/lane]', '?'):>4} lds={k.get('LDS Size [bytes/block]', '?'):>6} "
                  f"occ={k.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
