"""Per-kernel resource usage (VGPR / AGPR / SGPR / LDS / scratch / occupancy) of one HIP source
for gfx950, from the assembly's kernel descriptors (`hipcc --cuda-device-only -S`, the flags of
mxddp/_build.py).

    python scripts/kres.py mxddp/csrc/mnist_conv_bwd.hip [kernel-name-substring]
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_waits import compile_asm  # noqa: E402


def main():
    src = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    asm = compile_asm(src)
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", asm, re.S):
        name, body = m.group(1), m.group(2)
        if pat not in name:
            continue

        def f(k):
            x = re.search(r"\.amdhsa_" + k + r"\s+(\d+)", body)
            return int(x.group(1)) if x else -1
        vg, ag = f("next_free_vgpr"), f("accum_offset")
        occ = re.search(name.replace("$", r"\$") + r".*?; Occupancy:\s*(\d+)", asm, re.S)
        print(f"{name[:90]:90s} vgpr={vg:4d} accum_off={ag:4d} sgpr={f('next_free_sgpr'):3d} "
              f"lds={f('group_segment_fixed_size'):6d} scratch={f('private_segment_fixed_size'):5d}")
    for m in re.finditer(r"; Kernel info:\n; codeLenInByte.*?\n(?:;.*\n)*?", asm):
        pass


if __name__ == "__main__":
    main()
