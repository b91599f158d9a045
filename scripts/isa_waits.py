"""Where do a kernel's loads get waited for?  Compiles one HIP source for gfx950 to assembly
(`hipcc --cuda-device-only -S`, the flags of mxddp/_build.py) and prints, per kernel, a compressed
sequence of its global loads (G), vector-memory waits (W:vmcnt(N)), MFMAs (M), barriers (B) and
branches (J).  A `G.. W:vmcnt(0) M..` run inside a loop means the stage's prefetch is waited for
before the current stage's MFMAs -- the pattern that cost the ResNet-50 weight gradient 1-2 %
(docs/ROUND5.md, profiles/r5_wgload/).

    python scripts/isa_waits.py mxddp/csrc/nhwc_bf16.hip [kernel-name-substring]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mxddp import _build  # noqa: E402


def compile_asm(src: str) -> str:
    flags = [f for f in _build._common_flags() if f != "-c"]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        r = subprocess.run([_build.HIPCC] + flags + _build._includes() + ["--cuda-device-only", "-S", src, "-o", out],
                           capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr[-2000:])
        with open(out) as f:
            return f.read()


def summarise(body: str) -> str:
    seq = []
    for line in body.splitlines():
        line = line.strip()
        if not line or line.startswith(";"):
            continue
        op = line.split()[0]
        if line.endswith(":"):
            seq.append("L")
        elif op == "s_waitcnt" and "vmcnt" in line:
            seq.append("W:" + re.search(r"vmcnt\(\d+\)", line).group(0))
        elif op.startswith(("global_load", "buffer_load")):
            seq.append("G")
        elif op.startswith("v_mfma"):
            seq.append("M")
        elif op == "s_barrier":
            seq.append("B")
        elif op.startswith("s_cbranch") or op == "s_branch":
            seq.append("J")
    out, prev, n = [], None, 0
    for s in seq + [None]:
        if s == prev:
            n += 1
            continue
        if prev is not None:
            out.append(prev + (str(n) if n > 1 else ""))
        prev, n = s, 1
    return re.sub(r"(L J ?)+", "", " ".join(out))


def main():
    src = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    asm = compile_asm(src)
    for m in re.finditer(r"^(_Z\S+):", asm, re.M):
        sym = m.group(1)
        if pat not in sym:
            continue
        body = asm[m.end():asm.find(".Lfunc_end", m.end())]
        print(sym)
        print("   ", summarise(body))


if __name__ == "__main__":
    main()
