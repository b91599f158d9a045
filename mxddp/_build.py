"""In-tree build driver for the mxddp native extension (``mxddp/_C*.so``).

Every ``.hip`` / ``.cpp`` file under ``mxddp/csrc`` is compiled by ``hipcc`` for
``gfx950`` only (no hipify, no dual-platform paths) and linked into ONE pybind11
module.  The module is linked against the HIP runtime and RCCL that ship inside
the installed PyTorch-ROCm wheel (``torch/lib``), so the process ends up with a
single HIP runtime and a single RCCL instance shared with ``torch.distributed``.

Usage::

    python -m mxddp._build            # incremental
    python -m mxddp._build --clean    # full rebuild

The build is incremental (per-object content hash of source + headers + flags)
and parallel (``MAX_JOBS`` or 8 workers).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(os.path.dirname(PKG_DIR), "build", "mxddp")
ARCH = os.environ.get("MXDDP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> str:
    return os.path.join(PKG_DIR, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_lib() -> str:
    # Locate torch/lib without importing torch (import is slow on a cold image).
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("PyTorch is required to build mxddp")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _includes() -> list[str]:
    import pybind11

    return [
        "-I" + CSRC,
        "-I" + pybind11.get_include(),
        "-I" + sysconfig.get_paths()["include"],
        "-I/opt/rocm/include",
    ]


def _common_flags() -> list[str]:
    return [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-munsafe-fp-atomics",  # float atomicAdd -> global_atomic_add_f32 (no CAS loop)
        "-Wno-unused-result",
        "-DMXDDP_ARCH_GFX950=1",
    ]


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


def _sources() -> list[str]:
    srcs = []
    for ext in ("*.hip", "*.cpp"):
        srcs += glob.glob(os.path.join(CSRC, "**", ext), recursive=True)
    return sorted(srcs)


def stamp_path() -> str:
    return ext_path() + ".srcsha"


def source_digest() -> str:
    """Digest of every source and header under csrc plus the compile flags: the built module
    records it (``_C*.so.srcsha``) and ``mxddp.native()`` refuses a module whose digest no
    longer matches the tree (a stale .so shipped to a GPU box after a csrc edit)."""
    h = hashlib.sha256(" ".join(_common_flags()).encode())
    for p in sorted(_sources() + glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)):
        with open(p, "rb") as f:
            h.update(os.path.relpath(p, CSRC).encode())
            h.update(f.read())
    return h.hexdigest()


def is_stale() -> bool:
    try:
        with open(stamp_path()) as f:
            return f.read().strip() != source_digest()
    except OSError:
        return True


def _compile_one(src: str, flags: list[str], hdr_digest: str, force: bool) -> tuple[str, bool]:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    obj = os.path.join(BUILD_DIR, rel + ".o")
    stamp = obj + ".sha"
    with open(src, "rb") as f:
        digest = hashlib.sha256(f.read() + hdr_digest.encode() + " ".join(flags).encode()).hexdigest()
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return obj, False
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + flags + _includes() + lang + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(digest)
    return obj, True


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile + link under an exclusive file lock (several ranks may call native() at once)."""
    import fcntl

    os.makedirs(BUILD_DIR, exist_ok=True)
    with open(os.path.join(BUILD_DIR, ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and os.path.exists(ext_path()) and not is_stale():
            return ext_path()  # another process finished the build while we waited
        return _build_locked(force, verbose)


def _build_locked(force: bool, verbose: bool) -> str:
    flags = _common_flags()
    hdr = _headers_digest()
    srcs = _sources()
    jobs = int(os.environ.get("MAX_JOBS", "8"))
    objs: list[str] = []
    rebuilt = False
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        futs = {ex.submit(_compile_one, s, flags, hdr, force): s for s in srcs}
        for fut in cf.as_completed(futs):
            obj, did = fut.result()
            objs.append(obj)
            rebuilt |= did
            if verbose and did:
                print(f"[mxddp build] compiled {os.path.relpath(futs[fut], PKG_DIR)}", flush=True)
    out = ext_path()
    if rebuilt or force or not os.path.exists(out):
        tlib = _torch_lib()
        # Link against torch's own libamdhip64/librccl (no SONAME there, so the
        # NEEDED entries resolve to the copies torch already loaded).
        # Link with the host compiler: hipcc would put /opt/rocm/lib first and record the
        # versioned SONAMEs (libamdhip64.so.7), pulling a SECOND HIP runtime into the process.
        cmd = [os.environ.get("CXX", "g++"), "-shared", "-fPIC"] + sorted(objs) + [
            "-L" + tlib,
            "-Wl,-rpath," + tlib,
            "-lamdhip64",
            "-lrccl",
            "-o",
            out + ".tmp",
        ]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(out + ".tmp", out)
        if verbose:
            print(f"[mxddp build] linked {os.path.relpath(out, os.path.dirname(PKG_DIR))}", flush=True)
    with open(stamp_path(), "w") as f:
        f.write(source_digest())
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args()
    if a.clean and os.path.isdir(BUILD_DIR):
        shutil.rmtree(BUILD_DIR)
    build(force=a.clean)


if __name__ == "__main__":
    sys.exit(main())
