"""Build the in-tree native libraries (gfx950 HIP + host C).

Outputs (git-ignored; the first three travel to the GPU box with the gpurun
snapshot, oracle/_ref/ stays in this container: .gpurunignore lists it):
  dqdk_amd/lib/libdqdk_gpu.so   -- the product: HIP kernels + C ABI (include/dqdk_gpu.h)
  oracle/liboracle.so           -- test-only C restatement (oracle/Makefile)
  build/fetch_xsk_harness       -- test-only C consumer of include/dqdk_gpu.h (tests/c/)
  oracle/_ref/libref_tcpip.so   -- the reference's src/tcpip, built only where /root/reference exists
                                   (test-only checker, like liboracle.so)
  oracle/_ref/libref_tristan.so -- the reference's TRISTAN decode (oracle/ref_tristan.py), same condition
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "dqdk_amd" / "csrc"
LIBDIR = ROOT / "dqdk_amd" / "lib"
BUILD = ROOT / "build"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DQDK_OFFLOAD_ARCH", "gfx950")
REF = Path(os.environ.get("DQDK_REFERENCE", "/root/reference"))

HIP_SRCS = ["rx_kernels.hip", "egress_kernels.hip", "membench.hip", "dqdk_gpu.hip", "frame_processor.hip"]
C_SRCS = ["synth.c"]
HDRS = ["rx_kernels.h", "egress_kernels.h", "queue_internal.h", str(ROOT / "include" / "dqdk_gpu.h")]


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_gpu_lib(force: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    LIBDIR.mkdir(exist_ok=True)
    hdrs = [CSRC / h if not h.startswith("/") else Path(h) for h in HDRS]
    objs = []
    for src in HIP_SRCS:
        s = CSRC / src
        o = BUILD / (s.stem + ".o")
        if force or _stale(o, [s, *hdrs]):
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
                  "-c", str(s), "-o", str(o)])
        objs.append(o)
    for src in C_SRCS:
        s = CSRC / src
        o = BUILD / (s.stem + ".o")
        if force or _stale(o, [s, *hdrs]):
            _run(["gcc", "-O3", "-fPIC", "-std=gnu11", "-Wall", "-pthread", "-c", str(s), "-o", str(o)])
        objs.append(o)
    lib = LIBDIR / "libdqdk_gpu.so"
    if force or _stale(lib, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib),
              *map(str, objs), "-lpthread"])
    return lib


def build_c_harness(lib: Path, force: bool = False) -> Path:
    """tests/c/fetch_xsk_harness.c: a plain C program compiled against
    include/dqdk_gpu.h and linked with libdqdk_gpu.so (test-only)."""
    src = ROOT / "tests" / "c" / "fetch_xsk_harness.c"
    out = BUILD / "fetch_xsk_harness"
    if force or _stale(out, [src, ROOT / "include" / "dqdk_gpu.h", lib]):
        _run(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-I", str(ROOT / "include"), str(src), "-o", str(out),
              "-L", str(LIBDIR), "-ldqdk_gpu", "-Wl,-rpath,$ORIGIN/../dqdk_amd/lib", "-Wl,-rpath,/opt/rocm/lib"])
    return out


def build_oracle(force: bool = False) -> None:
    args = ["make", "-s", "-C", str(ROOT / "oracle")]
    if force:
        _run(args + ["clean"])
    _run(args)
    if (REF / "src" / "tcpip" / "ipv4.c").exists():
        _run(args + ["ref", f"REF={REF}"])
        tri = ROOT / "oracle" / "_ref" / "libref_tristan.so"
        if force or _stale(tri, [REF / "src" / "tristan.c", REF / "src" / "tristan.h", ROOT / "oracle" / "ref_tristan.py"]):
            _run([sys.executable, str(ROOT / "oracle" / "ref_tristan.py"), "--ref", str(REF), "--out", str(tri)])


def build_all(force: bool = False) -> None:
    lib = build_gpu_lib(force)
    build_c_harness(lib, force)
    build_oracle(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
