"""Build recipe for the native artefacts (no cmake/ninja needed).

    libvptmcm.so      hipcc, gfx950: HIP kernels + C-ABI (include/vptmcm.h), links RCCL
    vptmcm_napi.node  gcc: Node N-API shim over the C-ABI (host stays JavaScript)
    libvptsynth.so    gcc: synthetic benchmark volume generator
    oracle/liboracle.so  gcc: the CPU oracle (test infrastructure, built as the checker)

Everything lands in-tree under vpt-spectral-volume-rendering_amd/lib/ (git-ignored,
but shipped to the GPU box by gpurun's snapshot).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
LIB = PKG / "lib"
# tools/variants.py A/B builds: outside the package, so lib/ holds the product only
VARIANTS = REPO / "build" / "variants"
CSRC = PKG / "csrc"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = "gfx950"

# -ffp-contract=off and the default (correctly rounded) f32 div/sqrt are part of
# the arithmetic specification; never add -ffast-math here.
# -fno-slp-vectorize: gfx950's packed f32 ops (v_pk_add/mul_f32) issue at the
# same lane rate as two scalar ops, so SLP packing only adds v_mov shuffles
# (measured: march 8 % faster without it; results are identical either way).
HIP_FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-ffp-contract=off", "-fPIC",
             "-fno-slp-vectorize", "-Wall", "-Wno-unused-command-line-argument"]


def _run(cmd: list[str], cwd: Path | None = None) -> None:
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True, cwd=cwd)


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_hip(force: bool = False) -> Path:
    out = LIB / "libvptmcm.so"
    srcs = [CSRC / "kernels.hip", CSRC / "vptmcm.cpp"]
    deps = srcs + [CSRC / "kernels.h", CSRC / "march.h", CSRC / "mcm_device.h", CSRC / "stamp.h",
                   REPO / "include" / "vptmcm.h"]
    if force or _stale(out, deps):
        hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
        LIB.mkdir(parents=True, exist_ok=True)
        _run([hipcc, *HIP_FLAGS, "-shared", f"-I{REPO / 'include'}", *srcs, "-o", out,
              "-lrccl", f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}"])
    return out


# Debug builds the GPU tests load (tests/test_gpu_guard.py): guard zones and
# poisoned allocations / LDS with two poison bytes, volume-gather bounds flags
# (csrc/kernels.hip, VPT_GUARD). Test infrastructure, never the product.
GUARD_VARIANTS = {"guard": ["-DVPT_GUARD=1"], "guardff": ["-DVPT_GUARD=1", "-DVPT_POISON=0xFFu"]}


def build_guard(force: bool = False) -> list[Path]:
    from concurrent.futures import ThreadPoolExecutor
    srcs = [CSRC / "kernels.hip", CSRC / "vptmcm.cpp"]
    deps = srcs + [CSRC / "kernels.h", CSRC / "march.h", CSRC / "mcm_device.h", CSRC / "stamp.h",
                   REPO / "include" / "vptmcm.h"]
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    VARIANTS.mkdir(parents=True, exist_ok=True)

    def one(item):
        name, flags = item
        out = VARIANTS / f"libvptmcm_{name}.so"
        if force or _stale(out, deps):
            _run([hipcc, *HIP_FLAGS, *flags, "-shared", f"-I{REPO / 'include'}", *srcs, "-o", out,
                  "-lrccl", f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}"])
        return out
    with ThreadPoolExecutor(len(GUARD_VARIANTS)) as ex:
        return list(ex.map(one, GUARD_VARIANTS.items()))


def build_napi(force: bool = False) -> Path | None:
    out = LIB / "vptmcm_napi.node"
    src = PKG / "napi" / "vptmcm_napi.c"
    node_inc = Path("/usr/include/node")
    if not src.exists() or not (node_inc / "node_api.h").exists():
        print("skip N-API addon (no node headers)")
        return None
    deps = [src, REPO / "include" / "vptmcm.h", LIB / "libvptmcm.so"]
    if force or _stale(out, deps):
        _run(["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-Wall", f"-I{node_inc}",
              f"-I{REPO / 'include'}", src, "-o", out, f"-L{LIB}", "-lvptmcm",
              "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{ROCM / 'lib'}"])
    return out


def build_synth(force: bool = False) -> Path:
    out = LIB / "libvptsynth.so"
    src = PKG / "tools" / "vptsynth.c"
    if force or _stale(out, [src]):
        LIB.mkdir(parents=True, exist_ok=True)
        _run(["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-Wall", src, "-o", out, "-lm",
              "-lpthread"])
    return out


def build_oracle(force: bool = False) -> Path:
    """The CPU oracle is test infrastructure; it is built here only as the checker."""
    odir = REPO / "oracle"
    args = ["make", "-C", odir, "-s"]
    if force:
        args.insert(1, "-B")
    _run(args)
    return odir / "liboracle.so"


def clean_stale_variants() -> None:
    """lib/ holds the product library only: A/B builds that older rounds left
    there (libvptmcm_<name>.so) are removed (variants now live in build/variants/)."""
    for p in LIB.glob("libvptmcm_*.so"):
        print(f"remove stale variant {p}", flush=True)
        p.unlink()


def build_all(force: bool = False) -> None:
    from concurrent.futures import ThreadPoolExecutor
    clean_stale_variants()
    with ThreadPoolExecutor(2) as ex:  # the product and the guard builds compile at once
        guard = ex.submit(build_guard, force)
        build_hip(force)
        guard.result()
    build_synth(force)
    build_napi(force)
    build_oracle(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
