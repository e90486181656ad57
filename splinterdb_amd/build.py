"""Build the HIP engine in-tree: splinterdb_amd/librf_amd.so (gfx950 only).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU container too.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "librf_amd.so")
LIB_STAMPS = os.path.join(HERE, "librf_amd_stamps.so")  # diagnostics: per-phase clock stamps
SOURCES = ["rf_kernels.hip", "rf_engine.cpp"]
HEADERS = ["rf_device.h", "rf_plan.h", "../../include/rf_amd.h", "../../include/rf_amd_diag.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def source_id():
    """16 hex digits of SHA-256 over the engine's sources and headers: compiled into the
    library (rf_amd_build_id), so a loaded library can be checked against the tree"""
    import hashlib
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def _stale(lib=LIB):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, stamps=False):
    """stamps=True builds the diagnostics library (tools/phase_times.py) with per-phase
    shader-clock stamps compiled into the build kernels."""
    lib = LIB_STAMPS if stamps else LIB
    if not force and not _stale(lib):
        return lib
    objs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + ("_stamps.o" if stamps else ".o"))
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-Wall", "-Wno-unused-function", f'-DRF_AMD_SRC_ID="{source_id()}"',
               "-c", os.path.join(CSRC, src), "-o", obj]
        if stamps:
            cmd.insert(1, "-DRF_PHASE_STAMPS")
        if src.endswith(".cpp"):
            cmd.insert(1, "-x")
            cmd.insert(2, "hip")
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = lib + ".tmp"
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs,
                   check=True)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, stamps="--stamps" in sys.argv))
