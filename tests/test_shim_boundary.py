"""The drop-in boundary at the reference's own interface (CPU checks).

shim/routing_filter_amd.c replaces vmware/splinterdb's src/routing_filter.c: it must compile
against the reference's src/routing_filter.h (so the compiler checks every prototype), and
define every function that header declares. oracle/_ref/libshim_rf.so is that shim linked
into the reference's own page stack (clockcache, mini_allocator, rc_allocator) and
librf_amd.so; without a HIP device its routing_filter_add must fail with ENODEV -- there is
no CPU fallback. tests/c/abi_smoke is a plain C client of librf_amd.so through
include/rf_amd.h. GPU behaviour of the shim: tests/test_gpu_shim.py.
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT
from oracle import refimpl as R

REF = "/root/reference"
XXH = "/usr/local/lib/python3.10/dist-packages/pyarrow/include/arrow/vendored/xxhash"
SHIM = os.path.join(ROOT, "shim", "routing_filter_amd.c")
need_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference tree absent")


def ref_flags():
    return ["-std=gnu11", "-D_GNU_SOURCE", "-DXXH_STATIC_LINKING_ONLY", "-DSPLINTERDB_PLATFORM_DIR=platform_linux",
            f"-I{XXH}", f"-I{REF}/include", f"-I{REF}/src", f"-I{REF}/src/platform_linux",
            f"-I{ROOT}/include", f"-I{ROOT}/shim"]


def declared_functions():
    """non-inline functions src/routing_filter.h declares (what a replacement must define)"""
    src = open(os.path.join(REF, "src", "routing_filter.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = set()
    for m in re.finditer(r"(?m)^([A-Za-z_][\w \*]*)\n(routing_filter_\w+)\(", src):
        if "static" not in m.group(1):
            out.add(m.group(2))
    # DEFINE_ASYNC_STATE(...) is followed by the coroutine's own prototype
    return sorted(out)


@need_ref
def test_shim_compiles_against_reference_header():
    """-Werror: a signature that differs from routing_filter.h's is a conflicting-types error,
    and every call into the reference's cache / mini_allocator / iterator API is checked"""
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-Wno-sign-compare"] + ref_flags() + [SHIM], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


@need_ref
def test_shim_defines_every_declared_function():
    decl = declared_functions()
    assert {"routing_filter_add", "routing_filter_lookup", "routing_filter_lookup_async",
            "routing_filter_dec_ref", "routing_filter_inc_ref", "routing_filter_estimate_unique_fp",
            "routing_filter_estimate_unique_keys", "routing_filter_estimate_unique_keys_from_count",
            "routing_filter_space_use_bytes", "routing_filter_verify", "routing_filter_print"} <= set(decl)
    tmp = os.path.join(ROOT, "oracle", "_ref", "shim_check.o")
    os.makedirs(os.path.dirname(tmp), exist_ok=True)
    r = subprocess.run(["gcc", "-c", "-O2", "-fPIC", "-o", tmp] + ref_flags() + [SHIM],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    nm = subprocess.run(["nm", "--defined-only", tmp], capture_output=True, text=True).stdout
    os.unlink(tmp)
    defined = set(re.findall(r" T (\w+)", nm))
    missing = [f for f in decl if f not in defined]
    assert not missing, missing


@pytest.mark.skipif(not R.available(R.SHIM_PATH), reason="oracle/_ref/libshim_rf.so not built")
def test_shim_library_has_no_cpu_fallback():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a HIP device is present")
    s = R.Stack(path=R.SHIM_PATH)
    with pytest.raises(RuntimeError, match="platform_status 19"):
        s.add([1, 2, 3])
    s.close()


def test_c_client_links_librf_amd():
    """a C program (not ctypes) built against include/rf_amd.h and linked with librf_amd.so"""
    exe = os.path.join(ROOT, "tests", "c", "abi_smoke")
    if not os.path.exists(exe):
        subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", f"-I{ROOT}/include",
                        os.path.join(ROOT, "tests", "c", "abi_smoke.c"), f"-L{ROOT}/splinterdb_amd",
                        "-l:librf_amd.so", "-Wl,-rpath,$ORIGIN/../../splinterdb_amd", "-o", exe], check=True)
    import torch
    args = [exe] + (["--expect-gpu"] if torch.cuda.device_count() > 0 else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_smoke:" in r.stdout
