"""CPU: the Go binding builds with the reference's toolchain, Go 1.9.x
(/root/reference .travis.yml:7-8) -- checked without Go, which the image
lacks: the binding uses no API newer than Go 1.9 (runtime.Pinner, unsafe.Slice
and friends), passes packet arrays only through the C shims of
include/contivcls_go.h, and the shims compile as strict C99 with gcc and link
against the in-tree library (go/shimtest, which runs on the GPU in
test_gpu_go_shims.py)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "contivcls", "contivcls.go")

# API added after Go 1.9, by version: what the binding must not name
POST_19 = [
    r"runtime\.Pinner", r"\.Pin\(", r"unsafe\.Slice", r"unsafe\.Add", r"unsafe\.String", r"unsafe\.SliceData",
    r"strings\.Builder", r"strings\.ReplaceAll", r"strings\.Cut", r"errors\.Is", r"errors\.As",
    r"errors\.Unwrap", r"errors\.Join", r"%w", r"io\.ReadAll", r"os\.ReadFile", r"os\.WriteFile",
    r"math\.MaxInt\b", r"\bany\b", r"sort\.Slice\b.*func\(.*\) bool", r"\[T ", r"min\(", r"max\(",
    r"atomic\.Int", r"atomic\.Uint", r"atomic\.Bool", r"sync\.OnceFunc", r"clear\(",
]


def _code(path):
    """The Go source without comments."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return "\n".join(line.split("//", 1)[0] for line in src.splitlines())


def test_go_binding_uses_only_go19_api():
    code = _code(GO)
    for pat in POST_19:
        assert not re.search(pat, code), pat


def test_go_binding_passes_no_go_pointers_in_go_memory():
    """cgo (Go 1.6+) refuses Go memory holding Go pointers: the SoA records are
    never built in Go -- every packet / connection call goes through a shim."""
    code = _code(GO)
    assert "C.cls_pkt_soa" not in code and "C.cls_conn_soa" not in code
    assert "C.cls_classify(" not in code and "C.cls_connect_batch(" not in code
    for shim in ("clsg_classify_v4", "clsg_classify_v16", "clsg_connect_v4", "clsg_connect_v16",
                 "clsg_engine_create", "clsg_batch_mirror"):
        assert "C." + shim + "(" in code, shim
    assert '#include "contivcls_go.h"' in open(GO).read()


def test_shims_compile_as_c99_and_link():
    out = os.path.join(ROOT, "go", "shimtest", "shimtest_cpu_check")
    try:
        r = subprocess.run(["gcc", "-O1", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                            "-I" + os.path.join(ROOT, "include"), "-o", out,
                            os.path.join(ROOT, "go", "shimtest", "shimtest.c"),
                            "-L" + os.path.join(ROOT, "vpp_amd"), "-lcontivcls",
                            "-Wl,-rpath-link,/opt/rocm/lib"], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    finally:
        if os.path.exists(out):
            os.remove(out)
