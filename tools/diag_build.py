"""Diagnostic library builder (never the product): psketch_amd/lib/libpsketch_craft_diag.so, linked
from the product's objects except the named translation units, which are compiled again with
-DCRAFT_STAMPS (s_memrealtime phase stamps, craft_device.h) and any extra defines.

    python tools/diag_build.py craft_sim craft_tile [-DNAME ...] [--out libname.so] [--no-stamps]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402

DIAG = os.path.join(REPO, "psketch_amd", "lib", "libpsketch_craft_diag.so")


def build(stamped=("craft_sim", "craft_tile"), defines=(), out=DIAG, stamps=True):
    ge.build()
    obj = os.path.join(REPO, "psketch_amd", "lib", "obj")
    dobj = os.path.join(REPO, "psketch_amd", "lib", "obj_diag" + "".join("_" + d[2:].lower() for d in defines))
    os.makedirs(dobj, exist_ok=True)
    objs = []
    for src in ge.SOURCES:
        base = os.path.splitext(src)[0]
        if base in stamped:
            o = os.path.join(dobj, base + ".o")
            subprocess.check_call([ge.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                                   *(["-DCRAFT_STAMPS"] if stamps else []), *defines, "-c", os.path.join(ge.CSRC, src), "-o", o])
        else:
            o = os.path.join(obj, base + ".o")
        objs.append(o)
    subprocess.check_call([ge.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    out = DIAG
    if "--out" in args:                  # another diagnostic library name under psketch_amd/lib/
        i = args.index("--out")
        out = os.path.join(REPO, "psketch_amd", "lib", args[i + 1])
        del args[i:i + 2]
    stamps = "--no-stamps" not in args        # an A/B variant of the product: the defines only
    args = [a for a in args if a != "--no-stamps"]
    names = [a for a in args if not a.startswith("-D")]
    build(tuple(names) or ("craft_sim", "craft_tile"), [a for a in args if a.startswith("-D")], out, stamps)
