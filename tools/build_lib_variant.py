#!/usr/bin/env python3
"""Build libnfsp with extra compiler flags into tools/bin/libnfsp_<tag>.so (A/B builds of the
whole engine; load one with NFSP_LIB=<path>):

    python tools/build_lib_variant.py <tag> [-DNAME=VALUE ...]
"""
import concurrent.futures as cf
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402


def main():
    tag, extra = sys.argv[1], sys.argv[2:]
    out = os.path.join(REPO, "tools", "bin")
    objdir = os.path.join(out, "obj_" + tag)
    os.makedirs(objdir, exist_ok=True)
    srcs = sorted(f for f in os.listdir(g.CSRC) if f.endswith(".hip"))
    objs = [os.path.join(objdir, s[:-4] + ".o") for s in srcs]
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(lambda so: g._run([g.HIPCC, *g.HIPFLAGS, *g.FILE_FLAGS.get(so[0], []), *extra, "-c",
                                       os.path.join(g.CSRC, so[0]), "-o", so[1]]), zip(srcs, objs)))
    lib = os.path.join(out, f"libnfsp_{tag}.so")
    g._run([g.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, *objs])
    print(lib)


if __name__ == "__main__":
    main()
