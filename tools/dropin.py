"""The reference-side drop-in of INTEGRATION.md §1, applied and built.

swap(main_cpp_text) applies the diff block of INTEGRATION.md §1 (read from
that file, so the documented change and the built one cannot drift apart).

build() writes the swapped reference src/main.cpp into a temporary
directory OUTSIDE this repository (the reference's sources never enter the
tree), compiles it with the reference's own flags and headers (the recipe of
oracle/build_ref.sh) plus include/, links libpfaai_hip.so, deletes the
temporary copy and leaves only the binary oracle/_ref/par_fastaai_hip.x
(git-ignored; travels to the GPU box like oracle/_ref/par_fastaai.x).  Skipped
where /root/reference is absent.  tests/test_gpu_dropin.py runs it.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("PFAAI_REFERENCE", "/root/reference")
OUT = os.path.join(ROOT, "oracle", "_ref", "par_fastaai_hip.x")


def diff_block():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"^## 1\..*?```diff\n(.*?)```", doc, re.S | re.M)
    if not m:
        raise RuntimeError("INTEGRATION.md §1 has no diff block")
    return m.group(1).splitlines()


def swap(src: str) -> str:
    """Apply INTEGRATION.md §1's diff to the text of the reference's main.cpp:
    per hunk (split at '@@' lines), the k-th removed line is replaced by the
    k-th added line; a hunk without removals inserts its added lines after
    its last context line."""
    hunks, cur = [], []
    for ln in diff_block():
        if ln.startswith("@@"):
            hunks.append(cur)
            cur = []
        elif ln.strip():
            cur.append(ln)
    hunks.append(cur)
    for h in hunks:
        minus = [x[1:] for x in h if x.startswith("-")]
        plus = [x[1:] for x in h if x.startswith("+")]
        ctx = [x[1:] for x in h if x.startswith(" ")]
        if minus:
            if len(minus) != len(plus):
                raise RuntimeError("each removed line needs its replacement")
            for o, n in zip(minus, plus):
                if src.count(o) != 1:
                    raise RuntimeError(f"main.cpp must contain {o!r} exactly once")
                src = src.replace(o, n)
        elif plus:
            if not ctx or src.count(ctx[-1]) != 1:
                raise RuntimeError("an insertion needs a unique context line")
            src = src.replace(ctx[-1], ctx[-1] + "\n" + "\n".join(plus))
    return src


def flags():
    return ["-std=c++17", "-fopenmp", f"-I{REF}/include", f"-I{REF}/ext/sqlite", f"-I{REF}/ext/fmt/include",
            f"-I{REF}/ext/CLI11/include", f"-I{REF}/ext/cereal/include", f"-I{ROOT}/include"]


def build(force=False):
    main = os.path.join(REF, "src", "main.cpp")
    if not os.path.exists(main):
        return None
    lib = os.path.join(ROOT, "parfastaai_amd", "lib", "libpfaai_hip.so")
    deps = [lib, os.path.join(ROOT, "include", "pfaai_hip.hpp"), os.path.join(ROOT, "include", "pfaai_dropin.hpp"),
            os.path.join(ROOT, "parfastaai_amd", "host", "scp_db.hpp"), os.path.join(ROOT, "INTEGRATION.md")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(d) <= os.path.getmtime(OUT) for d in deps):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    td = tempfile.mkdtemp(prefix="pfaai_dropin_")
    try:
        src = os.path.join(td, "main_hip.cpp")
        with open(src, "w") as f:
            f.write(swap(open(main).read()))
        cmd = ["g++", "-O2", "-DNDEBUG", *flags(), src, f"{REF}/ext/fmt/src/format.cc",
               "-L" + os.path.dirname(lib), "-lpfaai_hip", "-Wl,-rpath,$ORIGIN/../../parfastaai_amd/lib",
               "/lib/x86_64-linux-gnu/libsqlite3.so.0", "-ldl", "-o", OUT]
        print("+", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    finally:
        shutil.rmtree(td, ignore_errors=True)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
