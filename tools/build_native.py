"""Build recipes for the native pieces (no cmake, no pip).

  hip      parfastaai_amd/lib/libpfaai_hip.so   hipcc --offload-arch=gfx950
  diag     parfastaai_amd/lib/libpfaai_hip_diag.so  the same with -DPFAAI_DIAGNOSTICS
                                                (A/B kernel switches, ablations,
                                                stage clocks, k_rows_v2; the
                                                variant tests load it)
  cli      parfastaai_amd/lib/par_fastaai_amd   g++ host CLI over the C ABI
  syn      tools/_build/libpfaai_syn.so         synthetic DB generator
  rebuild  tools/_build/rebuild_xantho_db       C1 DB from the reference's fixtures
  oracle   oracle/_build/libpfaai_oracle.so     CPU oracle (test infra)
  ref      oracle/_ref/par_fastaai.x            the reference, from its own
                                                sources (only where
                                                /root/reference exists)
  dropin   oracle/_ref/par_fastaai_hip.x        the reference's main.cpp with
                                                INTEGRATION.md §1's swap, linked
                                                to libpfaai_hip.so (tools/dropin.py)
Everything is built in-tree so the snapshot that travels to the GPU box
carries the binaries.
"""
from __future__ import annotations

import os
import time
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # repo root
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PFAAI_ARCH", "gfx950")


def _run(cmd, cwd=ROOT):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


def _newer(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build_hip(force=False, diag=False):
    """libpfaai_hip.so from the translation units of parfastaai_amd/csrc
    (the C-ABI unit and one row-kernel unit per mode), compiled in parallel
    to objects under build/ and linked."""
    csrc = os.path.join(ROOT, "parfastaai_amd/csrc")
    units = sorted(f for f in os.listdir(csrc) if f.endswith(".hip"))
    deps = [os.path.join(csrc, f) for f in os.listdir(csrc)] + [os.path.join(ROOT, "include/pfaai_hip.h")]
    out = os.path.join(ROOT, "parfastaai_amd/lib", "libpfaai_hip_diag.so" if diag else "libpfaai_hip.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    objdir = os.path.join(ROOT, "build", "hip_diag" if diag else "hip")
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-Wall",
             "-I" + os.path.join(ROOT, "include"), *(["-DPFAAI_DIAGNOSTICS"] if diag else [])]
    objs = [os.path.join(objdir, u[:-4] + ".o") for u in units]
    from concurrent.futures import ThreadPoolExecutor

    # an object is rebuilt when its own unit or any shared header is newer
    # (a row-kernel unit takes ~4 min: editing the C-ABI unit alone must not
    # recompile them)
    headers = [d for d in deps if not d.endswith(".hip")]
    # (by object, not by the library: a header edited while an earlier build
    # compiled would otherwise be older than that build's library and never
    # reach the objects compiled before the edit)
    todo = [(u, o) for u, o in zip(units, objs) if force or _newer(o, [os.path.join(csrc, u), *headers])]
    if not todo and not _newer(out, objs):
        return out
    def compile_unit(u, o):
        # the object carries the time its compile STARTED: a header edited
        # while the compile ran is then newer than the object, and the next
        # build compiles the unit again instead of keeping a mixed library
        t0 = time.time()
        _run([HIPCC, *flags, "-c", "-o", o, os.path.join(csrc, u)])
        os.utime(o, (t0, t0))

    with ThreadPoolExecutor(max_workers=max(1, min(len(todo), int(os.environ.get("MAX_JOBS", "8"))))) as ex:
        futs = [ex.submit(compile_unit, u, o) for u, o in todo]
        for f in futs:
            f.result()  # re-raises a failed compile
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs, "-ldl"])
    return out


def build_syn(force=False):
    src = os.path.join(ROOT, "tools/syn_gen.c")
    out = os.path.join(ROOT, "tools/_build/libpfaai_syn.so")
    if force or _newer(out, [src]):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        _run(["gcc", "-O2", "-fPIC", "-shared", "-fopenmp", "-std=c11", "-o", out, src])
    return out


def build_rebuild_tool(force=False):
    src = os.path.join(ROOT, "tools/rebuild_xantho_db.cpp")
    out = os.path.join(ROOT, "tools/_build/rebuild_xantho_db")
    if force or _newer(out, [src, os.path.join(ROOT, "parfastaai_amd/host/sqlite_min.h")]):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-o", out, src, "/lib/x86_64-linux-gnu/libsqlite3.so.0"])
    return out


def build_oracle(force=False):
    src = os.path.join(ROOT, "oracle/pfaai_oracle.c")
    out = os.path.join(ROOT, "oracle/_build/libpfaai_oracle.so")
    if force or _newer(out, [src]):
        _run(["make", "-C", os.path.join(ROOT, "oracle")])
    return out


def build_cli(force=False):
    srcs = [os.path.join(ROOT, "parfastaai_amd/host", f) for f in ("par_fastaai_amd.cpp",)]
    hdrs = [os.path.join(ROOT, "parfastaai_amd/host", f) for f in os.listdir(os.path.join(ROOT, "parfastaai_amd/host"))]
    if not os.path.exists(srcs[0]):
        return None
    out = os.path.join(ROOT, "parfastaai_amd/lib/par_fastaai_amd")
    if force or _newer(out, srcs + hdrs + [os.path.join(ROOT, "include/pfaai_hip.h"),
                                           os.path.join(ROOT, "include/pfaai_hip.hpp")]):
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-fopenmp", "-I" + os.path.join(ROOT, "include"), "-o", out,
              *srcs, "-L" + os.path.join(ROOT, "parfastaai_amd/lib"), "-lpfaai_hip",
              "-Wl,-rpath,$ORIGIN", "/lib/x86_64-linux-gnu/libsqlite3.so.0", "-ldl"])
    return out


def build_ref(force=False):
    """The reference CLI compiled from its own sources under /root/reference
    (oracle/build_ref.sh); skipped where the reference is absent."""
    if not os.path.isdir("/root/reference/src"):
        return None
    out = os.path.join(ROOT, "oracle/_ref/par_fastaai.x")
    if force or not os.path.exists(out):
        _run(["bash", os.path.join(ROOT, "oracle/build_ref.sh")])
    return out


def build_all(force=False):
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=2) as ex:  # the two HIP builds' units compile side by side
        libs = [ex.submit(build_hip, force), ex.submit(build_hip, force, True)]
        outs = [f.result() for f in libs]
    outs += [build_syn(force), build_oracle(force), build_cli(force), build_rebuild_tool(force)]
    try:
        outs.append(build_ref(force))
    except subprocess.CalledProcessError as e:  # the reference build is optional
        print(f"reference build failed: {e}", file=sys.stderr)
    try:  # the reference's main.cpp with INTEGRATION.md §1's swap, over libpfaai_hip.so
        import dropin

        outs.append(dropin.build(force))
    except (subprocess.CalledProcessError, RuntimeError) as e:
        print(f"drop-in build failed: {e}", file=sys.stderr)
    return outs


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
