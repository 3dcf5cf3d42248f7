"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

Builds, into tools/_build/san/, with -fsanitize=address,undefined:
  par_fastaai_amd       the drop-in CLI's host path: argument parser, SQLite
                        loader (blob parsing, host/scp_db.hpp), datastruct,
                        CSV writer and fmt-exact double formatting
                        (host/output.hpp); it links the release
                        libpfaai_hip.so, which is not instrumented
  rebuild_xantho_db     the C1 DB rebuild tool (tools/rebuild_xantho_db.cpp)
  libpfaai_oracle.so    the CPU oracle (oracle/pfaai_oracle.c)
then runs the CPU tests that drive them -- tests/test_cli_host.py,
tests/test_c1_loader.py, tests/test_oracle.py, tests/test_zero_overlap.py --
against those builds (PFAAI_CLI / PFAAI_REBUILD_TOOL / PFAAI_ORACLE_LIB; the
oracle is dlopen'ed by Python, so libasan is preloaded into the interpreter).
Any sanitizer report aborts the process that hit it (halt_on_error,
-fno-sanitize-recover), which fails its test.

    python tools/sanitize.py          # exit status = pytest's
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_build", "san")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
TESTS = ["tests/test_cli_host.py", "tests/test_c1_loader.py", "tests/test_oracle.py", "tests/test_zero_overlap.py"]


def _newer(out, srcs):
    return not os.path.exists(out) or any(os.path.getmtime(s) > os.path.getmtime(out) for s in srcs)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=ROOT, check=True)


def build():
    os.makedirs(OUT, exist_ok=True)
    host = os.path.join(ROOT, "parfastaai_amd", "host")
    lib = os.path.join(ROOT, "parfastaai_amd", "lib")
    cli = os.path.join(OUT, "par_fastaai_amd")
    srcs = [os.path.join(host, f) for f in os.listdir(host)] + [os.path.join(ROOT, "include", f) for f in
                                                                 ("pfaai_hip.h", "pfaai_hip.hpp")]
    if _newer(cli, srcs):
        _run(["g++", "-std=c++17", *SAN, "-fopenmp", "-I" + os.path.join(ROOT, "include"), "-o", cli,
              os.path.join(host, "par_fastaai_amd.cpp"), "-L" + lib, "-lpfaai_hip", "-Wl,-rpath," + lib,
              "/lib/x86_64-linux-gnu/libsqlite3.so.0", "-ldl"])
    tool = os.path.join(OUT, "rebuild_xantho_db")
    src = os.path.join(ROOT, "tools", "rebuild_xantho_db.cpp")
    if _newer(tool, [src, os.path.join(host, "sqlite_min.h")]):
        _run(["g++", "-std=c++17", *SAN, "-o", tool, src, "/lib/x86_64-linux-gnu/libsqlite3.so.0"])
    orc = os.path.join(OUT, "libpfaai_oracle.so")
    src = os.path.join(ROOT, "oracle", "pfaai_oracle.c")
    if _newer(orc, [src]):
        _run(["gcc", "-std=c11", "-fPIC", "-shared", "-fno-fast-math", "-ffp-contract=off", *SAN, "-o", orc, src])
    return cli, tool, orc


def main(argv):
    cli, tool, orc = build()
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    ubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, PFAAI_CLI=cli, PFAAI_REBUILD_TOOL=tool, PFAAI_ORACLE_LIB=orc,
               # python itself is not instrumented: only the preloaded runtimes, no leak report for the
               # interpreter; every report is fatal
               LD_PRELOAD=" ".join(x for x in (asan, ubsan, os.environ.get("LD_PRELOAD", "")) if x),
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", *TESTS, *argv],
                       cwd=ROOT, env=env)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
