"""the host code runs clean under AddressSanitizer and
UndefinedBehaviorSanitizer -- the CLI's argument parser, SQLite blob loader,
datastruct and CSV / fmt writer, the C1 rebuild tool and the CPU oracle,
driven by their CPU tests (tools/sanitize.py builds them with
-fsanitize=address,undefined -fno-sanitize-recover=all; any report aborts)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_clean_under_asan_ubsan():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sanitize.py"), "-x"], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert " passed" in r.stdout and "failed" not in r.stdout
