#!/usr/bin/env python3
"""Per-kernel register and scratch use of a built library (gfx950 code
objects in its .hip_fatbin bundles): name, VGPRs, VGPR spills, scratch bytes
per lane.  A row-kernel change is checked with it before it goes to the GPU
(a spill in k_rows_pl is a slowdown the tests do not see).

    python tools/kernel_resources.py parfastaai_amd/lib/libpfaai_hip.so [--filter k_rows_pl] [--spills]
"""
import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
        data = open(fb, "rb").read()
    pos = 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", data, i + len(MAGIC))[0]
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                yield data[i + off:i + off + size]
        pos = i + len(MAGIC)


def kernels(co):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], capture_output=True,
                             text=True).stdout
    cur = {}
    for line in out.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s*(.*)$", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == "args":
            continue
        if k in ("name", "symbol") and k == "name" and "vgpr_count" in cur:
            yield cur
            cur = {}
        cur[k] = v
    if "vgpr_count" in cur:
        yield cur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--filter", default="")
    ap.add_argument("--spills", action="store_true", help="only kernels with VGPR spills or scratch")
    a = ap.parse_args()
    rows = {}
    for co in code_objects(a.lib):
        for k in kernels(co):
            name = k.get("name", "?")
            if a.filter and a.filter not in name:
                continue
            rows[name] = (int(k.get("vgpr_count", 0)), int(k.get("vgpr_spill_count", 0)),
                          int(k.get("private_segment_fixed_size", 0)))
    bad = 0
    for name, (v, sp, scr) in sorted(rows.items()):
        if a.spills and not (sp or scr):
            continue
        bad += bool(sp or scr)
        print(f"{v:4d} vgpr {sp:3d} spill {scr:4d} B scratch  {name}")
    print(f"{len(rows)} kernels, {bad} with spills / scratch", file=sys.stderr)


if __name__ == "__main__":
    main()
