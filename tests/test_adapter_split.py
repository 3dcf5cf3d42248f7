"""The C++ adapter's multi-device row split (include/pfaai_hip.hpp
pfaai::split_rows, used by ParFAAIHipImpl with several devices and by the
CLI's --devices) gives exactly the cuts of parfastaai_amd/shard.py:split_rows
that bench.py's ranks use (with the device's CU count: the round-tail
adjustment) -- one row-cost model on both paths (CPU only: the header's
split is compiled with g++ and no GPU is touched)."""
import os
import subprocess

import pytest

from parfastaai_amd.shard import split_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [(n, parts, ava, cus) for n in (0, 1, 2, 3, 7, 10, 48, 999, 2000, 10000, 40000, 100000, 123457)
         for parts in (1, 2, 3, 4, 7, 8) for ava in (True, False) for cus in (0, 256, 304, 80)]


@pytest.fixture(scope="module")
def split_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("split")
    src = d / "split.cpp"
    src.write_text(r'''
#include "pfaai_hip.hpp"
#include <cstdio>
int main() {
    long long n; int parts, ava, cus;
    while (std::scanf("%lld %d %d %d", &n, &parts, &ava, &cus) == 4) {
        for (auto c : pfaai::split_rows(n, parts, ava != 0, cus)) std::printf("%lld ", (long long)c);
        std::printf("\n");
    }
    return 0;
}
''')
    exe = d / "split"
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{ROOT}/include", "-o", str(exe), str(src), "-lpthread"],
                   check=True)
    return str(exe)


def test_cpp_split_equals_shard_split(split_exe):
    inp = "".join(f"{n} {p} {int(a)} {c}\n" for n, p, a, c in CASES)
    out = subprocess.run([split_exe], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    assert len(out) == len(CASES)
    for (n, parts, ava, cus), line in zip(CASES, out):
        cuts = [int(x) for x in line.split()]
        py = split_rows(n, parts, ava, cus=cus or None)
        assert cuts == [py[0][0]] + [hi for _, hi in py], (n, parts, ava, cus)
        assert cuts[0] == 0 and cuts[-1] == n and all(a <= b for a, b in zip(cuts, cuts[1:]))
