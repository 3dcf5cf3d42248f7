#!/usr/bin/env python3
"""Stale-memory check (round 6): fill most of the free device memory with
random bytes, release it to the driver, then run the C3 digest test
(tests/test_gpu_configs.py::test_c3_10k_all_vs_all_and_8way_rowblocks: F+G
load, full run, 8 row blocks, G-only reload) on a fresh context -- a kernel
or load step that read device memory before writing it would see the
garbage instead of zeros or an earlier run's values."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402


def main():
    free, total = torch.cuda.mem_get_info(0)
    n = int(free * 0.5) // 8
    g = torch.Generator(device="cuda:0").manual_seed(7)
    x = torch.randint(-(2 ** 62), 2 ** 62, (n,), dtype=torch.int64, device="cuda:0", generator=g)
    torch.cuda.synchronize()
    print(f"[garbage_c3] filled {n * 8 / 2 ** 30:.1f} GiB of {total / 2 ** 30:.1f} GiB with random bytes", flush=True)
    del x
    torch.cuda.empty_cache()
    import test_gpu_configs as T
    from parfastaai_amd import _capi
    eng = _capi.Engine(0)
    T.test_c3_10k_all_vs_all_and_8way_rowblocks(eng)
    eng.close()
    print("[garbage_c3] C3 digests equal after the garbage fill", flush=True)


if __name__ == "__main__":
    main()
