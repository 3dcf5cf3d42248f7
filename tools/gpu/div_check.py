"""Exhaustive check of the row kernels' fp64 division refinements vs IEEE '/'
(PFAAI_DIV_NEWTON = 0, 1, 2 Newton steps) over 1 <= c <= 65535, c <= d < 2^17."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402,F401
from parfastaai_amd import _capi  # noqa: E402

eng = _capi.Engine(0)
for ns in sys.argv[1:] or ["2", "1", "0"]:
    os.environ["PFAAI_DIV_NEWTON"] = ns
    t0 = time.time()
    print(f"newton={ns} mismatches={eng.debug_div_check(65535, (1 << 17) - 1)} ({time.time() - t0:.1f}s)", flush=True)
