"""The first pfaai_run after a load against the next ones (device time of
each, eng.timing), 10k all-vs-all: does the first carry a one-time cost, and
is it the load or the idle time before the run?

    python tools/gpu/first_step.py [n] [--busy] [--clock]

Cases (each a list of consecutive run times, ms):
  after_load          load, then 4 runs (rounds 3-4's observation: 7.9, 7.6, 7.4)
  after_idle_<ms>     steady runs, the host sleeps <ms>, then 4 runs
  after_load_spin     load, a ~30 ms torch matmul spin, then 4 runs
  after_idle_spin     steady runs, 200 ms sleep, the spin, then 4 runs
--busy: also keep the GPU busy (torch matmuls, ~50 ms) right before each load
(round 4's test).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parfastaai_amd import _capi, syn  # noqa: E402
from parfastaai_amd.datastruct import ParFAAIData  # noqa: E402

busy = "--busy" in sys.argv
args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 10000
g = syn.generate(n, 100)
ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
eng = _capi.Engine(0)
out = {"busy": busy}


def spin(ms=30.0):
    """Dense matmuls on the context's device for about ms."""
    a = torch.randn(4096, 4096, device="cuda:0")
    t0 = time.time()
    while (time.time() - t0) * 1e3 < ms:
        for _ in range(4):
            a = a @ a
            a = a / a.norm()
        torch.cuda.synchronize()


# --clock: the shader clock (MHz, tools/gpu/clkprobe.hip) measured by a
# 100-us probe on every CU right before each run; runs() then returns
# [ms, MHz] pairs
clock = "--clock" in sys.argv
if clock:
    import ctypes

    _clk = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libclkprobe.so"))
    _wall_mhz = _clk.clkprobe_wall_khz(0) // 1000
    _cus = torch.cuda.get_device_properties(0).multi_processor_count
    _cbuf = torch.zeros(2 * _cus, dtype=torch.int64, device="cuda:0")
    _sink = torch.zeros(256, dtype=torch.float32, device="cuda:0")


def shader_mhz():
    s = torch.cuda.current_stream().cuda_stream
    assert _clk.clkprobe_launch(ctypes.c_void_p(s), _cus, 100, _wall_mhz, ctypes.c_void_p(_cbuf.data_ptr()),
                                ctypes.c_void_p(_sink.data_ptr())) == 0
    torch.cuda.synchronize()
    c = _cbuf.view(-1, 2).cpu().double()
    return round(float((c[:, 0] / (c[:, 1] / _wall_mhz)).median()), 1)


def runs(k=4):
    ts = []
    for _ in range(k):
        mhz = shader_mhz() if clock else None
        eng.timing(reset=True)
        eng.run(0, rows, 0, d)
        _, b, r = eng.timing(reset=True)
        ts.append([round(b + r, 3), mhz] if clock else round(b + r, 3))
    return ts


d = None
for rep in range(2):
    if busy:
        spin(50)
    eng.load(**ds.problem())
    rows, pairs = eng.shape()
    d = eng.alloc(pairs * 8) if d is None else d
    out[f"after_load{rep}"] = runs()
for idle in (20, 200, 1000):
    runs(3)
    time.sleep(idle / 1e3)
    out[f"after_idle_{idle}ms"] = runs()
eng.load(**ds.problem())
spin(30)
out["after_load_spin"] = runs()
runs(3)
time.sleep(0.2)
spin(30)
out["after_idle_spin"] = runs()
print(json.dumps(out), flush=True)
