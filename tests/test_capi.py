"""The C-ABI library builds, loads and exports every symbol include/pfaai_hip.h
declares (CPU only: no compute calls)."""
import ctypes
import os
import re

import pytest

from parfastaai_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "pfaai_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(pfaai_\w+)\s*\(", src, re.M)))


def test_header_lists_exports():
    assert header_functions() == sorted(_capi.EXPORTS)


def test_library_exports_every_symbol():
    lib = _capi.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_abi_version():
    # the header, the binding and the library agree (__graft_entry__.build() asserts the last two)
    import re

    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "pfaai_hip.h")).read()
    v = int(re.search(r"#define PFAAI_ABI_VERSION (\d+)", hdr).group(1))
    assert v == _capi.ABI_VERSION == _capi.load_library().pfaai_version() == 6


def test_problem_struct_layout():
    # pfaai_problem: 6 x int32, int64, 9 pointers
    assert ctypes.sizeof(_capi.Problem) == 6 * 4 + 8 + 9 * 8


def test_no_silent_cpu_fallback_without_gpu():
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(_capi.PfaaiError):
        _capi.Engine(0)
    # the multi-device group: no device -> a HIP error, never a host fallback;
    # an empty device list is refused before the runtime is asked
    with pytest.raises(_capi.PfaaiError) as e:
        _capi.Group([0])
    assert e.value.code == 4  # PFAAI_RC_HIP
    with pytest.raises(_capi.PfaaiError) as e:
        _capi.Group([])
    assert e.value.code == 7  # PFAAI_RC_INVALID


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "parfastaai_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                txt = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "import oracle" not in txt and "pfaai_oracle" not in txt, f


AB_SWITCHES = (b"PFAAI_ROWS_KERNEL", b"PFAAI_XCD_CHUNK", b"PFAAI_PL_PRIO", b"PFAAI_PL_LAUNCH_COLS",
               b"PFAAI_PL_WINDOWS", b"PFAAI_BLK_THREADS", b"PFAAI_BLK_QT_SPLIT", b"PFAAI_BLK_END_TILE",
               b"PFAAI_BLK_END_U", b"PFAAI_PL_KWMAX", b"PFAAI_PL_BIGF", b"PFAAI_PL_NREG", b"PFAAI_PL_V",
               b"PFAAI_PL_NOWK4", b"PFAAI_TRACE_COMPUTE", b"PFAAI_PL_T24", b"PFAAI_PL_STAG", b"PFAAI_PL_REV", b"PFAAI_SORT_DIRECT")


def test_release_library_ignores_diagnostic_switches():
    """The result-changing ablations, the stage-clock instrumentation and
    every A/B kernel switch exist only in libpfaai_hip_diag.so
    (-DPFAAI_DIAGNOSTICS): the release library does not even contain their
    names, so no environment can change its kernel choice or results.  The
    rejected k_rows_v2 of rounds 2-4 is compiled into neither."""
    blob = open(_capi.LIB_PATH, "rb").read()
    for name in (b"PFAAI_ABLATE", b"PFAAI_BLK_ABLATE", b"PFAAI_PL_CLK", b"PFAAI_DIV_NEWTON") + AB_SWITCHES:
        assert name not in blob, name
    assert b"k_rows_v2" not in blob
    diag = open(_capi.DIAG_LIB_PATH, "rb").read()
    for name in AB_SWITCHES:
        assert name in diag, name
    assert b"k_rows_v2" not in diag
