"""The reference-side binding of INTEGRATION.md §1 compiles against the
reference's own headers (CPU only, g++ -fsyntax-only; skipped where
/root/reference is absent).

  * the documented swap (INTEGRATION.md §1's diff, applied by
    tools/dropin.swap) on the reference's src/main.cpp (read at test time,
    never copied into this repository): include pfaai_hip.hpp, the three
    data-structure classes wrapped in pfaai::DeviceE (no E), and
    `using PFImpl = pfaai::ParFAAIHipImpl<IdType, ValueType, PFDSInterface>;`
    -- main.cpp:193, 256, 324 (`PFImpl pfaaiImpl(data)`), 196/260/327
    (`print_aji`) and printOutput (main.cpp:133-175) then compile unchanged
    (tests/test_gpu_dropin.py runs the linked binary);
  * ParFAAIHipImpl explicitly instantiated (every member) for the three
    reference DSIT classes ParFAAIData / ParFAAIQSubData / ParFAAIQryTgtData
    and for the abstract DefaultDataStructInterface;
  * pfaai_hip.h next to interface.hpp: no enumerator collides with
    enum PFAAI_ERROR_CODE (interface.hpp:39-44).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
MAIN = os.path.join(REF, "src", "main.cpp")

pytestmark = pytest.mark.skipif(not os.path.exists(MAIN), reason="reference sources not present")


def _flags():
    return ["g++", "-std=c++17", "-fopenmp", "-fsyntax-only", "-w", f"-I{REF}/include", f"-I{REF}/ext/sqlite",
            f"-I{REF}/ext/fmt/include", f"-I{REF}/ext/CLI11/include", f"-I{REF}/ext/cereal/include",
            f"-I{ROOT}/include"]


def test_integration_swap_compiles_in_reference_main(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import dropin

    src = dropin.swap(open(MAIN).read())
    assert "using PFImpl = pfaai::ParFAAIHipImpl<IdType, ValueType, PFDSInterface>;" in src
    assert "using PFData = pfaai::DeviceE<ParFAAIData<IdType>>;" in src
    assert "ParFAAIImpl<IdType, ValueType>" not in src
    f = tmp_path / "main_hip.cpp"
    f.write_text(src)
    r = subprocess.run(_flags() + [str(f)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]


def test_adapter_instantiates_for_reference_dsit_classes(tmp_path):
    f = tmp_path / "inst.cpp"
    f.write_text(r'''
#include "pfaai/algorithm_impl.hpp"
#include "pfaai/ds_impl.hpp"
#include "pfaai/interface.hpp"
#include "pfaai_hip.h"
#include "pfaai_hip.hpp"
#include <type_traits>
using IdType = int;
using ValueType = double;
template class pfaai::ParFAAIHipImpl<IdType, ValueType, DefaultDataStructInterface<IdType>>;
template class pfaai::ParFAAIHipImpl<IdType, ValueType, ParFAAIData<IdType>>;
template class pfaai::ParFAAIHipImpl<IdType, ValueType, ParFAAIQSubData<IdType>>;
template class pfaai::ParFAAIHipImpl<IdType, ValueType, ParFAAIQryTgtData<IdType>>;
static_assert(std::is_same<pfaai::ParFAAIHipImpl<IdType, ValueType, ParFAAIData<IdType>>::JACType,
                           JACTuple<IdType>>::value, "JACType");
static_assert(PFAAI_OK == PFAAI_RC_OK && PFAAI_ERR_SQLITE_DB == PFAAI_RC_SQLITE_DB &&
              PFAAI_ERR_SQLITE_MEM_ALLOC == PFAAI_RC_SQLITE_MEM_ALLOC && PFAAI_ERR_CONSTRUCT == PFAAI_RC_CONSTRUCT,
              "codes 0..3 are the reference's");
int one_arg(const ParFAAIData<IdType>& a, const ParFAAIQSubData<IdType>& q, const ParFAAIQryTgtData<IdType>& t) {
    pfaai::ParFAAIHipImpl<IdType, ValueType, ParFAAIData<IdType>> x(a);
    pfaai::ParFAAIHipImpl<IdType, ValueType, ParFAAIQSubData<IdType>> y(q);
    pfaai::ParFAAIHipImpl<IdType, ValueType, ParFAAIQryTgtData<IdType>> z(t);
    return x.run() + y.run() + z.run() + (int)x.getJAC().size() + (int)x.getAJI().size();
}
''')
    r = subprocess.run(_flags() + [str(f)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
