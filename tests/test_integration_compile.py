"""The reference-side binding of INTEGRATION.md §1 compiles against the
reference's own headers (CPU only, g++ -fsyntax-only; skipped where
/root/reference is absent).

  * the documented swap applied to the reference's src/main.cpp (read at
    test time, never copied into this repository): include pfaai_hip.hpp and
    `using PFImpl = pfaai::ParFAAIHipImpl<IdType, ValueType, PFDSInterface>;`
    -- main.cpp:193, 256, 324 (`PFImpl pfaaiImpl(data)`), 196/260/327
    (`print_aji`) and printOutput (main.cpp:133-175) then compile unchanged;
  * ParFAAIHipImpl explicitly instantiated (every member) for the three
    reference DSIT classes ParFAAIData / ParFAAIQSubData / ParFAAIQryTgtData
    and for the abstract DefaultDataStructInterface;
  * pfaai_hip.h next to interface.hpp: no enumerator collides with
    enum PFAAI_ERROR_CODE (interface.hpp:39-44).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
MAIN = os.path.join(REF, "src", "main.cpp")

pytestmark = pytest.mark.skipif(not os.path.exists(MAIN), reason="reference sources not present")


def _flags():
    return ["g++", "-std=c++17", "-fopenmp", "-fsyntax-only", "-w", f"-I{REF}/include", f"-I{REF}/ext/sqlite",
            f"-I{REF}/ext/fmt/include", f"-I{REF}/ext/CLI11/include", f"-I{REF}/ext/cereal/include",
            f"-I{ROOT}/include"]


def _integration_swap():
    """The two lines INTEGRATION.md §1 tells a maintainer to change."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    inc = re.search(r'^\+(#include "pfaai_hip.hpp".*)$', doc, re.M).group(1)
    using = re.search(r"^\+(using PFImpl = .*;)\s*$", doc, re.M).group(1)
    return inc, using


def test_integration_swap_compiles_in_reference_main(tmp_path):
    inc, using = _integration_swap()
    src = open(MAIN).read()
    old = "using PFImpl = ParFAAIImpl<IdType, ValueType>;"
    assert old in src
    src = src.replace('#include "pfaai/scp_db.hpp"', '#include "pfaai/scp_db.hpp"\n' + inc, 1).replace(old, using)
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
