"""The drop-in's producer (pfaai::DeviceE, include/pfaai_dropin.hpp; VERDICT
r05 missing #2 / next #4) against the reference's own construction, on the
CPU: a probe compiled from the reference's headers builds the same DB twice,
once through the reference's ParFAAIData / ParFAAIQSubData construct()
(constructLc / constructF / constructT over the SQLite UNION ALL,
ds_helper.hpp:46-162 and scp_db.hpp:161-262) and once through
DeviceE<...>::construct() (the parallel `<p>_genomes` ingest), and compares
refLc, refLp, refT and refF element by element -- refF assembled from the
lists on demand.  Cases: the reference's fixture DBs xdb_subset1/2 (all-vs-
all), the rebuilt C1 DB with the reference's -q list (query subset), and a
DB whose `<p>_genomes` blobs disagree with `<p>_tetras` at equal counts
(make_ref_vectors.mutate_equal_count): DeviceE must fall back to the
reference's construction there and still produce its arrays.  Skipped where
the reference sources are absent (the GPU box)."""
import gzip
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "main.cpp")),
                                reason="reference sources not present")

PROBE = r'''
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>
#include "pfaai/ds_impl.hpp"
#include "pfaai/interface.hpp"
#include "pfaai/scp_db.hpp"
#include "pfaai_hip.hpp"
using IdType = int;
using SQLiteDB = SQLiteSCPDataBase<IdType, DatabaseNames>;

template <class A, class B>
static int compare(A& ref, B& dev) {
    if (ref.construct() != PFAAI_OK || dev.construct() != PFAAI_OK) return 2;
    const auto &F1 = ref.refF(), &F2 = dev.refF();
    bool f = F1.size() == F2.size();
    for (std::size_t i = 0; f && i < F1.size(); ++i) f = F1[i].first == F2[i].first && F1[i].second == F2[i].second;
    const bool l = ref.refLc() == dev.refLc() && ref.refLp() == dev.refLp();
    const bool t = ref.refT() == dev.refT();
    std::printf("fast=%d lc_lp=%d t=%d f=%d nf=%zu\n", (int)dev.fastIngest(), (int)l, (int)t, (int)f, F2.size());
    return l && t && f ? 0 : 1;
}

int main(int argc, char** argv) {
    SQLiteDB db(argv[1]);
    if (db.validate() != PFAAI_OK) return 3;
    if (argc > 2) {  // -q list
        std::vector<std::string> q;
        std::ifstream in(argv[2]);
        for (std::string s; std::getline(in, s);)
            if (!s.empty()) q.push_back(s);
        ParFAAIQSubData<IdType> ref(db, db.getMeta(), q);
        pfaai::DeviceE<ParFAAIQSubData<IdType>> dev(db, db.getMeta(), q);
        return compare(ref, dev);
    }
    ParFAAIData<IdType> ref(db, db.getMeta());
    pfaai::DeviceE<ParFAAIData<IdType>> dev(db, db.getMeta());
    return compare(ref, dev);
}
'''


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    import dropin
    d = tmp_path_factory.mktemp("probe")
    src = d / "probe.cpp"
    src.write_text(PROBE)
    exe = str(d / "probe")
    lib = os.path.join(ROOT, "parfastaai_amd", "lib")
    cmd = ["g++", "-O1", *dropin.flags(), str(src), f"{REF}/ext/fmt/src/format.cc", "-L" + lib, "-lpfaai_hip",
           f"-Wl,-rpath,{lib}", "/lib/x86_64-linux-gnu/libsqlite3.so.0", "-ldl", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def _unpack(tmp, name):
    out = os.path.join(tmp, name)
    with gzip.open(os.path.join(ROOT, "tests", "golden", name + ".gz")) as fi, open(out, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    return out


def _run(probe, *args):
    r = subprocess.run([probe, *args], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="8"))
    line = [x for x in r.stdout.splitlines() if x.startswith("fast=")]
    assert r.returncode == 0 and line, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return line[0]


@pytest.mark.parametrize("name", ["xdb_subset1.db", "xdb_subset2.db"])
def test_deviceE_all_equals_reference_construction(probe, tmp_path, name):
    assert _run(probe, _unpack(str(tmp_path), name)).startswith("fast=1 lc_lp=1 t=1 f=1")


def test_deviceE_qsub_c1_equals_reference_construction(probe, tmp_path):
    from test_c1_loader import rebuild_xantho
    db = rebuild_xantho(str(tmp_path))
    q = _unpack(str(tmp_path), "qsub_test_input.txt")
    assert _run(probe, db, q).startswith("fast=1 lc_lp=1 t=1 f=1")


def test_deviceE_falls_back_when_orientations_differ(probe, tmp_path):
    import make_ref_vectors as mk
    from parfastaai_amd import syn
    _, kw = mk.CASES["mismatch24"]
    db = str(tmp_path / "m.db")
    syn.write_db(db, **kw)
    assert _run(probe, db).startswith("fast=1 lc_lp=1 t=1 f=1")
    mk.mutate_equal_count(db)
    assert _run(probe, db).startswith("fast=0 lc_lp=1 t=1 f=1")
