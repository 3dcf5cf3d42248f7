"""Names of the reference's 20-genome xantho test DB (config C1), as data.

The DB itself (data/modified_xantho_fastaai2.db) is a missing blob upstream
(.MISSING_LARGE_BLOBS:1); its arrays are committed fixtures
(xanthodb_{f_array,lc_array,t_matrix}.bin) and its names are listed by the
reference's tests (tests/pfaai_tests.hpp:23-39 TESTDB_PROTEIN_SET, 80 SCP
accessions in protein-index order; :159-179 TESTDB_GENOME_SET, 20 genome
names in genome-id order).  This script copies those two string lists, and
nothing else, into tests/golden/xantho_names.txt ("P <acc>" / "G <name>"
lines) for tools/rebuild_xantho_db.cpp.

Run in the build container only (the reference is absent on the GPU box):
    python tests/golden/make_xantho_names.py
"""
import os
import re

SRC = "/root/reference/tests/pfaai_tests.hpp"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xantho_names.txt")


def string_list(text, macro):
    body = re.search(r"#define\s+" + macro + r"\s+\\\s*\{(.*?)\}", text, re.S).group(1)
    return re.findall(r'"([^"]+)"', body)


def main():
    text = open(SRC).read()
    prot = string_list(text, "TESTDB_PROTEIN_SET")
    gen = string_list(text, "TESTDB_GENOME_SET")
    assert len(prot) == 80 and len(gen) == 20, (len(prot), len(gen))
    with open(DST, "w") as f:
        f.writelines(f"P {p}\n" for p in prot)
        f.writelines(f"G {g}\n" for g in gen)
    print(f"wrote {DST}: {len(prot)} proteins, {len(gen)} genomes")


if __name__ == "__main__":
    main()
