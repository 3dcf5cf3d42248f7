"""Copy the reference's own test fixtures into tests/golden/ (gzip-compressed).

Provenance: every file listed in FIXTURES is a data file held by the reference's
own test-suite under /root/reference/data/ (see SURVEY.md §4 fixture inventory;
loaded by tests/pfaai_tests.cpp:49-120 of the reference).  They are inputs and
expected outputs (cereal binary archives, CSV matrices, SQLite DBs, query lists),
not source.  They are stored gzip-compressed so the repo stays small; the
loaders in parfastaai_amd/formats.py read them transparently.

Run (in the build container only; /root/reference is absent on the GPU box):
    python tests/golden/make_golden.py
"""
import gzip
import os
import shutil
import sys

SRC = "/root/reference/data"
DST = os.path.dirname(os.path.abspath(__file__))

FIXTURES = [
    # 20-genome xantho DB arrays + outputs (DB itself is a missing blob upstream)
    "xanthodb_lc_array.bin", "xanthodb_lp_array.bin", "xanthodb_f_array.bin",
    "xanthodb_t_matrix.bin", "xanthodb_jac.bin", "xanthodb_aji.bin",
    "xanthodb_e_size.bin", "xanthodb_e_starts.bin",
    "xanthodb_gpe_starts.bin", "xanthodb_gpe_ends.bin",
    "xanthodb_aji_matrix.csv", "xanthodb_aji_matrix_wheader.csv",
    # 4-genome subsets
    "xdb_subset1.db", "xdb_subset2.db", "xdb_subset_combo12.db",
    "xdb_subset1_lc_array.bin", "xdb_subset1_lp_array.bin", "xdb_subset1_f_array.bin",
    "xdb_subset1_t_matrix.bin", "xdb_subset1_sorted_e_array.bin",
    "xdb_subset1_jac.bin", "xdb_subset1_aji.bin", "xdb_subset1_aji_matrix_wheader.csv",
    "xdb_subset2_lc_array.bin", "xdb_subset2_lp_array.bin", "xdb_subset2_f_array.bin",
    "xdb_subset2_t_matrix.bin", "xdb_subset2_sorted_e_array.bin",
    "xdb_subset2_jac.bin", "xdb_subset2_aji.bin", "xdb_subset2_aji_matrix_wheader.csv",
    # query-subset (-q) mode on xantho
    "qsub_test_input.txt", "qsub_test_bad_input.txt",
    "xdb_qry_subset_jac.bin", "xdb_qry_subset_aji.bin",
    "qsub_test_output_matrix_wheader.csv",
    # query-vs-target (-r) mode subset1 x subset2
    "xdb_qt_lc_array.bin", "xdb_qt_lp_array.bin", "xdb_qt_f_array.bin",
    "xdb_qt_t_matrix.bin", "xdb_qt_combo_t_matrix.bin", "xdb_qt_sorted_e_array.bin",
    "xdb_qt_jac.bin", "xdb_qt_aji.bin",
]


def main():
    if not os.path.isdir(SRC):
        sys.exit(f"{SRC} not present (fixtures are only regenerated in the build container)")
    for name in FIXTURES:
        with open(os.path.join(SRC, name), "rb") as fi, \
                gzip.GzipFile(os.path.join(DST, name + ".gz"), "wb", mtime=0) as fo:
            shutil.copyfileobj(fi, fo)
    print(f"wrote {len(FIXTURES)} fixtures to {DST}")


if __name__ == "__main__":
    main()
