# One-off (round 6): the C3 digest test after the diagnostics-variant tests
# in one process, with this library and with a saved earlier build (PREV).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-c3ab}
mkdir -p $OUT
T="tests/test_gpu_stream.py::test_diagnostic_variants_equal_release_form tests/test_gpu_configs.py::test_c3_10k_all_vs_all_and_8way_rowblocks"
timeout -k 10 500 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $T > $OUT/cur.txt 2>&1
rc=$?
echo "cur rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PFAAI_HIP_LIB=$PREV timeout -k 10 500 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $T > $OUT/prev.txt 2>&1
echo "prev rc=$?"
