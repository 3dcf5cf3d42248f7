#!/bin/bash
# Build the reference CLI (par_fastaai.x) from its own sources where they lie
# under /root/reference, into oracle/_ref/ (git-ignored; travels to the GPU
# box inside the snapshot).  Recipe from SURVEY.md §8c: the reference's
# sqlite3.c amalgamation is a missing blob, so it links the system
# libsqlite3.so.0 through the reference's own vendored sqlite3.h.  Nothing is
# copied out of /root/reference and nothing is written into it.
# Used only as a checker / CPU baseline (tests, bench.py cpu_baseline).
set -euo pipefail
R=${PFAAI_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
mkdir -p "$OUT"
g++ -std=c++17 -O2 -fopenmp -DNDEBUG \
    -I"$R/include" -I"$R/ext/sqlite" -I"$R/ext/fmt/include" \
    -I"$R/ext/CLI11/include" -I"$R/ext/cereal/include" \
    "$R/src/main.cpp" "$R/ext/fmt/src/format.cc" \
    /lib/x86_64-linux-gnu/libsqlite3.so.0 -ldl \
    -o "$OUT/par_fastaai.x"
echo "built $OUT/par_fastaai.x"
