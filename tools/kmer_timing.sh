#!/bin/bash
# GPU box: swap in the ROGTK_KMER_TIMING library (box copy only) and print k_kmer_lds's phase split.
# Build it here first (a copy of the library with -DROGTK_KMER_TIMING in HIPFLAGS, saved as tools/ab/kt.so).
set -eu
cd "$GRAFT_REPO_ROOT"
cp tools/ab/kt.so rogtk_amd/librogtk_hip.so
timeout -k 10 180 python3 tools/kmer_timing.py "$@"
