#!/bin/bash
# GPU box: k_local_cc per-phase clocks alone and inside the pipeline (tools/lcc_timing.py)
# with the timing build tools/ab/lcct.so installed for the run, then the default library back.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
cp rogtk_amd/librogtk_hip.so gpurun_out/.orig.so
cp tools/ab/${LCC_SO:-lcct}.so rogtk_amd/librogtk_hip.so
timeout -k 10 240 python3 tools/lcc_timing.py > gpurun_out/lcc_timing.log 2>&1
rc=$?
cp gpurun_out/.orig.so rogtk_amd/librogtk_hip.so
echo "lcc_timing rc=$rc"; tail -3 gpurun_out/lcc_timing.log
exit $rc
