#!/bin/bash
# GPU box: interleaved A/B of library builds (the one parameterised A/B tool).
#   AB_ORDER   build names in run order; tools/ab/<name>.so must exist   (default "base new base new")
#   AB_CMD     the measured command, one JSON line last on stdout         (default: bench.py C2, 30 steps)
#   AB_KEYS    space-separated JSON keys printed per run (dotted = nested) (default "ms_per_step value")
#   AB_ENV_<name>  extra environment for that build's runs, e.g. AB_ENV_new="ROGTK_X=1"
#   AB_SO_<name>   the library a name runs (default tools/ab/<name>.so), e.g. AB_SO_ev=new
#   AB_ARGS_<name> extra arguments appended to AB_CMD for that name
#   PRE_TESTS  optional pytest selection run first on the LAST build of AB_ORDER ("" = none)
#   AB_T       per-run time limit in seconds (default 240)
# Stops at the first failing step; leaves the last build of AB_ORDER installed.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
ORDER=${AB_ORDER:-base new base new}
CMD=${AB_CMD:-python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-end-to-end --no-c3 --sustain-seconds 1}
KEYS=${AB_KEYS:-ms_per_step value}
last=${ORDER##* }
cp rogtk_amd/librogtk_hip.so gpurun_out/.orig.so 2>/dev/null
lastso="AB_SO_$last"; lastso=${!lastso:-$last}
if [ -n "${PRE_TESTS:-}" ]; then
    cp tools/ab/$lastso.so rogtk_amd/librogtk_hip.so
    timeout -k 10 ${TEST_T:-600} python3 -u -m pytest $PRE_TESTS -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_pretests.log 2>&1
    rc=$?; echo "pre-tests ($last) rc=$rc"; tail -3 gpurun_out/ab_pretests.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for v in $ORDER; do
    i=$((i + 1))
    soname="AB_SO_$v"; cp tools/ab/${!soname:-$v}.so rogtk_amd/librogtk_hip.so
    envname="AB_ENV_$v"; extra=${!envname:-}
    argname="AB_ARGS_$v"; args=${!argname:-}
    env $extra timeout -k 10 ${AB_T:-240} $CMD $args > gpurun_out/ab_${i}_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab_${i}_$v.log; exit $rc; }
    python3 - "$v" "$KEYS" gpurun_out/ab_${i}_$v.log <<'EOF'
import json, sys
name, keys, path = sys.argv[1], sys.argv[2].split(), sys.argv[3]
j = json.loads([l for l in open(path).read().splitlines() if l.startswith("{")][-1])
def get(d, k):
    for p in k.split("."):
        d = d.get(p) if isinstance(d, dict) else None
    return d
print(name, " ".join(f"{k}={get(j, k)}" for k in keys), flush=True)
EOF
done
cp tools/ab/$lastso.so rogtk_amd/librogtk_hip.so
