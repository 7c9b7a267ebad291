# A/B of two builds of librogtk_hip.so (tools/kt/old.so vs tools/kt/new.so, box copy only) on bench.py; tools only.
set -e
mkdir -p gpurun_out; : > gpurun_out/ab.log
for round in 1 2; do
  for v in old new; do
    cp tools/kt/$v.so rogtk_amd/librogtk_hip.so
    for w in ${WS:-1 8}; do
      r=$(timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --emulate-ranks $w 2>>gpurun_out/ab.err | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['ms_per_step'])")
      echo "$v W=$w $r" | tee -a gpurun_out/ab.log
    done
  done
done
