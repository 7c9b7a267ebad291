# Pipeline / mark-variant comparison on the GPU box (tools only; not part of the product).
set -e
mkdir -p gpurun_out
: > gpurun_out/exp.log
for a in "--depth 3" "--depth 3 --score-alone" "--depth 3 --mark fused --score-alone" "--depth 2 --score-alone"; do
  echo "== $a" >> gpurun_out/exp.log
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline $a 2>>gpurun_out/exp.err | python -c "import json,sys; j=json.loads(sys.stdin.readlines()[-1]); print(j['ms_per_step'], j['roofline']['frac'], j['kernels_us'])" >> gpurun_out/exp.log
done
cat gpurun_out/exp.log
