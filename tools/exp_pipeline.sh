set -e
mkdir -p gpurun_out
for a in "--depth 1" "--depth 3" "--depth 3 --prio=-1,0,0" "--depth 3 --prio=0,-1,0" "--depth 3 --prio=-1,-1,0" "--depth 2"; do
  echo "== $a" >> gpurun_out/exp.log
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline $a 2>>gpurun_out/exp.err | python -c "import json,sys; j=json.loads(sys.stdin.readlines()[-1]); print(j['ms_per_step'], j['kernels_us'])" >> gpurun_out/exp.log
done
cat gpurun_out/exp.log
