# Per-rank step time at N = 1, 2, 4, 8 emulated on one GPU (bench.py --emulate-ranks; tools only).
set -e
mkdir -p gpurun_out
: > gpurun_out/scal.log
for w in 1 2 4 8; do
  echo "== W=$w" >> gpurun_out/scal.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-ranks $w 2>>gpurun_out/scal.err | python -c "import json,sys; j=json.loads(sys.stdin.readlines()[-1]); print(j['ms_per_step'], j['value'], j['config']['n_distinct'], j['config']['n_clusters'], j['kernels_us'])" >> gpurun_out/scal.log
done
cat gpurun_out/scal.log
