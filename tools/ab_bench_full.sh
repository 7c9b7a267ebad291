# A/B of two builds (abtmp/old.so vs abtmp/new.so): full bench JSON per run -> gpurun_out/ab_full.log
set -e
mkdir -p gpurun_out; : > gpurun_out/ab_full.log
for round in 1 2; do
  for v in old new; do
    cp abtmp/$v.so rogtk_amd/librogtk_hip.so
    r=$(timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline 2>>gpurun_out/ab.err | tail -1)
    echo "$v $r" >> gpurun_out/ab_full.log
    echo "$v $(echo "$r" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['ms_per_step'], j['roofline']['frac'], j['roofline']['isolated']['avg_us'], j['kernels_us']['score_packed'], j['kernels_us']['cluster_mark'], j['kernels_us']['cluster_assign'])")"
  done
done
