# A/B of an environment knob on bench.py: ENVA vs ENVB (e.g. ENVB="ROGTK_LABEL_BY_INDEX=1")
set -e
mkdir -p gpurun_out; : > gpurun_out/ab_env.log
for round in 1 2; do
  for v in A B; do
    if [ $v = A ]; then E="${ENVA:-}"; else E="${ENVB:-}"; fi
    r=$(env $E timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline 2>>gpurun_out/ab.err | tail -1)
    echo "$v $r" >> gpurun_out/ab_env.log
    echo "$v $(echo "$r" | python -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels_us']; print(j['ms_per_step'], j['roofline']['frac'], k['score_packed'], k['cluster_mark'], k['cluster_label'], k['cluster_assign'], j['config']['n_clusters'])")"
  done
done
