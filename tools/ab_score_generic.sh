set -u
for g in 0 1 0 1; do ROGTK_SCORE_GENERIC=$g timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --iso-launches 20 > gpurun_out/b.log 2>&1 || exit 1; python -c "import json,sys; j=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print('generic', sys.argv[1], j['ms_per_step'], j['roofline']['frac'], j['roofline']['isolated']['avg_us'])" $g; done
